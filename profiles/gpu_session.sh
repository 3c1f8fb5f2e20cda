#!/bin/bash
# One GPU-box session: parity tests, the bench line, a rocprofv3 kernel-trace summary and the
# per-phase ablation of k_small.  Usage (repo root, on the box): bash profiles/gpu_session.sh <tag>
# Every GPU step has its own time limit; the script stops at the first failure.
set -u -o pipefail
TAG=${1:-r01}
R=$(pwd)
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest-gpu
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "gpu tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
step bench
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
step rocprof-stats
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$R/bench.py" --steps 10 --cpu-sample 0 > "$OUT/prof.log" 2>&1) \
  || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -type f | head -20; find "$OUT/prof" -name '*kernel_stats.csv' -exec head -6 {} \;
step ablate
timeout -k 10 300 python -u profiles/ablate.py > "$OUT/ablate.log" 2>&1 || { echo "ablate failed"; tail -20 "$OUT/ablate.log"; exit 1; }
tail -1 "$OUT/ablate.log"
if [ "${PMC:-1}" = 1 ]; then
  step pmc
  bash profiles/collect_pmc.sh "$OUT/pmc" || exit 1
  python profiles/pmc_bench_summary.py "$OUT/pmc" "$OUT/pmc_summary.json" | head -60
  step pmc-ablate
  bash profiles/collect_pmc_ablate.sh "$OUT/pmca" || exit 1
  python profiles/pmc_summary.py "$OUT/pmca" > "$OUT/pmca_summary.json"; head -80 "$OUT/pmca_summary.json"
fi
step prune
find "$OUT" -type f -size +2M -print -delete
du -sh "$OUT"
step done
