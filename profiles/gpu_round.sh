#!/bin/bash
# One GPU call per milestone: the -m gpu suite, smoke(), the driver's default bench line (with the
# CPU baselines), then the C2/C3 rocprofv3 stats + PMC passes (prof_round.sh) and the streaming
# end-to-end file timing.  Usage (repo root, on the box): bash profiles/gpu_round.sh <tag> [skip-e2e]
set -u -o pipefail
TAG=$1
R=$(pwd)
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
echo "[$(date +%T)] pytest-gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "[$(date +%T)] smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[$(date +%T)] bench (driver default)"
timeout -k 10 400 python -u bench.py > "$OUT/bench_default.log" 2>&1 || { tail -20 "$OUT/bench_default.log"; exit 1; }
tail -1 "$OUT/bench_default.log" | cut -c1-400
echo "[$(date +%T)] ablate"
timeout -k 10 200 python -u profiles/ablate.py --config C3 --kernel large > "$OUT/ablate_C3.log" 2>&1 || { tail -20 "$OUT/ablate_C3.log"; exit 1; }
tail -1 "$OUT/ablate_C3.log"
timeout -k 10 200 python -u profiles/ablate.py --config C2 > "$OUT/ablate_C2.log" 2>&1 || { tail -20 "$OUT/ablate_C2.log"; exit 1; }
tail -1 "$OUT/ablate_C2.log"
[ "${NOPROF:-0}" = 1 ] || bash profiles/prof_round.sh "$TAG/prof" || exit 1
if [ "${2:-}" != "skip-e2e" ]; then
  echo "[$(date +%T)] e2e stream"
  timeout -k 10 500 python -u profiles/e2e_stream.py --families 1000000 --threads 16 > "$OUT/e2e_stream.log" 2>&1 \
    || { tail -20 "$OUT/e2e_stream.log"; exit 1; }
  tail -5 "$OUT/e2e_stream.log"
fi
echo "[$(date +%T)] done"
