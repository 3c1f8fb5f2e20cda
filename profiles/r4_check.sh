#!/bin/bash
# Round-4 GPU check: the -m gpu suite (the parity / fp64 / stream files first, then the rest),
# smoke(), the driver's default bench line, optional extra bench configs and the end-to-end timing
# of the given modes.  Usage (repo root, on the box):
#   bash profiles/r4_check.sh <tag> [e2e modes, comma-separated] [bench configs, comma-separated]
set -u -o pipefail
TAG=$1
OUT="gpurun_out/$TAG"
mkdir -p "$OUT"
echo "[$(date +%T)] pytest-gpu (parity, fp64, stream)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_stream.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_a.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu_a.log" | head -20; tail -5 "$OUT/pytest_gpu_a.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_a.log"
echo "[$(date +%T)] pytest-gpu (the rest)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  --deselect tests/test_gpu_parity.py --deselect tests/test_gpu_fp64.py --deselect tests/test_gpu_stream.py \
  > "$OUT/pytest_gpu_b.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu_b.log" | head -20; tail -5 "$OUT/pytest_gpu_b.log"; exit 1; }
tail -1 "$OUT/pytest_gpu_b.log"
echo "[$(date +%T)] smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
for cfg in $(echo "${3:-}" | tr ',' ' '); do
  echo "[$(date +%T)] bench $cfg"
  timeout -k 10 400 python -u bench.py --config "$cfg" --cpu-sample 0 > "$OUT/bench_$cfg.log" 2>&1 || { tail -20 "$OUT/bench_$cfg.log"; exit 1; }
  tail -1 "$OUT/bench_$cfg.log" | cut -c1-300
done
if [ -n "${2:-}" ]; then
  echo "[$(date +%T)] e2e $2"
  timeout -k 10 800 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --modes "$2" > "$OUT/e2e.log" 2>&1 \
    || { tail -20 "$OUT/e2e.log"; exit 1; }
  tail -4 "$OUT/e2e.log" | cut -c1-600
fi
echo "[$(date +%T)] done"
