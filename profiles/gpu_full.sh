#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke(), then the C2 (headline) and C3 benches without the
# CPU baseline.  Usage: bash profiles/gpu_full.sh <tag>
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for c in C2 C3; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 --cpu-sample-1core 0 > "$OUT/bench_$c.log" 2>&1 || { echo "bench $c failed"; tail -20 "$OUT/bench_$c.log"; exit 1; }
  echo "$c $(tail -1 "$OUT/bench_$c.log" | cut -c1-300)"
done
