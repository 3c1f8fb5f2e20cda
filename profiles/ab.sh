#!/bin/bash
# A/B of k_small builds on the GPU box: parity tests on the default build, then bench + per-phase
# ablation for each library given.  Usage: bash profiles/ab.sh <tag> <lib.so>...
set -u -o pipefail
TAG=$1; shift
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { echo "gpu tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u bench.py --cpu-sample 0 > "$OUT/bench_$n.log" 2>&1 \
    || { echo "bench $n failed"; tail -20 "$OUT/bench_$n.log"; exit 1; }
  echo "$n $(tail -1 "$OUT/bench_$n.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u profiles/ablate.py > "$OUT/ablate_$n.log" 2>&1 \
    || { echo "ablate $n failed"; tail -20 "$OUT/ablate_$n.log"; exit 1; }
  tail -1 "$OUT/ablate_$n.log"
done
