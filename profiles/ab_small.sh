#!/bin/bash
# A/B of k_small builds on the GPU box: the C0-C2 GPU parity tests per library, then the C2 and C1
# bench per library.  Usage: bash profiles/ab_small.sh <tag> <lib.so>...
set -u -o pipefail
TAG=$1; shift
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "C0 or C1 or C2 or golden or reference or empty or messy" --timeout 200 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 \
    || { echo "gpu tests failed ($n)"; tail -30 "$OUT/pytest_$n.log"; exit 1; }
  echo "$n $(tail -1 "$OUT/pytest_$n.log")"
done
for c in ${CFGS:-C2 C1}; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 --steps 20 > "$OUT/bench_${c}_$n.log" 2>&1 \
      || { echo "bench $c $n failed"; tail -20 "$OUT/bench_${c}_$n.log"; exit 1; }
    echo "$c $n $(tail -1 "$OUT/bench_${c}_$n.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["small_kernel_ms"], r["large_kernel_ms"])')"
  done
done
