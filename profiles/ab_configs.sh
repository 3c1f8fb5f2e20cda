#!/bin/bash
# A/B of kernel builds on the GPU box over several configs: GPU parity on each library (first
# library's full suite, large-family tests for the rest), then bench per config and library.
# Usage: bash profiles/ab_configs.sh <tag> "<configs>" <lib.so>...
set -u -o pipefail
TAG=$1; CFGS=$2; shift 2
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 \
    || { echo "gpu tests failed ($n)"; tail -30 "$OUT/pytest_$n.log"; exit 1; }
  echo "$n $(tail -1 "$OUT/pytest_$n.log")"
done
for c in $CFGS; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 > "$OUT/bench_${c}_$n.log" 2>&1 \
      || { echo "bench $c $n failed"; tail -20 "$OUT/bench_${c}_$n.log"; exit 1; }
    echo "$c $n $(tail -1 "$OUT/bench_${c}_$n.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms"], r["large_kernel_ms"])')"
  done
done
