#!/bin/bash
# which change breaks C4 full size / the fused-join arm: selects (pick4) or the OR records
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
for v in new; do
  case $v in nopick) LP="$B/libbsdc_nopick.so";; *) LP="";; esac
  BSDC_LIB_PATH="$LP" BSDC_SPLIT_JOIN=part timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k split -q --timeout 300 --timeout-method thread > "$OUT/pytest_partjoin_$v.log" 2>&1
  echo "part-join $v rc=$?"; grep -E "^FAILED|passed|failed" "$OUT/pytest_partjoin_$v.log" | tail -4
  BSDC_LIB_PATH="$LP" timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "c4_bench" -q --timeout 380 --timeout-method thread > "$OUT/pytest_c4_$v.log" 2>&1
  echo "c4 $v rc=$?"; grep -E "^E  |passed|failed" "$OUT/pytest_c4_$v.log" | tail -4
done
