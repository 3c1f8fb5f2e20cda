#!/bin/bash
# The -m gpu tests selected by -k <expr> against each library given (BSDC_LIB_PATH), then the
# default build.  Usage: bash profiles/ab_test.sh <tag> <expr> <lib.so>...
set -u -o pipefail
TAG=$1; K=$2; shift 2
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for lib in "$@" default; do
  n=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset BSDC_LIB_PATH; else export BSDC_LIB_PATH=$(realpath "$lib"); fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 240 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -1 "$OUT/pytest_$n.log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
