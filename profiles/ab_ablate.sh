#!/bin/bash
# Per-phase ablation of alternative builds (BSDC_LIB_PATH) on one GPU box, after the default
# build's parity tests.  Usage: bash profiles/ab_ablate.sh <tag> <config> <small|large> <lib.so>...
set -u -o pipefail
TAG=$1; CFG=$2; KER=$3; shift 3
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 200 python -u profiles/ablate.py --config $CFG --kernel $KER > "$OUT/ablate_${CFG}_$n.log" 2>&1 \
    || { echo "ablate $n failed"; tail -20 "$OUT/ablate_${CFG}_$n.log"; exit 1; }
  echo "$n $(tail -1 "$OUT/ablate_${CFG}_$n.log")"
done
