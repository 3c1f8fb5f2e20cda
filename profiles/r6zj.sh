#!/bin/bash
# Round 6: k_large's staging priority dropped before the record metadata loop (le0) instead of after
# the staging reduction (the tree), C3 and C4
set -o pipefail
O=gpurun_out/r6zj
mkdir -p $O
for i in 1 2; do
  for n in cur le0; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C3 --steps 10 --cpu-sample 0 --no-tags-leg > $O/c3_${i}_$n.log 2>&1 || exit 4
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 5
  done
done
