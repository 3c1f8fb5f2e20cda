#!/bin/bash
# Round 6, tag-leg store ablation (profiles/tag_variants.py st1 st2 st3): the fast path's tag
# stores one at a time; the tree's library is the control
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
for i in 1 2; do
  for n in tree st1 st2 st3; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/tv_${i}_$n.log 2>&1 || exit 5
  done
done
