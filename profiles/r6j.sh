#!/bin/bash
# Round 6, tag-leg ablation on the whole-dword stores (profiles/tag_variants.py nofast st1 nocount)
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
for i in 1 2; do
  for n in tree nofast st1 nocount; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/tv_${i}_$n.log 2>&1 || exit 5
  done
done
