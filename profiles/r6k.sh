#!/bin/bash
# Round 6: kernel-argument output pointers re-read where they are stored through (fewer SGPR
# spills) -- tags only (vol) and tags + the consensus stores (volall) against the tree
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
for i in 1 2; do
  for n in tree vol volall; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/tv_${i}_$n.log 2>&1 || exit 5
  done
done
