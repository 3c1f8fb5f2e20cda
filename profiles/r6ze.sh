#!/bin/bash
# Round 6: wave-priority variants, second set -- pe (k_small staging + k_large staging at 3), pf (pe +
# k_large convert's reference-load issue at 3), pg (k_small from the kernel's table loads on + k_large staging)
set -o pipefail
O=gpurun_out/r6ze
mkdir -p $O
for i in 1 2; do
  for n in prev pe pg; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
  done
  for n in prev pe pf pg; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C3 --steps 10 --cpu-sample 0 --no-tags-leg > $O/c3_${i}_$n.log 2>&1 || exit 4
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 5
  done
done
