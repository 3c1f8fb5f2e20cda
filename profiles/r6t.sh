#!/bin/bash
# Round 6: k_small waves per SIMD capped by LDS padding (profiling builds, -DSMALL_CAP_WAVES=5, 6)
# against the tree (7 by registers), C2 and C4, alternated
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
for i in 1 2; do
  for n in tree cap6 cap5; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
