#!/bin/bash
# Round 6: k_small wave priority (s_setprio) A/B -- SMALL_PRIO=1 (staging issues at priority 3),
# SMALL_PRIO=2 (the phases after staging at priority 2) against the tree's library, C2 and C4
set -o pipefail
O=gpurun_out/r6zc
mkdir -p $O
for i in 1 2; do
  for lib in profiles/_build/libbsdc_prev.so profiles/_build/libbsdc_prio1.so profiles/_build/libbsdc_prio2.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
