#!/bin/bash
# Round 6: k_join at priority 3 through its table loads + k_large from the kernel entry (qa); k_small
# image chunk loads in flight per lane 2 (qb) and 8 (qc) under the priority default; against cur
set -o pipefail
O=gpurun_out/r6zh
mkdir -p $O
for i in 1 2; do
  for n in cur qb qc; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 --no-tags-leg > $O/c2_${i}_$n.log 2>&1 || exit 3
  done
  for n in cur qa; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C3 --steps 10 --cpu-sample 0 --no-tags-leg > $O/c3_${i}_$n.log 2>&1 || exit 4
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 5
  done
done
