#!/bin/bash
# Round 6: k_small cut for 8 waves per SIMD with no VGPR spill (-DSMALL_WAVES=8 -DSMALL_SGPRS=96:
# 63 VGPRs, SGPRs spilled to VGPR lanes) against the tree (65 VGPRs, 7 waves), C2 and C4
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
for i in 1 2; do
  for n in tree w8; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
