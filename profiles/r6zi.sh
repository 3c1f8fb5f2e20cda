#!/bin/bash
# Round 6: k_small at 8 waves per SIMD (SMALL_WAVES=8: 63 VGPRs, 54 SGPRs spilled to VGPR lanes)
# under the wave-priority default, against the tree (7 waves)
set -o pipefail
O=gpurun_out/r6zi
mkdir -p $O
for i in 1 2; do
  for n in cur w8; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
