#!/bin/bash
# Round 6: wave-priority variants -- k_small staging at priority 3 until the window loads (pa), until
# the image loads (pb), until staging ends (pc), at priority 1 (pd); pa + k_large staging at 3 (pe)
set -o pipefail
O=gpurun_out/r6zd
mkdir -p $O
for i in 1 2; do
  for n in prev pa pb pc pd; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
  done
  for n in prev pa pe; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C3 --steps 10 --cpu-sample 0 --no-tags-leg > $O/c3_${i}_$n.log 2>&1 || exit 4
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 5
  done
done
