#!/bin/bash
# Round 6: k_small's tables by LDS-DMA with the workgroup barrier at the end of staging (tdma) --
# parity subset on that library, then C2 / C4 A/B against the tree's (cur)
set -o pipefail
O=gpurun_out/r6zg
mkdir -p $O
BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_tdma.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "parity or fp64 or c2 or C2 or batches or golden or tags or small" --timeout 300 --timeout-method thread > $O/pytest_tdma.log 2>&1 || exit 2
for i in 1 2; do
  for n in cur tdma; do
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
