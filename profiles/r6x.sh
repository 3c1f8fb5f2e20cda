#!/bin/bash
# Round 6: k_large's overlap task map by multiply-high (TaskDiv) and 16-B task entries -- large /
# split / C3 / C4 parity, then C3 and C4 A/B against the previous library
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "split or c3 or C3 or c4 or C4 or large or join or messy or golden or tool" --timeout 300 --timeout-method thread > $O/pytest_large.log 2>&1 || exit 2
for i in 1 2; do
  for lib in profiles/_build/libbsdc_prev.so bsseqconsensusreads_amd/libbsdc.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --config C3 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c3_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
