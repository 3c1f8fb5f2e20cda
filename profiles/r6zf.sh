#!/bin/bash
# Round 6: the wave-priority default (k_small from its table loads to its window loads, k_large's
# staging) -- GPU suite and smoke on the new default, then C2 / C4 A/B against the previous library,
# and the pack-at-priority arm (pi)
set -o pipefail
O=gpurun_out/r6zf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
for i in 1 2; do
  for lib in profiles/_build/libbsdc_prev.so bsseqconsensusreads_amd/libbsdc.so profiles/_build/libbsdc_pi.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 4
  done
done
