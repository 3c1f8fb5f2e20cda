#!/bin/bash
# Round 6: k_small's overlap dwords flattened over the wave (prefix sum of the templates' dwords)
# -- parity, then C2 / C4 A/B against the previous library
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
for i in 1 2; do
  for lib in profiles/_build/libbsdc_prev.so bsseqconsensusreads_amd/libbsdc.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_$n.log 2>&1 || exit 3
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 4
  done
done
