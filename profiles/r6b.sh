#!/bin/bash
# Round 6, second GPU session: the GPU suite with deferred long-span templates, the bench line,
# CLI wall time one process vs two ranks on GPU 0
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit 3
timeout -k 10 600 python -u profiles/e2e_cli.py --families 1000000 --reps 2 > $O/e2e_cli.log 2>&1 || exit 4
# A/B: k_small's list entry by one scalar load (the tree's library) against the build before it
for i in 1 2; do
  for lib in profiles/_build/libbsdc_head.so bsseqconsensusreads_amd/libbsdc.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 --no-tags-leg > $O/ab_${i}_$n.log 2>&1 || exit 5
  done
done
