#!/bin/bash
# Round 6: the tag leg's whole-dword single-strand stores -- tag parity, then the bench twice
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_tags.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/bench_$i.log 2>&1 || exit 3
done
