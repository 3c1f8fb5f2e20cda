#!/bin/bash
# Round 6: the rank path on seven contigs (region cuts) and the other rank / long-span GPU tests
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_fleet.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ranks.log 2>&1 || exit 2
