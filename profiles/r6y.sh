#!/bin/bash
# Round 6: the N-rank bench rehearsed on one GPU (2 and 4 ranks on device 0, gloo collectives)
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_ranks.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_bench_ranks.log 2>&1 || exit 2
timeout -k 10 300 python -u profiles/rehearse_bench_ranks.py --ranks 2 -- --steps 10 --cpu-sample 0 --no-tags-leg > $O/rehearse_2x1M.log 2>&1 || exit 3
timeout -k 10 300 python -u profiles/rehearse_bench_ranks.py --ranks 4 -- --families 250000 --steps 10 --cpu-sample 0 --no-tags-leg > $O/rehearse_4x250K.log 2>&1 || exit 4
