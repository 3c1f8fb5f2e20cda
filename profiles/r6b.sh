#!/bin/bash
# Round 6, second GPU session: the GPU suite with deferred long-span templates, the bench line,
# CLI wall time one process vs two ranks on GPU 0
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || exit 3
timeout -k 10 600 python -u profiles/e2e_cli.py --families 1000000 --reps 2 > $O/e2e_cli.log 2>&1 || exit 4
