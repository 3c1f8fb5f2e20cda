#!/bin/bash
# Round 6, first GPU session: the staging probe, the GPU suite after the dead-arm removal, a bench line
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u profiles/probe_stage.py > $O/probe.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench.log 2>&1 || exit 3
