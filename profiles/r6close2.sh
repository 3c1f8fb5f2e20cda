#!/bin/bash
# Round 6 closing check on the final tree (wave-priority default): the whole GPU suite, smoke and
# the default bench line (C2, CPU baseline)
set -o pipefail
O=gpurun_out/r6close2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 4
