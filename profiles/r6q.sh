#!/bin/bash
# Round 6 closing check on the final tree: the whole GPU suite, smoke, the default bench line
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 4
