#!/bin/bash
# Round 6 closing check on the final tree (after the k_join clamp): the whole GPU suite, smoke,
# the default bench line (C2, CPU baseline), C4's bench line, and rocprofv3 stats + spans + PMC
# of C4 (the kernel that changed)
set -o pipefail
O=gpurun_out/r6close
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --config C4 --cpu-sample 100000 --cpu-sample-1core 20000 > $O/bench_C4.log 2>&1 || exit 5
CONFIGS="C4" timeout -k 10 900 bash profiles/prof_round.sh r6close/prof > $O/prof_round.log 2>&1 || exit 6
