#!/bin/bash
# Round 6 final profile (tree at this commit): rocprofv3 kernel-trace stats + launch-set spans +
# PMC passes of bench.py on C2, C3 and C4 (profiles/prof_round.sh)
set -o pipefail
CONFIGS="C2 C3 C4" timeout -k 10 1100 bash profiles/prof_round.sh r06final > gpurun_out/r06final.log 2>&1 || exit 2
