#!/bin/bash
# Round 6: k_small per-phase stops on C2 (profiles/ablate.py), the tree's library
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 300 python profiles/ablate.py --config C2 > $O/ablate_C2.log 2>&1 || exit 2
