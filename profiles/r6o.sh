#!/bin/bash
# Round 6: k_large per-phase stops on C3 (profiles/ablate.py --kernel large)
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 400 python profiles/ablate.py --config C3 --kernel large > $O/ablate_C3.log 2>&1 || exit 2
