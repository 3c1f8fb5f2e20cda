#!/bin/bash
# Round 6: k_small per-phase PMC on C2 (instructions, waits, LDS bank conflicts per phase)
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
bash profiles/collect_pmc_ablate.sh $O/pmc_ablate --config C2 > $O/pmc_ablate.log 2>&1 || exit 2
python profiles/pmc_phases.py $O/pmc_ablate small > $O/pmc_phases_C2.txt 2>&1 || exit 3
find $O -type f -size +2M -delete
