#!/bin/bash
# Round 6: byte-width FETCH/WRITE calibration, and C4's large set split per kernel instance
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
bash profiles/calib_fetch.sh $O/calib > $O/calib.log 2>&1 || exit 2
bash profiles/collect_pmc.sh $O/pmc_C4 --config C4 > $O/pmc_C4.log 2>&1 || exit 3
python profiles/pmc_instances.py $O/pmc_C4 $O/pmc_C4_instances.json > /dev/null || exit 4
find $O -type f -size +2M -delete
