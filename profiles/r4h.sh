#!/bin/bash
# Round-4: smaller parts (BSDC_PART_CAP) and cutting the 1- / 2-per-CU classes too (BSDC_SPLIT_FROM)
set -u -o pipefail
CFGS="C4" bash profiles/ab_r4.sh r4h cap26k=-:BSDC_PART_CAP=26000 cap22k=-:BSDC_PART_CAP=22000 cap18k=-:BSDC_PART_CAP=18000 \
  s4cap27k=-:BSDC_PART_CAP=27840,BSDC_SPLIT_FROM=4 s3cap27k=-:BSDC_PART_CAP=27840,BSDC_SPLIT_FROM=3 || exit 1
CFGS="C3" bash profiles/ab_r4.sh r4h base=- s4cap27k=-:BSDC_PART_CAP=27840,BSDC_SPLIT_FROM=4 s3cap27k=-:BSDC_PART_CAP=27840,BSDC_SPLIT_FROM=3
