#!/bin/bash
# Round-4: part size A/B on C4 (BSDC_PART_CAP: the part arena cap, i.e. 5 / 4 / 3 / 2 workgroups per CU)
set -u -o pipefail
CFGS="C4" bash profiles/ab_r4.sh r4g cap27k=-:BSDC_PART_CAP=27840 cap36k=-:BSDC_PART_CAP=36032 cap49k=- cap77k=-:BSDC_PART_CAP=76992 nopart=-:BSDC_PART_CAP=0
