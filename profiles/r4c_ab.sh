set -u -o pipefail
CFGS="C4 C3" bash profiles/ab_r4.sh r4c base=- nopart=-:BSDC_PART_CAP=0 split4=-:BSDC_SPLIT_FROM=4 split3=-:BSDC_SPLIT_FROM=3 persist=ablibs/libbsdc_persist.so \
 && CFGS="C2" bash profiles/ab_r4.sh r4c base=- persist=ablibs/libbsdc_persist.so \
 && CONFIGS="C4" SKIP_PMC=1 bash profiles/prof_round.sh r4c
