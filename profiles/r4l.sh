#!/bin/bash
# Round-4: the part -> join chain launched before the classes (-DSPLIT_FIRST=1) on C4, twice each.
set -u -o pipefail
CFGS="C4" bash profiles/ab_r4.sh r4l base=- splitfirst=ablibs/libbsdc_splitfirst.so base2=- splitfirst2=ablibs/libbsdc_splitfirst.so
