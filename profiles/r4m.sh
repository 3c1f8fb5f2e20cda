#!/bin/bash
# Round-4: k_small's register budget cut for 8 waves per SIMD (-DSMALL_WAVES=8) against 7.
set -u -o pipefail
CFGS="C2 C1" bash profiles/ab_r4.sh r4m base=- w8=ablibs/libbsdc_w8.so base2=- w8b=ablibs/libbsdc_w8.so
