#!/bin/bash
# Round-4: k_small's queue walking two reads at a time (ablibs/libbsdc_q2.so): parity + fp64 suites
# through it, then C2 / C1 / C4 bench against the same source without the change (libbsdc_base.so).
set -u -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_q2.so) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_q2.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_q2.log | head; tail -5 $OUT/pytest_q2.log; exit 1; }
tail -1 $OUT/pytest_q2.log
CFGS="C2 C1 C4" bash profiles/ab_r4.sh r4n base=ablibs/libbsdc_base.so q2=ablibs/libbsdc_q2.so base2=ablibs/libbsdc_base.so q2b=ablibs/libbsdc_q2.so
