#!/bin/bash
# Round-4: k_large's LDS-heavy classes at 768 threads (three waves per set in the vote;
# -DLARGE_THREADS_BIG=768) against 512: parity through both builds, then C3 / C4 bench.
set -u -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $OUT/pytest_512.log 2>&1 || { echo "tests 512 failed"; grep -E "FAILED|Error" $OUT/pytest_512.log | head; tail -5 $OUT/pytest_512.log; exit 1; }
tail -1 $OUT/pytest_512.log
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_t768.so) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_768.log 2>&1 || { echo "tests 768 failed"; grep -E "FAILED|Error" $OUT/pytest_768.log | head; tail -5 $OUT/pytest_768.log; exit 1; }
tail -1 $OUT/pytest_768.log
CFGS="C3 C4" bash profiles/ab_r4.sh r4p t512=- t768=ablibs/libbsdc_t768.so t512b=- t768b=ablibs/libbsdc_t768.so
