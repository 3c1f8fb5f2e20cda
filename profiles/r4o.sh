#!/bin/bash
set -u -o pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_parity.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest_parity.log | head; tail -5 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
