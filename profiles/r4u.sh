#!/bin/bash
# Round-4: split families in groups, each group's parts and join on a stream of their own
# (BSDC_SPLIT_GROUPS 1 / 2 / 4 / 8): parity, then C4 bench.
set -u -o pipefail
OUT=gpurun_out/r4u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
BSDC_SPLIT_GROUPS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k split --timeout 300 \
  --timeout-method thread > $OUT/pytest_g1.log 2>&1 || { echo "tests g1 failed"; tail -5 $OUT/pytest_g1.log; exit 1; }
tail -1 $OUT/pytest_g1.log
CFGS="C4" bash profiles/ab_r4.sh r4u g1=-:BSDC_SPLIT_GROUPS=1 g2=-:BSDC_SPLIT_GROUPS=2 g4=- g8=-:BSDC_SPLIT_GROUPS=8 g1b=-:BSDC_SPLIT_GROUPS=1 g4b=-
