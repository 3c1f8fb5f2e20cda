#!/bin/bash
# Round-4: fused join (the family's last part joins it; -DJOIN_FUSED=1): part-mode parity through
# that build, then C4 / C3 bench against the in-tree build (separate k_join dispatch).
set -u -o pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_joinfused.so) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
  -k "split or large or C4" --timeout 300 --timeout-method thread > $OUT/pytest_fused.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_fused.log | head; tail -5 $OUT/pytest_fused.log; exit 1; }
tail -1 $OUT/pytest_fused.log
CFGS="C4 C3" bash profiles/ab_r4.sh r4i base=- fused=ablibs/libbsdc_joinfused.so
