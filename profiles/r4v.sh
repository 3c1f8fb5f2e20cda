#!/bin/bash
# Round-4 cleanup check: parity / fp64 / stream suites, smoke and the C2 / C4 bench after the
# persistent and split-first variants left the code.
set -u -o pipefail
OUT=gpurun_out/r4v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_stream.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
CFGS="C2 C4" bash profiles/ab_r4.sh r4v head=-
