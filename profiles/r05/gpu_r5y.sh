#!/bin/bash
# parity with 512-thread workgroups from the 3-per-CU class: parity (large/split), C3 + C4 full size
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_batches.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "c3 or c4" -x -q --timeout 900 --timeout-method thread > "$OUT/pytest_full.log" 2>&1 \
  || { echo "full size failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_full.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_full.log"
