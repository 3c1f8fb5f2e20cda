#!/bin/bash
# rank-parallel file path + k_pair parity on the GPU
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_fleet.py "tests/test_gpu_parity.py::test_pair_small_kernel_vs_oracle" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
grep -E "PASSED|FAILED" "$OUT/pytest.log" | tail -12; tail -1 "$OUT/pytest.log"
