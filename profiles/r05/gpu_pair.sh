#!/bin/bash
# Round 5: k_pair (two families per wavefront) parity + the C2 bench against k_small on one box.
# Usage: bash profiles/r05/gpu_pair.sh <tag> [pytest -k expr]
set -u -o pipefail
TAG=$1
K=${2:-}
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -v -k "$K" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
fi
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-tags-leg > "$OUT/bench_pair.log" 2>&1 || { tail -20 "$OUT/bench_pair.log"; exit 1; }
tail -1 "$OUT/bench_pair.log" | cut -c1-400
BSDC_SMALL_KERNEL=wave timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-tags-leg > "$OUT/bench_wave.log" 2>&1 || { tail -20 "$OUT/bench_wave.log"; exit 1; }
tail -1 "$OUT/bench_wave.log" | cut -c1-400
