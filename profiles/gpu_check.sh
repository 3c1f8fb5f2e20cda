#!/bin/bash
# One GPU call: parity (the whole -m gpu suite, or the tests named in $TESTS), then the C2 bench and
# the per-phase ablations of both kernels.  Usage: bash profiles/gpu_check.sh <tag> [pytest -k expr]
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "gpu tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "gpu tests failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
fi
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u profiles/ablate.py --config C3 --kernel large > "$OUT/ablate_C3.log" 2>&1 || { tail -20 "$OUT/ablate_C3.log"; exit 1; }
tail -1 "$OUT/ablate_C3.log"
timeout -k 10 200 python -u profiles/ablate.py --config C2 > "$OUT/ablate_C2.log" 2>&1 || { tail -20 "$OUT/ablate_C2.log"; exit 1; }
tail -1 "$OUT/ablate_C2.log"
