#!/bin/bash
# Round-3 A/B on the GPU box: the whole -m gpu suite on the in-tree build, then the C2 / C3 / C4 bench
# per library (BSDC_LIB_PATH).  Usage (repo root): bash profiles/ab_round3.sh <tag> <lib.so>...
set -u -o pipefail
TAG=$1; shift
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" "$OUT/pytest_gpu.log" | head -20; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
for c in ${CFGS:-C2 C3 C4}; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    BSDC_LIB_PATH=$(realpath "$lib") timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 --steps 20 > "$OUT/bench_${c}_$n.log" 2>&1 \
      || { echo "bench $c $n failed"; tail -20 "$OUT/bench_${c}_$n.log"; exit 1; }
    echo "$c $n $(tail -1 "$OUT/bench_${c}_$n.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["small_kernel_ms"], r["large_kernel_ms"], d.get("tags_ms_per_step"))')"
  done
done
