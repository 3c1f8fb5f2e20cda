#!/bin/bash
# dispatch order: small families first (default) vs large first, C3 and C4 steps; parity on large-first
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
BSDC_LARGE_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_lf.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_lf.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_lf.log"
for c in C3 C4; do
  for lf in 0 1; do
    BSDC_LARGE_FIRST=$lf timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_lf$lf.log" 2>&1 || { tail -20 "$OUT/bench_${c}_lf$lf.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_lf$lf.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c large_first=$lf ms', d['ms_per_step'], 'value', d['value'])"
  done
done
