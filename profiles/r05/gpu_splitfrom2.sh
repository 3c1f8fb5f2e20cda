#!/bin/bash
# cutting the 2-per-CU class into parts again, now that part records are smaller (C3, C4)
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in C3 C4; do
  for v in 4 3 4b 3b; do
    BSDC_SPLIT_FROM=${v:0:1} timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c split_from $v ms', d['ms_per_step'], 'small', r.get('small_kernel_ms'), 'large', r.get('large_kernel_ms'))"
  done
done
