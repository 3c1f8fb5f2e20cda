#!/bin/bash
# which large classes to cut into parts now that parts stage in chunks: C3 and C4
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in C3 C4; do
  for sf in 5 4 3 2; do
    BSDC_SPLIT_FROM=$sf timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_sf$sf.log" 2>&1 || { tail -20 "$OUT/bench_${c}_sf$sf.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_sf$sf.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c split_from $sf ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
  done
done
