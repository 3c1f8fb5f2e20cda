#!/bin/bash
# which families k_small takes: the small-arena cap (bigger small families go to k_large)
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in C3 C4 C2; do
  for cap in 24576 16384 12288 8192; do
    BSDC_SMALL_CAP=$cap timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_cap$cap.log" 2>&1 || { tail -20 "$OUT/bench_${c}_cap$cap.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_cap$cap.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c cap $cap ms', d['ms_per_step'], 'small', r['small_kernel_ms'], 'large', r['large_kernel_ms'])"
  done
done
