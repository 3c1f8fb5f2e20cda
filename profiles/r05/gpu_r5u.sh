#!/bin/bash
# part size A/B on C4 after contiguous part images (BSDC_PART_CAP: 5, 4, 3 parts per CU)
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for cap in 27840 36032 49680; do
  BSDC_PART_CAP=$cap timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 2 --cpu-sample 0 --no-tags-leg > "$OUT/bench_C4_cap$cap.log" 2>&1 || { tail -20 "$OUT/bench_C4_cap$cap.log"; exit 1; }
  tail -1 "$OUT/bench_C4_cap$cap.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 cap $cap ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
done
