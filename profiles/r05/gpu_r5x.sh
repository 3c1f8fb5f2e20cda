#!/bin/bash
# k_large: 512-thread workgroups from the 3-per-CU class on (LARGE_BIG_BUCKET=2) vs from the 2-per-CU class (3)
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in C3 C4; do
  for v in default big2; do
    if [ $v = default ]; then LP=""; else LP="$(pwd)/profiles/_build/libbsdc_$v.so"; fi
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'])"
  done
done
