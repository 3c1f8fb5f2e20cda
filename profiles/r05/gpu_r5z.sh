#!/bin/bash
# k_large knobs re-tuned at the new class widths: C3 and C4 large set per variant
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in C3 C4; do
  for v in default vu8 vu2 ou4 cu8 su4; do
    if [ $v = default ]; then LP=""; else LP="$(pwd)/profiles/_build/libbsdc_$v.so"; fi
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'])"
  done
done
