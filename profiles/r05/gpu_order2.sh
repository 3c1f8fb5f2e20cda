#!/bin/bash
# small buckets dispatched longest first (BSDC_SMALL_ORDER=work) vs by arena size
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
BSDC_SMALL_ORDER=work timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for c in C2 C4; do
  for v in size work size2 work2; do
    case $v in size*) O=size;; *) O=work;; esac
    BSDC_SMALL_ORDER=$O timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'small', r.get('small_kernel_ms'), 'large', r.get('large_kernel_ms'))"
  done
done
