#!/bin/bash
# C4 large leg: split chain first vs last, k_join vs part join
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or large" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for v in "BSDC_SPLIT_LAST=0" "BSDC_SPLIT_LAST=1" "BSDC_SPLIT_JOIN=part"; do
  env $v timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_C4_$v.log" 2>&1 || { tail -20 "$OUT/bench_C4_$v.log"; exit 1; }
  tail -1 "$OUT/bench_C4_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 $v ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
done
