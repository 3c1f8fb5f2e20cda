#!/bin/bash
# per-batch small-cap router (batch.route_small_cap): parity (C3 batches now route), full-size C3,
# and A/B against BSDC_SMALL_ROUTE=0 on C2, C3, C4
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "c3" -x -q --timeout 380 --timeout-method thread > "$OUT/pytest_c3.log" 2>&1 \
  || { echo "c3 tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_c3.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_c3.log"
for c in C3 C4 C2; do
  for v in off on off2 on2; do
    case $v in off*) R=0;; *) R=1;; esac
    BSDC_SMALL_ROUTE=$R timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'small', r.get('small_kernel_ms'), 'large', r.get('large_kernel_ms'), 'frac', r['frac'])"
  done
done
