#!/bin/bash
# part join (one-lane release/acquire): split-family parity, C4 full size, C4 bench A/B
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or large" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for j in kernel part; do
  BSDC_SPLIT_JOIN=$j timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_C4_$j.log" 2>&1 || { tail -20 "$OUT/bench_C4_$j.log"; exit 1; }
  tail -1 "$OUT/bench_C4_$j.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 $j ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_c4.log" 2>&1 \
  || { echo "c4 full size failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_c4.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_c4.log"
