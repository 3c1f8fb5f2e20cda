#!/bin/bash
# parity (tags + wide rows, part join), rank path, C4 full size; benches C2 (tags leg) and C4 A/B split join
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ranks.py tests/test_gpu_fleet.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"; tail -1 "$OUT/pytest.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_c4.log" 2>&1 \
  || { echo "c4 full size failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_c4.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_c4.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'tags_ms', d['tags_ms_per_step'], d['tags_roofline'])"
for j in part kernel; do
  BSDC_SPLIT_JOIN=$j timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_C4_$j.log" 2>&1 || { tail -20 "$OUT/bench_C4_$j.log"; exit 1; }
  tail -1 "$OUT/bench_C4_$j.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 $j ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
done
