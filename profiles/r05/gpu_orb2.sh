#!/bin/bash
# the tag instance's part records as vectors too: parity (both join arms), C4 full size, C4 A/B
# with the tag leg
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
BSDC_SPLIT_JOIN=part timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k split -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_partjoin.log" 2>&1 \
  || { echo "part-join tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_partjoin.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_partjoin.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" -x -q --timeout 380 --timeout-method thread > "$OUT/pytest_c4.log" 2>&1 \
  || { echo "c4 tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_c4.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_c4.log"
for v in head new head2 new2; do
  case $v in head*) LP="$B/libbsdc_head.so";; *) LP="";; esac
  BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 2 --cpu-sample 0 > "$OUT/bench_C4_$v.log" 2>&1 || { tail -20 "$OUT/bench_C4_$v.log"; exit 1; }
  tail -1 "$OUT/bench_C4_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 $v ms', d['ms_per_step'], 'large_ms', r.get('large_kernel_ms'), 'tags_ms', d.get('tags_ms_per_step'))"
done
