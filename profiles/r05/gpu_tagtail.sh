#!/bin/bash
# tag leg: a set's last dword written whole (zeros past its length) instead of byte by byte
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for v in head new head2 new2; do
  case $v in head*) LP="$B/libbsdc_head.so";; *) LP="";; esac
  BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/bench_C2_$v.log" 2>&1 || { tail -20 "$OUT/bench_C2_$v.log"; exit 1; }
  tail -1 "$OUT/bench_C2_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 $v ms', d['ms_per_step'], 'tags', d.get('tags_ms_per_step'), d['tags_roofline']['vs_headline_ms'])"
done
