#!/bin/bash
# k_large without scratch (per-set figures as selects) vs HEAD; the C2 tag leg with LDS-DMA quals
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for c in C4 C3; do
  for v in head new head2 new2; do
    case $v in head*) LP="$B/libbsdc_head.so";; *) LP="";; esac
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'large_ms', r.get('large_kernel_ms'), 'tags_ms', d.get('tags_ms_per_step'))"
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/bench_C2_tags.log" 2>&1 || { tail -20 "$OUT/bench_C2_tags.log"; exit 1; }
tail -1 "$OUT/bench_C2_tags.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['ms_per_step'], 'tags', d.get('tags_ms_per_step'), d['tags_roofline']['vs_headline_ms'])"
timeout -k 10 200 bash profiles/calib_fetch.sh "$OUT/calib" > "$OUT/calib.log" 2>&1 || { tail -20 "$OUT/calib.log"; exit 1; }
cat "$OUT/calib.log"
