#!/bin/bash
# k_join: branch-free part loop (default 512 threads, 4 parts in flight) and width / depth variants
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or large" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for v in default j512_8 j256_4 j256_8; do
  if [ $v = default ]; then LP=""; else LP="$(pwd)/profiles/_build/libbsdc_$v.so"; fi
  BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_C4_$v.log" 2>&1 || { tail -20 "$OUT/bench_C4_$v.log"; exit 1; }
  tail -1 "$OUT/bench_C4_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C4 $v ms', d['ms_per_step'], 'large_ms', r['large_kernel_ms'], 'large_frac', r['large_frac'])"
done
