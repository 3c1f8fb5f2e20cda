#!/bin/bash
# k_large: quals staged by LDS-DMA in LDS arenas (LARGE_QDMA) -- parity first (forced k_large,
# parts, full-size C3 / C4), then C3 / C4 A/B
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
BSDC_LIB_PATH="$B/libbsdc_lqdma.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
BSDC_LIB_PATH="$B/libbsdc_lqdma.so" timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -k "c3 or c4" -x -q --timeout 450 --timeout-method thread > "$OUT/pytest_full.log" 2>&1 \
  || { echo "full-size tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_full.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_full.log"
for c in C3 C4; do
  for v in reg dma reg2 dma2; do
    case $v in reg*) LP="";; *) LP="$B/libbsdc_lqdma.so";; esac
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'small', r.get('small_kernel_ms'), 'large', r.get('large_kernel_ms'))"
  done
done
