#!/bin/bash
# k_small: families per wavefront in turn (SMALL_FPW), C2 / C4; parity of the FPW=2 build first
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
BSDC_LIB_PATH="$B/libbsdc_fpw2.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_fpw2.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_fpw2.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_fpw2.log"
for c in C2 C4; do
  for v in 1 2 4 1b 2b 4b; do
    case ${v:0:1} in 1) LP="";; *) LP="$B/libbsdc_fpw${v:0:1}.so";; esac
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --no-tags-leg > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c fpw $v ms', d['ms_per_step'], 'small', r.get('small_kernel_ms'))"
  done
done
