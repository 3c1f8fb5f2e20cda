#!/bin/bash
# parity of both small kernels + A/B bench + ablations (k_pair vs k_small)
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
for kern in pair wave; do
  BSDC_SMALL_KERNEL=$kern timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-tags-leg --cpu-sample 0 > "$OUT/bench_$kern.log" 2>&1 || { tail -20 "$OUT/bench_$kern.log"; exit 1; }
  tail -1 "$OUT/bench_$kern.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$kern', d['ms_per_step'], d['roofline']['frac'])"
  BSDC_SMALL_KERNEL=$kern timeout -k 10 200 python -u profiles/ablate.py --config C2 > "$OUT/ablate_$kern.log" 2>&1 || { tail -5 "$OUT/ablate_$kern.log"; exit 1; }
  tail -1 "$OUT/ablate_$kern.log"
done
