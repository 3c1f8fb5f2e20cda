#!/bin/bash
# k_small staging: LDS-DMA quals (SMALL_QDMA) A/B, with the no-unpack probe (SMALL_PROBE=2, wrong
# results) bounding what the base unpack costs; parity of the DMA arm first
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
BSDC_LIB_PATH="$B/libbsdc_qdma.so" timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_qdma.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_qdma.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_qdma.log"
for v in default qdma p2 p2q default2 qdma2; do
  case $v in default|default2) LP="";; qdma2) LP="$B/libbsdc_qdma.so";; *) LP="$B/libbsdc_$v.so";; esac
  BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-tags-leg --cpu-sample 0 > "$OUT/bench_$v.log" 2>&1 || { tail -20 "$OUT/bench_$v.log"; exit 1; }
  tail -1 "$OUT/bench_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['frac'])"
done
BSDC_LIB_PATH="" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/bench_tags.log" 2>&1 || { tail -20 "$OUT/bench_tags.log"; exit 1; }
tail -1 "$OUT/bench_tags.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tags leg', d['ms_per_step'], d.get('tags_ms_per_step'), d.get('tags_roofline'))"
for v in default qdma; do
  if [ $v = default ]; then LP=""; else LP="$B/libbsdc_$v.so"; fi
  BSDC_LIB_PATH="$LP" timeout -k 10 200 python -u profiles/ablate.py --config C2 > "$OUT/ablate_$v.log" 2>&1 || { tail -5 "$OUT/ablate_$v.log"; exit 1; }
  tail -1 "$OUT/ablate_$v.log"
done
