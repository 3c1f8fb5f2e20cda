#!/bin/bash
# parity (incl. tags, wide rows on C4), rank path, k_pair arm, then the bench with the tag leg
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ranks.py tests/test_gpu_fleet.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"; tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-sample 0 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'tags_ms', d['tags_ms_per_step'])"
