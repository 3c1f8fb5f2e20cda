#!/bin/bash
# Round-4: the whole -m gpu suite (parity / fp64 / stream first, then the rest) and smoke().
set -u -o pipefail
T=${1:-r4tests}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py tests/test_gpu_stream.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/pytest_gpu_a.log 2>&1 \
  || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu_a.log | head -20; tail -5 $OUT/pytest_gpu_a.log; exit 1; }
tail -1 $OUT/pytest_gpu_a.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  --deselect tests/test_gpu_parity.py --deselect tests/test_gpu_fp64.py --deselect tests/test_gpu_stream.py \
  > $OUT/pytest_gpu_b.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu_b.log | head -20; tail -5 $OUT/pytest_gpu_b.log; exit 1; }
tail -1 $OUT/pytest_gpu_b.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for c in C4 C3; do
  timeout -k 10 400 python -u bench.py --config $c --cpu-sample 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  echo "$c $(tail -1 $OUT/bench_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r.get("small_kernel_ms"), r.get("large_kernel_ms"), d.get("tags_ms_per_step"))')"
done
echo "[$(date +%T)] done"
