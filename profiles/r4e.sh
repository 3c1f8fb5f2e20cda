#!/bin/bash
# Round-4 fleet check: the GPU fleet tests, then the end-to-end fleet with one and two workers on
# GPU 0 beside the one-process stream (profiles/e2e_stream.py, 1M C2 families, GPU BGZF).
set -u -o pipefail
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fleet.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu_fleet.log 2>&1 || { echo "fleet tests failed"; grep -E "FAILED|Error" $OUT/pytest_gpu_fleet.log | head; tail -5 $OUT/pytest_gpu_fleet.log; exit 1; }
tail -1 $OUT/pytest_gpu_fleet.log
for w in 1 2; do
  echo "[$(date +%T)] e2e fleet $w worker(s)"
  timeout -k 10 600 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --workers $w \
    --modes stream_gpubgzf,fleet_gpubgzf > $OUT/e2e_fleet$w.log 2>&1 || { tail -20 $OUT/e2e_fleet$w.log; exit 1; }
  grep -E "^(stream_gpubgzf|fleet_gpubgzf) " $OUT/e2e_fleet$w.log | cut -c1-700
  tail -1 $OUT/e2e_fleet$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if 'identical' in k})"
done
echo "[$(date +%T)] done"
