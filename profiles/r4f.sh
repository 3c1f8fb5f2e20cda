#!/bin/bash
# Round-4: part-mode staging from the part records' own slot / length (one load), checked and
# timed: the part-mode parity tests, C4 bench with part mode on / off, the per-class times with the
# side streams off, then the fleet end to end with one worker (materialize on the planner thread).
set -u -o pipefail
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "split or large or C4" --timeout 300 \
  --timeout-method thread > $OUT/pytest_parts.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_parts.log | head; tail -5 $OUT/pytest_parts.log; exit 1; }
tail -1 $OUT/pytest_parts.log
CFGS="C4" bash profiles/ab_r4.sh r4f base=- nopart=-:BSDC_PART_CAP=0 || exit 1
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_nofork.so) CONFIGS="C4" SKIP_PMC=1 bash profiles/prof_round.sh r4f/nofork > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
echo "[$(date +%T)] e2e fleet 1 worker"
timeout -k 10 600 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --workers 1 \
  --modes stream_gpubgzf,fleet_gpubgzf > $OUT/e2e_fleet1.log 2>&1 || { tail -20 $OUT/e2e_fleet1.log; exit 1; }
grep -E "^(stream_gpubgzf|fleet_gpubgzf) " $OUT/e2e_fleet1.log | cut -c1-900
echo "[$(date +%T)] done"
