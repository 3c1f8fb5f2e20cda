#!/bin/bash
# Round-4: the join with its parts' set lengths in LDS and four parts' loads in flight: part-mode
# parity, then C4 bench and kernel stats.
set -u -o pipefail
OUT=gpurun_out/r4j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "split or large or C4" --timeout 300 \
  --timeout-method thread > $OUT/pytest_parts.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_parts.log | head; tail -5 $OUT/pytest_parts.log; exit 1; }
tail -1 $OUT/pytest_parts.log
CFGS="C4" bash profiles/ab_r4.sh r4j base=- || exit 1
CONFIGS="C4" SKIP_PMC=1 bash profiles/prof_round.sh r4j > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
grep -E "k_join|k_large" $OUT/prof_C4/bench_kernel_stats.csv | cut -c1-40,100-200 | head; cat $OUT/span_C4.json
