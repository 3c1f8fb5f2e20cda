#!/bin/bash
# Round-4: compact part sums (a one-base column's single int32 sum instead of four): part-mode
# parity, C4 bench, C4 PMC traffic.
set -u -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "split or large or C4" --timeout 300 \
  --timeout-method thread > $OUT/pytest_parts.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_parts.log | head; tail -5 $OUT/pytest_parts.log; exit 1; }
tail -1 $OUT/pytest_parts.log
CFGS="C4" bash profiles/ab_r4.sh r4k base=- || exit 1
bash profiles/collect_pmc.sh $OUT/pmc_C4 --config C4 > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
python profiles/pmc_bench_summary.py $OUT/pmc_C4 $OUT/pmc_C4.json > /dev/null && python -c "
import json; d=json.load(open('$OUT/pmc_C4.json'))['k_large']; print('k_large GB/dispatch', round(d['hbm_bytes_per_dispatch']/1e9,4), 'x6 =', round(6*d['hbm_bytes_per_dispatch']/1e9,3))"
find $OUT -type f -size +2M -delete
