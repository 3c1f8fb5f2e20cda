#!/bin/bash
# Bench lines of the non-headline configs (C0, C1, C3, C4 and C5 on one GPU) with a bounded CPU
# baseline each.  Usage (repo root, on the box): bash profiles/bench_configs.sh <tag>
set -u -o pipefail
OUT=gpurun_out/${1:-cfg}; mkdir -p $OUT
for c in C0 C1 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-sample 100000 --cpu-sample-1core 20000 > $OUT/bench_$c.log 2>&1 \
    || { echo "bench $c failed"; tail -20 $OUT/bench_$c.log; exit 1; }
  echo "$c $(tail -1 $OUT/bench_$c.log | cut -c1-300)"
done
timeout -k 10 400 python -u bench.py --config C5 --families 6000000 --steps 5 --cpu-sample 0 > $OUT/bench_C5.log 2>&1 \
  || { echo "bench C5 failed"; tail -20 $OUT/bench_C5.log; exit 1; }
echo "C5 $(tail -1 $OUT/bench_C5.log | cut -c1-300)"
