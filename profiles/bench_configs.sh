set -u -o pipefail
OUT=gpurun_out/v12cfg; mkdir -p $OUT
for c in C0 C1 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-sample 100000 > $OUT/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 $OUT/bench_$c.log; exit 1; }
  echo "$c $(tail -1 $OUT/bench_$c.log | cut -c1-400)"
done
timeout -k 10 300 python -u profiles/e2e.py > $OUT/e2e.log 2>&1 || { echo e2e failed; tail -20 $OUT/e2e.log; exit 1; }
tail -5 $OUT/e2e.log
