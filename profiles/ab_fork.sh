set -u -o pipefail
OUT=gpurun_out/ab_fork; mkdir -p $OUT
BSDC_LIB_PATH=$(realpath abl/libbsdc_fork.so) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batches.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_fork.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_fork.log; exit 1; }
tail -1 $OUT/pytest_fork.log
for c in C2 C3 C4; do for n in base fork; do
  BSDC_LIB_PATH=$(realpath abl/libbsdc_$n.so) timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 --steps 20 > $OUT/bench_${c}_$n.log 2>&1 || { echo "bench $c $n failed"; tail -20 $OUT/bench_${c}_$n.log; exit 1; }
  echo "$c $n $(tail -1 $OUT/bench_${c}_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["small_kernel_ms"], r["large_kernel_ms"])')"
done; done
