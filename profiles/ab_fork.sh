#!/bin/bash
# A/B of the side-stream fan-out (BSDC_FORK / BSDC_FORK_STREAMS builds under abl/): GPU parity of
# the first library, then the C2 / C3 / C4 bench per library.  Usage: bash profiles/ab_fork.sh <tag> <lib.so>...
set -u -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
BSDC_LIB_PATH=$(realpath $1) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batches.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in C2 C3 C4; do for lib in "$@"; do
  n=$(basename $lib .so)
  BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 300 python -u bench.py --config $c --cpu-sample 0 --steps 20 > $OUT/bench_${c}_$n.log 2>&1 || { echo "bench $c $n failed"; tail -20 $OUT/bench_${c}_$n.log; exit 1; }
  echo "$c $n $(tail -1 $OUT/bench_${c}_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["small_kernel_ms"], r["large_kernel_ms"])')"
done; done
