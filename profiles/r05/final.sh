#!/bin/bash
# Round-5 final measurements on one box.  Usage: bash profiles/r05/final.sh <tag> <stage>
#   tests  : the whole -m gpu suite (timed) and smoke()
#   bench  : bench lines C2 (tags leg + CPU baseline), C3, C4; rocprofv3 kernel stats + spans
#   pmc    : PMC passes (FETCH/WRITE + instruction counts) for C2, C3, C4
#   e2e    : end-to-end file path: one-GPU stream, ranks (2 on GPU 0), fleet, step 1
set -u -o pipefail
T=$1; STAGE=$2
OUT="$(pwd)/gpurun_out/$T"
mkdir -p "$OUT"
case $STAGE in
tests)
  s0=$(date +%s)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "gpu suite failed"; grep -E "FAIL|Error" "$OUT/pytest_gpu.log" | tail -20; exit 1; }
  echo "suite_seconds $(( $(date +%s) - s0 ))"; tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
  ;;
bench)
  timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" | cut -c1-300
  for c in C3 C4; do
    timeout -k 10 400 python -u bench.py --config $c --cpu-sample 0 > "$OUT/bench_$c.log" 2>&1 || { tail -20 "$OUT/bench_$c.log"; exit 1; }
    tail -1 "$OUT/bench_$c.log" | cut -c1-200
  done
  CONFIGS="C2 C3 C4" SKIP_PMC=1 bash profiles/prof_round.sh $T > "$OUT/prof_round.log" 2>&1 || { tail -20 "$OUT/prof_round.log"; exit 1; }
  grep -E "done|failed" "$OUT/prof_round.log"
  ;;
pmc)
  for c in C2 C3 C4; do
    bash profiles/collect_pmc.sh "$OUT/pmc_$c" --config $c > "$OUT/pmc_$c.log" 2>&1 || { tail -20 "$OUT/pmc_$c.log"; exit 1; }
    python profiles/pmc_bench_summary.py "$OUT/pmc_$c" "$OUT/pmc_$c.json" > /dev/null || exit 1
    echo "pmc $c ok"
  done
  TAGS=1 bash profiles/collect_pmc.sh "$OUT/pmc_C2_tags" --config C2 > "$OUT/pmc_C2_tags.log" 2>&1 || { tail -20 "$OUT/pmc_C2_tags.log"; exit 1; }
  python profiles/pmc_bench_summary.py "$OUT/pmc_C2_tags" "$OUT/pmc_C2_tags.json" > /dev/null || exit 1
  find "$OUT" -type f -size +2M -delete
  echo "pmc done"
  ;;
e2e)
  timeout -k 10 900 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --workers 2 \
    --modes stream_gpubgzf,ranks_gpubgzf,stream,ranks,fleet_gpubgzf,molecular_stream > "$OUT/e2e.log" 2>&1 || { tail -20 "$OUT/e2e.log"; exit 1; }
  tail -1 "$OUT/e2e.log" | cut -c1-400
  ;;
esac
