#!/bin/bash
# Round profile on one GPU box: rocprofv3 kernel-trace stats of bench.py on C2 (headline) and C3,
# then the PMC passes of both (HBM traffic, instruction counts) and their summaries.
# Usage (repo root, on the box): [CONFIGS="C2 C3 C4"] [SKIP_PMC=1] bash profiles/prof_round.sh <tag>
set -u -o pipefail
TAG=${1:-r02}
R=$(pwd)
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS:-C2 C3}; do
  echo "[$(date +%T)] stats $c"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o bench -- \
      python3 "$R/bench.py" --config $c --steps 20 --cpu-sample 0 --cpu-sample-1core 0 --no-tags-leg > "$OUT/prof_$c.log" 2>&1) \
    || { echo "rocprof $c failed"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  tail -1 "$OUT/prof_$c.log" | cut -c1-200
  find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cat {} \;
  # launch-set spans (the side streams overlap a set's dispatches: DESIGN.md 5.4)
  python profiles/trace_span.py "$(find "$OUT/prof_$c" -name '*kernel_trace.csv' | head -1)" "$OUT/prof_$c.log" "$OUT/span_$c.json" || exit 1
  # the family kernels' rows of the trace (the whole trace is too large to keep)
  python profiles/trace_filter.py "$(find "$OUT/prof_$c" -name '*kernel_trace.csv' | head -1)" "$OUT/trace_k_$c.csv" || exit 1
  find "$OUT/prof_$c" -type f -size +2M -delete
done
for c in ${CONFIGS:-C2 C3}; do
  [ -n "${SKIP_PMC:-}" ] && break
  echo "[$(date +%T)] pmc $c"
  bash profiles/collect_pmc.sh "$OUT/pmc_$c" --config $c || exit 1
  python profiles/pmc_bench_summary.py "$OUT/pmc_$c" "$OUT/pmc_$c.json" > /dev/null || exit 1
done
find "$OUT" -type f -size +2M -print -delete
echo "[$(date +%T)] done"
