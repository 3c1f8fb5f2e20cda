#!/bin/bash
# Round-4: the consensus-tag instances (the drop-in's default BAM output) profiled: rocprofv3 stats
# of bench with its tag leg, and the PMC passes with the tag instances summarised apart (TAGS=1).
set -u -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r4s
mkdir -p $OUT
export TMPDIR=/tmp
for c in C2 C4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o bench -- \
      python3 "$R/bench.py" --config $c --steps 20 --cpu-sample 0 --cpu-sample-1core 0 > "$OUT/prof_$c.log" 2>&1) \
    || { echo "rocprof $c failed"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_tags_$c.csv" \;
  find "$OUT/prof_$c" -type f -size +2M -delete
  TAGS=1 bash profiles/collect_pmc.sh "$OUT/pmc_$c" --config $c > "$OUT/pmc_$c.log" 2>&1 || { tail "$OUT/pmc_$c.log"; exit 1; }
  python profiles/pmc_bench_summary.py "$OUT/pmc_$c" "$OUT/pmc_tags_$c.json" > /dev/null || exit 1
  find "$OUT/pmc_$c" -type f -size +2M -delete
  python -c "
import json; d=json.load(open('$OUT/pmc_tags_$c.json'))
for k,v in d.items(): print('$c', k, v.get('dispatches_per_counter'), round(v.get('hbm_bytes_per_dispatch',0)/1e9,4), v.get('per_wave',{}).get('SQ_INSTS_VALU'))"
done
