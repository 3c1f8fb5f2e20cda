#!/bin/bash
# Round-4 final measurements on one box: bench lines for C2 / C3 / C4, rocprofv3 kernel stats,
# trace spans and PMC passes of the same configs, and the end-to-end file path.
set -u -o pipefail
T=${1:-r4final}
OUT=gpurun_out/$T
mkdir -p $OUT
echo "[$(date +%T)] bench"
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
for c in C3 C4; do
  timeout -k 10 400 python -u bench.py --config $c --cpu-sample 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
done
CONFIGS="C2 C3 C4" bash profiles/prof_round.sh $T > $OUT/prof_round.log 2>&1 || { tail -20 $OUT/prof_round.log; exit 1; }
grep -E "trace_span|stats|pmc|done" $OUT/prof_round.log | cut -c1-200
echo "[$(date +%T)] e2e"
timeout -k 10 700 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --workers 1 \
  --modes stream_gpubgzf,stream_fastq_gpubgzf,fleet_gpubgzf,molecular_stream > $OUT/e2e.log 2>&1 || { tail -20 $OUT/e2e.log; exit 1; }
tail -1 $OUT/e2e.log | cut -c1-300
echo "[$(date +%T)] done"
