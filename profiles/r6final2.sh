#!/bin/bash
# Round 6 final, part 2: the default bench line (C2, CPU baseline included), the tag instance's PMC
# on C2, bench lines of C3 and C4 with bounded CPU baselines, smoke
set -o pipefail
O=gpurun_out/r06final
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 2
TAGS=1 timeout -k 10 600 bash profiles/collect_pmc.sh $O/pmc_C2_tags --config C2 > $O/pmc_C2_tags.log 2>&1 || exit 3
python profiles/pmc_bench_summary.py $O/pmc_C2_tags $O/pmc_C2_tags.json > /dev/null || exit 4
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-sample 100000 --cpu-sample-1core 20000 > $O/bench_$c.log 2>&1 || exit 5
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 6
find $O -type f -size +2M -delete
