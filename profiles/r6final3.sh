#!/bin/bash
# Round 6 final profile after the wave-priority change (profiles/r06/final2/): smoke; rocprofv3
# kernel-trace stats + launch-set spans + PMC passes of bench.py on C2, C3, C4; the tag instance's
# PMC on C2; then the bench lines (reading the fresh PMC for roofline.traffic): C2 default with the
# CPU baseline, C3 and C4 with bounded CPU baselines
set -o pipefail
O=gpurun_out/r6final3
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
CONFIGS="C2 C3 C4" timeout -k 10 1100 bash profiles/prof_round.sh r6final3/prof > $O/prof_round.log 2>&1 || exit 3
TAGS=1 timeout -k 10 600 bash profiles/collect_pmc.sh $O/pmc_C2_tags --config C2 > $O/pmc_C2_tags.log 2>&1 || exit 4
python profiles/pmc_bench_summary.py $O/pmc_C2_tags $O/pmc_C2_tags.json > /dev/null || exit 5
for c in C2 C3 C4; do cp $O/prof/pmc_$c.json profiles/pmc_$c.json || exit 6; done
cp $O/pmc_C2_tags.json profiles/pmc_C2_tags.json || exit 6
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 7
for c in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-sample 100000 --cpu-sample-1core 20000 > $O/bench_$c.log 2>&1 || exit 8
done
find $O -type f -size +2M -delete
