#!/bin/bash
# Round 6: the parts' OR rows back to back -- split-family parity, C4 A/B against the previous
# library, C4's large set per kernel instance (PMC)
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "split or c4 or C4 or large or join" --timeout 300 --timeout-method thread > $O/pytest_split.log 2>&1 || exit 2
for i in 1 2; do
  for lib in profiles/_build/libbsdc_prev.so bsseqconsensusreads_amd/libbsdc.so; do
    n=$(basename $lib .so)
    BSDC_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 3
  done
done
bash profiles/collect_pmc.sh $O/pmc_C4 --config C4 > $O/pmc_C4.log 2>&1 || exit 4
python profiles/pmc_instances.py $O/pmc_C4 $O/pmc_C4_instances.json > /dev/null || exit 5
python profiles/pmc_bench_summary.py $O/pmc_C4 $O/pmc_C4.json > /dev/null || exit 6
find $O -type f -size +2M -delete
