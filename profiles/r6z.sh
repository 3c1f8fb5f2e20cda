#!/bin/bash
# Round 6: does k_join's near-tie fallback (the whole family again in its HBM arena) carry C4's
# join reads?  FETCH / WRITE per kernel instance and the C4 step, with the fallback compiled out
# (wrong on tie columns: profiling only) against the tree
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
for n in tree notie; do
  BSDC_LIB_PATH=$(realpath profiles/_build/libbsdc_$n.so) timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_$n.log 2>&1 || exit 3
  R=$(pwd)
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && BSDC_LIB_PATH=$R/profiles/_build/libbsdc_$n.so timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex 'k_small|k_large|k_join' --output-format csv -d $R/$O/pmc_$n/p_$c -o pmc -- python3 $R/bench.py --config C4 --steps 3 --warmup 1 --cpu-sample 0 --no-tags-leg > $R/$O/pmc_${n}_$c.log 2>&1) || exit 4
  done
  python profiles/pmc_instances.py $O/pmc_$n $O/instances_$n.json > /dev/null || exit 5
done
