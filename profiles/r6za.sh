#!/bin/bash
# Round 6: k_join's part loads -- slots past the family's last part load nothing (np), and also
# lanes past the part's set length (lane) -- against the tree: split/large parity, C4 step and
# per-instance FETCH / WRITE
set -o pipefail
O=gpurun_out/r6za
mkdir -p $O
R=$(pwd)
for n in np lane; do
  BSDC_LIB_PATH=$R/profiles/_build/libbsdc_$n.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "split or c4 or C4 or join" --timeout 300 --timeout-method thread > $O/pytest_$n.log 2>&1 || exit 2
done
for i in 1 2; do
  for n in tree np lane; do
    BSDC_LIB_PATH=$R/profiles/_build/libbsdc_$n.so timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_$n.log 2>&1 || exit 3
  done
done
for n in tree np lane; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && BSDC_LIB_PATH=$R/profiles/_build/libbsdc_$n.so timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex 'k_large|k_join' --output-format csv -d $R/$O/pmc_$n/p_$c -o pmc -- python3 $R/bench.py --config C4 --steps 3 --warmup 1 --cpu-sample 0 --no-tags-leg > $R/$O/pmc_${n}_$c.log 2>&1) || exit 4
  done
  python profiles/pmc_instances.py $O/pmc_$n $O/instances_$n.json > /dev/null || exit 5
done
