#!/bin/bash
# k_pair vs k_small on C2: rocprofv3 kernel stats + two SQ counter passes each (separate runs).
# Usage (GPU box, repo root): bash profiles/r05/pmc_ab.sh <tag>
set -u -o pipefail
OUT=$(realpath -m "gpurun_out/$1")
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-sample 0 --no-tags-leg"
for kern in pair wave; do
  export BSDC_SMALL_KERNEL=$kern
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_small|k_pair' --output-format csv \
      -d "$OUT/stats_$kern" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/stats_$kern.log" 2>&1 || { echo "stats $kern failed"; tail -5 "$OUT/stats_$kern.log"; exit 1; }
  i=0
  for grp in \
    "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex 'k_small|k_pair' --output-format csv \
        -d "$OUT/p${i}_$kern" -o pmc -- python3 "$R/bench.py" $ARGS > "$OUT/p${i}_$kern.log" 2>&1 || { echo "pass $i $kern failed"; tail -5 "$OUT/p${i}_$kern.log"; exit 1; }
  done
  echo "$kern ok"
done
cd "$R"
for kern in pair wave; do
  BSDC_SMALL_KERNEL=$kern timeout -k 10 200 python -u profiles/ablate.py --config C2 > "$OUT/ablate_$kern.log" 2>&1 || { tail -5 "$OUT/ablate_$kern.log"; exit 1; }
  tail -1 "$OUT/ablate_$kern.log"
done
