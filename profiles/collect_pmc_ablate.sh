#!/bin/bash
# PMC per ablation phase of k_small: rocprofv3 over profiles/ablate.py (12 dispatches per phase,
# in PHASES order).  Usage: [KREGEX=k_large] bash profiles/collect_pmc_ablate.sh <out_dir> [ablate args...]
set -u
OUT=$(realpath -m "$1"); shift
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_small}" --output-format csv \
      -d "$OUT/p$i" -o pmc -- python3 "$R/profiles/ablate.py" --families ${FAMS:-300000} --reps 10 "$@" > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
