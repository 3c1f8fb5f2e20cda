#!/bin/bash
# LDS-side PMC per ablation phase (unaligned stalls, bank / address conflicts, FIFO full, LDS
# waits): rocprofv3 over profiles/ablate.py.  Usage: KREGEX=k_large bash profiles/collect_pmc_lds.sh <out> [ablate args]
set -u
OUT=$(realpath -m "$1"); shift
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
  "SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_small}" --output-format csv \
      -d "$OUT/p$i" -o pmc -- python3 "$R/profiles/ablate.py" --families ${FAMS:-300000} --reps 10 "$@" > "$OUT/p$i.log" 2>&1 \
      || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
