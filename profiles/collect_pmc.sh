#!/bin/bash
# PMC passes for the family kernels (one rocprofv3 run per counter group; MI355X_MICROARCH.md
# "rocprofv3 PMC slots": <= 8 SQ, <= 4 TCC counters per pass).  Usage (on the GPU box, repo root):
#   bash profiles/collect_pmc.sh <out_dir> [bench args...]
set -u
OUT=$(realpath -m "$1"); shift
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# TAGS=1: keep bench's consensus-tag leg (the k_small<true> / k_large tag instances, summarised apart)
if [ "${TAGS:-0}" = 1 ]; then ARGS="--steps 3 --warmup 1 --cpu-sample 0 $*"; else ARGS="--steps 3 --warmup 1 --cpu-sample 0 --no-tags-leg $*"; fi
i=0
for grp in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex 'k_small|k_large|k_join' --output-format csv \
      -d "$OUT/p$i" -o pmc -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
