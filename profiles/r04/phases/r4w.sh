#!/bin/bash
# Round-4 end state per phase: ablation times (C2 small, C3 and C4 large) and the per-phase PMC of
# k_small on C2, for DESIGN 5.3's "where k_small stands".  Usage (repo root, on the box):
# bash profiles/r4w.sh <tag>
set -u -o pipefail
TAG=$1
R=$(pwd)
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
for a in "C2 small" "C3 large" "C4 large"; do
  set -- $a
  echo "[$(date +%T)] ablate $1 $2"
  timeout -k 10 200 python -u profiles/ablate.py --config $1 --kernel $2 > "$OUT/ablate_$1.log" 2>&1 || { tail -20 "$OUT/ablate_$1.log"; exit 1; }
  tail -1 "$OUT/ablate_$1.log"
done
echo "[$(date +%T)] pmc-ablate C2 small"
FAMS=300000 bash profiles/collect_pmc_ablate.sh "$OUT/pmca_C2" --config C2 || exit 1
python profiles/pmc_summary.py "$OUT/pmca_C2" > "$OUT/pmca_C2.json" || exit 1
find "$OUT" -type f -size +2M -print -delete
echo "[$(date +%T)] done"
