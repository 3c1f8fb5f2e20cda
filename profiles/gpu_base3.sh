#!/bin/bash
# Round-3 baseline at HEAD: GPU suite, smoke, default bench, ablation, rocprofv3 stats + PMC for
# C2/C3/C4, per-phase PMC of k_small (C2) and k_large (C3) for the LDS-conflict attribution.
# Usage (repo root, on the box): bash profiles/gpu_base3.sh <tag>
set -u -o pipefail
TAG=$1
R=$(pwd)
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
NOPROF=1 bash profiles/gpu_round.sh "$TAG" skip-e2e || exit 1
timeout -k 10 200 python -u profiles/ablate.py --config C4 --kernel large > "$OUT/ablate_C4.log" 2>&1 || { tail -20 "$OUT/ablate_C4.log"; exit 1; }
tail -1 "$OUT/ablate_C4.log"
CONFIGS="C2 C3 C4" bash profiles/prof_round.sh "$TAG/prof" || exit 1
echo "[$(date +%T)] pmc-ablate C2 small"
FAMS=300000 bash profiles/collect_pmc_ablate.sh "$OUT/pmca_C2" --config C2 || exit 1
python profiles/pmc_summary.py "$OUT/pmca_C2" > "$OUT/pmca_C2.json" || exit 1
echo "[$(date +%T)] pmc-ablate C3 large"
KREGEX=k_large FAMS=100000 bash profiles/collect_pmc_ablate.sh "$OUT/pmca_C3" --config C3 --kernel large || exit 1
python profiles/pmc_summary.py "$OUT/pmca_C3" large > "$OUT/pmca_C3.json" || exit 1
find "$OUT" -type f -size +2M -print -delete
echo "[$(date +%T)] base done"
