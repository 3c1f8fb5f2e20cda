#!/bin/bash
# Round-4 k_large / fleet measurements: per-class dispatch times with the side streams off
# (-DBSDC_FORK=0, ablibs/libbsdc_nofork.so) on C4 (part mode on / off) and C3, the C4 PMC passes
# of the in-tree build, and the end-to-end fleet with one worker beside the one-process stream.
set -u -o pipefail
mkdir -p gpurun_out/r4d
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_nofork.so) CONFIGS="C4 C3" SKIP_PMC=1 bash profiles/prof_round.sh r4d/nofork || exit 1
BSDC_LIB_PATH=$(realpath ablibs/libbsdc_nofork.so) BSDC_PART_CAP=0 CONFIGS="C4" SKIP_PMC=1 bash profiles/prof_round.sh r4d/nofork_nopart || exit 1
CFGS="C4" bash profiles/ab_r4.sh r4d base=- splitfirst=ablibs/libbsdc_splitfirst.so nopart=-:BSDC_PART_CAP=0 || exit 1
bash profiles/collect_pmc.sh gpurun_out/r4d/pmc_C4 --config C4 || exit 1
python profiles/pmc_bench_summary.py gpurun_out/r4d/pmc_C4 gpurun_out/r4d/pmc_C4.json > /dev/null || exit 1
find gpurun_out/r4d -type f -size +2M -delete
echo "[$(date +%T)] e2e fleet 1 worker"
timeout -k 10 600 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --workers 1 \
  --modes stream_gpubgzf,fleet_gpubgzf > gpurun_out/r4d/e2e_fleet1.log 2>&1 || { tail -20 gpurun_out/r4d/e2e_fleet1.log; exit 1; }
tail -3 gpurun_out/r4d/e2e_fleet1.log | cut -c1-400
echo "[$(date +%T)] done"
