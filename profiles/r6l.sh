#!/bin/bash
# Round 6: hardware queues per process (HIP's GPU_MAX_HW_QUEUES, 4 by default) against the side
# streams' overlap, C2 and C4, alternated
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 20 --cpu-sample 0 > $O/c2_${i}_q$q.log 2>&1 || exit 3
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --config C4 --steps 20 --cpu-sample 0 --no-tags-leg > $O/c4_${i}_q$q.log 2>&1 || exit 4
  done
done
