#!/bin/bash
# Round-4: the stream decoder's own breakdown (BSDC_STREAM_PROF: fill = read + inflate, split =
# record scan + family keys, select = the family-complete cut, emit) on the 1M-family e2e input.
set -u -o pipefail
OUT=gpurun_out/r4r
mkdir -p $OUT
BSDC_STREAM_PROF=1 timeout -k 10 600 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --modes stream_gpubgzf,stream_fastq_gpubgzf \
  > $OUT/e2e.log 2>&1 || { tail -20 $OUT/e2e.log; exit 1; }
grep -E "bsdc stream|^stream" $OUT/e2e.log | cut -c1-700
