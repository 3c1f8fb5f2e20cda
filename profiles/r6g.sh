#!/bin/bash
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
bash profiles/calib_fetch.sh $O/calib > $O/calib.log 2>&1 || exit 2
find $O -type f -size +2M -delete
