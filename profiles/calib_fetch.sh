#!/bin/bash
# FETCH_SIZE / WRITE_SIZE against known byte counts per access width (profiles/calib_fetch.hip).
# Usage (GPU box, repo root, after building profiles/_build/calib_fetch): bash profiles/calib_fetch.sh <out_dir>
set -u -o pipefail
OUT=$(realpath -m "$1")
R=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d "$OUT/c$i" -o pmc -- "$R/profiles/_build/calib_fetch" > "$OUT/c$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/c$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
per = collections.defaultdict(float)  # (kernel, counter, dispatch) -> KiB, summed over the rows
for f in glob.glob(out + "/c*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(k, r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
last = {}
for (k, c, d), v in sorted(per.items()):
    last[(k, c)] = v  # the second round's dispatch (the highest id) of each kernel
B = 1 << 30
for (k, c), v in sorted(last.items()):
    print("%-28s %-11s %14.0f B  = %.3f x the bytes moved" % (k, c, v * 1024, v * 1024 / B))
PY
