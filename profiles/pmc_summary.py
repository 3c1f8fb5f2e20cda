"""Summarise profiles/collect_pmc_ablate.sh output: per-phase counter means per wave (family)."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
PH = ["launch", "tables", "staging", "convert", "extend", "overlap", "srcreads+lists", "vote-preamble", "vote-main", "vote-queue", "full"]
if len(sys.argv) > 2 and sys.argv[2] == "large":  # profiles/ablate.py LARGE_PHASES
    PH = ["launch", "tables", "staging", "convert", "extend", "overlap-wild", "overlap-templates", "overlap", "srcreads",
          "filter+lists", "vote-sums", "vote", "full"]
RUNS = 12  # 2 warmup + 10 timed per phase
res = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    disp = sorted({int(r["Dispatch_Id"]) for r in rows})
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    nb = len(disp) // (len(PH) * RUNS)  # dispatches per run (one per non-empty LDS bucket)
    for k, name in enumerate(PH):
        ids = disp[nb * (RUNS * k + 2): nb * (RUNS * k + RUNS)]
        for i in ids:
            for c, v in per[i].items():
                res[name][c] += v
        res[name]["_n"] = len(ids)
out = {}
for name in PH:
    w = res[name].get("SQ_WAVES") or res["full"].get("SQ_WAVES", 1) * 0 or 1
    out[name] = {c: round(v / w, 1) if c != "_n" else v for c, v in sorted(res[name].items())}
print(json.dumps(out, indent=1))
