"""Per template instance of the family kernels (k_large<IN_LDS, G, TAGS, PART>, k_join<TAGS>, ...):
FETCH_SIZE / WRITE_SIZE per launch set from profiles/collect_pmc.sh output, so the large set's
bytes split into its whole families, its parts and the join.  A launch set is
one k_join dispatch (one per step).  Reads are reported raw and x2 (MI355X_MICROARCH.md's
correction for 16-B-per-lane reads; profiles/calib_fetch.sh for the other widths).
Usage: python profiles/pmc_instances.py <collect_pmc out dir> [out.json]"""
import collections
import csv
import glob
import json
import re
import sys

d = sys.argv[1]
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        c = r["Counter_Name"]
        if c not in ("FETCH_SIZE", "WRITE_SIZE"):
            continue
        m = re.search(r"(k_\w+<[^>]*>)", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        k = m.group(1) if m else r["Kernel_Name"][:80]
        tot[(k, c)] += float(r["Counter_Value"]) * 1024
        disp[(k, c)].add((f, int(r["Dispatch_Id"])))
sets = max(len(v) for (k, c), v in disp.items() if k.startswith("k_join") and c == "FETCH_SIZE")
out = {"launch_sets": sets, "kernels": {}}
for k in sorted({k for k, _ in tot}):
    fr = tot.get((k, "FETCH_SIZE"), 0.0) / sets
    wr = tot.get((k, "WRITE_SIZE"), 0.0) / sets
    out["kernels"][k] = {"dispatches_per_set": len(disp.get((k, "FETCH_SIZE"), ())) / sets,
                         "fetch_raw_MB": round(fr / 1e6, 1), "read_x2_MB": round(2 * fr / 1e6, 1),
                         "write_MB": round(wr / 1e6, 1)}
js = json.dumps(out, indent=1)
print(js)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(js)
