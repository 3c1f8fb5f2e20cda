"""Per-phase PMC table from a collect_pmc*.sh run over profiles/ablate.py: counter deltas between
consecutive ablation phases, per wave, for one grid size (or all).
Usage: python profiles/pmc_phases.py <dir with p1/, p2/> <small|large> [grid]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
d, kind = sys.argv[1], sys.argv[2]
grid = int(sys.argv[3]) if len(sys.argv) > 3 else None
import importlib.util  # noqa: E402
src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ablate.py")).read()
ns = {}
exec(src[src.index("PHASES = "):src.index("ap = argparse")], ns)
phases = [p for p, _ in (ns["PHASES"] if kind == "small" else ns["LARGE_PHASES"])]
res = {}
for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        by[int(r["Dispatch_Id"])]["_grid"] = int(r["Grid_Size"])
    ids = sorted(by)
    nb = len(ids) // (12 * len(phases))
    per = 12 * nb
    for i, ph in enumerate(phases):
        tot = collections.Counter()
        for x in ids[i * per:(i + 1) * per][2 * nb:]:
            if grid is None or by[x]["_grid"] == grid:
                for k, v in by[x].items():
                    if k != "_grid":
                        tot[k] += v / 10
        res.setdefault(ph, collections.Counter()).update(tot)
keys = sorted({k for v in res.values() for k in v if k != "SQ_WAVES"})
print("%-18s" % "phase (per wave)" + "".join("%12s" % k[3:15] for k in keys))
prev = None
for ph in phases:
    v = res[ph]
    w = v.get("SQ_WAVES", 1) or 1
    cur = {k: v.get(k, 0) / w for k in keys}
    row = cur if prev is None else {k: cur[k] - prev[k] for k in keys}
    print("%-18s" % ph + "".join("%12.0f" % row[k] for k in keys))
    prev = cur
