"""Summarise profiles/collect_pmc.sh output: per-kernel counter means per dispatch, plus HBM
traffic per launch with the gfx950 correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE
reports half the bytes of wide streaming reads, so reads = 2 x FETCH_SIZE; WRITE_SIZE is exact.
Both counters are in KiB.  Usage: python profiles/pmc_bench_summary.py <collect_pmc out dir> [out.json]"""
import collections
import csv
import glob
import json
import re
import sys

d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"]][(f, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
# every template instance of a kernel (k_large<true, 256>, <true, 512>, <false, 512>; one
# dispatch per bucket) under its name: mean per dispatch x dispatches per launch set = per set
grouped = collections.defaultdict(dict)
for k, disp in per.items():
    m = re.search(r"(k_small|k_pair|k_large|k_join|k_tie)", k)
    name = m.group(1) if m else k[:60]
    if name == "k_small" and "k_small<true" in k:  # the consensus-tag instance (BSDC_MODE_TAGS) on its own
        name = "k_small_tags"
    elif (name == "k_large" and re.search(r"k_large<(true|false), \d+, true", k)) or "k_join<true" in k or "k_tie<true" in k:
        name = "k_large_tags"  # (k_large<IN_LDS, G, TAGS, PART>, k_join<TAGS>)
    elif name in ("k_join", "k_tie"):  # the split families' join: one more dispatch of the k_large launch set
        name = "k_large"
    grouped[name].update({(k,) + key: v for key, v in disp.items()})
out = {}
for name, disp in grouped.items():
    sums = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for _, cs in disp.items():
        for c, v in cs.items():
            sums[c] += v
            cnt[c] += 1
    means = {c: sums[c] / cnt[c] for c in sums}
    o = {"dispatches_per_counter": max(cnt.values()), "mean_per_dispatch": {c: round(v, 1) for c, v in sorted(means.items())}}
    if "SQ_WAVES" in means and means["SQ_WAVES"]:
        w = means["SQ_WAVES"]
        o["per_wave"] = {c: round(means[c] / w, 1) for c in sorted(means) if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES",)}
    if "FETCH_SIZE" in means:
        o["fetch_bytes_raw"] = means["FETCH_SIZE"] * 1024
        o["read_bytes_corrected"] = 2 * means["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in means:
        o["write_bytes"] = means["WRITE_SIZE"] * 1024
    if "read_bytes_corrected" in o and "write_bytes" in o:
        o["hbm_bytes_per_dispatch"] = o["read_bytes_corrected"] + o["write_bytes"]
    out[name] = o
js = json.dumps(out, indent=1)
print(js)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(js)
