"""Launch-set spans of the bench's roofline kernel from a rocprofv3 kernel trace.

Since the bucket dispatches of one bsdc_run fan out over side streams, the
dispatches of one launch set overlap, and rocprofv3's mean duration per dispatch no longer adds
up to the set's time.  The caller's stream still orders the sets: each set starts after the one
before has ended.  bench.py's roofline leg for the dominant kernel is its last `max(5, steps)` sets
of that kernel alone (the k_small-only leg, then the k_large-only leg).  This takes the last
sets × dispatches_per_launch dispatches of that kernel in start order, cuts them into sets, and
prints the mean span (first start to last end) next to the bench's HIP-event time for the same
sets and the per-set sum of dispatch durations (what --stats adds up), as JSON.
Usage: python profiles/trace_span.py <kernel_trace.csv> <bench log> [out.json]
"""
import csv
import json
import sys


def main():
    trace, log = sys.argv[1], sys.argv[2]
    line = [x for x in open(log) if x.startswith("{") and '"metric"' in x][-1]
    d = json.loads(line)
    r = d["roofline"]
    kern, per, nsets = r["kernel"], int(r["dispatches_per_launch"]), max(5, int(d["steps"]))
    rows = []
    with open(trace, newline="") as f:
        for x in csv.DictReader(f):
            k = x["Kernel_Name"]
            if kern + "<" in k or (kern == "k_large" and ("k_join<" in k or "k_tie<" in k)):  # (split families' join)
                rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"])))
    rows.sort()
    take = rows[-nsets * per:]
    assert len(take) == nsets * per, "trace holds %d %s dispatches, need %d" % (len(rows), kern, nsets * per)
    sets = [take[i * per:(i + 1) * per] for i in range(nsets)]
    # sets do not overlap (the caller's stream orders them); if they seem to, the per-set
    # dispatch count is off and the spans below are not the sets'
    overlap = any(b[0][0] < max(e for _, e in a) for a, b in zip(sets, sets[1:]))
    span = sum(max(e for _, e in s) - s[0][0] for s in sets) / nsets / 1e6
    summed = sum(e - s0 for s in sets for s0, e in s) / nsets / 1e6
    out = {"kernel": kern, "sets": nsets, "dispatches_per_set": per, "trace_span_ms_per_set": round(span, 4),
           "bench_event_ms_per_set": r["kernel_ms"], "sum_of_dispatch_ms_per_set": round(summed, 4),
           "span_vs_event": round(span / r["kernel_ms"], 4), "sets_overlap": overlap}
    txt = json.dumps(out)
    print(txt)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
