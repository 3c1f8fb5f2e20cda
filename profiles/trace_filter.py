"""Keep the family kernels' rows (k_small, k_large, k_join) of a rocprofv3 kernel trace, with the
columns the span / per-class analyses need, numbered by dispatch order.
Usage: python profiles/trace_filter.py <kernel_trace.csv> <out.csv>"""
import csv
import re
import sys

KEEP = ("Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
        "Stream_Id", "Correlation_Id")


def main():
    src, dst = sys.argv[1], sys.argv[2]
    with open(src, newline="") as f, open(dst, "w", newline="") as g:
        r = csv.DictReader(f)
        cols = [c for c in KEEP if c in r.fieldnames]
        w = csv.writer(g)
        w.writerow(cols)
        for x in r:
            if re.search(r"k_small|k_pair|k_large|k_join|k_tie", x["Kernel_Name"]):
                w.writerow([x[c] for c in cols])


if __name__ == "__main__":
    main()
