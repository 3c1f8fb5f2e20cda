"""Times the reference's own tools 1 and 2 on the C0 / C1 workloads (CPU timing
step 1).  TEST INFRASTRUCTURE: runs only in the build container, where /root/reference exists; the
reference never travels to the GPU box.

The tools are imported through the pysam / rich_click stand-ins of make_golden.py (their record
model; in-memory JSON "BAM" files), so BGZF I/O is not included and the stand-in's accessors are
slower than pysam's C ones.  The stand-in's own file read / write time is measured separately
and reported next to the tool time.  The tools are single-threaded: 1 core.

    python tests/golden/time_reference_tools.py [--families 10000] [--configs C1,C0] [--out profiles/r02/...json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (the stand-ins)

from bsseqconsensusreads_amd import records as R  # noqa: E402
from bsseqconsensusreads_amd import synth  # noqa: E402


def to_dicts(raw):
    """RawRecords (synthetic) -> the stand-in's record dicts (MI with its /A|/B, MC, RX)."""
    out = []
    nt = R.NT16_TO_ASCII
    for k in range(raw.n):
        o, L = int(raw.seq_off[k]), int(raw.l_seq[k])
        seq = nt[raw.seq[o:o + L]].tobytes().decode()
        qual = (raw.qual[o:o + L] + 33).tobytes().decode()
        cig = [[int(c) & 0xF, int(c) >> 4] for c in raw.record_cigar(k)]
        strand = "A" if raw.mi_strand[k] == 0 else "B"
        out.append({"name": "t%d" % raw.name_id[k], "flag": int(raw.flag[k]), "tid": int(raw.tid[k]),
                    "pos": int(raw.pos[k]), "mapq": 60, "cigar": cig, "seq": seq, "qual": qual,
                    "next_tid": int(raw.next_tid[k]), "next_pos": int(raw.next_pos[k]), "tlen": int(raw.tlen[k]),
                    "tags": [["MC", "Z", "%dM" % L], ["MI", "Z", "%d/%s" % (raw.mi_id[k], strand)],
                             ["RX", "Z", "ACGT-TGCA"]]})
    # coordinate order, as the step-5 input is sorted
    out.sort(key=lambda d: (d["tid"], d["pos"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=10_000)
    ap.add_argument("--configs", default="C1,C0")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if not os.path.isdir(mg.REF_ROOT):
        print("reference checkout absent; nothing to do")
        return 0
    mg._install_stubs()
    t1 = mg._load(os.path.join(mg.REF_ROOT, "tools", "1.convert_AG_to_CT.py"), "_ref_tool1")
    t2 = mg._load(os.path.join(mg.REF_ROOT, "tools", "2.extend_gap.py"), "_ref_tool2")
    results = []
    for cfg in a.configs.split(","):
        s = synth.generate(cfg, a.families, seed=42, device="cpu", genome_len=2_000_000)
        codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
        contigs = {"chrS": R.NT16_TO_ASCII[codes].tobytes().decode()}
        header = {"references": [{"name": "chrS", "length": len(codes)}]}
        recs = to_dicts(s.raw)
        tmp = tempfile.mkdtemp(prefix="bsdc_time_")
        fa, i1, o1, o2 = (os.path.join(tmp, x) for x in ("ref.json", "in.json", "t1.json", "t2.json"))
        with open(fa, "w") as fh:
            json.dump({"contigs": contigs}, fh)
        with open(i1, "w") as fh:
            json.dump({"header": header, "records": recs}, fh)
        # the stand-in's own file cost: read the input and write it back, as each tool does
        c0 = time.perf_counter()
        with open(i1) as fh:
            d = json.load(fh)
        with open(os.path.join(tmp, "io.json"), "w") as fh:
            json.dump(d, fh)
        io_s = time.perf_counter() - c0
        c0 = time.perf_counter()
        t1.main.callback(input_bam=i1, output_bam=o1, reference=fa)
        tool1_s = time.perf_counter() - c0
        c0 = time.perf_counter()
        t2.main.callback(input_bam=o1, output_bam=o2)
        tool2_s = time.perf_counter() - c0
        n = s.n_fam
        r = {"config": cfg, "families": n, "records": s.raw.n, "cores": 1,
             "tool1_s": round(tool1_s, 2), "tool2_s": round(tool2_s, 2), "standin_io_s_per_tool": round(io_s, 2),
             "tool1_families_per_s": round(n / tool1_s, 1), "tool2_families_per_s": round(n / tool2_s, 1),
             "tools12_families_per_s": round(n / (tool1_s + tool2_s), 1),
             "tools12_families_per_s_excl_standin_io": round(n / max(tool1_s + tool2_s - 2 * io_s, 1e-9), 1)}
        print(json.dumps(r), flush=True)
        results.append(r)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"generator": "tests/golden/time_reference_tools.py", "host": os.uname().nodename,
                       "results": results}, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
