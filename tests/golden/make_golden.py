"""Golden-vector generator for the step-5 B-strand conversion (tool 1) and gap extension (tool 2).

TEST INFRASTRUCTURE ONLY.  Run in the build container, where the read-only reference checkout
exists at /root/reference; it never runs on the GPU box and nothing in the product imports it.

It loads the reference's own scripts
  /root/reference/tools/1.convert_AG_to_CT.py   (main:33-186)
  /root/reference/tools/2.extend_gap.py         (main:145-190)
through importlib with two stand-in modules registered in sys.modules first:
  * ``rich_click`` -> ``click`` (only the decorators are used), and
  * ``pysam``      -> the in-memory model below.  pysam/htslib is not installed in this image
    (SURVEY.md section 8c), so the model restates the pysam semantics the two tools rely on:
    assigning ``seq``/``query_sequence`` clears the qualities, ``qual`` is the phred+33 string,
    ``query_qualities`` an array of ints, ``pos``/``cigar`` alias ``reference_start``/
    ``cigartuples``, ``reference_end`` counts M/D/N/=/X, ``set_tag`` replaces-and-appends, and
    ``FastaFile.fetch`` clamps at the contig end like faidx.
Record streams are exchanged with the tools through small JSON files standing in for BAM.

The fixtures written (data only: inputs and the reference's outputs) are
  tests/golden/tool1_fuzz.json.gz      fuzzed records through tool 1
  tests/golden/tool12_families.json.gz MI families through tool 1 then tool 2
  tests/golden/tool2_missing_mi.json.gz the tool-2 missing-MI error case
Usage:  python tests/golden/make_golden.py   (skips itself when /root/reference is absent)
"""
from __future__ import annotations

import array
import gzip
import importlib.util
import json
import os
import random
import sys
import tempfile
import types

REF_ROOT = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

# --------------------------------------------------------------------------------------------
# pysam stand-in
# --------------------------------------------------------------------------------------------

_REF_CONSUMING = (0, 2, 3, 7, 8)


class AlignedSegment:
    """Minimal model of pysam.AlignedSegment as used by the two tools."""

    def __init__(self, d):
        self.query_name = d["name"]
        self.flag = d["flag"]
        self.reference_id = d["tid"]
        self.reference_start = d["pos"]
        self.mapping_quality = d.get("mapq", 60)
        cig = d.get("cigar")
        self._cigar = [tuple(c) for c in cig] if cig else None
        self._seq = d["seq"] if d.get("seq") else None
        q = d.get("qual")
        self._qual = None if q is None else [ord(c) - 33 for c in q]
        self.next_reference_id = d.get("next_tid", -1)
        self.next_reference_start = d.get("next_pos", -1)
        self.template_length = d.get("tlen", 0)
        self._tags = [list(t) for t in d.get("tags", [])]

    def to_dict(self):
        return {
            "name": self.query_name,
            "flag": self.flag,
            "tid": self.reference_id,
            "pos": self.reference_start,
            "mapq": self.mapping_quality,
            "cigar": [list(c) for c in self._cigar] if self._cigar else [],
            "seq": self._seq or "",
            "qual": None if self._qual is None else "".join(chr(q + 33) for q in self._qual),
            "next_tid": self.next_reference_id,
            "next_pos": self.next_reference_start,
            "tlen": self.template_length,
            "tags": [list(t) for t in self._tags],
        }

    # --- sequence / qualities (pysam: setting the sequence resets the qualities) ---
    @property
    def query_sequence(self):
        return self._seq

    @query_sequence.setter
    def query_sequence(self, v):
        self._seq = v if v else None
        self._qual = None

    seq = query_sequence

    @property
    def query_qualities(self):
        return None if self._qual is None else array.array("B", self._qual)

    @query_qualities.setter
    def query_qualities(self, v):
        if v is None:
            self._qual = None
            return
        v = list(v)
        n = len(self._seq or "")
        if len(v) != n:
            raise ValueError("quality and sequence mismatch: %i != %i" % (len(v), n))
        self._qual = v

    @property
    def qual(self):
        return None if self._qual is None else "".join(chr(q + 33) for q in self._qual)

    @qual.setter
    def qual(self, v):
        if v is None:
            self._qual = None
            return
        self.query_qualities = [ord(c) - 33 for c in v]

    # --- position / cigar ---
    @property
    def pos(self):
        return self.reference_start

    @pos.setter
    def pos(self, v):
        self.reference_start = v

    @property
    def cigartuples(self):
        return None if not self._cigar else list(self._cigar)

    @cigartuples.setter
    def cigartuples(self, v):
        self._cigar = [tuple(c) for c in v] if v else None

    cigar = cigartuples

    @property
    def reference_end(self):
        if self.flag & 4 or not self._cigar:
            return None
        return self.reference_start + sum(l for op, l in self._cigar if op in _REF_CONSUMING)

    # --- tags ---
    def has_tag(self, tag):
        return any(t[0] == tag for t in self._tags)

    def get_tag(self, tag):
        for t in self._tags:
            if t[0] == tag:
                return t[2]
        raise KeyError("tag '%s' not present" % tag)

    def set_tag(self, tag, value, value_type=None, replace=True):
        self._tags = [t for t in self._tags if t[0] != tag]
        if value is None:
            return
        if value_type is None:
            value_type = "i" if isinstance(value, int) else "Z"
        self._tags.append([tag, value_type, value])


class AlignmentFile:
    def __init__(self, path, mode="r", template=None, header=None, **kw):
        self.path = path
        self.mode = mode
        if "r" in mode:
            with open(path) as fh:
                d = json.load(fh)
            self.header = d["header"]
            self._records = d["records"]
        else:
            self.header = template.header if template is not None else header
            self._out = []

    def get_reference_name(self, tid):
        return self.header["references"][tid]["name"]

    def __iter__(self):
        for r in self._records:
            yield AlignedSegment(r)

    def write(self, read):
        self._out.append(read.to_dict())

    def close(self):
        if "w" in self.mode and self._out is not None:
            with open(self.path, "w") as fh:
                json.dump({"header": self.header, "records": self._out}, fh)
            self._out = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
        return False


class FastaFile:
    def __init__(self, path):
        with open(path) as fh:
            self._contigs = json.load(fh)["contigs"]

    def fetch(self, reference, start=None, end=None):
        seq = self._contigs[reference]  # KeyError for an unknown contig, like faidx
        return seq[start:end]


def _install_stubs():
    import click

    pysam = types.ModuleType("pysam")
    pysam.AlignedSegment = AlignedSegment
    pysam.AlignmentFile = AlignmentFile
    pysam.FastaFile = FastaFile
    pysam.CMATCH = 0
    bcftools = types.ModuleType("pysam.bcftools")
    pysam.bcftools = bcftools
    sys.modules["pysam"] = pysam
    sys.modules["pysam.bcftools"] = bcftools
    sys.modules["rich_click"] = click


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# --------------------------------------------------------------------------------------------
# synthetic inputs
# --------------------------------------------------------------------------------------------

IUPAC = "RYMKSWN"


def make_reference(rng):
    contigs = {}
    for name, n in (("chr1", 4000), ("chr2", 600), ("chrM", 180)):
        s = []
        for i in range(n):
            r = rng.random()
            if s and s[-1] == "C" and r < 0.25:
                s.append("G")  # CpG enrichment so the CpG rules fire often
            else:
                s.append(rng.choice("ACGT"))
        s = "".join(s)
        # lowercase (soft-masked) stretches, N runs and the odd IUPAC code
        s = list(s)
        for _ in range(n // 400 + 1):
            a = rng.randrange(n)
            for j in range(a, min(n, a + rng.randint(5, 60))):
                s[j] = s[j].lower()
        for _ in range(n // 1000 + 1):
            a = rng.randrange(n)
            for j in range(a, min(n, a + rng.randint(1, 8))):
                s[j] = "N"
        for _ in range(3):
            s[rng.randrange(n)] = rng.choice(IUPAC)
        contigs[name] = "".join(s)
    header = {
        "references": [
            {"name": "chr1", "length": len(contigs["chr1"])},
            {"name": "chr2", "length": len(contigs["chr2"])},
            {"name": "chrM", "length": len(contigs["chrM"])},
            {"name": "chrUn_absent", "length": 300},  # in the header, not in the FASTA
        ],
        "read_groups": [{"ID": "A", "LB": "libA", "SM": "S"}],
    }
    return contigs, header


def bs_convert(seq, top, rng, meth_cpg=0.75, meth_other=0.005):
    """Bisulfite/EM-seq conversion of a forward-orientation ref window."""
    out = list(seq.upper())
    for i, b in enumerate(out):
        if top and b == "C":
            cpg = i + 1 < len(out) and out[i + 1] == "G"
            if rng.random() > (meth_cpg if cpg else meth_other):
                out[i] = "T"
        elif (not top) and b == "G":
            cpg = i > 0 and seq[i - 1].upper() == "C"
            if rng.random() > (meth_cpg if cpg else meth_other):
                out[i] = "A"
    return out


def mutate(bases, rng, err=0.01, nrate=0.005):
    for i in range(len(bases)):
        r = rng.random()
        if r < err:
            bases[i] = rng.choice("ACGT")
        elif r < err + nrate:
            bases[i] = "N"
        elif bases[i] not in "ACGT":
            bases[i] = "N"
    return bases


def rand_qual(n, rng):
    return "".join(chr(33 + rng.choice((2, 12, 25, 30, 37, 37, 37, 40, 41))) for _ in range(n))


def ref_window(contigs, header, tid, pos, n):
    name = header["references"][tid]["name"]
    s = contigs.get(name)
    if s is None:
        return "".join(random.choice("ACGT") for _ in range(n))
    w = s[pos:pos + n]
    return w + "".join("A" for _ in range(n - len(w)))


def cigar_len_query(cig):
    return sum(l for op, l in cig if op in (0, 1, 4, 7, 8))


def cigar_len_ref(cig):
    return sum(l for op, l in cig if op in (0, 2, 3, 7, 8))


def random_cigar(rng, L, kind):
    """Cigar with query length L."""
    if kind == "M":
        return [[0, L]]
    if kind == "S5":
        a = rng.randint(1, 12)
        return [[4, a], [0, L - a]]
    if kind == "S3":
        a = rng.randint(1, 12)
        return [[0, L - a], [4, a]]
    if kind == "SS":
        a, b = rng.randint(1, 8), rng.randint(1, 8)
        return [[4, a], [0, L - a - b], [4, b]]
    if kind == "I":
        a = rng.randint(10, L - 20)
        i = rng.randint(1, 3)
        return [[0, a], [1, i], [0, L - a - i]]
    if kind == "D":
        a = rng.randint(10, L - 20)
        return [[0, a], [2, rng.randint(1, 4)], [0, L - a]]
    if kind == "H5":
        return [[5, rng.randint(1, 10)], [0, L]]
    if kind == "H3S":
        a = rng.randint(1, 6)
        return [[0, L - a], [4, a], [5, 3]]
    if kind == "EQX":
        a = rng.randint(5, L - 5)
        return [[7, a], [8, 1], [7, L - a - 1]]
    if kind == "N":
        a = rng.randint(10, L - 10)
        return [[0, a], [3, rng.randint(5, 30)], [0, L - a]]
    raise ValueError(kind)


def mc_string(cig):
    return "".join("%d%s" % (l, "MIDNSHP=X"[op]) for op, l in cig)


def fuzz_records(rng, contigs, header, n):
    flags = [0, 1, 83, 99, 147, 163] * 6 + [65, 129, 81, 161, 97, 145, 339, 355, 403, 419, 2131, 2145, 16, 4]
    kinds = ["M"] * 12 + ["S5", "S3", "SS", "I", "D", "H5", "H3S", "EQX", "N"]
    recs = []
    for k in range(n):
        tid = rng.choice([0, 0, 0, 1, 1, 2, 3])
        clen = header["references"][tid]["length"]
        L = rng.choice([150, 150, 150, 151, 100, 36, 75, 149])
        kind = rng.choice(kinds)
        cig = random_cigar(rng, L, kind)
        rlen = cigar_len_ref(cig)
        r = rng.random()
        if r < 0.05:
            pos = 0
        elif r < 0.15:
            pos = max(0, clen - rlen + rng.randint(-3, 2))
        else:
            pos = rng.randrange(0, max(1, clen - rlen))
        win = ref_window(contigs, header, tid, pos, L + 4)
        top = rng.random() < 0.5
        # start the query at the first aligned base; leading clips get random bases
        lead = cig[0][1] if cig[0][0] == 4 else (cig[1][1] if len(cig) > 1 and cig[0][0] == 5 and cig[1][0] == 4 else 0)
        body = bs_convert(win, top, rng)
        q = "".join(rng.choice("ACGT") for _ in range(lead)) + "".join(body)
        q = list(q[:L])
        while len(q) < L:
            q.append(rng.choice("ACGT"))
        if rng.random() < 0.3:
            # bias: put 'A' after C of CpG sites to exercise the C,A -> T,G rule
            for i in range(L - 1):
                if q[i] == "C" and rng.random() < 0.3:
                    q[i + 1] = "A"
        q = mutate(q, rng)
        seq = "".join(q)
        flag = rng.choice(flags)
        if flag == 4:
            flag = 0
        recs.append({
            "name": "q%05d" % k, "flag": flag, "tid": tid, "pos": pos, "mapq": 60,
            "cigar": cig, "seq": seq, "qual": rand_qual(L, rng),
            "next_tid": tid, "next_pos": pos + rng.randint(0, 300), "tlen": rng.randint(-400, 400),
            "tags": [["MI", "Z", "%d/%s" % (k, rng.choice("AB"))], ["RX", "Z", "ACGT-TTGA"]],
        })
    return recs


def make_template(rng, contigs, header, mi, strand, top, tid, s, e, L, cig1="M", cig2="M", rx="AAC-GGT"):
    """One read pair of fragment [s, e) on contig tid. top -> 99/147, else 83/163."""
    name = "t%s_%s_%d" % (mi, strand, rng.randrange(10**6))
    recs = []
    frag = ref_window(contigs, header, tid, s, e - s)
    conv = bs_convert(frag, top, rng)
    if top:
        specs = [(99, s, conv[:L], cig1), (147, e - L, conv[len(conv) - L:], cig2)]
    else:
        specs = [(163, s, conv[:L], cig1), (83, e - L, conv[len(conv) - L:], cig2)]
    out = []
    for flag, pos, body, kind in specs:
        cig = random_cigar(rng, L, kind)
        q = list(body)
        # realign query to the cigar very roughly (indels are just shifts; fine for golden vectors)
        q = mutate(q[:L], rng, err=0.003)
        out.append((flag, pos, "".join(q), cig))
    (f1, p1, s1, c1), (f2, p2, s2, c2) = out
    tlen = e - s
    for (flag, pos, seq, cig), (mflag, mpos, mseq, mcig) in (((f1, p1, s1, c1), (f2, p2, s2, c2)), ((f2, p2, s2, c2), (f1, p1, s1, c1))):
        recs.append({
            "name": name, "flag": flag, "tid": tid, "pos": pos, "mapq": 60, "cigar": cig,
            "seq": seq, "qual": rand_qual(len(seq), rng),
            "next_tid": tid, "next_pos": mpos, "tlen": tlen if pos <= mpos else -tlen,
            "tags": [["MC", "Z", mc_string(mcig)], ["MI", "Z", "%s/%s" % (mi, strand)],
                     ["RX", "Z", rx if strand == "A" else "-".join(rx.split("-")[::-1])]],
        })
    return recs


def family_records(rng, contigs, header, nfam):
    recs = []
    for k in range(nfam):
        mi = str(k)
        tid = rng.choice([0, 0, 0, 1, 2])
        clen = header["references"][tid]["length"]
        L = rng.choice([150, 150, 151, 100, 60])
        flen = rng.randint(L + 2, min(clen - 1, L + 250)) if clen > L + 4 else L + 2
        r = rng.random()
        s = 0 if r < 0.03 else rng.randrange(0, max(1, clen - flen))
        e = min(clen, s + flen)
        if e - s < L:
            s, e = 0, min(clen, L + 2)
            L = min(L, e - s)
        ab_top = rng.random() < 0.5
        shape = rng.random()
        fam = []
        if shape < 0.55:  # the pipeline as written: 1 template per strand
            k1 = rng.choice(["M"] * 10 + ["S5", "S3", "SS", "I", "D", "H5"])
            k2 = rng.choice(["M"] * 10 + ["S5", "S3", "SS", "I", "D", "H3S"])
            fam += make_template(rng, contigs, header, mi, "A", ab_top, tid, s, e, L, k1, k2)
            fam += make_template(rng, contigs, header, mi, "B", not ab_top, tid, s, e, L,
                                 rng.choice(["M"] * 12 + ["S5", "SS"]), rng.choice(["M"] * 12 + ["S3", "SS"]))
        elif shape < 0.70:  # only one strand
            fam += make_template(rng, contigs, header, mi, rng.choice("AB"), rng.random() < 0.5, tid, s, e, L)
        elif shape < 0.85:  # several templates per strand
            for _ in range(rng.randint(1, 3)):
                fam += make_template(rng, contigs, header, mi, "A", ab_top, tid, s, e, L)
            for _ in range(rng.randint(0, 3)):
                fam += make_template(rng, contigs, header, mi, "B", not ab_top, tid, s, e, L)
        else:  # odd groups: duplicated flags, flags 0/1, dropped flags
            fam += make_template(rng, contigs, header, mi, "A", ab_top, tid, s, e, L)
            odd = rng.choice(["dup", "flag0", "flag1", "drop97", "single"])
            t = make_template(rng, contigs, header, mi, "B", not ab_top, tid, s, e, L)
            if odd == "dup":
                t[0]["flag"] = fam[0]["flag"]
            elif odd == "flag0":
                t[0]["flag"] = 0
            elif odd == "flag1":
                t[0]["flag"] = 1
            elif odd == "drop97":
                t[0]["flag"] = 97
            elif odd == "single":
                t = t[:1]
            fam += t
        recs += fam
    # interleave families a little, as a coordinate sort would (tool 2 groups by first-seen MI)
    rng.shuffle(recs)
    recs.sort(key=lambda r: (r["tid"], r["pos"] // 40))
    return recs


def main():
    if not os.path.isdir(REF_ROOT):
        print("reference checkout absent; nothing to do")
        return 0
    _install_stubs()
    t1 = _load(os.path.join(REF_ROOT, "tools", "1.convert_AG_to_CT.py"), "_ref_tool1")
    t2 = _load(os.path.join(REF_ROOT, "tools", "2.extend_gap.py"), "_ref_tool2")

    rng = random.Random(20250620)
    contigs, header = make_reference(rng)
    tmp = tempfile.mkdtemp(prefix="bsdc_golden_")
    fa = os.path.join(tmp, "ref.json")
    with open(fa, "w") as fh:
        json.dump({"contigs": contigs}, fh)

    def run_tool1(recs):
        ip, op = os.path.join(tmp, "t1_in.json"), os.path.join(tmp, "t1_out.json")
        with open(ip, "w") as fh:
            json.dump({"header": header, "records": recs}, fh)
        t1.main.callback(input_bam=ip, output_bam=op, reference=fa)
        with open(op) as fh:
            return json.load(fh)["records"]

    def run_tool2(recs):
        ip, op = os.path.join(tmp, "t2_in.json"), os.path.join(tmp, "t2_out.json")
        with open(ip, "w") as fh:
            json.dump({"header": header, "records": recs}, fh)
        t2.main.callback(input_bam=ip, output_bam=op)
        with open(op) as fh:
            return json.load(fh)["records"]

    # 1) tool 1 fuzz
    fz = fuzz_records(rng, contigs, header, 2500)
    fz_out = run_tool1(fz)
    # 2) families through tools 1 and 2
    fam = family_records(rng, contigs, header, 700)
    fam_t1 = run_tool1(fam)
    fam_t2 = run_tool2(fam_t1)
    # 3) missing MI -> ValueError in tool 2 (tools/2.extend_gap.py:179-180)
    miss = family_records(random.Random(7), contigs, header, 3)
    for r in miss:
        if r["flag"] in (99, 147):
            r["tags"] = [t for t in r["tags"] if t[0] != "MI"]
            break
    miss_t1 = run_tool1(miss)
    try:
        run_tool2(miss_t1)
        miss_err = None
    except ValueError as e:
        miss_err = str(e)

    meta = {"generator": "tests/golden/make_golden.py", "reference": "tools/1.convert_AG_to_CT.py, tools/2.extend_gap.py"}
    with gzip.open(os.path.join(HERE, "tool1_fuzz.json.gz"), "wt") as fh:
        json.dump({"meta": meta, "contigs": contigs, "header": header, "input": fz, "tool1": fz_out}, fh)
    with gzip.open(os.path.join(HERE, "tool12_families.json.gz"), "wt") as fh:
        json.dump({"meta": meta, "contigs": contigs, "header": header, "input": fam, "tool1": fam_t1, "tool2": fam_t2}, fh)
    with gzip.open(os.path.join(HERE, "tool2_missing_mi.json.gz"), "wt") as fh:
        json.dump({"meta": meta, "contigs": contigs, "header": header, "input": miss, "tool1": miss_t1, "tool2_error": miss_err}, fh)
    print("fuzz: %d in -> %d out; families: %d in -> %d t1 -> %d t2; missing-MI error: %r" % (
        len(fz), len(fz_out), len(fam), len(fam_t1), len(fam_t2), miss_err))
    return 0


if __name__ == "__main__":
    sys.exit(main())
