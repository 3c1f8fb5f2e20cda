"""Shared test helpers: golden fixtures and record comparisons."""
import gzip
import json
import os

import numpy as np

from bsseqconsensusreads_amd import records as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_golden(name):
    with gzip.open(os.path.join(GOLDEN, name), "rt") as fh:
        return json.load(fh)


def golden_inputs(g):
    raw = R.records_from_dicts(g["input"])
    names = [c["name"] for c in g["header"]["references"]]
    ref = R.Reference.from_contigs(names, g["contigs"], header_lengths=[c["length"] for c in g["header"]["references"]])
    return raw, ref


def compare_records(golden_out, produced, raw, inputs, what=""):
    """golden_out: list of fixture dicts (reference tool output, in order);
    produced: an OracleRecords / OutRecords with .record(k); inputs: fixture input dicts."""
    n = len(produced.src)
    assert n == len(golden_out), "%s: %d records vs golden %d" % (what, n, len(golden_out))
    for k in range(n):
        g = golden_out[k]
        p = produced.record(k)
        src = inputs[p["src"]]
        ctx = "%s record %d (%s flag %d)" % (what, k, g["name"], g["flag"])
        assert src["name"] == g["name"] and src["flag"] == g["flag"], ctx + ": wrong record/order"
        assert p["pos"] == g["pos"], ctx + ": pos %d vs %d" % (p["pos"], g["pos"])
        gc = [(l << 4) | op for op, l in g["cigar"]]
        assert [int(x) for x in p["cigar"]] == gc, ctx + ": cigar %s vs %s" % (
            R.cigar_string(p["cigar"]), R.cigar_string(gc))
        gs = R.encode_seq(g["seq"]) if g["seq"] else np.zeros(0, np.uint8)
        assert np.array_equal(p["seq"], gs), ctx + ": seq\n%s\n%s" % (R.decode_seq(p["seq"]), g["seq"])
        gq = np.frombuffer(g["qual"].encode(), np.uint8) - 33 if g["qual"] is not None else None
        assert gq is not None and np.array_equal(p["qual"], gq), ctx + ": qual"
        gt = {t[0]: t[2] for t in g["tags"]}
        st = {t[0]: t[2] for t in src["tags"]}
        for t in ("RD", "LA"):
            exp = gt.get(t, None)
            got = p[t.lower()] if p[t.lower()] >= 0 else st.get(t, None)
            assert exp == got, ctx + ": tag %s %r vs %r" % (t, got, exp)
        # every other tag passes through
        assert {k: v for k, v in gt.items() if k not in ("RD", "LA")} == {k: v for k, v in st.items() if k not in ("RD", "LA")}, ctx


def trim_tails(raw, frac=0.3, seed=1, min_len=30):
    """Adapter-trimmed reads: a fraction of records lose a random number of 3' bases (sequencing
    orientation: the end of a forward read, the start of a reverse one), cigar and position
    adjusted.  Simple-cigar records only; others pass unchanged."""
    rng = np.random.default_rng(seed)
    b = R._Builder()
    for k in range(raw.n):
        seq, qual = raw.record_seq(k).copy(), raw.record_qual(k).copy()
        cig = [int(x) for x in raw.record_cigar(k)]
        flag, pos, L = int(raw.flag[k]), int(raw.pos[k]), len(seq)
        if len(cig) == 1 and (cig[0] & 0xF) == R.OP_M and L > min_len and rng.random() < frac:
            cut = int(rng.integers(1, L - min_len))
            if flag & 16:  # reverse read: its 3' end is the leftmost bases
                seq, qual, pos = seq[cut:], qual[cut:], pos + cut
            else:
                seq, qual = seq[:L - cut], qual[:L - cut]
            cig = [((L - cut) << 4) | R.OP_M]
        tags = [("MI", "Z", "%s/%s" % (raw.mi_id[k], "A" if raw.mi_strand[k] == 0 else "B")),
                ("MC", "Z", "%dM" % L)]
        b.add(("t%d" % raw.name_id[k]).encode(), flag, int(raw.tid[k]), pos, 60, cig, seq, qual,
              int(raw.next_tid[k]), int(raw.next_pos[k]), int(raw.tlen[k]), R.encode_aux(tags), tags)
    return b.finish()


def near_tie_votes(raw, n_pos=6, seed=3, qlo=80, qhi=93, p_n=0.1, n_alleles=2):
    """Adversarial vote columns (a copy of `raw`): per family, `n_pos` reference positions inside
    its forward reads' span get, in every record covering them, a random A/C/G/T base (`n_alleles`
    alleles per position) at a random quality in [qlo, qhi] (an N at Q2 with probability p_n).  High
    qualities make the per-read likelihoods nearly equal (lr[q] saturates at the post-UMI error
    rate), so columns where the bases disagree are near ties -- fgbio's fp64 sums separate them,
    2^-20 fixed point does not."""
    import dataclasses
    rng = np.random.default_rng(seed)
    seq, qual = raw.seq.copy(), raw.qual.copy()
    pos = raw.pos.astype(np.int64)
    fam = raw.mi_id.astype(np.int64)
    L = raw.l_seq.astype(np.int64)
    fwd = (raw.flag & 16) == 0
    n_fam = int(fam.max()) + 1 if raw.n else 0
    start = np.full(n_fam, np.iinfo(np.int64).max)
    np.minimum.at(start, fam[fwd], pos[fwd])
    P = start[:, None] + rng.integers(20, 130, size=(n_fam, n_pos))
    alle = rng.choice(np.array([1, 2, 4, 8], np.uint8), size=(n_fam, n_pos, n_alleles))
    for k in range(raw.n):
        f = int(fam[k])
        j = P[f] - pos[k]
        ok = (j >= 0) & (j < L[k])
        for i in np.nonzero(ok)[0]:
            o = int(raw.seq_off[k] + j[i])
            if rng.random() < p_n:
                seq[o], qual[o] = 15, 2
            else:
                seq[o] = alle[f, i, int(rng.integers(0, n_alleles))]
                qual[o] = int(rng.integers(qlo, qhi + 1))
    return dataclasses.replace(raw, seq=seq, qual=qual)


def assert_bam_matches_oracle(out_bam, in_bam, fasta, what=""):
    """The step-5 output BAM, record by record (R1, R2 per emitted family, TemplateCoordinate
    order): name suffix, SEQ and QUAL against oracle/ on the whole input file."""
    from bsseqconsensusreads_amd import bam
    from oracle import oracle
    _, whole = bam.read_bam(in_bam, threads=4)
    ref = bam.read_fasta(fasta, bam.read_bam_header(in_bam))
    r = oracle.run(whole, ref, threads=8)
    em = np.nonzero(r.status == 1)[0]
    _, out = bam.read_bam(out_bam, threads=4)
    assert out.n == 2 * em.shape[0], "%s: %d records vs %d" % (what, out.n, 2 * em.shape[0])
    for j, f in enumerate(em):
        mi = whole.mi_names[int(r.fam_mi[f])]
        mi = mi if isinstance(mi, bytes) else mi.encode()
        for e in range(2):
            k = 2 * j + e
            n = int(r.cons_len[f, e])
            ctx = "%s family %d end %d" % (what, f, e)
            assert int(out.l_seq[k]) == n, ctx
            assert np.array_equal(out.record_seq(k), r.cons_seq[f, e, :n]), ctx + ": SEQ"
            assert np.array_equal(out.record_qual(k), r.cons_qual[f, e, :n]), ctx + ": QUAL"
            assert out.qname(k).endswith(b":" + mi), ctx + ": name"
    return int(out.n)
