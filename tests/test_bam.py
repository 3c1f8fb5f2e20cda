"""Host BAM/BGZF codec (libbsdc_io, include/bsdc_io.h) and the duplex output records
(SURVEY.md 8a row 8, 8f ranks 1-2).  CPU only: round trips, an independent BGZF reader/writer
written here with zlib, the RX consensus against a Python restatement, and the output records of
the oracle's consensus."""
import gzip
import struct
import zlib

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, batch, synth
from bsseqconsensusreads_amd import records as R
from oracle import oracle


def _header(ref):
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(ref.names, ref.lengths)) + "@RG\tID:rg1\tSM:s1\tLB:libA\n"
    return bam.BamHeader(text, list(ref.names), np.asarray(ref.lengths, np.int64))


def _messy(n_fam=400, seed=3):
    s = synth.generate("C2", n_fam, seed=seed, device="cpu", genome_len=100_000)
    return s, synth.messify(s.raw, frac=0.3, seed=seed)


def _same_records(a: R.RawRecords, b: R.RawRecords):
    assert a.n == b.n
    for k in ("flag", "tid", "pos", "mapq", "l_seq", "next_tid", "next_pos", "tlen", "mi_strand", "n_cig"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert np.array_equal(a.seq, b.seq) and np.array_equal(a.qual, b.qual)
    assert np.array_equal(a.cigar, b.cigar)
    for k in range(a.n):
        assert a.names[int(a.name_id[k])] == b.names[int(b.name_id[k])]
        if a.mi_id[k] < 0:
            assert b.mi_id[k] < 0
        else:
            assert a.mi_names[int(a.mi_id[k])] == b.mi_names[int(b.mi_id[k])]
        ma = a.mc_cigar[a.mc_off[k]:a.mc_off[k] + a.mc_n[k]] if a.mc_off[k] >= 0 else None
        mb = b.mc_cigar[b.mc_off[k]:b.mc_off[k] + b.mc_n[k]] if b.mc_off[k] >= 0 else None
        assert (ma is None) == (mb is None) and (ma is None or np.array_equal(ma, mb))


def test_round_trip(tmp_path):
    s, raw = _messy()
    hdr = _header(s.ref)
    p = str(tmp_path / "a.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=6, threads=4)
    h2, raw2 = bam.read_bam(p, threads=4)
    assert h2.text == hdr.text and h2.ref_names == hdr.ref_names
    assert np.array_equal(h2.ref_lens, hdr.ref_lens)
    _same_records(raw, raw2)
    # aux bytes survive untouched, and the family builder sees the same families
    for k in range(0, raw.n, 97):
        assert raw2.aux[k] == raw.aux[k]
    f1 = batch.build_family_batch(raw, "full", s.ref)
    f2 = batch.build_family_batch(raw2, "full", s.ref)
    assert np.array_equal(f1.src, f2.src) and np.array_equal(f1.fam_off, f2.fam_off)


def _py_bgzf_read(path):
    """Independent reader: BGZF is multi-member gzip."""
    with gzip.open(path, "rb") as f:
        return f.read()


def _py_bgzf_write(path, data: bytes, block=40000):
    out = bytearray()
    for i in range(0, len(data), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        cd = c.compress(chunk) + c.flush()
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(cd) + 25)
        out += cd + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes([31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0])
    open(path, "wb").write(bytes(out))


def test_bgzf_interoperates_with_zlib(tmp_path):
    s, raw = _messy(200, seed=4)
    hdr = _header(s.ref)
    p = str(tmp_path / "b.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=1, threads=2)
    data = _py_bgzf_read(p)
    assert data[:4] == b"BAM\1"
    l_text = struct.unpack("<i", data[4:8])[0]
    assert data[8:8 + l_text].decode() == hdr.text
    # rewrite the same stream with other block boundaries (records split across blocks)
    q = str(tmp_path / "c.bam")
    _py_bgzf_write(q, data, block=777)
    _, raw3 = bam.read_bam(q, threads=3)
    _same_records(raw, raw3)


def test_zlib_and_libdeflate_backends_agree(tmp_path):
    """The codec deflates / inflates with libdeflate when the system has it, else zlib
    (BSDC_ZLIB forces zlib): each backend reads what the other wrote, to the same records."""
    import os
    import subprocess
    import sys
    s, raw = _messy(150, seed=5)
    hdr = _header(s.ref)
    a = str(tmp_path / "default.bam")
    bam.write_bam(a, hdr, bam.records_to_bam(raw), level=5, threads=2)
    b = str(tmp_path / "zlib.bam")
    code = ("import sys; sys.path.insert(0, %r); from bsseqconsensusreads_amd import bam; "
            "h, r = bam.read_bam(%r, 2); bam.write_bam(%r, h, bam.records_to_bam(r), level=5, threads=2)"
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), a, b))
    subprocess.run([sys.executable, "-c", code], check=True, env=dict(os.environ, BSDC_ZLIB="1"))
    assert _py_bgzf_read(a) == _py_bgzf_read(b)  # the same BAM stream, whatever the compressed bytes
    _, rb = bam.read_bam(b, threads=2)
    _same_records(raw, rb)


def test_corrupt_input_fails_loudly(tmp_path):
    p = tmp_path / "bad.bam"
    p.write_bytes(b"not a bam at all")
    with pytest.raises(OSError, match="BGZF"):
        bam.read_bam(str(p))
    s, raw = _messy(50, seed=5)
    good = tmp_path / "g.bam"
    bam.write_bam(str(good), _header(s.ref), bam.records_to_bam(raw))
    b = bytearray(good.read_bytes())
    b[40] ^= 0xFF  # inside the first block's deflate data
    (tmp_path / "x.bam").write_bytes(bytes(b))
    with pytest.raises(OSError):
        bam.read_bam(str(tmp_path / "x.bam"))


def _py_rx(rxs, strands):
    vals = []
    for rx, st in zip(rxs, strands):
        if rx is None:
            continue
        if st == 1 and "-" in rx:
            a, b2 = rx.split("-", 1)
            rx = b2 + "-" + a
        vals.append(rx)
    if not vals:
        return ""
    lens = [len(v) for v in vals]
    L = max(set(lens), key=lambda l: (lens.count(l), -lens.index(l)))
    out = []
    for j in range(L):
        col = [v[j] for v in vals if len(v) == L]
        cnt = {c: col.count(c) for c in set(col)}
        top = max(cnt.values())
        best = [c for c in cnt if cnt[c] == top]
        out.append(best[0] if len(best) == 1 else "N")
    return "".join(out)


def test_rx_consensus_matches_restatement():
    rng = np.random.default_rng(9)
    b = R._Builder()
    fams, rxs, strands = [], [], []
    k = 0
    for f in range(300):
        recs = []
        u1 = "".join(rng.choice(list("ACGT"), 6))
        u2 = "".join(rng.choice(list("ACGT"), 6))
        for j in range(int(rng.integers(1, 6))):
            st = int(rng.integers(0, 2))
            rx = (u1 + "-" + u2) if st == 0 else (u2 + "-" + u1)
            rx = "".join(c if rng.random() > 0.1 else "T" for c in rx)
            if rng.random() < 0.05:
                rx = rx[:-1]
            has = rng.random() > 0.05
            tags = [("MI", "Z", "%d/%s" % (f, "AB"[st]))] + ([("RX", "Z", rx)] if has else [])
            b.add(b"r%d" % k, 99, 0, 10, 60, [(4 << 4)], np.ones(4, np.uint8), np.full(4, 30, np.uint8), 0, 10, 0,
                  R.encode_aux(tags), tags)
            recs.append(k)
            rxs.append(rx if has else None)
            strands.append(st)
            k += 1
        fams.append(recs)
    raw = b.finish()
    off = np.zeros(len(fams) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in fams])
    cons = type("C", (), {})()
    cons.fam_rec_off = off
    cons.fam_src = np.concatenate([np.asarray(x, np.int64) for x in fams])
    cons.status = np.ones(len(fams), np.uint8)
    cons.fam_mi = np.asarray([raw.mi_id[x[0]] for x in fams], np.int32)
    cons.length = np.ones((len(fams), 2), np.int32)
    cons.seq = np.ones((len(fams), 2, 16), np.uint8)
    cons.qual = np.full((len(fams), 2, 16), 30, np.uint8)
    recs = bam.duplex_records(cons, raw, "pfx", threads=3)
    for f, members in enumerate(fams):
        want = _py_rx([rxs[i] for i in members], [strands[i] for i in members])
        got = R.aux_get(recs.aux[2 * f], "RX") or ""
        assert got == want, (f, got, want)


def test_duplex_records_of_the_oracle_consensus(tmp_path):
    s, raw = _messy(300, seed=6)
    res = oracle.run(raw, s.ref)
    stride = res.cons_seq.shape[2]
    cons = type("C", (), {})()
    cons.fam_rec_off, cons.fam_src = res.fam_rec_off, res.fam_src
    cons.status, cons.fam_mi, cons.length = res.status.astype(np.uint8), res.fam_mi, res.cons_len
    cons.seq, cons.qual = res.cons_seq, res.cons_qual
    hdr = _header(s.ref)
    recs = bam.duplex_records(cons, raw, bam.read_name_prefix(hdr))
    p = str(tmp_path / "out.bam")
    bam.write_bam(p, bam.output_header(hdr), recs)
    h2, out = bam.read_bam(p)
    em = np.nonzero(res.status == 1)[0]
    assert out.n == 2 * em.shape[0]
    assert np.array_equal(out.flag, np.tile([77, 141], em.shape[0]))
    assert (out.tid == -1).all() and (out.pos == -1).all() and (out.n_cig == 0).all()
    assert "@RG\tID:A\tSM:s1\tLB:libA" in h2.text and h2.text.startswith("@HD\tVN:1.6\tSO:unsorted")
    for i, f in enumerate(em):
        mi = raw.mi_names[int(res.fam_mi[f])]
        for e in range(2):
            k = 2 * i + e
            assert out.names[int(out.name_id[k])] == ("libA:%s" % mi).encode()
            assert out.mi_names[int(out.mi_id[k])] == mi and R.aux_get(out.aux[k], "RG") == "A"
            L = int(res.cons_len[f, e])
            o = int(out.seq_off[k])
            assert int(out.l_seq[k]) == L
            assert np.array_equal(out.seq[o:o + L], res.cons_seq[f, e, :L])
            assert np.array_equal(out.qual[o:o + L], res.cons_qual[f, e, :L])
    assert stride > 0


def test_fasta_reader(tmp_path):
    s = synth.generate("C2", 10, seed=8, device="cpu", genome_len=5_000)
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    letters = R.NT16_TO_ASCII[codes].tobytes().decode()
    fa = tmp_path / "g.fa"
    fa.write_text(">chrX other words\nACGTNNNN\nacgt\n>%s\n%s\n" % (
        s.ref.names[0], "\n".join(letters[i:i + 60] for i in range(0, len(letters), 60))))
    hdr = bam.BamHeader("", [s.ref.names[0], "chrMissing"], np.asarray([len(letters), 5], np.int64))
    ref = bam.read_fasta(str(fa), hdr)
    assert ref.contig_off[1] == -1
    got = R.unpack_nibbles(ref.packed, ref.n_nibbles)[ref.contig_off[0]:ref.contig_off[0] + ref.contig_len[0]]
    assert np.array_equal(got, codes)


def _py_fastq(recs, mate):
    """Python restatement of picard SamToFastq's record text for first (mate 1) / second (2) of pair."""
    out = []
    for k in range(recs.n):
        fl = int(recs.flag[k])
        if fl & 0xB00 or not fl & 1 or bool(fl & 0x40) != (mate == 1):
            continue
        s = recs.seq[recs.seq_off[k]:recs.seq_off[k + 1]]
        q = recs.qual[recs.seq_off[k]:recs.seq_off[k + 1]]
        seq = R.NT16_TO_ASCII[s].tobytes().decode()
        if fl & 16:
            seq = seq[::-1].translate(str.maketrans("ACGTMRWSYKVHDBN=", "TGCAKYWSRMBDHVN="))
            q = q[::-1]
        out.append("@%s/%d\n%s\n+\n%s\n" % (recs.names[k].decode(), mate, seq, (q + 33).tobytes().decode()))
    return "".join(out)


def test_fastq_of_the_oracle_consensus(tmp_path):
    s, raw = _messy(300, seed=9)
    res = oracle.run(raw, s.ref)
    cons = type("C", (), {})()
    cons.fam_rec_off, cons.fam_src = res.fam_rec_off, res.fam_src
    cons.status, cons.fam_mi, cons.length = res.status.astype(np.uint8), res.fam_mi, res.cons_len
    cons.seq, cons.qual = res.cons_seq, res.cons_qual
    recs = bam.duplex_records(cons, raw, "libA")
    p1, p2 = str(tmp_path / "r_1.fq.gz"), str(tmp_path / "r_2.fq.gz")
    bam.write_fastq(p1, p2, recs, level=5, threads=3)
    for p, mate in ((p1, 1), (p2, 2)):
        with gzip.open(p, "rt") as fh:
            assert fh.read() == _py_fastq(recs, mate)


def test_fastq_orientation_and_errors(tmp_path):
    b = R._Builder()
    seq = np.asarray([1, 2, 4, 8, 15], np.uint8)
    for nm, fl in ((b"a", 77), (b"a", 141), (b"b", 83), (b"b", 163), (b"c", 77 | 0x100), (b"d", 77 | 0x200),
                   (b"d", 141 | 0x200)):
        b.add(nm, fl, -1, -1, 0, [], seq, np.asarray([30, 31, 32, 33, 2], np.uint8), -1, -1, 0, b"", [("MI", "Z", "1/A")])
    recs = bam.records_to_bam(b.finish())
    p1, p2 = str(tmp_path / "x_1.fq.gz"), str(tmp_path / "x_2.fq.gz")
    bam.write_fastq(p1, p2, recs)
    with gzip.open(p1, "rt") as fh:
        assert fh.read() == "@a/1\nACGTN\n+\n?@AB#\n@b/1\nNACGT\n+\n#BA@?\n"
    with gzip.open(p2, "rt") as fh:
        assert fh.read() == "@a/2\nACGTN\n+\n?@AB#\n@b/2\nACGTN\n+\n?@AB#\n"
    for bad in (((b"a", 77),), ((b"a", 77), (b"z", 141)), ((b"a", 141), (b"a", 77)), ((b"a", 4),)):
        b = R._Builder()
        for nm, fl in bad:
            b.add(nm, fl, -1, -1, 0, [], seq, np.full(5, 30, np.uint8), -1, -1, 0, b"", [("MI", "Z", "1/A")])
        with pytest.raises(ValueError):
            bam.write_fastq(p1, p2, bam.records_to_bam(b.finish()))


def test_family_image_matches_numpy():
    """libbsdc_io's family image (batch.build_family_batch) against a numpy restatement of the
    per-base scatter and the BAM nibble packing."""
    s, raw = _messy(300, seed=11)
    rng = np.random.default_rng(1)
    n = raw.n
    L = raw.l_seq.astype(np.int64)
    cap4 = (L + 2 + 3) & ~np.int64(3)
    dst = np.zeros(n, np.int64)
    dst[1:] = np.cumsum(cap4 + 4 * rng.integers(0, 3, n))[:-1]
    n_slots = int(dst[-1] + cap4[-1]) + 64
    src = raw.seq_off.astype(np.int64)
    packed = np.zeros(n_slots // 2, np.uint8)
    qual = np.zeros(n_slots, np.uint8)
    bam.family_image(src, L, dst, raw.seq, raw.qual, n_slots, packed, qual, threads=4)
    codes = np.zeros(n_slots, np.uint8)
    q2 = np.zeros(n_slots, np.uint8)
    for k in range(n):
        codes[dst[k] + 1:dst[k] + 1 + L[k]] = raw.seq[src[k]:src[k] + L[k]]
        q2[dst[k] + 1:dst[k] + 1 + L[k]] = raw.qual[src[k]:src[k] + L[k]]
    assert np.array_equal(packed, R.pack_nibbles(codes)) and np.array_equal(qual, q2)
    with pytest.raises(ValueError):
        bam.family_image(src, L, dst + 1, raw.seq, raw.qual, n_slots, packed, qual)


def _expected_tags(ss, f, e, L, molecular):
    """fgbio createSamRecord's consensus tags of record (f, e), restated in Python (the C++
    encoder bsdc_consensus_tags is checked against this; fgbio itself: PARITY UNPINNED)."""
    def per_read(d, er, names):
        return [(names[0], int(d.max())), (names[1], int(d.min())), (names[2], np.float32(er.sum()) / np.float32(d.sum()))]
    if molecular:
        d, er = ss["depth"][f, e, :L].astype(np.int64), ss["err"][f, e, :L].astype(np.int64)
        return per_read(d, er, "cD cM cE".split()) + [("cd", list(d)), ("ce", list(er))]
    sa, sb = (0, 3) if e == 0 else (1, 2)
    la, lb = ss["len"][f, sa] > 0, ss["len"][f, sb] > 0
    a = sa if la else sb
    col = lambda s, k: ss[k][f, s, :L].astype(np.int64)  # noqa: E731
    ad, ae = col(a, "depth"), col(a, "err")
    tags = []
    if la and lb:
        bd, be = col(sb, "depth"), col(sb, "err")
        ab, bb, aq, bq = col(sa, "base"), col(sb, "base"), col(sa, "qual"), col(sb, "qual")
        raw = np.where(ab == bb, ab, np.where(aq > bq, ab, np.where(bq > aq, bb, ab)))
        td = ad + bd
        te = np.where(ab == raw, ae, ad) + np.where(bb == raw, be, bd)
        tags += per_read(td, te, "cD cM cE".split()) + per_read(ad, ae, "aD aM aE".split())
        tags += per_read(bd, be, "bD bM bE".split())
    else:
        tags += per_read(ad, ae, "cD cM cE".split()) + per_read(ad, ae, "aD aM aE".split())
    tags += [("ad", list(ad)), ("ae", list(ae)), ("ac", R.NT16_TO_ASCII[col(a, "base")].tobytes().decode()),
             ("aq", (col(a, "qual") + 33).astype(np.uint8).tobytes().decode())]
    if la and lb:
        tags += [("bd", list(bd)), ("be", list(be)), ("bc", R.NT16_TO_ASCII[col(sb, "base")].tobytes().decode()),
                 ("bq", (col(sb, "qual") + 33).astype(np.uint8).tobytes().decode())]
    return tags


def _check_tags(out, res, em, molecular):
    n_two = 0
    for i, f in enumerate(em):
        for e in range(2):
            k = 2 * i + e
            got = [(t, v) for t, _, v in R.parse_aux(bytes(out.aux[k])) if t not in ("RG", "MI", "RX")]
            exp = _expected_tags(res.ss, f, e, int(res.cons_len[f, e]), molecular)
            assert [t for t, _ in got] == [t for t, _ in exp], (f, e)
            for (t, g), (_, x) in zip(got, exp):
                if t.endswith("E"):
                    assert np.float32(g) == x or (np.isnan(g) and np.isnan(x)), (f, e, t, g, x)
                else:
                    assert g == x, (f, e, t)
            n_two += any(t == "bd" for t, _ in got)
    return n_two


def _cons_of(res, with_ss=True):
    cons = type("C", (), {})()
    cons.fam_rec_off, cons.fam_src = res.fam_rec_off, res.fam_src
    cons.status, cons.fam_mi, cons.length = res.status.astype(np.uint8), res.fam_mi, res.cons_len
    cons.seq, cons.qual = res.cons_seq, res.cons_qual
    cons.ss = res.ss if with_ss else None
    return cons


def test_consensus_tags_of_the_oracle_consensus(tmp_path):
    """fgbio's per-read / per-base consensus tags from the restatement's
    single-strand reads, through the native encoder, the BAM writer and the reader."""
    s, raw = _messy(300, seed=8)
    res = oracle.run(raw, s.ref)
    ss = res.ss
    assert (ss["err"] <= ss["depth"]).all() and (ss["depth"] >= 0).all()
    hdr = _header(s.ref)
    p = str(tmp_path / "t.bam")
    bam.write_bam(p, bam.output_header(hdr), bam.duplex_records(_cons_of(res), raw, "x"))
    _, out = bam.read_bam(p)
    em = np.nonzero(res.status == 1)[0]
    assert out.n == 2 * em.shape[0]
    assert _check_tags(out, res, em, False) > 0  # both-strand records are covered
    # one-strand families (AB-only / BA-only ends) are covered too
    one = [(f, e) for f in em for e in range(2) if (res.ss["len"][f, [0, 1][e]] > 0) != (res.ss["len"][f, [3, 2][e]] > 0)]
    assert one


def test_consensus_tags_of_wide_families():
    """Depths past a byte: the kernels' layout (u8 depth / err, exact u16 rows for the families of
    256+ records, device.fetch ss_wide) encodes the same tags as the u16 statistics, which equal
    the Python restatement"""
    from bsseqconsensusreads_amd import batch
    s, raw = _messy(120, seed=12)
    res = oracle.run(raw, s.ref)
    ss = dict(res.ss)
    F = ss["len"].shape[0]
    big = np.zeros(F, bool)
    big[::3] = True  # every third family: depths in the hundreds / thousands
    ss["depth"] = np.where(big[:, None, None], ss["depth"].astype(np.int64) * 137, ss["depth"]).astype(np.uint16)
    ss["err"] = np.where(big[:, None, None], ss["err"].astype(np.int64) * 131, ss["err"]).astype(np.uint16)
    assert ss["depth"].max() > 255
    res.ss = ss
    em = np.nonzero(res.status == 1)[0]
    t16 = bam.consensus_tags(_cons_of(res), em)
    wide = np.where(big, np.cumsum(big) - 1, -1).astype(np.int32)
    ss8 = {"len": ss["len"], "base": ss["base"], "qual": ss["qual"],
           "depth": np.minimum(ss["depth"], 255).astype(np.uint8), "err": np.minimum(ss["err"], 255).astype(np.uint8),
           "wide": wide, "wdepth": ss["depth"][big], "werr": ss["err"][big]}
    d16, e16 = batch.ss_stats16(ss8)
    assert np.array_equal(d16, ss["depth"]) and np.array_equal(e16, ss["err"])
    c8 = _cons_of(res)
    c8.ss = ss8
    t8 = bam.consensus_tags(c8, em)
    assert np.array_equal(t8.off, t16.off) and np.array_equal(t8.buf, t16.buf)
    for i, f in enumerate(em[:40]):
        for e in range(2):
            k = 2 * i + e
            got = [(t, v) for t, _, v in R.parse_aux(bytes(t8.buf[t8.off[k]:t8.off[k + 1]]))]
            exp = _expected_tags(ss, f, e, int(res.cons_len[f, e]), False)
            assert [t for t, _ in got] == [t for t, _ in exp]
            for (t, g), (_, x) in zip(got, exp):
                if not t.endswith("E"):
                    assert g == x, (f, e, t)


def test_molecular_tags_of_the_oracle_consensus(tmp_path):
    from bsseqconsensusreads_amd import pipeline
    s, raw = _messy(200, seed=9)
    raw = R.take(raw, np.lexsort((raw.mi_strand, raw.mi_id)))
    rm = pipeline.molecular_records(raw)
    res = oracle.run(rm, s.ref, run_tools=False, family_order="mi-group")
    p = str(tmp_path / "m.bam")
    bam.write_bam(p, bam.output_header(_header(s.ref)), bam.duplex_records(_cons_of(res), rm, "x", molecular=True))
    _, out = bam.read_bam(p)
    em = np.nonzero(res.status == 1)[0]
    assert out.n == 2 * em.shape[0]
    assert _check_tags(out, res, em, True) == 0


def _raw_stream(tmp_path, n_fam=20, seed=6):
    """(uncompressed BAM bytes, offset of the first record) of a small valid file."""
    s, raw = _messy(n_fam, seed=seed)
    p = str(tmp_path / "ok.bam")
    bam.write_bam(p, _header(s.ref), bam.records_to_bam(raw))
    data = bytearray(_py_bgzf_read(p))
    l_text = struct.unpack("<i", data[4:8])[0]
    o = 8 + l_text
    n_ref = struct.unpack("<i", data[o:o + 4])[0]
    o += 4
    for _ in range(n_ref):
        ln = struct.unpack("<i", data[o:o + 4])[0]
        o += 4 + ln + 4
    return data, o


def test_truncated_files_fail_loudly(tmp_path):
    """A BAM cut anywhere -- inside the magic, the header, a record, a block, or just before the
    EOF block -- is refused or read to its last whole block, never read past."""
    s, raw = _messy(60, seed=7)
    good = tmp_path / "g.bam"
    bam.write_bam(str(good), _header(s.ref), bam.records_to_bam(raw), level=1)
    b = good.read_bytes()
    for cut in (1, 10, 17, 18, 30, len(b) // 3, len(b) // 2, len(b) - 29, len(b) - 28, len(b) - 1):
        t = tmp_path / ("t%d.bam" % cut)
        t.write_bytes(b[:cut])
        try:
            _, r2 = bam.read_bam(str(t))
        except OSError:
            continue
        assert r2.n <= raw.n  # a cut at a block boundary: the records of the whole blocks
    # the same stream re-blocked so that records straddle blocks, then cut mid-record
    data, _ = _raw_stream(tmp_path)
    q = tmp_path / "q.bam"
    _py_bgzf_write(str(q), bytes(data[:len(data) - 100]), block=333)
    with pytest.raises(OSError, match="truncated"):
        bam.read_bam(str(q))


@pytest.mark.parametrize("what", ["block_size_small", "block_size_past_end", "l_read_name_zero", "n_cigar_huge",
                                  "l_seq_huge", "l_seq_negative", "aux_bad_type", "aux_Z_unterminated",
                                  "aux_B_huge_count", "aux_B_bad_subtype", "l_text_huge", "ref_name_len_huge"])
def test_malformed_bam_fields_fail_loudly(tmp_path, what):
    """Hand-damaged fields of valid BGZF content: every length the parser trusts is checked (the
    sanitizer run, tests/sanitize/run.sh, runs these under ASan/UBSan)."""
    data, o = _raw_stream(tmp_path)
    bs = struct.unpack("<i", data[o:o + 4])[0]
    r = o + 4  # first record's body
    l_name = data[r + 8]
    n_cig = struct.unpack("<H", data[r + 12:r + 14])[0]
    l_seq = struct.unpack("<i", data[r + 16:r + 20])[0]
    aux = r + 32 + l_name + 4 * n_cig + (l_seq + 1) // 2 + l_seq
    end = r + bs
    if what == "block_size_small":
        data[o:o + 4] = struct.pack("<i", 20)
    elif what == "block_size_past_end":
        data[o:o + 4] = struct.pack("<i", len(data))
    elif what == "l_read_name_zero":
        data[r + 8] = 0
    elif what == "n_cigar_huge":
        data[r + 12:r + 14] = struct.pack("<H", 0xFFFF)
    elif what == "l_seq_huge":
        data[r + 16:r + 20] = struct.pack("<i", 0x7FFFFFFF)
    elif what == "l_seq_negative":
        data[r + 16:r + 20] = struct.pack("<i", -5)
    elif what == "aux_bad_type":
        data[aux + 2] = ord("q")
    elif what == "aux_Z_unterminated":
        # the record's last aux byte is the final NUL of a Z field: make it a letter
        assert data[end - 1] == 0
        data[end - 1] = ord("x")
    elif what in ("aux_B_huge_count", "aux_B_bad_subtype"):
        # replace the record's aux block by one B array of the same size
        n = end - aux
        assert n >= 8
        sub, cnt = (b"C", 0x7FFFFFF0) if what == "aux_B_huge_count" else (b"k", 1)
        data[aux:end] = b"XBB" + sub + struct.pack("<I", cnt) + bytes(n - 8)
    elif what == "l_text_huge":
        data[4:8] = struct.pack("<I", 0xFFFFFFF0)
    elif what == "ref_name_len_huge":
        l_text = struct.unpack("<i", data[4:8])[0]
        p = 8 + l_text + 4
        data[p:p + 4] = struct.pack("<i", 0x7FFFFFF0)
    q = tmp_path / "m.bam"
    _py_bgzf_write(str(q), bytes(data), block=5000)
    with pytest.raises(OSError):
        bam.read_bam(str(q))


def test_unpack_nibbles_matches_numpy():
    """The consensus rows' nibble unpack (libbsdc_io) = the numpy statement."""
    a = np.random.default_rng(7).integers(0, 256, size=(1000, 2, 40), dtype=np.uint8)
    want = np.empty((1000, 2, 80), np.uint8)
    want[:, :, 0::2] = a >> 4
    want[:, :, 1::2] = a & 0xF
    assert np.array_equal(bam.unpack_nibbles(a, threads=3), want)
    assert bam.unpack_nibbles(np.zeros((0, 2, 8), np.uint8)).shape == (0, 2, 16)
