"""Streaming step-5 I/O: the bounded-memory BAM reader (bsdc_bam_stream_*)
and writer (bsdc_bam_writer_*), CPU only.  The chunks of a coordinate-sorted BAM partition its
records (each chunk in file order); no template or MI family straddles two chunks; the chunks'
family plans (C++ plan, TemplateCoordinate order) concatenate to the whole file's plan; the
streaming writer writes the bytes write_bam writes.  tests/test_gpu_stream.py runs bam.step5_stream against bam.step5."""
import os

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, batch, synth
from bsseqconsensusreads_amd import records as R


@pytest.fixture(autouse=True, params=["serial", "parallel"])
def family_assignment(request, monkeypatch):
    """Every test runs with the stream's MI family assignment serial and in parallel (sharded by
    hash; bsdc_io.cpp stream_split uses it from BSDC_STREAM_PAR_MIN records per split on)."""
    monkeypatch.setenv("BSDC_STREAM_PAR_MIN", "1000000000" if request.param == "serial" else "0")
    return request.param


def _header(ref):
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(ref.names, ref.lengths)) + "@RG\tID:rg1\tSM:s1\tLB:libA\n"
    return bam.BamHeader(text, list(ref.names), np.asarray(ref.lengths, np.int64))


def _sorted_bam(tmp_path, cfg="C2", n_fam=1500, messy=0.2, seed=5, genome_len=400_000, mate_unmapped=0.0):
    s = synth.generate(cfg, n_fam, seed=seed, device="cpu", genome_len=genome_len)
    raw = synth.messify(s.raw, frac=messy, seed=seed) if messy else s.raw
    if mate_unmapped:  # some families' mates flagged unmapped (GroupReadsByUmi keeps such templates in
        # families of their own): their templates sort after every other template of the contig
        fam = np.random.default_rng(seed).random(int(raw.mi_id.max()) + 1) < mate_unmapped
        raw.flag[fam[np.maximum(raw.mi_id, 0)] & (raw.mi_id >= 0)] |= 8
    raw = R.take(raw, np.lexsort((raw.pos, raw.tid)))  # coordinate-sorted, as the step-5 input is
    p = str(tmp_path / "in.bam")
    bam.write_bam(p, _header(s.ref), bam.records_to_bam(raw), level=1, threads=4)
    return s, p


def _ident(raw: R.RawRecords):
    """record identity across chunk-local name ids: (QNAME, flag)"""
    return [(raw.names[int(raw.name_id[k])], int(raw.flag[k])) for k in range(raw.n)]


def test_chunks_partition_the_file(tmp_path):
    """every record in exactly one chunk, decoded as the whole-file reader decodes it, and the
    records of a chunk in file order"""
    s, p = _sorted_bam(tmp_path)
    h, whole = bam.read_bam(p, threads=4)
    parts = list(bam.stream_bam(p, threads=4, chunk_bytes=60_000, slack=2000, read_size=32_768))
    assert len(parts) > 5
    assert all(ph.text == h.text and ph.ref_names == h.ref_names for ph, _ in parts)
    idw = _ident(whole)
    where = {x: k for k, x in enumerate(idw)}
    assert len(where) == whole.n
    seen = []
    for _, r in parts:
        ks = np.asarray([where[x] for x in _ident(r)], np.int64)
        assert (np.diff(ks) > 0).all()  # file order within the chunk
        seen.append(ks)
        for k in ("flag", "tid", "pos", "mapq", "l_seq", "next_tid", "next_pos", "tlen", "mi_strand", "n_cig"):
            assert np.array_equal(getattr(r, k), getattr(whole, k)[ks]), k
        for j in range(0, r.n, 29):
            w = int(ks[j])
            assert np.array_equal(r.record_seq(j), whole.record_seq(w))
            assert np.array_equal(r.record_qual(j), whole.record_qual(w))
            assert np.array_equal(r.record_cigar(j), whole.record_cigar(w))
            assert r.aux[j] == whole.aux[w]
            mi = r.mi_names[int(r.mi_id[j])] if r.mi_id[j] >= 0 else None
            assert mi == (whole.mi_names[int(whole.mi_id[w])] if whole.mi_id[w] >= 0 else None)
    allk = np.sort(np.concatenate(seen))
    assert np.array_equal(allk, np.arange(whole.n))


def test_no_family_or_template_straddles_chunks(tmp_path):
    s, p = _sorted_bam(tmp_path, messy=0.0)
    seen_mi, seen_name = {}, {}
    # the default read size holds the whole file: chunks stay about chunk_bytes anyway
    for i, (_, r) in enumerate(bam.stream_bam(p, threads=2, chunk_bytes=40_000, slack=2000)):
        for k in range(r.n):
            if r.mi_id[k] >= 0:
                assert seen_mi.setdefault(r.mi_names[int(r.mi_id[k])], i) == i
            assert seen_name.setdefault(r.names[int(r.name_id[k])], i) == i
    assert max(seen_mi.values()) > 5


@pytest.mark.parametrize("cfg,mate_unmapped", [("C1", 0.0), ("C2", 0.0), ("C2", 0.03)])
def test_chunk_plans_concatenate_to_the_file_plan(tmp_path, cfg, mate_unmapped):
    """the families of the chunks, in chunk order, are the file's families in TemplateCoordinate
    order: the same MI runs with the same records in the same order"""
    s, p = _sorted_bam(tmp_path, cfg=cfg, n_fam=800, messy=0.15, seed=9, mate_unmapped=mate_unmapped)
    _, whole = bam.read_bam(p, threads=4)
    pw = batch.plan_families(whole, "full", s.ref)
    idw = _ident(whole)
    want = [(whole.mi_names[int(pw.fam_mi[f])], [idw[int(k)] for k in pw.order[pw.fam_off[f]:pw.fam_off[f + 1]]])
            for f in range(pw.n_fam)]
    got = []
    n_chunks = 0
    for _, r in bam.stream_bam(p, threads=4, chunk_bytes=50_000, slack=2000, read_size=20_000):
        n_chunks += 1
        pc = batch.plan_families(r, "full", s.ref)
        idr = _ident(r)
        got += [(r.mi_names[int(pc.fam_mi[f])], [idr[int(k)] for k in pc.order[pc.fam_off[f]:pc.fam_off[f + 1]]])
                for f in range(pc.n_fam)]
    assert n_chunks > 3
    assert got == want


def test_streaming_writer_writes_write_bam_bytes(tmp_path):
    s, p = _sorted_bam(tmp_path, n_fam=600)
    h, raw = bam.read_bam(p, threads=4)
    recs = bam.records_to_bam(raw)
    a, b = str(tmp_path / "a.bam"), str(tmp_path / "b.bam")
    bam.write_bam(a, h, recs, level=5, threads=4)
    w = bam.BamWriter(b, h, level=5)
    n = recs.n
    for lo, hi in ((0, 7), (7, n // 3), (n // 3, n // 3), (n // 3, n)):
        w.add(bam.take_records(recs, np.arange(lo, hi)), threads=3)
    w.close(threads=2)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_stream_of_a_truncated_file_fails_loudly(tmp_path):
    s, p = _sorted_bam(tmp_path, n_fam=300)
    data = open(p, "rb").read()
    t = str(tmp_path / "t.bam")
    open(t, "wb").write(data[: len(data) * 2 // 3])
    with pytest.raises(OSError):
        for _ in bam.stream_bam(t, threads=2, chunk_bytes=20_000, read_size=8192):
            pass


def test_header_only_read(tmp_path):
    s, p = _sorted_bam(tmp_path, n_fam=50)
    h = bam.read_bam_header(p)
    h2, _ = bam.read_bam(p)
    assert h.text == h2.text and h.ref_names == h2.ref_names and np.array_equal(h.ref_lens, h2.ref_lens)
    assert os.path.getsize(p) > 0


def test_unsorted_input_fails_loudly(tmp_path):
    s = synth.generate("C2", 200, seed=3, device="cpu", genome_len=100_000)
    p = str(tmp_path / "u.bam")
    raw = R.take(s.raw, np.random.default_rng(0).permutation(s.raw.n))
    bam.write_bam(p, _header(s.ref), bam.records_to_bam(raw), level=1)
    with pytest.raises(OSError, match="coordinate-sorted"):
        for _ in bam.stream_bam(p, threads=2, chunk_bytes=10_000):
            pass


def test_buffer_pool_reuse_and_trim():
    """bam.BufferPool (the stream reader's record arrays): the smallest free buffer that fits is
    reused, a new one is made when none fits, and the free list keeps its `keep` largest."""
    p = bam.BufferPool(keep=2)
    a = p.take(1000)
    assert a.size >= 1000
    p.give(a)
    assert p.take(500) is a  # reused
    b, c, d = p.take(100), p.take(5000), p.take(300)
    for x in (a, b, c, d):
        p.give(x)
    assert len(p.free) == 2 and sorted(x.size for x in p.free) == sorted([a.size, c.size])
    p.give(None)
    assert len(p.free) == 2
    big = p.take(4000)
    assert big is c
