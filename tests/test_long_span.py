"""Long-span templates in the one-process stream (include/bsdc_io.h
bsdc_bam_stream_set_defer; reference: main.snake.py:152's external TemplateCoordinate sort and the
100 GB RAM note, README.md:83).

A template whose mate lies kilobases to megabases away on the same contig would hold every family
after its key in memory until the stream reaches its far end.  The stream defers such templates
(and the families whose keys may interleave with theirs) to a spill, runs the spill as a second
pass and splices its families in at their keys.  Checked here on the CPU with the oracle stand-in
of tests/test_stream_pipeline.py: the output equals the stream without deferral (which holds
everything) byte for byte after decompression, and oracle/ on the whole file record by record;
the stream's buffered bytes stay within a fixed multiple of chunk_bytes, where without deferral
they grow to most of the file."""
import gzip
import json

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, synth
from bsseqconsensusreads_amd import records as R
from helpers import assert_bam_matches_oracle
from test_stream_pipeline import standin  # noqa: F401 -- (the fixture)

CHUNK = 60_000
READ = 16 << 10  # compressed bytes per refill: small, so that the buffer is what the selection holds


def _long_input(tmp, n_fam=2500, genome_len=6_000_000, frac=0.02, seed=23, cross=0.0):
    s = synth.generate("C2", n_fam, seed=seed, device="cpu", genome_len=genome_len, long_frac=frac,
                       long_span=(20_000, 2_500_000), long_giant=True)
    raw = s.raw
    if cross:  # some templates' R2 moved onto a second contig (mate on another contig)
        rng = np.random.default_rng(seed)
        fam_x = rng.random(int(raw.mi_id.max()) + 1) < cross
        by_name = {}
        for k in range(raw.n):
            by_name.setdefault(int(raw.name_id[k]), []).append(k)
        for ks in by_name.values():
            if len(ks) != 2 or raw.mi_id[ks[0]] < 0 or not fam_x[int(raw.mi_id[ks[0]])]:
                continue
            i, j = (ks[0], ks[1]) if raw.flag[ks[0]] & 64 else (ks[1], ks[0])
            P = int(rng.integers(1000, 35_000))
            raw.tid[j], raw.pos[j] = 1, P
            raw.next_tid[i], raw.next_pos[i] = 1, P
            raw.next_tid[j], raw.next_pos[j] = 0, raw.pos[i]
            raw.tlen[i] = raw.tlen[j] = 0
        codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
        c0 = R.NT16_TO_ASCII[codes[:int(s.ref.contig_len[0])]].tobytes()
        c1 = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 40_000).tobytes())
        names = [s.ref.names[0], "chrX2"]
        ref = R.Reference.from_contigs(names, {names[0]: c0, names[1]: c1}, keep_letters=False)
    else:
        ref = s.ref
    raw = R.take(raw, np.lexsort((raw.pos, raw.tid)))
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(ref.names, ref.lengths)) + "@RG\tID:A\tSM:s\tLB:L\n"
    hdr = bam.BamHeader(text, list(ref.names), np.asarray(ref.lengths, np.int64))
    p = str(tmp / "in.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=1, threads=4)
    fa = str(tmp / "g.fa")
    codes = R.unpack_nibbles(ref.packed, ref.n_nibbles)
    with open(fa, "wb") as fh:
        for i, n in enumerate(ref.names):
            o, ln = int(ref.contig_off[i]), int(ref.contig_len[i])
            fh.write((">%s\n" % n).encode() + R.NT16_TO_ASCII[codes[o:o + ln]].tobytes() + b"\n")
    span = np.abs(raw.next_pos.astype(np.int64) - raw.pos.astype(np.int64))
    return raw, p, fa, span


def _stream(standin, tmp, p, fa, tag, **kw):  # noqa: F811
    out = str(tmp / ("%s.bam" % tag))
    fq = (str(tmp / ("%s_1.fq.gz" % tag)), str(tmp / ("%s_2.fq.gz" % tag)))
    info = bam.step5_stream(p, fa, out, engine=standin, threads=2, level=1, fastq=fq, chunk_bytes=CHUNK, slack=2000,
                            read_size=READ, **kw)
    return info, [gzip.decompress(open(x, "rb").read()) for x in (out,) + fq], out


@pytest.mark.parametrize("cross", [0.0, 0.05])
def test_long_span_stream_is_bounded_and_exact(standin, tmp_path, cross):  # noqa: F811
    raw, p, fa, span = _long_input(tmp_path, cross=cross)
    assert (span > 20_000).sum() >= 40 and span.max() > 3_000_000  # (the giant spans > half the contig)
    held, ref_bytes, _ = _stream(standin, tmp_path, p, fa, "held", defer=0)
    info, got, out = _stream(standin, tmp_path, p, fa, "defer", defer=1000)
    assert info["spilled_bytes"] > 0 and info["spliced_families"] > 40
    json.dumps(info)  # (the CLI prints it: plain numbers only)
    for a, b in zip(got, ref_bytes):  # (BAM and the FASTQ pair decompress to the same bytes)
        assert a == b
    for k in ("families", "families_emitted", "records_out", "records_in"):
        assert info[k] == held[k], k
    # memory: without deferral the giant template holds most of the file; with it a few chunks
    _, whole = bam.read_bam(p, threads=2)
    total = int(whole.l_seq.astype(np.int64).sum()) * 2  # (a lower bound on the record bytes)
    assert held["peak_buffered"] > total // 3, (held["peak_buffered"], total)
    assert info["peak_buffered"] <= 8 * CHUNK, (info["peak_buffered"], CHUNK)
    assert_bam_matches_oracle(out, p, fa, "long-span stream") > 0
    assert not [f for f in (tmp_path).iterdir() if f.name.startswith(".")], "spill files left behind"


def test_no_far_templates_writes_in_place(standin, tmp_path):  # noqa: F811
    """Without far templates the deferring stream writes the file in place: the same compressed
    bytes as with deferral off."""
    s = synth.generate("C2", 800, seed=5, device="cpu", genome_len=300_000)
    raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(s.ref.names, s.ref.lengths))
    hdr = bam.BamHeader(text, list(s.ref.names), np.asarray(s.ref.lengths, np.int64))
    p = str(tmp_path / "in.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=1, threads=2)
    fa = str(tmp_path / "g.fa")
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    with open(fa, "wb") as fh:
        fh.write((">%s\n" % s.ref.names[0]).encode() + R.NT16_TO_ASCII[codes].tobytes() + b"\n")
    a, b = str(tmp_path / "a.bam"), str(tmp_path / "b.bam")
    bam.step5_stream(p, fa, a, engine=standin, threads=2, level=1, chunk_bytes=CHUNK, slack=2000, defer=0)
    info = bam.step5_stream(p, fa, b, engine=standin, threads=2, level=1, chunk_bytes=CHUNK, slack=2000)
    assert info["deferred_families"] == 0 and info["spliced_families"] == 0
    assert open(a, "rb").read() == open(b, "rb").read()


def test_spill_entries_sort_back_to_file_order():
    """bsdc_spill_sort: entries {coordinate, sequence, record} from several streams, out of order,
    come back as their records sorted by (coordinate, sequence), stably; a truncated spill fails"""
    rng = np.random.default_rng(3)
    ents, want = [], []
    for k in range(300):
        c, q = int(rng.integers(0, 50)), int(rng.integers(0, 1 << 40))
        body = bytes(rng.integers(0, 256, int(rng.integers(32, 90)), dtype=np.uint8))
        rec = len(body).to_bytes(4, "little") + body
        ents.append((c, q, k, rec))
    order = sorted(ents, key=lambda e: (e[0], e[1], e[2]))
    data = b"".join(c.to_bytes(8, "little", signed=True) + q.to_bytes(8, "little", signed=True) + r
                    for c, q, _, r in ents)
    got, n = bam.spill_sorted_records(data)
    assert n == 300 and got == b"".join(e[3] for e in order)
    with pytest.raises(ValueError):
        bam.spill_sorted_records(data[:-5])


def test_long_span_stream_c4_giant_families(standin, tmp_path):  # noqa: F811
    """C4's skewed families (up to hundreds of templates per molecule) with 3% long-span templates:
    a deferred template whose molecule is large joins or defers with it whole; the stream's bytes
    equal the stream without deferral and oracle/"""
    s = synth.generate("C4", 800, seed=11, device="cpu", genome_len=4_000_000, long_frac=0.03,
                       long_span=(20_000, 1_500_000), long_giant=True)
    raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))
    ref = s.ref
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(ref.names, ref.lengths)) + "@RG\tID:A\tSM:s\tLB:L\n"
    hdr = bam.BamHeader(text, list(ref.names), np.asarray(ref.lengths, np.int64))
    p = str(tmp_path / "in.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=1, threads=4)
    fa = str(tmp_path / "g.fa")
    codes = R.unpack_nibbles(ref.packed, ref.n_nibbles)
    with open(fa, "wb") as fh:
        for i, n in enumerate(ref.names):
            o, ln = int(ref.contig_off[i]), int(ref.contig_len[i])
            fh.write((">%s\n" % n).encode() + R.NT16_TO_ASCII[codes[o:o + ln]].tobytes() + b"\n")
    held, ref_bytes, _ = _stream(standin, tmp_path, p, fa, "held", defer=0)
    info, got, out = _stream(standin, tmp_path, p, fa, "defer", defer=1000)
    assert info["spilled_bytes"] > 0
    for a, b in zip(got, ref_bytes):
        assert a == b
    assert assert_bam_matches_oracle(out, p, fa, "stream, C4 long-span") > 0
