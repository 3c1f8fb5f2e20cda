"""The streaming, pipelined file-level step 5 (bam.step5_stream: bounded-memory reader, C++ family
formation per chunk, GPU batches, streaming writer) writes the bytes the whole-file step 5
(bam.step5) writes, on a coordinate-sorted synthetic BAM cut into many chunks, and those records
are oracle/'s on the whole file, record by record."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, synth
from bsseqconsensusreads_amd import records as R
from helpers import assert_bam_matches_oracle

pytestmark = pytest.mark.gpu


def _inputs(tmp_path, cfg, n_fam, messy, seed):
    s = synth.generate(cfg, n_fam, seed=seed, device="cpu", genome_len=300_000)
    raw = synth.messify(s.raw, frac=messy, seed=seed) if messy else s.raw
    raw = R.take(raw, np.lexsort((raw.pos, raw.tid)))
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in
                                                    zip(s.ref.names, s.ref.lengths)) + "@RG\tID:A\tSM:s\tLB:L\n"
    hdr = bam.BamHeader(text, list(s.ref.names), np.asarray(s.ref.lengths, np.int64))
    inp = str(tmp_path / "in.bam")
    bam.write_bam(inp, hdr, bam.records_to_bam(raw), level=1, threads=4)
    fa = str(tmp_path / "g.fa")
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    with open(fa, "wb") as fh:
        fh.write((">%s\n" % s.ref.names[0]).encode() + R.NT16_TO_ASCII[codes].tobytes() + b"\n")
    return inp, fa


@pytest.mark.parametrize("cfg,messy", [("C2", 0.0), ("C1", 0.2)])
def test_stream_writes_the_whole_file_bytes(engine, tmp_path, cfg, messy):
    inp, fa = _inputs(tmp_path, cfg, 1200, messy, 17)
    a, b = str(tmp_path / "whole.bam"), str(tmp_path / "stream.bam")
    ia = bam.step5(inp, fa, a, engine=engine, threads=4, level=5)
    stats = {}
    ib = bam.step5_stream(inp, fa, b, engine=engine, threads=4, level=5, chunk_bytes=80_000, slack=2000,
                          stats=stats)
    assert ib["chunks"] > 3
    for k in ("records_in", "families", "families_emitted", "records_out"):
        assert ia[k] == ib[k], k
    assert open(a, "rb").read() == open(b, "rb").read()
    assert assert_bam_matches_oracle(b, inp, fa, "stream %s" % cfg) == ib["records_out"]


@pytest.mark.parametrize("messy", [0.0, 0.15])
def test_molecular_stream_writes_the_whole_file_bytes(engine, tmp_path, messy):
    """Step 1 (bam.molecular_stream, cut between MI runs) == the whole-file step 1 (bam.molecular),
    byte for byte over many chunks, and oracle/'s records on the whole file -- with Q0-Q3
    disagreement columns, whose Q1 calls step 1 keeps (main.snake.py:54).  The GPU BGZF variant
    reads back as the same records."""
    from test_fgbio_vote import low_quality_votes
    from test_molecular_stream import assert_molecular_outputs_match_oracle, grouped_bam
    s, p0 = grouped_bam(tmp_path, n_fam=1500, messy=messy, seed=19)
    _, whole = bam.read_bam(p0)
    p = str(tmp_path / "low.bam")
    bam.write_bam(p, bam.read_bam_header(p0), bam.records_to_bam(low_quality_votes(whole, seed=2)), level=1)
    a, b, c = (str(tmp_path / n) for n in ("whole.bam", "stream.bam", "gpubgzf.bam"))
    fq = (str(tmp_path / "s1.fq.gz"), str(tmp_path / "s2.fq.gz"))
    ia = bam.molecular(p, a, engine=engine, threads=4, level=5)
    ib = bam.molecular_stream(p, b, engine=engine, threads=4, level=5, fastq=fq, chunk_bytes=60_000)
    assert ib["chunks"] > 3
    for k in ("records_in", "families", "families_emitted", "records_out"):
        assert ia[k] == ib[k], k
    assert open(a, "rb").read() == open(b, "rb").read()
    n, q1 = assert_molecular_outputs_match_oracle(b, fq, p, min_cbq=0)
    assert n == ib["records_out"] and q1 > 20
    bam.molecular_stream(p, c, engine=engine, threads=4, level=5, chunk_bytes=60_000, gpu_bgzf=True)
    _, ra = bam.read_bam(a)
    _, rc = bam.read_bam(c)
    assert ra.n == rc.n and np.array_equal(ra.seq, rc.seq) and np.array_equal(ra.qual, rc.qual)
    assert engine.params.min_consensus_base_quality == 2  # the shared engine's own flags are back
