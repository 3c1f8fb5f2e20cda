"""Step 1 in bounded memory (rule call_consensus_reads_molecular, main.snake.py:46-55; SURVEY.md 8f
rank 3), CPU only: the run chunker (bsdc_bam_stream_next_runs) partitions a GroupReadsByUmi-ordered
BAM between runs of one MI value, so every chunk's MI runs (pipeline.molecular_records) are whole
and concatenate to the file's; bam.molecular_stream's thread pipeline, with its GPU stage answered
by oracle/ (tests/fleet_standin.OracleRunner, TEST INFRASTRUCTURE ONLY), writes the BAM (with tags)
and FASTQ pair oracle/ computes on the whole file, record by record.  tests/test_gpu_stream.py runs
it against bam.molecular on the GPU."""
import contextlib
import types

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, device, pipeline, synth
from bsseqconsensusreads_amd import records as R
from fleet_standin import OracleRunner
from oracle import oracle


def grouped_bam(tmp_path, cfg="C2", n_fam=900, messy=0.1, seed=3):
    """A GroupReadsByUmi-like BAM: each MI's /A then /B molecule contiguous (not coordinate-sorted)."""
    s = synth.generate(cfg, n_fam, seed=seed, device="cpu", genome_len=300_000)
    raw = synth.messify(s.raw, frac=messy, seed=seed) if messy else s.raw
    raw = R.take(raw, np.lexsort((raw.mi_strand, raw.mi_id)))
    text = "@HD\tVN:1.6\tSO:unsorted\tGO:query\n" + "".join(
        "@SQ\tSN:%s\tLN:%d\n" % (n, l) for n, l in zip(s.ref.names, s.ref.lengths)) + "@RG\tID:A\tSM:s\tLB:L\n"
    hdr = bam.BamHeader(text, list(s.ref.names), np.asarray(s.ref.lengths, np.int64))
    p = str(tmp_path / "grouped.bam")
    bam.write_bam(p, hdr, bam.records_to_bam(raw), level=1, threads=4)
    return s, p


def _mi_values(raw):
    sfx = {0: "/A", 1: "/B"}
    return [raw.mi_names[int(raw.mi_id[k])] + sfx.get(int(raw.mi_strand[k]), "") if raw.mi_id[k] >= 0 else ""
            for k in range(raw.n)]


def test_run_chunks_partition_the_file_between_runs(tmp_path):
    s, p = grouped_bam(tmp_path)
    _, whole = bam.read_bam(p, threads=4)
    mw = _mi_values(whole)
    parts = [c.decode(2)[1] for c in bam.stream_chunks(p, 2, chunk_bytes=50_000, read_size=16_384, runs=True)]
    assert len(parts) > 5
    k0 = 0
    prev_last = None
    for r in parts:
        m = _mi_values(r)
        assert m == mw[k0:k0 + r.n]  # the file's records, in order
        for j in range(0, r.n, 17):
            assert r.names[int(r.name_id[j])] == whole.names[int(whole.name_id[k0 + j])]
            assert np.array_equal(r.record_seq(j), whole.record_seq(k0 + j))
            assert np.array_equal(r.record_qual(j), whole.record_qual(k0 + j))
        assert m[0] != prev_last  # a chunk opens a new MI run
        prev_last = m[-1]
        k0 += r.n
    assert k0 == whole.n
    # the chunks' runs concatenate to the file's runs (names and members)
    want = pipeline.molecular_records(whole)
    got_names, got_sizes = [], []
    for r in parts:
        rm = pipeline.molecular_records(r)
        got_names += list(rm.mi_names)
        got_sizes += np.bincount(rm.mi_id[rm.mi_id >= 0]).tolist()
    assert got_names == list(want.mi_names)
    assert got_sizes == np.bincount(want.mi_id[want.mi_id >= 0]).tolist()


def test_run_chunks_of_one_long_run_and_of_an_empty_file(tmp_path):
    s, p = grouped_bam(tmp_path, n_fam=40, messy=0.0)
    _, whole = bam.read_bam(p)
    one = R.take(whole, np.arange(whole.n))
    one.mi_id[:] = 0
    one.mi_strand[:] = 0
    one.aux = None  # (records_to_bam then writes MI from mi_id / mi_strand)
    q = str(tmp_path / "one.bam")
    hdr = bam.read_bam_header(p)
    bam.write_bam(q, hdr, bam.records_to_bam(one), level=1)
    parts = list(bam.stream_chunks(q, 1, chunk_bytes=2_000, runs=True))
    assert len(parts) == 1 and parts[0].decode()[1].n == whole.n  # a run is never cut
    e = str(tmp_path / "empty.bam")
    bam.write_bam(e, hdr, bam.records_to_bam(R.records_from_dicts([])), level=1)
    assert list(bam.stream_chunks(e, 1, chunk_bytes=2_000, runs=True)) == []


class _HostPool:
    def images(self, n_slots):
        return np.empty(n_slots // 2 + 64, np.uint8), np.empty(n_slots, np.uint8)

    def reset(self):
        pass


class _MolecularRunner(OracleRunner):
    """oracle/ as CallMolecularConsensusReads: vote only, MI-run families, the engine's mask."""

    min_cbq = 2

    def _result(self, raw):
        return oracle.run(raw, self.ref, threads=2, run_tools=False, family_order="mi-group",
                          min_consensus_base_quality=self.min_cbq)


class _Engine:
    device = "cpu"

    def __init__(self):
        self.runner = _MolecularRunner(0)
        self.runner.ref = types.SimpleNamespace(names=[], contig_off=[], contig_len=[], letters={})
        self.flag_log = []

    @contextlib.contextmanager
    def flags(self, **kw):
        old = self.runner.min_cbq
        self.runner.min_cbq = kw.get("min_consensus_base_quality", old)
        self.flag_log.append(self.runner.min_cbq)
        try:
            yield self
        finally:
            self.runner.min_cbq = old

    def close(self):
        pass


@pytest.fixture
def standin(monkeypatch):
    monkeypatch.setattr(device, "PinnedPool", _HostPool)
    orig = pipeline.materialize_ranges

    def materialize_ranges(plan, ranges, images=None):
        fbs = orig(plan, ranges, images)
        for fb in fbs:
            fb._raw = plan.raw
        return fbs

    def run_batches(engine, batches, mode, tags=False, timing=None):
        assert mode == pipeline.MODE_VOTE
        return [pipeline.consensus_from_output(fb, engine.runner.run_batch(fb, mode, tags, R.take(fb._raw, np.asarray(
            fb.src, np.int64)))) for fb in batches]
    monkeypatch.setattr(pipeline, "materialize_ranges", materialize_ranges)
    monkeypatch.setattr(pipeline, "run_batches", run_batches)
    return _Engine()


def assert_molecular_outputs_match_oracle(out_bam, fastq, in_bam, min_cbq=0):
    """step 1's BAM (R1, R2 per emitted run, file order) and FASTQ text against oracle/ on the
    whole file's runs."""
    import gzip
    _, whole = bam.read_bam(in_bam, threads=4)
    rm = pipeline.molecular_records(whole)
    r = oracle.run(rm, types.SimpleNamespace(names=[], contig_off=[], contig_len=[], letters={}), threads=4,
                   run_tools=False, family_order="mi-group", min_consensus_base_quality=min_cbq)
    em = np.nonzero(r.status == 1)[0]
    n = 0
    if out_bam is not None:
        _, out = bam.read_bam(out_bam, threads=4)
        assert out.n == 2 * em.shape[0]
        for j, f in enumerate(em):
            for e in range(2):
                k, L = 2 * j + e, int(r.cons_len[f, e])
                assert out.qname(k).endswith((":" + rm.mi_names[int(r.fam_mi[f])]).encode())
                assert np.array_equal(out.record_seq(k), r.cons_seq[f, e, :L])
                assert np.array_equal(out.record_qual(k), r.cons_qual[f, e, :L])
        n = out.n
    if fastq is not None:
        with gzip.open(fastq[1], "rt") as fh:
            lines = fh.read().split("\n")
        assert len(lines) == 4 * em.shape[0] + 1
        for j, f in enumerate(em[:200]):
            L = int(r.cons_len[f, 1])
            assert lines[4 * j].endswith(":%s/2" % rm.mi_names[int(r.fam_mi[f])])
            assert lines[4 * j + 3] == (r.cons_qual[f, 1, :L] + 33).tobytes().decode()
    return n, int((r.cons_qual[np.arange(r.cons_qual.shape[2])[None, None, :] < r.cons_len[:, :, None]] == 1).sum())


def test_molecular_stream_pipeline_matches_oracle(standin, tmp_path):
    from test_fgbio_vote import low_quality_votes
    s, p0 = grouped_bam(tmp_path, n_fam=700, seed=8)
    _, whole = bam.read_bam(p0)
    low = low_quality_votes(whole, seed=4)  # Q1 calls kept at step 1's mask 0
    p = str(tmp_path / "low.bam")
    bam.write_bam(p, bam.read_bam_header(p0), bam.records_to_bam(low), level=1)
    out, fq = str(tmp_path / "m.bam"), (str(tmp_path / "m1.fq.gz"), str(tmp_path / "m2.fq.gz"))
    stats = {}
    info = bam.molecular_stream(p, out, engine=standin, threads=2, level=1, fastq=fq, chunk_bytes=50_000, stats=stats)
    assert info["chunks"] > 4 and standin.flag_log == [0]
    n, q1 = assert_molecular_outputs_match_oracle(out, fq, p, min_cbq=0)
    assert n == info["records_out"] and q1 > 20


def test_run_names_vectorised_equal_the_string_path():
    """pipeline.molecular_records on a decoded BAM's packed MI table (the streaming path) names the
    runs exactly as the per-run string path does: MI + "/A" or "/B", "" without an MI."""
    from bsseqconsensusreads_amd import pipeline
    from bsseqconsensusreads_amd.bam import StringTable
    names = ["7", "12", "103", "x"]
    tab = StringTable.from_list(names)
    ids = np.array([0, 0, 1, -1, 2, 2, 3, 1], np.int32)
    strands = np.array([0, 1, 1, -1, 0, -1, 1, 0], np.int8)
    got = pipeline._run_names(tab, ids, strands)
    sfx = {0: "/A", 1: "/B", -1: ""}
    want = [names[i] + sfx[s] if i >= 0 else "" for i, s in zip(ids, strands)]
    assert [got[k] for k in range(len(want))] == want
    assert len(pipeline._run_names(tab, ids[:0], strands[:0])) == 0
