"""Batched execution on the GPU: a stream cut into many device batches gives the same consensus
as one batch (and as oracle/), and the workgroup-per-family kernel reproduces the reference
tools' own golden records byte for byte (k_large's tool-1 / tool-2 code: contig-end windows, RD)."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, pipeline, synth
from bsseqconsensusreads_amd import records as R
from helpers import compare_records, golden_inputs, load_golden
from oracle import oracle
from test_gpu_parity import assert_consensus_equal, assert_ss_equal

pytestmark = pytest.mark.gpu


def _same(a, b, what):
    for k in ("fam_mi", "status", "length", "fam_rec_off", "fam_src"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), "%s: %s" % (what, k)
    w = min(a.seq.shape[2], b.seq.shape[2])
    assert np.array_equal(a.seq[:, :, :w], b.seq[:, :, :w]) and np.array_equal(a.qual[:, :, :w], b.qual[:, :, :w])


@pytest.mark.parametrize("messy", [0.0, 0.25])
def test_many_batches_equal_one(engine, messy):
    s = synth.generate("C2", 900, seed=17, device="cpu", genome_len=150_000)
    raw = synth.messify(s.raw, frac=messy, seed=4) if messy else s.raw
    engine.load_reference(s.ref)
    one, _ = pipeline.run_step5(engine, raw, tags=True)
    many, _ = pipeline.run_step5(engine, raw, tags=True, batch_bases=6000)
    assert len(pipeline.plan_ranges(batch.plan_families(raw, "full", s.ref), 6000)) > 30
    _same(one, many, "batched")
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(many, ref, "batched vs oracle")
    assert_ss_equal(many, ref, "batched vs oracle")


def test_split_extension_batched(engine):
    s = synth.generate("C0", 500, seed=15, device="cpu", genome_len=100_000)
    raw = s.raw
    for k in np.nonzero(raw.flag == 163)[0][3:40:9]:
        raw.next_tid[int(k)] = 1
    assert batch.plan_families(raw, "full", s.ref).split_ext
    engine.load_reference(s.ref)
    cons, _ = pipeline.run_step5(engine, raw, batch_bases=3000)
    assert_consensus_equal(cons, oracle.run(raw, s.ref), "split + batched")


def _force_large(monkeypatch, where):
    real_m, real_b = batch.materialize, batch.build_family_batch

    def glob(fb):
        nb = len(fb.large_buckets)
        top = max(max(fb.large_arenas), batch.LARGE_LDS_MAX + 16)
        if where == "global":  # every large family in the last (HBM scratch) bucket
            fb.large_buckets = [np.zeros((0, 4), np.uint32)] * (nb - 1) + [fb.large_fams]
            fb.large_arenas = [16] * (nb - 1) + [top]
        elif where == "two-scratch":  # two buckets beyond the LDS budget, dispatched concurrently
            lf = fb.large_fams
            h = lf.shape[0] // 2
            fb.large_buckets = [np.zeros((0, 4), np.uint32)] * (nb - 2) + [lf[:h], lf[h:]]
            fb.large_arenas = [16] * (nb - 2) + [top + 4096, top + 8192]
        return fb
    monkeypatch.setattr(pipeline, "materialize",
                        lambda plan, f0, f1, small_cap=0, images=None: glob(real_m(plan, f0, f1, 0, images=images)))
    monkeypatch.setattr(pipeline, "build_family_batch",
                        lambda r, mode="full", ref=None, small_cap=0, **kw: glob(real_b(r, mode, ref, small_cap=0, **kw)))


@pytest.mark.parametrize("where", ["lds", "global"])
def test_large_kernel_tool1_fuzz_matches_reference(engine, where, monkeypatch):
    """k_large's two-dword tool-1 tasks (contig-end masking, RD, the seed) against the
    reference's own tool-1 output on the fuzz fixture."""
    _force_large(monkeypatch, where)
    g = load_golden("tool1_fuzz.json.gz")
    raw, ref = golden_inputs(g)
    engine.load_reference(ref)
    compare_records(g["tool1"], pipeline.run_tool1(engine, raw), raw, g["input"], "k_large tool1 fuzz " + where)


@pytest.mark.parametrize("where", ["lds", "global"])
def test_large_kernel_tools12_match_reference(engine, where, monkeypatch):
    _force_large(monkeypatch, where)
    g = load_golden("tool12_families.json.gz")
    raw, ref = golden_inputs(g)
    engine.load_reference(ref)
    compare_records(g["tool1"], pipeline.run_tool1(engine, raw), raw, g["input"], "k_large tool1 families")
    cons, t2 = pipeline.run_step5(engine, raw, dump=True)
    compare_records(g["tool2"], t2, raw, g["input"], "k_large fused tool2 dump " + where)
    assert_consensus_equal(cons, oracle.run(raw, ref), "k_large golden families")


def test_two_scratch_buckets_vs_oracle(engine, monkeypatch):
    """two large buckets beyond the LDS budget run concurrently on the side streams, each
    in its own region of the HBM scratch buffer (no two dispatches share an arena)."""
    _force_large(monkeypatch, "two-scratch")
    s = synth.generate("C3", 60, seed=29, device="cpu", genome_len=200_000)
    engine.load_reference(s.ref)
    cons, _ = pipeline.run_step5(engine, s.raw, tags=True)
    ref = oracle.run(s.raw, s.ref)
    assert_consensus_equal(cons, ref, "two scratch buckets")
    assert_ss_equal(cons, ref, "two scratch buckets")


def test_large_kernel_dump_vs_oracle_contig_ends(engine, monkeypatch):
    """k_large's tool-1/2 records on a genome small enough that many windows run past the contig
    end (the fuzz fixture's case at scale), against oracle/'s tool-2 records."""
    _force_large(monkeypatch, "lds")
    s = synth.generate("C1", 300, seed=19, device="cpu", genome_len=6_000)
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    short = R.Reference.from_codes(["chrS"], [codes[:3300]])  # reads past 3300 convert against N
    assert (s.raw.pos > 3300 - 160).sum() > 100
    engine.load_reference(short)
    cons, t2 = pipeline.run_step5(engine, s.raw, dump=True)
    ref = oracle.run(s.raw, short)
    assert np.array_equal(t2.src, ref.tool2.src) and np.array_equal(t2.pos, ref.tool2.pos)
    assert np.array_equal(t2.seq, ref.tool2.seq) and np.array_equal(t2.qual, ref.tool2.qual)
    assert np.array_equal(t2.cigar, ref.tool2.cigar)
    assert_consensus_equal(cons, ref, "k_large contig ends")
