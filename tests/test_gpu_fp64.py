"""The HIP vote against the independent fp64 restatement of fgbio (tests/fgbio_vote.py), through
the C-ABI: single-strand reads (BSDC_MODE_TAGS) and duplex consensus on C0-C4 and on adversarial
near-tie columns, in both kernels (k_small, and k_large with every family forced into it).

Bar (north_star): consensus bases bit-exact and quals within +-1 of fgbio's double-precision
log-space arithmetic, on every column: exact ties (the same multiset of qualities on two bases)
included, where fgbio's pick is the rounding of its read-order double sums and the kernels' near-tie
path (fp64_pick) reproduces it.  Counts are printed (run with -s) and asserted.
"""
import numpy as np
import pytest

import fgbio_vote as fv
from bsseqconsensusreads_amd import batch, pipeline, synth
from helpers import near_tie_votes
from oracle import oracle
from test_fgbio_vote import CASES, assert_fp64_bar, low_quality_votes
from test_gpu_parity import assert_consensus_equal, assert_ss_equal

pytestmark = pytest.mark.gpu


def _gpu_vs_fp64(engine, raw, ref, run_tools, what, molecular=False):
    engine.load_reference(ref)
    min_cbq = 0 if molecular else 2  # main.snake.py:54 vs the duplex caller's single-strand caller
    if molecular:
        cons, raw = pipeline.run_molecular(engine, raw, tags=True)
        r = oracle.run(raw, ref, keep_sources=True, run_tools=False, family_order="mi-group",
                       min_consensus_base_quality=0)
    else:
        if run_tools:
            cons, _ = pipeline.run_step5(engine, raw, tags=True)
        else:
            cons = pipeline.run_duplex(engine, raw, tags=True)
        r = oracle.run(raw, ref, keep_sources=True, run_tools=run_tools)
    assert_consensus_equal(cons, r, what)      # GPU == fixed-point restatement, bit for bit
    assert_ss_equal(cons, r, what)
    src = r.sources
    stride = cons.ss["base"].shape[2]
    ss = fv.ss_vote(src["count"], src["len"], src["base"], src["qual"], stride, min_cbq=min_cbq)
    em = np.nonzero((cons.status & 1) != 0)[0]  # (the kernels' single-strand reads: emitted families)
    c = fv.compare_ss({"len": cons.ss["len"][em], "base": cons.ss["base"][em], "qual": cons.ss["qual"][em]},
                      {k: v[em] for k, v in ss.items()})
    assert_fp64_bar(c, what)
    # duplex consensus vs fgbio fp64 duplex of the fp64 single-strand reads
    st, ln, b, q = fv.duplex(ss)
    assert np.array_equal(st, (cons.status & 1).astype(np.int32)) and np.array_equal(ln, cons.length)
    w = min(b.shape[2], cons.seq.shape[2])
    live = np.arange(w)[None, None, :] < ln[:, :, None]
    db = live & (cons.seq[:, :, :w] != b[:, :, :w])
    dq = np.abs(cons.qual[:, :, :w].astype(np.int64) - q[:, :, :w].astype(np.int64))
    print(what, "duplex columns %d, base diffs %d, qual +-1 %d, qual >1 %d" % (
        int(live.sum()), int(db.sum()), int((live & (dq == 1)).sum()), int((live & (dq > 1)).sum())))
    # a duplex column can differ only where one of its single-strand inputs does (a +-1 qual); with
    # none of those (the usual case), the duplex reads are identical
    same = np.ones(b.shape, bool)
    for e, (sa, sb) in enumerate(((0, 3), (1, 2))):
        for st_ in (sa, sb):
            same[:, e, :w] &= (cons.ss["base"][:, st_, :w] == ss["base"][:, st_, :w]) & \
                              (cons.ss["qual"][:, st_, :w] == ss["qual"][:, st_, :w])
    same[(cons.status & 1) == 0] = True  # (no duplex read there: ln is 0)
    assert not (db & same[:, :, :w]).any(), what + ": duplex base differs from fgbio fp64"
    assert not (live & (dq > 0) & same[:, :, :w]).any(), what + ": duplex qual differs from fgbio fp64"
    if c["qual_pm1"] == 0 and c["n_boundary"] == 0:
        assert int(db.sum()) == 0 and int((live & (dq > 0)).sum()) == 0
    return cons


@pytest.mark.parametrize("cfg,n,qlo", CASES)
def test_gpu_vote_vs_fgbio_fp64(engine, cfg, n, qlo):
    s = synth.generate(cfg, n, seed=11, device="cpu", genome_len=400_000)
    raw = s.raw if qlo is None else near_tie_votes(s.raw, qlo=qlo, seed=5)
    _gpu_vs_fp64(engine, raw, s.ref, qlo is None, "%s n=%d q>=%s" % (cfg, n, qlo))


@pytest.mark.parametrize("qlo", [84, 88])
def test_gpu_large_kernel_near_ties_vs_fgbio_fp64(engine, qlo, monkeypatch):
    """Every family through k_large (its near-tie path in `resolve` and the tag pass)."""
    s = synth.generate("C1", 800, seed=13, device="cpu", genome_len=200_000)
    raw = near_tie_votes(s.raw, qlo=qlo, seed=7)
    real = batch.materialize
    monkeypatch.setattr(pipeline, "materialize",
                        lambda plan, f0, f1, small_cap=0, images=None: real(plan, f0, f1, small_cap=0, images=images))
    _gpu_vs_fp64(engine, raw, s.ref, False, "k_large q>=%d" % qlo)


def _force_large(monkeypatch):
    real = batch.materialize
    monkeypatch.setattr(pipeline, "materialize",
                        lambda plan, f0, f1, small_cap=0, images=None: real(plan, f0, f1, small_cap=0, images=images))


@pytest.mark.parametrize("kernel", ["small", "large"])
@pytest.mark.parametrize("caller", ["duplex", "molecular"])
def test_gpu_min_consensus_base_quality(engine, kernel, caller, monkeypatch):
    """Q0-Q3 disagreement columns (Q1 calls, all-N columns) in both kernels and both callers:
    step 5's duplex caller masks single-strand Q < 2 to (N, 2), step 1 (main.snake.py:54,
    --min-consensus-base-quality=0) keeps the call at Q1; GPU == oracle/ bit for bit, and both
    within the fp64 bar of fgbio's arithmetic.  The engine's own flags are restored afterwards."""
    from bsseqconsensusreads_amd import records as R
    s = synth.generate("C1", 600, seed=17, device="cpu", genome_len=200_000)
    raw = low_quality_votes(s.raw, seed=9)
    if caller == "molecular":
        raw = R.take(raw, np.lexsort((raw.mi_strand, raw.mi_id)))
    if kernel == "large":
        _force_large(monkeypatch)
    cons = _gpu_vs_fp64(engine, raw, s.ref, False, "low-quality %s %s" % (caller, kernel),
                        molecular=caller == "molecular")
    w = cons.ss["qual"].shape[2]
    em = (cons.status & 1) != 0
    live = (np.arange(w)[None, None, :] < cons.ss["len"][:, :, None]) & em[:, None, None]
    q1 = int((live & (cons.ss["qual"] == 1)).sum())
    assert (q1 > 50) if caller == "molecular" else (q1 == 0)
    assert engine.params.min_consensus_base_quality == 2
