"""The vote's arithmetic against an independent fp64 restatement of fgbio (tests/fgbio_vote.py).

oracle/ (== the HIP kernels, bit for bit: tests/test_gpu_parity.py) votes in fixed point.  Here its
single-strand reads are compared with fgbio's double-precision log-space vote on the same source
reads, on C0-C4 and on adversarial near-tie columns (disagreeing bases at qualities 80-93, where
the per-read likelihoods differ by less than 2^-20 nats).  Bar (north_star): bases bit-exact on
every column -- exact ties included (the same quality multiset on two bases), where fgbio's pick is
the rounding of its read-order double sums and the vote reproduces it -- and qualities within +-1.
The counts are printed (`pytest -s`) and asserted.
"""
import numpy as np
import pytest

import fgbio_vote as fv
from bsseqconsensusreads_amd import _lib, synth
from helpers import near_tie_votes
from oracle import oracle

CASES = [("C0", 2000, None), ("C1", 1000, None), ("C2", 2000, None), ("C3", 100, None), ("C4", 800, None),
         ("C1", 1500, 80), ("C2", 2000, 84), ("C1", 1500, 20), ("C4", 600, 88)]


def fp64_check(raw, ref, run_tools=True, **kw):
    r = oracle.run(raw, ref, keep_sources=True, run_tools=run_tools, **kw)
    src = r.sources
    stride = r.ss["base"].shape[2]
    ss = fv.ss_vote(src["count"], src["len"], src["base"], src["qual"], stride,
                    min_cbq=kw.get("min_consensus_base_quality", 2))
    return r, ss, fv.compare_ss(r.ss, ss)


def assert_fp64_bar(c, what):
    print(what, c)
    assert c["columns"] > 0
    assert c["base_diff"] == 0, "%s: bases differ from fgbio fp64: %s" % (what, c)
    assert c["tie_diff"] == 0, "%s: an exact tie resolved unlike fgbio's read-order sums: %s" % (what, c)
    assert c["qual_gt1"] == 0 and c["n_boundary_bad"] == 0, "%s: quality off by more than 1: %s" % (what, c)


@pytest.mark.parametrize("cfg,n,qlo", CASES)
def test_oracle_vote_vs_fgbio_fp64(cfg, n, qlo):
    s = synth.generate(cfg, n, seed=11, device="cpu", genome_len=400_000)
    raw = s.raw if qlo is None else near_tie_votes(s.raw, qlo=qlo, seed=5)
    r, ss, c = fp64_check(raw, s.ref, run_tools=qlo is None)
    assert_fp64_bar(c, "%s n=%d q>=%s" % (cfg, n, qlo))
    # duplex: where both single-strand inputs agree exactly, the duplex column agrees exactly
    st, ln, b, q = fv.duplex(ss)
    assert np.array_equal(st, r.status) and np.array_equal(ln, r.cons_len)
    same_in = np.ones(b.shape, bool)
    w = b.shape[2]
    for e, (sa, sb) in enumerate(((0, 3), (1, 2))):
        for sset in (sa, sb):
            m = min(w, r.ss["base"].shape[2])
            same_in[:, e, :m] &= (r.ss["base"][:, sset, :m] == ss["base"][:, sset, :m]) & \
                                 (r.ss["qual"][:, sset, :m] == ss["qual"][:, sset, :m])
    live = np.arange(w)[None, None, :] < ln[:, :, None]
    m = min(w, r.cons_seq.shape[2])
    bad = live[:, :, :m] & same_in[:, :, :m] & ((b[:, :, :m] != r.cons_seq[:, :, :m]) | (q[:, :, :m] != r.cons_qual[:, :, :m]))
    assert not bad.any()


def test_near_tie_columns_exist_and_exact_ties_resolve():
    """The adversarial sets really are adversarial: at high qualities the 2^-20 ratios collide, so the
    fixed-point sums alone cannot order those columns, and the sets hold exact-tie columns (fp64
    gap 0) whose pick is fgbio's summation rounding -- all resolved as fgbio resolves them."""
    lr = np.asarray(oracle.tables()[0], np.int64)
    assert len(set(lr[85:94].tolist())) < 9
    s = synth.generate("C2", 2000, seed=11, device="cpu", genome_len=400_000)
    raw = near_tie_votes(s.raw, qlo=84, seed=5)
    _, ss, c = fp64_check(raw, s.ref, run_tools=False)
    assert c["tie_columns"] > 0 and c["tie_diff"] == 0 and c["base_diff"] == 0, c
    # and columns whose true sums tie (the same quality multiset on two bases) but whose read-order
    # double sums differ by rounding alone: there fgbio's pick is that rounding, and base_diff == 0
    # above says the vote reproduced it
    live = np.arange(ss["gap"].shape[2])[None, None, :] < ss["len"][:, :, None]
    assert np.count_nonzero(live & (ss["gap"] > 0) & (ss["gap"] < 1e-9)) > 0


def test_fp64_tables_match_library_and_restatement():
    """fgbio's per-read log-space terms: libbsdc (the kernels' copy), oracle/ and tests/fgbio_vote.py
    compute them independently; the near-tie pick sums them, so they must be the same doubles."""
    lib = _lib.load()
    for pre, post in ((45.0, 30.0), (40.0, 25.0), (45.0, 20.0)):
        lnc = np.zeros(256, np.float64)
        lne3 = np.zeros(256, np.float64)
        lib.bsdc_model_tables_fp64(pre, post, lnc.ctypes.data, lne3.ctypes.data)
        o_c, o_e = oracle.tables_fp64(pre, post)
        _, f_c, f_e = fv.qual_tables(post)
        assert np.array_equal(lnc.view(np.uint64), o_c.view(np.uint64))
        assert np.array_equal(lne3.view(np.uint64), o_e.view(np.uint64))
        assert np.array_equal(lnc.view(np.uint64), f_c.view(np.uint64))
        assert np.array_equal(lne3.view(np.uint64), f_e.view(np.uint64))
        # and the fixed-point ratio is their difference, to half a unit of 2^-20
        lr = np.asarray(oracle.tables(pre, post)[0], np.int64)
        assert np.all(np.abs(lr / 2.0 ** 20 - (lnc - lne3)) < 2.0 ** -20)


def test_fp64_worked_values():
    """one Q37 read -> Q29; a duplex agreement of two such -> Q58."""
    count = np.array([[1, 0, 0, 1]], np.int32)
    lens = np.array([1, 1])
    ss = fv.ss_vote(count, lens, np.array([2, 2], np.uint8), np.array([37, 37], np.uint8), 16)
    assert ss["base"][0, 0, 0] == 2 and ss["qual"][0, 0, 0] == 29
    count = np.array([[1, 1, 0, 0]], np.int32)
    ss = fv.ss_vote(count, lens, np.array([2, 2], np.uint8), np.array([37, 37], np.uint8), 16)
    st, ln, b, q = fv.duplex(ss)
    assert st[0] == 1 and ln[0, 0] == 1 and q[0, 0, 0] == 29  # one strand: passes through
    count = np.array([[1, 1, 1, 1]], np.int32)
    ss = fv.ss_vote(count, np.ones(4, np.int64), np.full(4, 2, np.uint8), np.full(4, 37, np.uint8), 16)
    st, ln, b, q = fv.duplex(ss)
    assert q[0, 0, 0] == 58 and b[0, 0, 0] == 2
    # an exact two-read tie: fp64 and fixed point both see a tie
    count = np.array([[2, 0, 0, 0]], np.int32)
    ss = fv.ss_vote(count, np.ones(2, np.int64), np.array([1, 2], np.uint8), np.array([30, 30], np.uint8), 16)
    assert ss["gap"][0, 0, 0] == 0 and ss["tied"][0, 0, 0] == 0b11


def low_quality_votes(raw, seed=5):
    """Columns of four disagreeing low-quality reads: per family 16 positions, each record covering
    one shows a random A/C/G/T (four alleles) at Q0-Q3, or N -- single-strand calls of Q1 (three
    reads A, C, G at one quality: P(error) 2/3) and depth-0 columns (only Ns) among them."""
    return near_tie_votes(raw, n_pos=16, qlo=0, qhi=3, p_n=0.15, n_alleles=4, seed=seed)


def test_min_consensus_base_quality_worked_values():
    """--min-consensus-base-quality: three reads A, C, G at Q30 in one set give
    P(error) ~ 2/3 -> Q1.  Inside the duplex caller (mask 2) that column is (N, 2); step 1
    (main.snake.py:54, mask 0) keeps fgbio's pick at Q1.  A column whose reads are all N is a
    no-call under either mask."""
    count = np.array([[3, 0, 0, 0]], np.int32)
    b, q = np.array([1, 2, 4], np.uint8), np.array([30, 30, 30], np.uint8)
    ss2 = fv.ss_vote(count, np.ones(3, np.int64), b, q, 16, min_cbq=2)
    ss0 = fv.ss_vote(count, np.ones(3, np.int64), b, q, 16, min_cbq=0)
    assert (ss2["base"][0, 0, 0], ss2["qual"][0, 0, 0]) == (15, 2)
    assert ss0["qual"][0, 0, 0] == 1 and ss0["base"][0, 0, 0] in (1, 2, 4)
    nn = fv.ss_vote(np.array([[2, 0, 0, 0]], np.int32), np.ones(2, np.int64), np.array([15, 15], np.uint8),
                    np.array([30, 30], np.uint8), 16, min_cbq=0)
    assert (nn["base"][0, 0, 0], nn["qual"][0, 0, 0]) == (15, 2)


@pytest.mark.parametrize("min_cbq", [2, 0])
def test_low_quality_columns_vs_fgbio_fp64(min_cbq):
    """The restatement's mask against fgbio fp64 on Q0-Q3 disagreement columns, both thresholds:
    Q1 calls exist and keep their base at 0, and are (N, 2) at 2."""
    s = synth.generate("C1", 1500, seed=11, device="cpu", genome_len=400_000)
    raw = low_quality_votes(s.raw)
    r, ss, c = fp64_check(raw, s.ref, run_tools=False, min_consensus_base_quality=min_cbq)
    assert_fp64_bar(c, "low-quality mask %d" % min_cbq)
    assert c["n_boundary"] == 0  # the same threshold on both sides: no N flips at all
    live = np.arange(r.ss["qual"].shape[2])[None, None, :] < r.ss["len"][:, :, None]
    q1 = live & (r.ss["qual"] == 1)
    nq2 = live & (r.ss["base"] == 15) & (r.ss["qual"] == 2)
    if min_cbq == 0:
        assert q1.sum() > 100 and np.isin(r.ss["base"][q1], [1, 2, 4, 8]).all()
    else:
        assert q1.sum() == 0 and nq2.sum() > 100


def test_molecular_low_quality_vs_fgbio_fp64():
    """Step 1's caller (mask 0, MI runs, no BA side) on the same columns."""
    from bsseqconsensusreads_amd import pipeline
    from bsseqconsensusreads_amd import records as R
    s = synth.generate("C1", 800, seed=12, device="cpu", genome_len=400_000)
    raw = low_quality_votes(s.raw, seed=6)
    rm = pipeline.molecular_records(R.take(raw, np.lexsort((raw.mi_strand, raw.mi_id))))
    r, ss, c = fp64_check(rm, s.ref, run_tools=False, family_order="mi-group", min_consensus_base_quality=0)
    assert_fp64_bar(c, "molecular low-quality")
    live = np.arange(r.cons_qual.shape[2])[None, None, :] < r.cons_len[:, :, None]
    assert (live & (r.cons_qual == 1)).sum() > 50
