"""The vote's arithmetic against an independent fp64 restatement of fgbio (tests/fgbio_vote.py).

oracle/ (== the HIP kernels, bit for bit: tests/test_gpu_parity.py) votes in fixed point.  Here its
single-strand reads are compared with fgbio's double-precision log-space vote on the same source
reads, on C0-C4 and on adversarial near-tie columns (disagreeing bases at qualities 80-93, where
the per-read likelihoods differ by less than 2^-20 nats).  Bar (north_star): bases bit-exact
(except exact ties, where fgbio's own pick is the rounding of its summation order and the
fixed-point vote must pick one of the tied bases), qualities within +-1.  The counts are printed
(`pytest -s`) and asserted.
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
    ss = fv.ss_vote(src["count"], src["len"], src["base"], src["qual"], stride)
    return r, ss, fv.compare_ss(r.ss, ss)


def assert_fp64_bar(c, what):
    print(what, c)
    assert c["columns"] > 0
    assert c["base_diff"] == 0, "%s: bases differ from fgbio fp64 outside exact ties: %s" % (what, c)
    assert c["tie_off_set"] == 0, "%s: an exact tie resolved to a base outside the tied set: %s" % (what, c)
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


def test_near_tie_columns_exist_and_need_2e40():
    """The adversarial set really is adversarial: the fixed-point 2^-20 sums alone pick a different
    base than fgbio fp64 on some columns (so the 2^-40 refinement is what keeps the bar)."""
    lr = np.asarray(oracle.tables()[0], np.int64)
    lr40 = oracle.tables40()
    # high qualities: 2^-20 ratios collide, the 2^-40 ones do not
    assert len(set(lr[85:94].tolist())) < 9
    assert len(set(lr40[85:94].tolist())) == 9
    x = fv.qual_tables(30.0)
    ratio = x[1] - x[2]  # ln P(correct) - ln P(error)/3 = the per-read likelihood ratio
    assert np.all(np.abs(lr40 / 2.0 ** 40 - ratio) < 1e-9)


def test_tables40_match_library():
    lib = _lib.load()
    for pre, post in ((45.0, 30.0), (40.0, 25.0)):
        a = np.zeros(256, np.int64)
        lib.bsdc_model_tables40(pre, post, a.ctypes.data)
        assert np.array_equal(a, oracle.tables40(pre, post))
        lr = oracle.tables(pre, post)[0]
        assert np.all(np.abs(a - (np.asarray(lr, np.int64) << 20)) <= (1 << 19) + 1)


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
