"""An independent fp64 restatement of fgbio's single-strand vote and duplex combine (TEST
INFRASTRUCTURE ONLY -- the checker of the vote's arithmetic, never the product).

The kernels and oracle/ vote in exact fixed point: likelihood sums in
2^-20 nats, a float32 exp, float thresholds; on a near tie they take fgbio's own pick, the four
double-precision sums added read by read in fgbio's read order.  fgbio computes the whole model in
double-precision log space.  This module restates fgbio's arithmetic the way fgbio writes it,
sharing no table and no code with either (main.snake.py:163 for the flags):

  ConsensusCaller.ConsensusBaseBuilder.add   per read with an A/C/G/T base:
      pErr  = probabilityOfErrorTwoTrials(ln e_post, ln e(q))          (log space)
      L[b] += not(pErr) for the read's base, pErr - ln 3 for the three others
  ConsensusBaseBuilder.call
      b*    = first maximum of L over A, C, G, T
      pErr  = not(L[b*] - or(L))                                        (or = logsumexp)
      pErr' = probabilityOfErrorTwoTrials(ln e_pre, pErr)
      Q     = min(93, floor(-10 pErr' / ln 10 + 0.001))                (PhredScore.fromLogProbability)
  VanillaUmiConsensusCaller: depth 0 (fewer contributions than min-reads 1) or
      Q < min-consensus-base-quality -> (N, 2): 2 inside the duplex caller, 0 for step 1
  LogProbability: or(a, b) = max + log1p(exp(min - max)); and(a, b) = a + b;
      aOrNotB(a, b) = a + log1p(-exp(b - a)); not(x) = log(-expm1(x)) near 0, log1p(-exp(x)) else;
      probabilityOfErrorTwoTrials(x, y) = aOrNotB(or(x, y), ln(4/3) + x + y)   (x + y - 4/3 x y)
  DuplexConsensusCaller.duplexConsensus: per column of min(len): agree -> sum, disagree -> the
      higher quality's base with the difference, equal -> (N, 2); capped at 93; N or 2 -> (N, 2);
      a strand absent -> the other passes through.

fgbio is not vendored, so this is a restatement of its published behaviour, not a
pinned copy: the comparison bounds how far the fixed-point vote can be from fp64 log space.  Input:
the source reads oracle/ records per set (oracle.run(..., keep_sources=True)), i.e. everything
before the vote, whose integer stages are checked elsewhere.
"""
from __future__ import annotations

import math

import numpy as np

LN10 = math.log(10.0)
LN3 = math.log(3.0)
LN43 = math.log(4.0 / 3.0)
ONE_HOT = {1: 0, 2: 1, 4: 2, 8: 3}  # nt16 A, C, G, T
N_CODE = 15


def _or2(a, b):
    m, n = np.maximum(a, b), np.minimum(a, b)
    with np.errstate(invalid="ignore"):
        return np.where(np.isneginf(m), m, m + np.log1p(np.exp(n - m)))


def _not(x):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(x > -math.log(2.0), np.log(-np.expm1(x)), np.log1p(-np.exp(x)))


def _a_or_not_b(a, b):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(np.isneginf(b), a, a + np.log1p(-np.exp(b - a)))


def error_two_trials(x, y):
    """LogProbability.probabilityOfErrorTwoTrials: ln(p1 + p2 - 4/3 p1 p2) from ln p1, ln p2."""
    return _a_or_not_b(_or2(x, y), LN43 + x + y)


def _or_s(a, b):
    m, n = max(a, b), min(a, b)
    return m if m == -math.inf else m + math.log1p(math.exp(n - m))


def _not_s(x):
    return math.log(-math.expm1(x)) if x > -math.log(2.0) else math.log1p(-math.exp(x))


def _a_or_not_b_s(a, b):
    return a if b == -math.inf else a + math.log1p(-math.exp(b - a))


def qual_tables(post: float):
    """Per phred 0..255: ln P(error), ln P(correct), ln P(error)/3 of one read after the post-UMI step.
    Scalar `math` calls (the C library's log / exp / log1p / expm1, the functions fgbio's JVM math
    also rounds correctly almost everywhere), not numpy's vectorised ones: the per-read terms are
    what fgbio adds up, so they must be the exact doubles."""
    x = -post * LN10 / 10.0
    p_err = np.array([_a_or_not_b_s(_or_s(x, -q * LN10 / 10.0), LN43 + x + -q * LN10 / 10.0)
                      for q in range(256)], np.float64)
    return p_err, np.array([_not_s(v) for v in p_err], np.float64), p_err - LN3


def phred_from_ln(ln_p):
    with np.errstate(invalid="ignore"):
        q = np.floor(-10.0 * (ln_p / LN10) + 0.001)
    return np.minimum(q, 93).astype(np.int64)


def ss_vote(count, lens, base, qual, stride, pre=45.0, post=30.0, min_cbq=2):
    """Single-strand consensus of every (family, set) from its source reads.

    count [F, 4] reads per set, lens / flat base (nt16) / qual per read in family / set order.
    -> dict: len [F, 4]; base, qual [F, 4, stride]; gap [F, 4, stride] = L(b*) - L(second)
    (fp64 nats); tied [F, 4, stride] one-hot mask of the bases whose sum equals the maximum (0 where
    no read has an A/C/G/T)."""
    F = count.shape[0]
    nrow = 4 * F
    cnt = count.reshape(-1).astype(np.int64)
    lens = np.asarray(lens, np.int64)
    set_of = np.repeat(np.arange(nrow, dtype=np.int64), cnt)
    lc = np.zeros(nrow, np.int64)
    if lens.shape[0]:
        np.maximum.at(lc, set_of, lens)
    out_len = lc.reshape(F, 4).astype(np.int32)
    tot = int(lens.sum())
    roff = np.cumsum(lens) - lens
    rid = np.repeat(np.arange(lens.shape[0], dtype=np.int64), lens)
    col = np.arange(tot, dtype=np.int64) - roff[rid]
    row = set_of[rid] * stride + col
    b = np.asarray(base[:tot], np.int64)
    q = np.asarray(qual[:tot], np.int64)
    bidx = np.full(tot, -1, np.int64)
    for code, k in ONE_HOT.items():
        bidx[b == code] = k
    ok = bidx >= 0
    _, p_cor, p_err3 = qual_tables(post)
    L = np.zeros((4, nrow * stride), np.float64)
    r_ok, b_ok, q_ok = row[ok], bidx[ok], q[ok]
    for k in range(4):  # np.bincount sums in entry order: read by read for each column, as fgbio adds them
        w = np.where(b_ok == k, p_cor[q_ok], p_err3[q_ok])
        L[k] = np.bincount(r_ok, weights=w, minlength=nrow * stride)
    depth = np.bincount(r_ok, minlength=nrow * stride)
    best = np.argmax(L, axis=0)  # first maximum
    m = L[best, np.arange(nrow * stride)]
    tot_ln = m + np.log(np.exp(L - m[None, :]).sum(0))
    p_err = _not(m - tot_ln)
    p_adj = error_two_trials(np.full_like(p_err, -pre * LN10 / 10.0), p_err)
    Q = phred_from_ln(p_adj)
    srt = np.sort(L, axis=0)
    gap = srt[3] - srt[2]
    tied = np.zeros(nrow * stride, np.int64)
    for k in range(4):
        tied |= np.where((L[k] == m) & (depth > 0), 1 << k, 0)
    live = np.arange(stride)[None, :] < lc[:, None]
    nocall = (Q < min_cbq) | (depth == 0)
    callb = np.where(nocall, N_CODE, 1 << best).reshape(nrow, stride)
    callq = np.where(nocall, 2, Q).reshape(nrow, stride)
    return {"len": out_len,
            "base": np.where(live, callb, 0).astype(np.uint8).reshape(F, 4, stride),
            "qual": np.where(live, callq, 0).astype(np.uint8).reshape(F, 4, stride),
            "gap": gap.reshape(F, 4, stride), "tied": np.where(live, tied.reshape(nrow, stride), 0).reshape(F, 4, stride)}


def duplex(ss):
    """DuplexConsensusCaller.duplexConsensus on the four single-strand reads per family:
    R1 = AB-R1 (+) BA-R2, R2 = AB-R2 (+) BA-R1 -> (status, len [F, 2], base / qual [F, 2, stride])."""
    ln = ss["len"].astype(np.int64)
    F, _, stride = ss["base"].shape
    has = ln > 0
    out_b = np.zeros((F, 2, stride), np.uint8)
    out_q = np.zeros((F, 2, stride), np.uint8)
    out_l = np.zeros((F, 2), np.int32)
    cols = np.arange(stride)[None, :]
    for e, (sa, sb) in enumerate(((0, 3), (1, 2))):
        ha, hb = has[:, sa], has[:, sb]
        ba, qa = ss["base"][:, sa].astype(np.int64), ss["qual"][:, sa].astype(np.int64)
        bb, qb = ss["base"][:, sb].astype(np.int64), ss["qual"][:, sb].astype(np.int64)
        same = ba == bb
        rb = np.where(same, ba, np.where(qa > qb, ba, np.where(qb > qa, bb, ba)))
        rq = np.where(same, qa + qb, np.where(qa > qb, qa - qb, np.where(qb > qa, qb - qa, 2)))
        rq = np.minimum(rq, 93)
        mask = (ba == N_CODE) | (bb == N_CODE) | (rq == 2)
        rb = np.where(mask, N_CODE, rb)
        rq = np.where(mask, 2, rq)
        both = ha & hb
        L = np.where(both, np.minimum(ln[:, sa], ln[:, sb]), np.where(ha, ln[:, sa], np.where(hb, ln[:, sb], 0)))
        b = np.where(both[:, None], rb, np.where(ha[:, None], ba, bb))
        q = np.where(both[:, None], rq, np.where(ha[:, None], qa, qb))
        live = cols < L[:, None]
        out_b[:, e] = np.where(live, b, 0)
        out_q[:, e] = np.where(live, q, 0)
        out_l[:, e] = L
    emit = (has[:, 0] | has[:, 3]) & (has[:, 1] | has[:, 2])
    out_l[~emit] = 0
    return emit.astype(np.int32), out_l, out_b, out_q


def compare_ss(got: dict, ref: dict) -> dict:
    """Kernel / oracle single-strand reads (`got`: len, base, qual [F, 4, stride], nt16) against
    this restatement (`ref` from ss_vote).  Returns counts: columns compared, base differences (every
    column, exact ties included: the vote takes fgbio's fp64 read-order pick on near ties, so a tie
    of the same quality multiset on two bases must resolve as fgbio's summation rounds it), the
    exact-tie columns (fp64 gap 0 between two bases, depth > 0) and the base differences among
    them, and the quality differences by size."""
    assert np.array_equal(got["len"], ref["len"]), "single-strand lengths differ"
    stride = min(got["base"].shape[2], ref["base"].shape[2])
    live = np.arange(stride)[None, None, :] < ref["len"][:, :, None]
    gb, rb = got["base"][:, :, :stride].astype(np.int64), ref["base"][:, :, :stride].astype(np.int64)
    gq, rq = got["qual"][:, :, :stride].astype(np.int64), ref["qual"][:, :, :stride].astype(np.int64)
    tie = live & (ref["gap"][:, :, :stride] == 0) & (np.bitwise_count(ref["tied"][:, :, :stride].astype(np.uint64)) > 1)
    diff_b = live & (gb != rb)
    dq = np.abs(gq - rq)
    # a base called N on one side only: the quality sits at the Q2 boundary (2 vs 1 -> N); allowed as a +-1
    n_flip = live & ((gb == N_CODE) != (rb == N_CODE))
    return {"columns": int(live.sum()),
            "base_diff": int((diff_b & ~n_flip).sum()),
            "tie_columns": int(tie.sum()),
            "tie_diff": int((tie & diff_b & ~n_flip).sum()),
            "n_boundary": int(n_flip.sum()),
            "n_boundary_bad": int((n_flip & (np.maximum(gq, rq) > 2)).sum()),
            "qual_pm1": int((live & (dq == 1)).sum()),
            "qual_gt1": int((live & ~n_flip & (dq > 1)).sum())}
