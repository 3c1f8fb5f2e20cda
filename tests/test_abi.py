"""CPU checks of the C-ABI library: it loads without a GPU, exports what include/bsdc.h declares,
and its host-side model tables / arena sizes agree with the oracle and the batch builder."""
import re
import os

import numpy as np

from bsseqconsensusreads_amd import _lib, batch
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "bsdc.h")).read()
    declared = set(re.findall(r"\b(bsdc_[a-z_0-9]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.bsdc_abi_version() == _lib.BSDC_ABI_VERSION


def test_model_tables_bit_identical_to_oracle():
    lib = _lib.load()
    for pre, post in ((45.0, 30.0), (40.0, 25.0), (60.0, 40.0)):
        lr = np.zeros(256, np.int64)
        thr = np.zeros(94, np.float32)
        lib.bsdc_model_tables(pre, post, lr.ctypes.data, thr.ctypes.data)
        olr, othr = oracle.tables(pre, post)
        assert np.array_equal(lr, olr)
        assert np.array_equal(thr.view(np.uint32), othr.view(np.uint32))


def test_model_tables_follow_fgbio_formula():
    """lr[q] = ln(1-a) - ln(a/3), a = e_post + e(q) - 4/3 e_post e(q) (fixed point 2^40);
    threshold k: S <= thr[k] <=> floor(-10 log10 p' + 0.001) >= k."""
    lr, thr = oracle.tables(45.0, 30.0)
    ep, epre = 10 ** -3.0, 10 ** -4.5
    for q in (0, 2, 10, 20, 30, 37, 40, 60, 93):
        e = 10 ** (-q / 10)
        a = ep + e - 4 / 3 * ep * e
        assert abs(lr[q] / 2.0 ** 20 - (np.log1p(-a) - np.log(a / 3))) < 1e-6
    # worked value: one Q37 read -> S = 3 e^-lr[37] -> Q29
    S = 3 * np.exp(-lr[37] / 2.0 ** 20)
    Q = max(k for k in range(94) if k == 0 or S <= thr[k])
    p = S / (1 + S)
    pp = epre + p - 4 / 3 * epre * p
    assert Q == 29 == int(np.floor(-10 * np.log10(pp) + 0.001))


def test_det_expf_accuracy():
    for x in np.linspace(-80, 0, 2001).astype(np.float32):
        v = oracle.det_expf(float(x))
        assert abs(v / np.exp(np.float64(x)) - 1) < 1e-6, x


def test_arena_formulas_match_library():
    lib = _lib.load()
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = int(rng.integers(1, 600))
        sl = int(rng.integers(0, 400 * n))
        ml = int(rng.integers(0, 400))
        co = int(rng.integers(0, 3)) * int(rng.integers(0, 50))
        assert lib.bsdc_family_arena_bytes(n, sl, ml, co) == int(batch.large_arena_bytes(n, sl, ml, co))
        img = 32 * int(rng.integers(1, 200))
        nc = int(rng.integers(0, min(n, 64) + 1))
        assert lib.bsdc_small_arena_bytes(min(n, 64), img, nc, co, ml) == int(
            batch.small_arena_bytes(min(n, 64), img, nc, co, ml))


def test_agreement_tables_exhaustive():
    """The kernel's agreement-case shortcut (integer thresholds on the likelihood sum) gives the
    same phred as the full float arithmetic of oracle/ for EVERY sum up to past saturation."""
    lib = _lib.load()
    for pre, post in ((45.0, 30.0), (40.0, 20.0)):
        qlo = np.zeros(2048, np.uint8)
        dthr = np.zeros(48, np.int32)
        lib.bsdc_agree_tables(pre, post, qlo.ctypes.data, dthr.ctypes.data)
        _, thr = oracle.tables(pre, post)
        assert oracle.check_agree_tables(qlo, dthr, thr, (1 << 27) + 1000) == -1


def test_phred_buckets_match_threshold_scan():
    """The kernels' phred of the general (disagreement) case -- bucket lower bound Tables::sq, then
    step up while S <= thr[q + 1] -- equals oracle/'s rule (the largest k with S <= thr[k]) on
    every 2^7-th float in [0, 4) (S = the sum of three exp terms <= 1) and on every threshold and
    its float neighbours."""
    lib = _lib.load()
    for pre, post in ((45.0, 30.0), (40.0, 20.0), (93.0, 93.0), (10.0, 5.0)):
        sq = np.zeros(144, np.uint8)
        lib.bsdc_phred_buckets(pre, post, sq.ctypes.data)
        _, thr = oracle.tables(pre, post)
        thr = np.concatenate([np.asarray(thr, np.float32)[:94], np.float32([-1.0, -1.0])])
        bits = np.arange(0, 0x40800000, 1 << 7, dtype=np.uint32)
        t = thr[1:94][thr[1:94] > 0]
        bits = np.concatenate([bits, t.view(np.uint32) - 1, t.view(np.uint32), t.view(np.uint32) + 1])
        bits = bits[bits < 0x40800000]
        S = bits.view(np.float32)
        want = np.searchsorted(-thr[1:94], -S, side="right")  # thr is non-increasing
        j = np.clip((bits >> 21).astype(np.int64) - ((127 - 32) << 2), 0, 135)
        q = sq[j].astype(np.int64)
        for _ in range(94):
            up = (q < 93) & (S <= thr[np.minimum(q + 1, 95)])
            if not up.any():
                break
            q = q + up
        bad = np.nonzero(q != want)[0]
        assert bad.size == 0, (pre, post, S[bad[:5]], q[bad[:5]], want[bad[:5]])
