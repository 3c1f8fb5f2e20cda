"""Parity at BASELINE.json's full size: the bench workload itself (C2, configs[1]: 1M duplex
families, 2x150 bp, Poisson(4) templates, seed 42 -- the batch `bench.py` times), every family
against oracle/ bit-exact, plus size-independent properties of the resident-batch step:

- idempotence: a second step over the same resident batch writes the same bytes (the kernels
  read only their inputs; `bench.py` times K such steps);
- output invariants on every family: bases are A/C/G/T/N codes, quals in [1, 93], every
  emitted end has a non-zero length no longer than the batch's longest record + 1.

C3 (configs[2], 200K deep families) and C4 (configs[3], skewed) run at a 20K-family sample of
their full-size model: the oracle restatement needs minutes for the whole C3 batch.
"""
import numpy as np
import pytest
import torch

from bsseqconsensusreads_amd import batch, synth
from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_VOTE
from bsseqconsensusreads_amd.pipeline import consensus_from_output
from oracle import oracle

pytestmark = pytest.mark.gpu
FULL = MODE_CONVERT | MODE_EXTEND | MODE_VOTE
ACGTN = np.array([1, 2, 4, 8, 15])


def _compare_all(cons, ref, what):
    """Vectorised bit-exact comparison of every family's two consensus reads."""
    assert np.array_equal(cons.fam_mi, ref.fam_mi), what + ": family order"
    st = (cons.status & 1).astype(np.int32)
    bad = np.nonzero(st != ref.status)[0]
    assert bad.size == 0, "%s: status differs at families %s" % (what, bad[:10])
    assert np.array_equal(cons.length, ref.cons_len), what + ": lengths"
    w = int(ref.cons_len.max()) if ref.cons_len.size else 0
    live = np.arange(w)[None, None, :] < ref.cons_len[:, :, None]
    for name, g, r in (("bases", cons.seq, ref.cons_seq), ("quals", cons.qual, ref.cons_qual)):
        diff = (g[:, :, :w] != r[:, :, :w]) & live
        if diff.any():
            f, e, c = (int(x[0]) for x in np.nonzero(diff))
            raise AssertionError("%s: %s differ (%d columns), first at family %d end %d column %d: gpu %d oracle %d"
                                 % (what, name, int(diff.sum()), f, e, c, g[f, e, c], r[f, e, c]))
    return live


def _run_resident(engine, fb):
    db = engine.upload(fb)
    engine.run(db, FULL)
    torch.cuda.synchronize()
    a = db.fetch()
    engine.run(db, FULL)
    torch.cuda.synchronize()
    b = db.fetch()
    return a, b


def test_bench_workload_c2_full_size(engine):
    s = synth.generate("C2", 1_000_000, seed=42, device="cuda")  # bench.py's rank-0 batch
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    assert fb.n_fam > 1_000_000 and not fb.split_ext
    engine.load_reference(s.ref)
    a, b = _run_resident(engine, fb)
    for k in ("status", "len", "seq", "qual"):
        assert np.array_equal(a[k], b[k]), "second step over the resident batch differs in " + k
    cons = consensus_from_output(fb, a)
    ref = oracle.run(s.raw, s.ref, threads=16)
    live = _compare_all(cons, ref, "C2 1M")
    w = live.shape[2]
    seq, qual = cons.seq[:, :, :w], cons.qual[:, :, :w]
    assert np.isin(seq[live], ACGTN).all()
    q = qual[live]  # a duplex disagreement keeps |qa - qb|, which can be 1 (fgbio duplexConsensus)
    assert q.min() >= 1 and q.max() <= 93
    emitted = (cons.status & 1) != 0
    assert (cons.length[emitted] > 0).all()
    assert cons.length.max() <= int((fb.rec_lenflag & 0xFFFF).max()) + 1
    assert emitted.sum() > 0.8 * fb.n_fam


@pytest.mark.parametrize("cfg", ["C3", "C4"])
def test_deep_and_skewed_configs_sample(engine, cfg):
    s = synth.generate(cfg, 20_000, seed=42, device="cuda")
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    engine.load_reference(s.ref)
    a, b = _run_resident(engine, fb)
    for k in ("status", "len", "seq", "qual"):
        assert np.array_equal(a[k], b[k]), "%s: second step differs in %s" % (cfg, k)
    if fb.split_ext:
        pytest.skip("split extension partner: covered by test_split_extension_partner_falls_back")
    ref = oracle.run(s.raw, s.ref, threads=16)
    _compare_all(consensus_from_output(fb, a), ref, cfg + " 20K")
