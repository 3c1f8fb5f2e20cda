"""Parity at BASELINE.json's full sizes, every family against oracle/ bit-exact:

- C2 (configs[1]): 1M duplex families, 2x150 bp, Poisson(4) templates, seed 42 -- the batch
  `bench.py` times -- plus size-independent properties of the resident-batch step: idempotence (a
  second step over the same resident batch writes the same bytes) and output invariants (bases
  A/C/G/T/N, quals in [1, 93], lengths bounded by the longest record + 1);
- C3 (configs[2]): all 200K deep families (20-100 templates), same checks;
- C4 (configs[3]): the 1M-family batch `bench.py --config C4` times, every family, and a
  20K-family sample;
- C5 (configs[4], per-GPU shape): a C2-shaped stream larger than one batch's 32-bit slot range,
  cut into bounded batches that run back to back on one GPU and are gathered in order -- what each
  rank of a 2/4/8-GPU run does with its share of the 100M families.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from bsseqconsensusreads_amd import batch, pipeline, synth
from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_VOTE
from bsseqconsensusreads_amd.pipeline import consensus_from_output
from oracle import oracle

pytestmark = pytest.mark.gpu
# the box's CPU share (OMP_NUM_THREADS = 16 there); os.cpu_count() shows the whole machine
THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
FULL = MODE_CONVERT | MODE_EXTEND | MODE_VOTE
ACGTN = np.array([1, 2, 4, 8, 15])


def _oracle_async(raw, ref):
    """oracle/ on a thread (its C call drops the GIL), started before the GPU run so the two
    overlap; .result() gives the restatement's result."""
    ex = ThreadPoolExecutor(1)
    fut = ex.submit(oracle.run, raw, ref, threads=THREADS)
    ex.shutdown(wait=False)
    return fut


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
    fut = _oracle_async(s.raw, s.ref)
    a, b = _run_resident(engine, fb)
    for k in ("status", "len", "seq", "qual"):
        assert np.array_equal(a[k], b[k]), "second step over the resident batch differs in " + k
    cons = consensus_from_output(fb, a)
    ref = fut.result()
    live = _compare_all(cons, ref, "C2 1M")
    # (a duplex disagreement keeps |qa - qb|, which can be 1: fgbio duplexConsensus)
    _invariants(cons, live, int((fb.rec_lenflag & 0xFFFF).max()))
    assert ((cons.status & 1) != 0).sum() > 0.8 * fb.n_fam


def _invariants(cons, live, fb_max_len):
    w = live.shape[2]
    seq, qual = cons.seq[:, :, :w], cons.qual[:, :, :w]
    assert np.isin(seq[live], ACGTN).all()
    q = qual[live]
    assert q.min() >= 1 and q.max() <= 93
    emitted = (cons.status & 1) != 0
    assert (cons.length[emitted] > 0).all()
    assert cons.length.max() <= fb_max_len + 1


@pytest.mark.timeout(900)
def test_c3_full_size_every_family(engine):
    s = synth.generate("C3", 200_000, seed=42, device="cuda")  # bench.py --config C3
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    assert fb.n_fam >= 200_000 and not fb.split_ext and fb.large_fams.shape[0] > 100_000
    engine.load_reference(s.ref)
    fut = _oracle_async(s.raw, s.ref)
    a, b = _run_resident(engine, fb)
    for k in ("status", "len", "seq", "qual"):
        assert np.array_equal(a[k], b[k]), "C3: second step differs in " + k
    cons = consensus_from_output(fb, a)
    del fb, a, b
    ref = fut.result()
    live = _compare_all(cons, ref, "C3 200K")
    _invariants(cons, live, int(s.raw.l_seq.max()) + 1)


@pytest.mark.timeout(900)
def test_c4_bench_batch_every_family(engine):
    """bench.py --config C4's rank-0 input (1M skewed families, seed 42), through the step's own
    batching (pipeline.run_step5: the fused launch, or the two-launch fallback if a tool-2 partner
    straddles families), every family against oracle/."""
    s = synth.generate("C4", 1_000_000, seed=42, device="cuda")
    engine.load_reference(s.ref)
    fut = _oracle_async(s.raw, s.ref)
    cons, _ = pipeline.run_step5(engine, s.raw)
    ref = fut.result()
    live = _compare_all(cons, ref, "C4 1M")
    _invariants(cons, live, int(s.raw.l_seq.max()) + 1)


def test_c4_skewed_sample(engine):
    s = synth.generate("C4", 20_000, seed=42, device="cuda")
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    engine.load_reference(s.ref)
    a, b = _run_resident(engine, fb)
    for k in ("status", "len", "seq", "qual"):
        assert np.array_equal(a[k], b[k]), "C4: second step differs in " + k
    if fb.split_ext:
        pytest.skip("split extension partner: covered by test_split_extension_partner_falls_back")
    ref = oracle.run(s.raw, s.ref, threads=THREADS)
    _compare_all(consensus_from_output(fb, a), ref, "C4 20K")


@pytest.mark.timeout(900)
def test_c5_stream_beyond_one_batch(engine):
    """One GPU's share of C5: 3.7M C2-shaped families, more slots than 32-bit batch offsets hold,
    as >= 3 bounded batches run back to back (pipeline.run_step5 -> plan_families / plan_ranges
    / run_ranges / concat_consensus), gathered in order, every family bit-exact."""
    s = synth.generate("C2", 3_700_000, seed=5, device="cuda")
    engine.load_reference(s.ref)
    plan = batch.plan_families(s.raw, "full", s.ref)
    ranges = pipeline.plan_ranges(plan, 1 << 30)
    slots = int(plan.fam_bases().sum())
    assert len(ranges) >= 3 and slots > (1 << 32), (len(ranges), slots)
    fut = _oracle_async(s.raw, s.ref)
    cons, _ = pipeline.run_step5(engine, s.raw, batch_bases=1 << 30)
    assert cons.status.shape[0] == plan.n_fam
    ref = fut.result()
    live = _compare_all(cons, ref, "C5 stream %d batches" % len(ranges))
    _invariants(cons, live, int(s.raw.l_seq.max()) + 1)


@pytest.mark.timeout(900)
def test_c5_full_share(engine, capsys):
    """C5 (configs[4]) at its full per-GPU share for N = 8: 12.5M C2-shaped families, generated as
    bench.py --config C5 builds rank 0's share (batches of 1.5M families, seed 42 + batch index, one
    genome), each batch through pipeline.run_step5 and compared, every family, with oracle/ on that
    batch's records.  Progress goes to the terminal per batch (the suite's runner watches for
    silence)."""
    total, per, first, done, emitted = 12_500_000, 1_500_000, None, 0, 0
    # batch i's oracle runs on a thread while batch i + 1 is generated and run on the GPU
    pending = None

    def check(p):
        nonlocal emitted
        j, sj, cons, fut, upto = p
        ref = fut.result()
        live = _compare_all(cons, ref, "C5 share batch %d" % j)
        _invariants(cons, live, int(sj.raw.l_seq.max()) + 1)
        emitted += int(ref.status.sum())
        with capsys.disabled():
            print("\nC5 share: batch %d, %d / %d families bit-exact" % (j, upto, total), flush=True)

    i = 0
    while done < total:
        n = min(per, total - done)
        s = synth.generate("C2", n, seed=42 + i, device="cuda", reuse=first)
        if first is None:
            engine.load_reference(s.ref)
            first = s
        cons, _ = pipeline.run_step5(engine, s.raw)
        fut = _oracle_async(s.raw, s.ref)
        done += n
        if pending is not None:
            check(pending)
        pending = (i, s, cons, fut, done)
        del s, cons
        i += 1
    check(pending)
    assert done == total and emitted > 0.8 * total
