"""The C++ family formation (include/bsdc_host.h, csrc/bsdc_host.cpp) against the numpy statement
of batch.plan_families / batch.materialize (plan_families_py / materialize_py): every plan array
and every device-batch array equal, on clean and messy synthetic inputs (clips, indels, hard
clips, missing MC, unmapped mates), tool-2 output (vote mode), both family orders, small_cap 0
(every family large) and family ranges."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, hostplan, pipeline, synth
from oracle import oracle

PLAN_KEYS = ("order", "fam_off", "fam_mi", "t2_rank", "fam_split", "conv", "ext_right", "ext_left", "rd_in",
             "partner_raw", "sL", "L", "kfirst", "kn")
BATCH_KEYS = ("fam_off", "rec_off", "fam_entry", "rec_pos", "rec_lenflag", "rec_tid", "rec_link", "rec_win", "cig_off",
              "cig_info", "cigar", "rt", "seq", "qual", "src", "fam_mi", "t2_rank")


def _same_plan(a, b):
    for k in PLAN_KEYS:
        x, y = getattr(a, k), getattr(b, k)
        assert x.shape == y.shape and np.array_equal(x.astype(np.int64), y.astype(np.int64)), k


def _same_batch(a, b):
    for k in BATCH_KEYS:
        x, y = np.asarray(getattr(a, k)), np.asarray(getattr(b, k))
        assert x.shape == y.shape, (k, x.shape, y.shape)
        assert np.array_equal(x.astype(np.int64), y.astype(np.int64)), k
    for k in ("max_len", "n_bases", "n_slots", "split_ext", "small_arenas", "large_arenas"):
        assert getattr(a, k) == getattr(b, k), k
    for k in ("small_buckets", "large_buckets"):
        xa, xb = getattr(a, k), getattr(b, k)
        assert len(xa) == len(xb), k
        for u, v in zip(xa, xb):
            assert np.array_equal(np.asarray(u).reshape(-1), np.asarray(v).reshape(-1)), k


def _check(raw, mode, ref, order="template-coordinate", small_cap=batch.SMALL_ARENA_CAP, ranges=None):
    p_py = batch.plan_families_py(raw, mode, ref, order)
    p_c = hostplan.plan_families(raw, mode, ref, order)
    _same_plan(p_c, p_py)
    for a, b in ranges or [(0, p_py.n_fam)]:
        _same_batch(hostplan.materialize(p_c, a, b, small_cap), batch.materialize_py(p_py, a, b, small_cap))
    return p_py


@pytest.mark.parametrize("cfg,messy", [("C0", 0.0), ("C2", 0.0), ("C2", 0.25), ("C4", 0.15), ("C1", 0.3)])
def test_full_mode_matches_numpy(cfg, messy):
    s = synth.generate(cfg, 300, seed=41, device="cpu", genome_len=120_000)
    raw = synth.messify(s.raw, frac=messy, seed=7) if messy else s.raw
    _check(raw, "full", s.ref)


def test_read_through_and_forced_large():
    s = synth.generate("C1", 400, seed=6, device="cpu", genome_len=200_000, frag=(140, 40, 60))
    _check(s.raw, "full", s.ref)
    _check(s.raw, "full", s.ref, small_cap=0)


def test_mi_group_order_and_ranges():
    s = synth.generate("C2", 500, seed=8, device="cpu", genome_len=150_000)
    raw = synth.messify(s.raw, frac=0.2, seed=3)
    _check(raw, "full", s.ref, order="mi-group")
    p = batch.plan_families_py(raw, "full", s.ref)
    from bsseqconsensusreads_amd import shard
    _check(raw, "full", s.ref, ranges=shard.plan_batches(p.fam_bases(), 5000))


def test_vote_mode_matches_numpy():
    s = synth.generate("C2", 400, seed=24, device="cpu", genome_len=60_000)
    res = oracle.run(s.raw, s.ref)
    raw2 = pipeline.raw_from_records(s.raw, res.tool2)
    _check(raw2, "vote", None)
    _check(raw2, "vote", None, order="mi-group")


def test_split_partner_and_missing_mi():
    s = synth.generate("C0", 400, seed=15, device="cpu", genome_len=100_000)
    raw = s.raw
    k = int(np.nonzero(raw.flag == 163)[0][7])
    raw.next_tid[k] = 1
    p = _check(raw, "full", s.ref)
    assert p.split_ext
    raw.mi_id[int(np.nonzero(raw.flag == 99)[0][3])] = -1
    with pytest.raises(batch.MissingMITag):
        hostplan.plan_families(raw, "full", s.ref)


def test_empty_input():
    s = synth.generate("C0", 10, seed=1, device="cpu", genome_len=20_000)
    from bsseqconsensusreads_amd import records as R
    raw = R.take(s.raw, np.zeros(0, np.int64))
    p = hostplan.plan_families(raw, "full", s.ref)
    assert p.n_fam == 0
    fb = hostplan.materialize(p, 0, 0, batch.SMALL_ARENA_CAP)
    assert fb.n_rec == 0 and fb.n_fam == 0
