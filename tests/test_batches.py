"""Bounded device batches on CPU (no GPU): a family plan cut into ranges materializes into
batches whose contents are exactly the one-batch contents, range by range -- the same records in
the same order, the same per-record words, the same family images (so the kernels, which only see
one family at a time, produce the same bytes; tests/test_gpu_batches.py checks the outputs)."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, pipeline, shard, synth


def _per_family_images(fb):
    """family id -> (bases bytes, quals bytes) of its image slots."""
    out = []
    ent = fb.fam_entry
    for f in range(fb.n_fam):
        base, img = int(ent[f, 3]), (int(ent[f, 2]) >> 8) * 32
        nib = np.empty(img, np.uint8)
        pk = fb.seq[base // 2:(base + img) // 2]
        nib[0::2], nib[1::2] = pk >> 4, pk & 0xF
        out.append((nib.tobytes(), fb.qual[base:base + img].tobytes()))
    return out


@pytest.mark.parametrize("messy", [0.0, 0.2])
def test_ranges_materialize_like_one_batch(messy):
    s = synth.generate("C2", 600, seed=8, device="cpu", genome_len=150_000)
    raw = synth.messify(s.raw, frac=messy, seed=3) if messy else s.raw
    plan = batch.plan_families(raw, "full", s.ref)
    whole = batch.materialize(plan, 0, plan.n_fam)
    ranges = shard.plan_batches(plan.fam_bases(), 4000)
    assert len(ranges) > 20 and ranges[0][0] == 0 and ranges[-1][1] == plan.n_fam
    parts = [batch.materialize(plan, a, b) for a, b in ranges]
    cat = lambda k: np.concatenate([getattr(p, k) for p in parts])  # noqa: E731
    for k in ("src", "rec_pos", "rec_lenflag", "rec_link", "rec_win", "fam_mi", "t2_rank"):
        assert np.array_equal(cat(k), getattr(whole, k)), k
    assert np.array_equal(np.concatenate([p.cig_info for p in parts]), whole.cig_info)
    imgs = [x for p in parts for x in _per_family_images(p)]
    assert imgs == _per_family_images(whole)
    # family sizes and the per-family record counts agree
    assert np.array_equal(np.concatenate([np.diff(p.fam_off.astype(np.int64)) for p in parts]),
                          np.diff(whole.fam_off.astype(np.int64)))
    assert all(not p.split_ext for p in parts) and not whole.split_ext


def test_plan_fam_bases_and_budget():
    s = synth.generate("C4", 300, seed=2, device="cpu", genome_len=100_000)
    plan = batch.plan_families(s.raw, "full", s.ref)
    fb = plan.fam_bases()
    L = plan.L[plan.order]
    assert fb.sum() == int((L + 2).sum())
    for a, b in pipeline.plan_ranges(plan, 50_000):
        assert fb[a:b].sum() <= 50_000 or b - a == 1
    assert pipeline.plan_ranges(plan) == [(0, plan.n_fam)]  # the default budget: one batch here


def test_split_partner_marks_both_families():
    s = synth.generate("C0", 400, seed=15, device="cpu", genome_len=100_000)
    raw = s.raw
    k = int(np.nonzero(raw.flag == 163)[0][7])
    raw.next_tid[k] = 1
    plan = batch.plan_families(raw, "full", s.ref)
    assert plan.split_ext and 1 <= int(plan.fam_split.sum()) <= 2
    assert batch.build_family_batch(raw, "full", s.ref).split_ext
