"""Bounded device batches on CPU (no GPU): a family plan cut into ranges materializes into
batches whose contents are exactly the one-batch contents, range by range -- the same records in
the same order, the same per-record words, the same family images (so the kernels, which only see
one family at a time, produce the same bytes; tests/test_gpu_batches.py checks the outputs)."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, pipeline, shard, synth
from bsseqconsensusreads_amd import records as R


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


def test_split_part_records_cover_each_family_once(monkeypatch):
    """k_large part mode's host cut (bsdc_split_count / bsdc_split_fill / bsdc_split_move via
    batch.split_hbm_bucket): every record of a cut family sits in exactly one part, whole templates
    stay together (a part-local mate points at the record's mate), each part's records lie back to
    back in the re-laid-out family image (its staged chunks from its first slot rounded down to 32),
    the family's first record leads its image, and every record's bases and quals moved with it."""
    from bsseqconsensusreads_amd import batch as B, synth
    s = synth.generate("C3", 300, seed=5, device="cpu", genome_len=200_000)
    fb = B.build_family_batch(s.raw, "full", s.ref)
    L = (fb.rec_lenflag & 0xFFFF).astype(np.int64)
    old_off = fb.rec_off.astype(np.int64).copy()
    codes = R.unpack_nibbles(fb.seq, 2 * fb.seq.shape[0]).copy()
    quals = fb.qual.copy()
    monkeypatch.setattr(B, "SPLIT_FROM", 0)  # every large bucket (C3 has no HBM-arena family)
    fb = B.split_hbm_bucket(fb, part_cap=12_000)
    sf = fb.split_fams.astype(np.int64)
    assert sf.shape[0] > 0
    parts, prec = fb.split_parts.astype(np.int64), fb.split_part_recs.astype(np.int64)
    codes2 = R.unpack_nibbles(fb.seq, 2 * fb.seq.shape[0])
    new_off = fb.rec_off.astype(np.int64)
    for row, f in enumerate(sf):
        fam, r0, n, p0, npart = f[0], f[1], f[2], f[4], f[5]
        base = int(old_off[r0:r0 + n].min())
        assert new_off[r0] == base  # (the whole-family fallback reads the image from there)
        seen, at = [], base
        for p in parts[p0:p0 + npart]:
            assert p[0] == fam and p[2] >> 8 == row  # (the part knows its split family's row)
            recs = prec[p[1]:p[1] + (p[2] & 0xFF)]
            a0 = int(recs[0][3] - recs[0][1])
            assert a0 % 32 == 0 and 0 <= recs[0][1] < 32
            for li, w in enumerate(recs):
                gi = int(w[0])
                seen.append(gi)
                cap = (L[gi] + 2 + 3) // 4 * 4
                assert w[3] == at == new_off[gi] and w[1] == at - a0 and (w[2] >> 16) == L[gi]
                a, b = int(old_off[gi]), int(new_off[gi])
                assert np.array_equal(codes2[b:b + cap], codes[a:a + cap]) and np.array_equal(fb.qual[b:b + cap], quals[a:a + cap])
                at += cap
                lm = int(w[2] & 0xFFFF)
                gm = int(fb.rec_link[gi] & 0xFFFF)
                if gm != 0xFFFF:  # the mate is in the same part, at its local index
                    assert lm != 0xFFFF and recs[lm][0] == r0 + gm
            assert p[3] == (at - a0 + 31) // 32 * 32  # (the staged image: whole 32-entry chunks)
        assert sorted(seen) == list(range(r0, r0 + n))


def test_route_small_cap_by_family_mix(monkeypatch):
    """route_small_cap: deep families (C3: most small-family records in arenas above 16 KB) go to
    k_large from 16 KB on; shallow and skewed mixes (C2, C4) keep the 24 KB cap; SMALL_ROUTE = False
    turns it off"""
    from bsseqconsensusreads_amd import synth
    got = {}
    for cfg, n in (("C2", 20000), ("C3", 3000), ("C4", 20000)):
        s = synth.generate(cfg, n, seed=3, device="cpu")
        plan = batch.plan_families(s.raw, "full", s.ref)
        got[cfg] = batch.route_small_cap(plan, 0, plan.n_fam)
        if cfg == "C3":
            fb = batch.materialize(plan, 0, plan.n_fam)  # (the routed cap reaches the plan)
            assert max(a for a, b in zip(fb.small_arenas, fb.small_buckets) if b.shape[0]) <= batch.MID_ARENA_CAP
            monkeypatch.setattr(batch, "SMALL_ROUTE", False)
            assert batch.route_small_cap(plan, 0, plan.n_fam) == batch.SMALL_ARENA_CAP
            monkeypatch.setattr(batch, "SMALL_ROUTE", True)
    assert got == {"C2": batch.SMALL_ARENA_CAP, "C3": batch.MID_ARENA_CAP, "C4": batch.SMALL_ARENA_CAP}
