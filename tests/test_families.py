"""Family formation: fgbio SortBam -s TemplateCoordinate + the duplex caller's
grouping of consecutive records with one MI base, on the tool-2 records.  PARITY UNPINNED (fgbio
is not vendored): the host batch builder and the oracle's C restatement are checked against each
other and against a third, pure-Python restatement of the comparator below.  CPU only."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, pipeline, synth
from bsseqconsensusreads_amd import records as R
from oracle import oracle

BIG = 2 ** 31 - 1


def _families(fb):
    off = fb.fam_off.astype(np.int64)
    return [fb.src[off[f]:off[f + 1]].tolist() for f in range(fb.n_fam)]


def _oracle_families(res):
    off = res.fam_rec_off
    return [res.fam_src[off[f]:off[f + 1]].tolist() for f in range(len(off) - 1)]


def _unclipped(cig, pos):
    ops = [(int(c) & 0xF, int(c) >> 4) for c in cig]
    lead = trail = 0
    i, j = 0, len(ops) - 1
    while i < len(ops) and ops[i][0] in (R.OP_S, R.OP_H):
        lead += ops[i][1]
        i += 1
    while j >= i and ops[j][0] in (R.OP_S, R.OP_H):
        trail += ops[j][1]
        j -= 1
    reflen = sum(l for o, l in ops if o in R.REF_CONSUMING)
    return pos - lead, pos + reflen - 1 + trail


def _python_tc_families(raw, t2):
    """Independent restatement: key per tool-2 record, Python sort, runs of one MI."""
    keys = []
    for k in range(len(t2.src)):
        r = t2.record(k)
        s = r["src"]
        fl = int(raw.flag[s])
        us, ue = _unclipped(r["cigar"], r["pos"])
        neg = bool(fl & 16)
        own = (int(raw.tid[s]), ue if neg else us, neg)
        if (fl & 1) and not (fl & 8):
            mneg = bool(fl & 32)
            if raw.mc_off[s] >= 0:
                mc = raw.mc_cigar[raw.mc_off[s]:raw.mc_off[s] + raw.mc_n[s]]
                mus, mue = _unclipped(mc, int(raw.next_pos[s]))
            else:
                mus = mue = int(raw.next_pos[s])
            mate = (int(raw.next_tid[s]), mue if mneg else mus, mneg)
        else:
            mate = (BIG, BIG, False)
        lo, hi, upper = (own, mate, False) if own <= mate else (mate, own, True)
        mi = raw.mi_names[raw.mi_id[s]].encode()
        keys.append(((lo[0], hi[0], lo[1], hi[1], lo[2], hi[2], mi, raw.names[raw.name_id[s]], upper, k), s))
    keys.sort(key=lambda x: x[0])
    fams, prev = [], None
    for _, s in keys:
        mi = int(raw.mi_id[s])
        if mi != prev:
            fams.append([])
            prev = mi
        fams[-1].append(int(s))
    return fams


@pytest.mark.parametrize("cfg,messy", [("C1", False), ("C2", False), ("C2", True), ("C4", False), ("C0", True)])
def test_template_coordinate_families_match_oracle(cfg, messy):
    # a dense genome so molecules interleave in TemplateCoordinate order
    s = synth.generate(cfg, 1500, seed=21, device="cpu", genome_len=30_000)
    raw = synth.messify(s.raw, frac=0.15, seed=5) if messy else s.raw
    fb = batch.build_family_batch(raw, "full", s.ref)
    res = oracle.run(raw, s.ref)
    assert _families(fb) == _oracle_families(res), "host vs oracle TemplateCoordinate families"
    assert np.array_equal(fb.fam_mi, res.fam_mi)
    assert _oracle_families(res) == _python_tc_families(raw, res.tool2)


def test_molecules_split_where_coordinates_disagree():
    """Multi-template strands: tool 1 moves the converted reads one base left, tool 2 does not act
    and the mate fields stay stale, so AB and BA of one molecule can sort apart."""
    s = synth.generate("C2", 3000, seed=22, device="cpu", genome_len=30_000)
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    assert fb.n_fam > len(np.unique(fb.fam_mi)), "expected some MI split into several families"
    grp = batch.build_family_batch(s.raw, "full", s.ref, family_order="mi-group")
    assert grp.n_fam == len(np.unique(grp.fam_mi))
    assert sorted(fb.src.tolist()) == sorted(grp.src.tolist())


def test_pipeline_as_written_splits_only_between_pairs():
    """One template per strand (post step-1): tool 2 lines the extension pairs (99, 163) and
    (83, 147) up on one key each, so a molecule can only split between the two pairs -- each
    extension partner stays in its record's family and the fused launch stays valid."""
    s = synth.generate("C0", 3000, seed=23, device="cpu", genome_len=30_000)
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    assert not fb.split_ext
    sizes = np.diff(fb.fam_off.astype(np.int64))
    assert set(sizes.tolist()) <= {2, 4}
    flags = fb.rec_lenflag >> 16
    off = fb.fam_off.astype(np.int64)
    for f in np.nonzero(sizes == 2)[0][:200]:
        assert sorted(flags[off[f]:off[f + 1]].tolist()) in ([99, 163], [83, 147])


def test_vote_mode_families_match_oracle():
    s = synth.generate("C2", 1500, seed=24, device="cpu", genome_len=30_000)
    ref = oracle.run(s.raw, s.ref)
    raw2 = pipeline.raw_from_records(s.raw, ref.tool2)
    fb = batch.build_family_batch(raw2, "vote")
    res2 = oracle.run(raw2, s.ref, run_tools=False)
    # raw2's record k is tool-2 record k: compare in raw2's index space
    assert _families(fb) == _oracle_families(res2)
    assert _oracle_families(res2) == _python_tc_families(raw2, res2.tool2)


def test_rd_prediction_matches_tool1():
    s = synth.generate("C2", 2000, seed=25, device="cpu", genome_len=50_000)
    raw = synth.messify(s.raw, frac=0.2, seed=6)
    res = oracle.run(raw, s.ref)
    _, conv = batch.tool1_plan(raw)
    sL, L, _, _ = batch._softclip_strip(raw)
    t1 = res.tool1
    sel = np.asarray([int(x) for k, x in enumerate(t1.src) if conv[int(x)]], np.int64)
    want = np.asarray([int(t1.rd[k]) for k, x in enumerate(t1.src) if conv[int(x)]]) == 1
    got = batch.predict_rd(raw, s.ref, sel, sL, L)
    assert sel.shape[0] > 100 and want.any()
    assert np.array_equal(got, want)


def test_molecular_runs():
    """Step 1's families (CallMolecularConsensusReads): consecutive records of one full MI tag,
    /A and /B apart, in input order; every record on the A side."""
    from bsseqconsensusreads_amd import pipeline

    s = synth.generate("C2", 60, seed=4, device="cpu", genome_len=50_000)
    raw = R.take(s.raw, np.lexsort((s.raw.mi_strand, s.raw.mi_id)))
    rm = pipeline.molecular_records(raw)
    assert (rm.mi_strand == 0).all()
    full = [raw.mi_names[int(raw.mi_id[k])] + "/" + "AB"[int(raw.mi_strand[k])] for k in range(raw.n)]
    runs = [full[0]] + [full[k] for k in range(1, raw.n) if full[k] != full[k - 1]]
    assert rm.mi_names == runs and len(set(runs)) == len(runs)
    assert all(rm.mi_names[int(rm.mi_id[k])] == full[k] for k in range(raw.n))
    fb = batch.build_family_batch(rm, "vote", family_order="mi-group")
    assert fb.n_fam == len(runs) and np.array_equal(fb.fam_mi, np.arange(len(runs)))


def test_take_round_trip():
    s = synth.generate("C4", 40, seed=5, device="cpu", genome_len=50_000)
    raw = synth.messify(s.raw, frac=0.3, seed=5)
    idx = np.random.default_rng(0).permutation(raw.n)
    t = R.take(raw, idx)
    back = R.take(t, np.argsort(idx))
    for k in ("flag", "pos", "l_seq", "seq", "qual", "cigar", "n_cig", "mc_n", "mc_cigar", "mi_id", "name_id"):
        assert np.array_equal(getattr(back, k), getattr(raw, k)), k


def test_cli_arguments():
    from bsseqconsensusreads_amd import cli

    a = cli.parse(["step5", "--reference", "g.fa", "in.bam", "out.bam", "--threads", "3"])
    assert (a.cmd, a.reference, a.input, a.output, a.threads, a.fastq1) == ("step5", "g.fa", "in.bam", "out.bam", 3, None)
    a = cli.parse(["molecular", "in.bam", "-", "--fastq1", "a", "--fastq2", "b"])
    assert a.output == "-" and (a.fastq1, a.fastq2) == ("a", "b")
    for bad in (["step5", "in.bam", "out.bam"], ["molecular", "in.bam", "-"], ["molecular", "i", "o", "--fastq1", "a"]):
        with pytest.raises(SystemExit):
            cli.parse(bad)


def test_clips_reflen_vs_loop():
    """_clips_reflen (one-op fast path + the per-op expansion) against a loop over the cigar ops:
    leading / trailing S+H and the reference-consuming length, absent and all-clip cigars included."""
    rng = np.random.default_rng(3)
    n = 4000
    cnt = rng.integers(-1, 6, n)
    cnt[rng.random(n) < 0.5] = 1
    c = np.maximum(cnt, 0)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(c)[:-1]
    off[cnt <= 0] = -1
    cig = (rng.integers(1, 200, c.sum()) << 4 | rng.choice([0, 1, 2, 3, 4, 5, 7, 8], c.sum())).astype(np.uint32)
    want = ([], [], [])
    for o, k in zip(off, cnt):
        ops = [(int(x) & 15, int(x) >> 4) for x in cig[o:o + k]] if k > 0 else []
        i, lead = 0, 0
        while i < len(ops) and ops[i][0] in (R.OP_S, R.OP_H):
            lead += ops[i][1]
            i += 1
        j, trail = len(ops) - 1, 0
        while j >= i and ops[j][0] in (R.OP_S, R.OP_H):
            trail += ops[j][1]
            j -= 1
        for lst, v in zip(want, (lead, trail, sum(ln for op, ln in ops if op in R.REF_CONSUMING))):
            lst.append(v)
    for g, w in zip(batch._clips_reflen(cig, off, cnt), want):
        assert np.array_equal(g, np.asarray(w))
