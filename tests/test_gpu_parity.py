"""HIP path (through the C-ABI) against the reference tools' golden outputs and the CPU restatement.

Bar: bit-exact everywhere -- tool 1 / tool 2 records (seq, qual, pos, cigar, tags) against the
reference's own outputs, consensus bases AND qualities against oracle/ (the vote's fixed-point
sums and shared phred thresholds make the qualities exact too; north_star allows +-1).
"""
import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, pipeline, synth
from bsseqconsensusreads_amd import records as R
from helpers import compare_records, golden_inputs, load_golden, trim_tails
from oracle import oracle

pytestmark = pytest.mark.gpu


def assert_consensus_equal(cons, ref, what=""):
    assert np.array_equal(cons.fam_mi, ref.fam_mi), what + ": family order"
    st = (cons.status & 1).astype(np.int32)
    bad = np.nonzero(st != ref.status)[0]
    assert bad.size == 0, "%s: status differs at families %s" % (what, bad[:10])
    assert np.array_equal(cons.length, ref.cons_len), what + ": lengths"
    F = len(ref.status)
    for f in range(F):
        for e in range(2):
            n = int(ref.cons_len[f, e])
            if not np.array_equal(cons.seq[f, e, :n], ref.cons_seq[f, e, :n]):
                d = np.nonzero(cons.seq[f, e, :n] != ref.cons_seq[f, e, :n])[0]
                raise AssertionError("%s: family %d end %d bases differ at %s: gpu %s oracle %s" % (
                    what, f, e, d[:8], cons.seq[f, e, d[:8]], ref.cons_seq[f, e, d[:8]]))
            if not np.array_equal(cons.qual[f, e, :n], ref.cons_qual[f, e, :n]):
                d = np.nonzero(cons.qual[f, e, :n] != ref.cons_qual[f, e, :n])[0]
                raise AssertionError("%s: family %d end %d quals differ at %s: gpu %s oracle %s" % (
                    what, f, e, d[:8], cons.qual[f, e, d[:8]], ref.cons_qual[f, e, d[:8]]))


def assert_ss_equal(cons, ref, what=""):
    """The single-strand reads and consensus-tag column statistics (BSDC_MODE_TAGS) of every
    emitted family and set equal the restatement's (the kernels compute them inside the vote, which
    runs for the families whose consensus pair is written: the tags ride on those records), and
    the single-strand lengths of every family."""
    assert cons.ss is not None, what + ": no tag outputs"
    assert np.array_equal(cons.ss["len"], ref.ss["len"]), what + ": single-strand lengths"
    d16, e16 = batch.ss_stats16(cons.ss)  # (the kernels' bytes + the wide families' exact rows)
    got = {"base": cons.ss["base"], "qual": cons.ss["qual"], "depth": d16, "err": e16}
    for f in np.nonzero(ref.status == 1)[0]:
        for s in range(4):
            n = int(ref.ss["len"][f, s])
            for k in ("base", "qual", "depth", "err"):
                g, r = got[k][f, s, :n].astype(np.int64), ref.ss[k][f, s, :n].astype(np.int64)
                if not np.array_equal(g, r):
                    d = np.nonzero(g != r)[0]
                    raise AssertionError("%s: family %d set %d %s differs at %s: gpu %s oracle %s" % (
                        what, f, s, k, d[:8], g[d[:8]], r[d[:8]]))


def force_large(monkeypatch, where):
    """Route every family of every batch through k_large: arena in LDS ("lds") or, with every
    family in the last bucket, in HBM scratch ("global")."""
    real = batch.materialize

    def forced(plan, f0, f1, small_cap=0, images=None):
        fb = real(plan, f0, f1, small_cap=0, images=images)
        if where == "global":
            nb = len(fb.large_buckets)
            fb.large_buckets = [np.zeros((0, 4), np.uint32)] * (nb - 1) + [fb.large_fams]
            fb.large_arenas = [16] * (nb - 1) + [max(max(fb.large_arenas), batch.LARGE_LDS_MAX + 16)]
        return fb

    monkeypatch.setattr(batch, "materialize", forced)
    monkeypatch.setattr(pipeline, "materialize", forced)


# (the same golden vectors through k_large: tests/test_gpu_batches.py)
def test_tool1_fuzz_matches_reference(engine):
    g = load_golden("tool1_fuzz.json.gz")
    raw, ref = golden_inputs(g)
    engine.load_reference(ref)
    out = pipeline.run_tool1(engine, raw)
    compare_records(g["tool1"], out, raw, g["input"], "gpu tool1 fuzz")


def test_tools12_families_match_reference(engine):
    g = load_golden("tool12_families.json.gz")
    raw, ref = golden_inputs(g)
    engine.load_reference(ref)
    compare_records(g["tool1"], pipeline.run_tool1(engine, raw), raw, g["input"], "gpu tool1 families")
    cons, t2 = pipeline.run_step5(engine, raw, dump=True)
    compare_records(g["tool2"], t2, raw, g["input"], "gpu fused tool2 dump")
    assert_consensus_equal(cons, oracle.run(raw, ref), "golden families consensus")


def test_tool2_alone_on_reference_tool1_output(engine):
    g = load_golden("tool12_families.json.gz")
    raw1 = R.records_from_dicts(g["tool1"])
    out = pipeline.run_tool2(engine, raw1)
    compare_records(g["tool2"], out, raw1, g["tool1"], "gpu tool2 alone")


def test_missing_mi_raises(engine):
    g = load_golden("tool2_missing_mi.json.gz")
    raw, ref = golden_inputs(g)
    with pytest.raises(ValueError, match="does not have MI tag"):
        pipeline.run_step5(engine, raw)


@pytest.mark.parametrize("cfg", ["C0", "C1", "C2", "C3", "C4"])
def test_synthetic_configs_vs_oracle(engine, cfg):
    # C1 at its stated size (BASELINE.json configs[0]: 10K families)
    n = {"C0": 3000, "C1": 10_000, "C2": 3000, "C3": 150, "C4": 1200}[cfg]
    s = synth.generate(cfg, n, seed=11, device="cpu", genome_len=2_000_000 if cfg == "C1" else 400_000)
    if cfg == "C4":  # the deep-set vote path (a strand/end set of more than 128 reads) is exercised
        fb = batch.build_family_batch(s.raw, "full", s.ref)
        assert np.diff(fb.fam_off.astype(np.int64)).max() > 600
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, s.raw, dump=True, tags=True)
    ref = oracle.run(s.raw, s.ref, threads=8)
    assert_consensus_equal(cons, ref, cfg)
    assert_ss_equal(cons, ref, cfg)
    # the fused kernel's tool-2 state equals the restatement's tool-2 records
    assert np.array_equal(t2.src, ref.tool2.src)
    assert np.array_equal(t2.pos, ref.tool2.pos)
    assert np.array_equal(t2.seq, ref.tool2.seq)
    assert np.array_equal(t2.qual, ref.tool2.qual)
    assert np.array_equal(t2.cigar, ref.tool2.cigar)


def test_messy_records_vs_oracle(engine):
    """soft/hard clips, I/D ops (complex cigars, alignment filter), N runs, trailing Ns."""
    s = synth.generate("C2", 800, seed=5, device="cpu", genome_len=200_000)
    raw = synth.messify(s.raw, frac=0.25, seed=9)
    engine.load_reference(s.ref)
    cons, _ = pipeline.run_step5(engine, raw, tags=True)
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(cons, ref, "messy")
    assert_ss_equal(cons, ref, "messy")


@pytest.mark.parametrize("read_len,trim", [(100, 0.0), (250, 0.0), (150, 0.4), (300, 0.2)])
def test_read_lengths_vs_oracle(engine, read_len, trim):
    """2x100 / 2x250 / 2x300 runs and adapter-trimmed reads of mixed lengths (columns past a read's
    end, consensus lengths set by the longest read, wider arenas and output strides)."""
    s = synth.generate("C2", 600, seed=31, device="cpu", genome_len=200_000, read_len=read_len)
    raw = trim_tails(s.raw, trim, seed=4) if trim else s.raw
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, raw, dump=True, tags=True)
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(cons, ref, "L%d trim %.1f" % (read_len, trim))
    assert_ss_equal(cons, ref, "L%d" % read_len)
    assert np.array_equal(t2.seq, ref.tool2.seq) and np.array_equal(t2.pos, ref.tool2.pos)
    if trim:
        assert len(set(ref.cons_len[ref.status == 1].reshape(-1).tolist())) > 10


def test_read_through_trim_vs_oracle(engine):
    """short inserts: reads run past the (stale) mate end, fgbio trims them."""
    s = synth.generate("C1", 600, seed=6, device="cpu", genome_len=200_000, frag=(140, 40, 60))
    fb = batch.build_family_batch(s.raw, "full", s.ref)
    assert (fb.rec_link & batch.LINK_RT).any()
    engine.load_reference(s.ref)
    cons, _ = pipeline.run_step5(engine, s.raw)
    assert_consensus_equal(cons, oracle.run(s.raw, s.ref), "read-through")


@pytest.mark.parametrize("where", ["lds", "global"])
def test_large_family_kernel(engine, where, monkeypatch):
    """every family through the workgroup-per-family kernel (arena in LDS, or in HBM scratch)."""
    s = synth.generate("C2", 700, seed=12, device="cpu", genome_len=200_000)
    raw = synth.messify(s.raw, frac=0.1, seed=2)
    force_large(monkeypatch, where)
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, raw, dump=True, tags=True)
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(cons, ref, "large-" + where)
    assert_ss_equal(cons, ref, "large-" + where)
    for k in ("src", "pos", "seq", "qual", "cigar"):  # k_large's tool-2 state (extend + dump phases)
        assert np.array_equal(getattr(t2, k), getattr(ref.tool2, k)), "large-%s tool-2 %s" % (where, k)


def test_vote_only_on_tool2_output(engine):
    """callduplex alone (main.snake.py:155-164) on the restatement's own tool-2 records."""
    s = synth.generate("C0", 1000, seed=13, device="cpu", genome_len=200_000)
    ref = oracle.run(s.raw, s.ref)
    t2 = ref.tool2
    b = R._Builder()
    for k in range(len(t2.src)):
        r = t2.record(k)
        src = r["src"]
        tags = [("MI", "Z", "%d/%s" % (s.raw.mi_id[src], "A" if s.raw.mi_strand[src] == 0 else "B")),
                ("MC", "Z", "%dM" % s.raw.l_seq[src])]
        b.add(("t%d" % s.raw.name_id[src]).encode(), int(s.raw.flag[src]), 0, r["pos"], 60, [int(x) for x in r["cigar"]],
              r["seq"], r["qual"], 0, int(s.raw.next_pos[src]), int(s.raw.tlen[src]), R.encode_aux(tags), tags)
    raw2 = b.finish()
    cons = pipeline.run_duplex(engine, raw2)
    ref2 = oracle.run(raw2, s.ref, run_tools=False)
    assert_consensus_equal(cons, ref2, "vote-only")


def test_split_extension_partner_falls_back(engine):
    """A tool-2 4-group whose extension partners land in different TemplateCoordinate families
    (here: one 163 record's stale mate contig changed) runs the tools and callduplex as two
    launches; the result still equals the restatement's."""
    s = synth.generate("C0", 400, seed=15, device="cpu", genome_len=100_000)
    raw = s.raw
    k = int(np.nonzero(raw.flag == 163)[0][7])
    raw.next_tid[k] = 1
    fb = batch.build_family_batch(raw, "full", s.ref)
    assert fb.split_ext
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, raw, dump=True)
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(cons, ref, "split-fallback")
    assert np.array_equal(t2.src, ref.tool2.src) and np.array_equal(t2.seq, ref.tool2.seq)


def test_empty_and_repeatable(engine):
    s = synth.generate("C2", 300, seed=14, device="cpu", genome_len=100_000)
    engine.load_reference(s.ref)
    a, _ = pipeline.run_step5(engine, s.raw)
    b, _ = pipeline.run_step5(engine, s.raw)
    assert np.array_equal(a.seq, b.seq) and np.array_equal(a.qual, b.qual)
    empty = R.records_from_dicts([])
    c, _ = pipeline.run_step5(engine, empty)
    assert c.status.shape[0] == 0


def test_step5_bam_end_to_end(engine, tmp_path):
    """The file-level drop-in (bam.step5): input BAM + FASTA -> duplex consensus BAM, checked
    record by record against the restatement's consensus."""
    from bsseqconsensusreads_amd import bam

    s = synth.generate("C2", 800, seed=16, device="cpu", genome_len=60_000)
    raw = synth.messify(s.raw, frac=0.1, seed=9)
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    fa = tmp_path / "g.fa"
    fa.write_text(">%s\n%s\n" % (s.ref.names[0], R.NT16_TO_ASCII[codes].tobytes().decode()))
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tLB:L1\n" % (
        s.ref.names[0], len(codes)), [s.ref.names[0]], np.asarray([len(codes)], np.int64))
    bam.write_bam(str(tmp_path / "in.bam"), hdr, bam.records_to_bam(raw))
    st = bam.step5(str(tmp_path / "in.bam"), str(fa), str(tmp_path / "out.bam"), engine=engine)
    _, out = bam.read_bam(str(tmp_path / "out.bam"))
    ref = oracle.run(raw, s.ref)
    em = np.nonzero(ref.status == 1)[0]
    assert st["families_emitted"] == em.shape[0] and out.n == 2 * em.shape[0]
    for i, f in enumerate(em):
        for e in range(2):
            k = 2 * i + e
            L = int(ref.cons_len[f, e])
            o = int(out.seq_off[k])
            assert out.names[int(out.name_id[k])] == ("L1:%s" % raw.mi_names[int(ref.fam_mi[f])]).encode()
            assert np.array_equal(out.seq[o:o + L], ref.cons_seq[f, e, :L])
            assert np.array_equal(out.qual[o:o + L], ref.cons_qual[f, e, :L])
    # fgbio's consensus tags, from the kernels' single-strand reads, equal the ones the encoder
    # makes from the restatement's (tests/test_bam.py checks the encoder itself)
    from test_bam import _check_tags
    assert _check_tags(out, ref, em, False) > 0


def _grouped(cfg, n_fam, seed, messy=0.0):
    """A GroupReadsByUmi-like stream: every MI's /A and /B molecules contiguous."""
    s = synth.generate(cfg, n_fam, seed=seed, device="cpu", genome_len=200_000)
    raw = synth.messify(s.raw, frac=messy, seed=seed) if messy else s.raw
    return s, R.take(raw, np.lexsort((raw.mi_strand, raw.mi_id)))


@pytest.mark.parametrize("cfg,n_fam,messy", [("C1", 300, 0.0), ("C2", 800, 0.2), ("C3", 40, 0.0), ("C4", 150, 0.1)])
def test_molecular_vs_oracle(engine, cfg, n_fam, messy):
    """Step 1 (CallMolecularConsensusReads, main.snake.py:46-55): the same vote kernel over MI runs
    (no BA side); equal to the restatement run as callduplex on the run records."""
    s, raw = _grouped(cfg, n_fam, seed=21, messy=messy)
    cons, rm = pipeline.run_molecular(engine, raw, tags=True)
    ref = oracle.run(rm, s.ref, run_tools=False, family_order="mi-group", min_consensus_base_quality=0)
    assert_consensus_equal(cons, ref, "molecular " + cfg)
    assert_ss_equal(cons, ref, "molecular " + cfg)
    assert ((cons.status & 4) == 0).all()  # no BA side anywhere
    assert (cons.status & 1).sum() > 0.5 * len(rm.mi_names)


def test_cli_step5_and_molecular_files(engine, tmp_path):
    """The command lines the Snakemake rules call (bsseqconsensusreads_amd/cli.py): BAM + FASTQ
    outputs of both steps agree with each other and with the restatement."""
    import gzip

    from bsseqconsensusreads_amd import bam, cli

    s, raw = _grouped("C2", 300, seed=22)
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    fa = tmp_path / "g.fa"
    fa.write_text(">%s\n%s\n" % (s.ref.names[0], R.NT16_TO_ASCII[codes].tobytes().decode()))
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:unsorted\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tLB:L1\n" % (
        s.ref.names[0], len(codes)), [s.ref.names[0]], np.asarray([len(codes)], np.int64))
    inp = str(tmp_path / "in.bam")
    bam.write_bam(inp, hdr, bam.records_to_bam(raw))
    p = lambda n: str(tmp_path / n)  # noqa: E731
    assert cli.main(["step5", "--reference", str(fa), inp, p("d.bam"), "--fastq1", p("d1.fq.gz"),
                     "--fastq2", p("d2.fq.gz"), "--threads", "4"]) == 0
    assert cli.main(["molecular", inp, "-", "--fastq1", p("m1.fq.gz"), "--fastq2", p("m2.fq.gz")]) == 0
    assert cli.main(["molecular", p("missing.bam"), p("x.bam")]) == 1
    # an unsorted input is read whole under the default --stream auto; insisting on the stream fails
    assert cli.main(["step5", "--reference", str(fa), inp, p("u.bam"), "--stream", "true"]) == 1
    # a coordinate-sorted input streams by default, with the bytes of the whole-file path
    sinp = str(tmp_path / "in.sorted.bam")
    shdr = bam.BamHeader(hdr.text.replace("SO:unsorted", "SO:coordinate"), hdr.ref_names, hdr.ref_lens)
    bam.write_bam(sinp, shdr, bam.records_to_bam(R.take(raw, np.lexsort((raw.pos, raw.tid)))))
    assert cli.main(["step5", "--reference", str(fa), sinp, p("s_stream.bam"), "--chunk-mb", "1"]) == 0
    assert cli.main(["step5", "--reference", str(fa), sinp, p("s_whole.bam"), "--stream", "false"]) == 0
    assert open(p("s_stream.bam"), "rb").read() == open(p("s_whole.bam"), "rb").read()
    _, d = bam.read_bam(p("d.bam"))
    ref = oracle.run(raw, s.ref)
    em = np.nonzero(ref.status == 1)[0]
    assert d.n == 2 * em.shape[0]
    with gzip.open(p("d1.fq.gz"), "rt") as fh:
        lines = fh.read().split("\n")
    assert len(lines) == 4 * em.shape[0] + 1
    for i, f in enumerate(em[:50]):
        L = int(ref.cons_len[f, 0])
        assert lines[4 * i] == "@L1:%s/1" % raw.mi_names[int(ref.fam_mi[f])]
        assert lines[4 * i + 1] == R.NT16_TO_ASCII[ref.cons_seq[f, 0, :L]].tobytes().decode()
        assert lines[4 * i + 3] == (ref.cons_qual[f, 0, :L] + 33).tobytes().decode()
    rm = pipeline.molecular_records(raw)
    mref = oracle.run(rm, s.ref, run_tools=False, family_order="mi-group", min_consensus_base_quality=0)
    mem = np.nonzero(mref.status == 1)[0]
    with gzip.open(p("m2.fq.gz"), "rt") as fh:
        lines = fh.read().split("\n")
    assert len(lines) == 4 * mem.shape[0] + 1
    for i, f in enumerate(mem[:50]):
        L = int(mref.cons_len[f, 1])
        assert lines[4 * i] == "@L1:%s/2" % rm.mi_names[int(mref.fam_mi[f])]
        assert lines[4 * i + 1] == R.NT16_TO_ASCII[mref.cons_seq[f, 1, :L]].tobytes().decode()


def force_parts(monkeypatch, cap, seen):
    """Route every family through k_large's part mode where it can be cut (include/bsdc.h
    split_parts): all families large, all in the HBM bucket, then split_hbm_bucket with parts of at
    most `cap` LDS bytes; families that cannot be cut (complex cigars, tool-2 roles, one part) stay
    in the HBM bucket.  `seen` collects the batches."""
    real = batch.materialize
    monkeypatch.setattr(batch, "PART_CAP", 0)

    def forced(plan, f0, f1, small_cap=0, images=None):
        fb = real(plan, f0, f1, small_cap=0, images=images)
        nb = len(fb.large_buckets)
        fb.large_buckets = [np.zeros((0, 4), np.uint32)] * (nb - 1) + [fb.large_fams]
        fb.large_arenas = [16] * (nb - 1) + [max(max(fb.large_arenas), batch.LARGE_LDS_MAX + 16)]
        fb = batch.split_hbm_bucket(fb, part_cap=cap)
        seen.append(fb)
        return fb

    monkeypatch.setattr(batch, "materialize", forced)
    monkeypatch.setattr(pipeline, "materialize", forced)


@pytest.mark.parametrize("cfg,n_fam,messy,qlo,cap", [("C3", 60, 0.0, None, 20000), ("C3", 50, 0.1, None, 24000),
                                                    ("C1", 400, 0.0, 84, 10000), ("C4", 250, 0.05, None, 30000)])
def test_split_families_vs_oracle(engine, monkeypatch, cfg, n_fam, messy, qlo, cap):
    """k_large part mode: families cut into parts of whole templates (their sums in HBM, one join
    workgroup per family), bit-exact against oracle/ -- consensus, the tags' single-strand reads and
    statistics, and the tool-2 records the parts dump; with near-tie columns (q >= 84) the join
    sends those families whole through their HBM fallback arena."""
    from helpers import near_tie_votes
    s = synth.generate(cfg, n_fam, seed=23, device="cpu", genome_len=300_000)
    raw = synth.messify(s.raw, frac=messy, seed=3) if messy else s.raw
    if qlo:
        raw = near_tie_votes(raw, qlo=qlo, seed=8)
    seen = []
    force_parts(monkeypatch, cap, seen)
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, raw, dump=True, tags=True)
    n_split = sum(fb.split_fams.shape[0] for fb in seen)
    assert n_split > (0.8 * n_fam if cfg != "C4" and not messy else 0), n_split
    ref = oracle.run(raw, s.ref)
    assert_consensus_equal(cons, ref, "parts " + cfg)
    assert_ss_equal(cons, ref, "parts " + cfg)
    for k in ("src", "pos", "seq", "qual", "cigar"):
        assert np.array_equal(getattr(t2, k), getattr(ref.tool2, k)), "parts %s tool-2 %s" % (cfg, k)


@pytest.mark.parametrize("cfg,n_fam,cap", [("C3", 60, 20000), ("C4", 250, 30000)])
def test_split_families_without_tags_vs_oracle(engine, monkeypatch, cfg, n_fam, cap):
    """Part mode on the untagged launch (the FASTQ path: no single-strand outputs), bit-exact
    against oracle/."""
    s = synth.generate(cfg, n_fam, seed=29, device="cpu", genome_len=300_000)
    seen = []
    force_parts(monkeypatch, cap, seen)
    engine.load_reference(s.ref)
    cons, _ = pipeline.run_step5(engine, s.raw, tags=False)
    assert sum(fb.split_fams.shape[0] for fb in seen) > 0
    assert_consensus_equal(cons, oracle.run(s.raw, s.ref), "parts, no tags " + cfg)


def test_split_families_tools_only_launch_vs_oracle(engine, monkeypatch):
    """the split_ext fallback runs tools 1 + 2 as a launch of their own
    (MODE_CONVERT | EXTEND | DUMP, no vote), and materialize cuts its large families into parts all
    the same.  The parts dump their tool-2 records and stop before the vote, so no k_join may run
    over their never-written sums; the records and the consensus of the vote launch after it equal
    oracle/'s."""
    s = synth.generate("C4", 250, seed=37, device="cpu", genome_len=300_000)
    raw = s.raw  # (C4: singleton templates per strand, whose 4-record groups tool 2 extends, beside deep families)
    for k in np.nonzero(raw.flag == 163)[0][3:400:7]:
        raw.next_tid[int(k)] = 1
    assert batch.plan_families(raw, "full", s.ref).split_ext
    seen = []
    force_parts(monkeypatch, 12000, seen)
    engine.load_reference(s.ref)
    cons, t2 = pipeline.run_step5(engine, raw, dump=True, tags=True)
    assert sum(fb.split_fams.shape[0] for fb in seen) > 5
    ref = oracle.run(raw, s.ref)
    for k in ("src", "pos", "seq", "qual", "cigar"):
        assert np.array_equal(getattr(t2, k), getattr(ref.tool2, k)), "split_ext parts tool-2 %s" % k
    assert_consensus_equal(cons, ref, "split_ext parts")
    assert_ss_equal(cons, ref, "split_ext parts")


def test_split_families_molecular_vs_oracle(engine, monkeypatch):
    """Part mode under step 1's caller (MI runs, no BA side, --min-consensus-base-quality=0): the
    join masks with the context's own threshold, bit-exact against oracle/ at 0."""
    s, raw = _grouped("C3", 40, seed=31)
    seen = []
    force_parts(monkeypatch, 16000, seen)
    cons, rm = pipeline.run_molecular(engine, raw, tags=True)
    assert sum(fb.split_fams.shape[0] for fb in seen) > 0
    ref = oracle.run(rm, s.ref, run_tools=False, family_order="mi-group", min_consensus_base_quality=0)
    assert_consensus_equal(cons, ref, "parts molecular")
    assert_ss_equal(cons, ref, "parts molecular")
