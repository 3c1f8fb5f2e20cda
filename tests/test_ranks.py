"""Rank-parallel step 5 (bsseqconsensusreads_amd/ranks.py) on CPU: the parent picks rank
boundaries in the template keys' gaps (bsdc_bam_find_cut), spawned rank processes each decode the
record window around their key interval and compute and encode the records they own (the one-GPU
stream over a window, writing fragments), and the parent concatenates.  The ranks run tests/fleet_standin.py (oracle/ in the
kernels' output layout) in place of the GPU; tests/test_gpu_ranks.py runs them on the GPU."""
import gzip
import os

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, ranks
from helpers import assert_bam_matches_oracle
from test_fleet import STANDIN, _sorted_bam, sorted_input, write_fasta  # noqa: F401 -- (the module fixture)

SLACK = 2000


def _run(tmp, p, fa, tag, n, slack=SLACK, **kw):
    out = str(tmp / ("%s.bam" % tag))
    fq = (str(tmp / ("%s_1.fq.gz" % tag)), str(tmp / ("%s_2.fq.gz" % tag)))
    st = {}
    info = ranks.step5_ranks(p, fa, out, [0] * n, threads=2, fastq=fq, runner=STANDIN, chunk_bytes=80_000,
                             slack=slack, batch_bases=40_000, stats=st, **kw)
    return info, st, [gzip.decompress(open(x, "rb").read()) for x in (out,) + fq], out


@pytest.fixture(scope="module")
def one_range(sorted_input):  # noqa: F811
    s, p, fa, tmp = sorted_input
    return _run(tmp, p, fa, "one", 1)


def test_cuts_partition_the_records(sorted_input):  # noqa: F811
    """find_cut's boundaries are in key order, their windows overlap by about 2 x slack, and the
    ranks' windows with ownership keep every record exactly once, none foreign"""
    s, p, fa, tmp = sorted_input
    cuts = ranks.plan_cuts(p, 4, threads=2, slack=SLACK)
    assert len(cuts) == 3
    assert [c["key"] for c in cuts] == sorted(set(c["key"] for c in cuts))
    for c in cuts:
        assert c["start"] < c["end"]
        assert c["coord"] & 0xFFFFFFFF == c["key"][1]
    kept, read = 0, 0
    for r, rng in enumerate(ranks.windows_of(cuts)):
        st = {}
        for ch in bam.stream_chunks(p, 2, 80_000, SLACK, rng=rng, stats=st, owner=(r, cuts)):
            ch.discard()
        assert st["foreign"] == 0
        kept += st["n"] - st["dropped"]
        read += st["n"]
    assert kept == s.raw.n
    assert s.raw.n < read < 1.3 * s.raw.n


def _same_contig_keys(raw):
    """(contig, key position) of every record whose mate is mapped on its contig: the lower
    unclipped 5' end of the template (include/bsdc_io.cpp rec_key, restated)."""
    from test_families import _unclipped
    out = []
    for k in range(raw.n):
        fl = int(raw.flag[k])
        if not (fl & 1) or (fl & 8) or int(raw.next_tid[k]) != int(raw.tid[k]):
            continue
        us, ue = _unclipped(raw.record_cigar(k), int(raw.pos[k]))
        own = ue if fl & 16 else us
        if raw.mc_off[k] >= 0:
            mc = raw.mc_cigar[raw.mc_off[k]:raw.mc_off[k] + raw.mc_n[k]]
            mus, mue = _unclipped(mc, int(raw.next_pos[k]))
            mate = mue if fl & 32 else mus
        else:
            mate = int(raw.next_pos[k])
        out.append((int(raw.tid[k]), min(own, mate)))
    return np.array(out, np.int64).reshape(-1, 2)


def test_no_key_near_a_boundary(sorted_input):  # noqa: F811
    """No template key lies within KEY_GUARD positions of a boundary on its contig (so no family,
    whose keys lie within the tools' jitter of each other, straddles one)"""
    s, p, fa, tmp = sorted_input
    cuts = ranks.plan_cuts(p, 4, threads=2, slack=SLACK)
    keys = _same_contig_keys(s.raw)
    assert len(keys) > 0.5 * s.raw.n
    for c in cuts:
        tid = c["coord"] >> 32
        near = (keys[:, 0] == tid) & (np.abs(keys[:, 1] - c["key"][1]) <= bam.KEY_GUARD)
        assert not near.any()


@pytest.mark.parametrize("n", [2, 3])
def test_ranks_write_the_records_of_one(sorted_input, one_range, n):  # noqa: F811
    """N ranks: the BAM and FASTQ pair decompress to the bytes of the one-range run, and every rank
    keeps about 1/N of the records and reads its share plus 2 x slack positions"""
    s, p, fa, tmp = sorted_input
    info1, _, ref_bytes, _ = one_range
    info, st, got, _ = _run(tmp, p, fa, "n%d" % n, n)
    assert info["ranks"] == n and not info["cuts_fallback"]
    for a, b in zip(got, ref_bytes):
        assert a == b
    assert info["records_in"] == info1["records_in"] == s.raw.n
    total = s.raw.n
    assert sum(st["rank_records"]) == total
    assert max(st["rank_records"]) <= total / n + 0.15 * total, st["rank_records"]
    assert max(st["rank_read"]) <= total / n + 0.2 * total, st["rank_read"]
    assert min(st["rank_records"]) > 0


def test_ranks_records_equal_whole_file_oracle(sorted_input, one_range):  # noqa: F811
    s, p, fa, tmp = sorted_input
    assert_bam_matches_oracle(one_range[3], p, fa, "ranks")


def test_foreign_records_fall_back_to_one_range(sorted_input, one_range):  # noqa: F811
    """A boundary whose owner cannot read some of its records (here: windows with no margin and
    no key gap, so the mates past the boundary of templates owned before it are read only by the
    next rank) is caught by the ranks' foreign counts and the file is rerun as one range: the
    same bytes"""
    s, p, fa, tmp = sorted_input
    bad = bam.find_cut(p, os.path.getsize(p) // 2, 2, min_span=0, slack=0, guard=0)
    assert bad is not None and bad["start"] == bad["end"]
    info, st, got, _ = _run(tmp, p, fa, "bad", 2, cuts=[bad])
    assert info["cuts_fallback"] and info["ranks"] == 1
    for a, b in zip(got, one_range[2]):
        assert a == b
    with pytest.raises(ranks.ForeignRecords, match="foreign record"):
        _run(tmp, p, fa, "bad2", 2, cuts=[bad], on_foreign="raise")
    assert not [f for f in os.listdir(tmp) if f.startswith(".")], "fragments left behind"


def test_rank_failure_reaches_the_caller(sorted_input, tmp_path):  # noqa: F811
    s, p, fa, _ = sorted_input
    with pytest.raises(RuntimeError, match="stand-in failure on batch 3"):
        ranks.step5_ranks(p, fa, str(tmp_path / "x.bam"), [0, 0], threads=2, runner="fleet_standin:FailingRunner",
                          chunk_bytes=80_000, slack=SLACK, batch_bases=40_000)
    assert not [f for f in os.listdir(tmp_path) if f.startswith(".")], "fragments left behind"





def test_small_file_gets_fewer_ranks(tmp_path):
    """A file too small for N key gaps 2 x slack apart runs on the ranks the cuts allow (here 1,
    with a 300-position genome share per rank impossible), and still writes the one-range bytes"""
    s, p = _sorted_bam(tmp_path, cfg="C2", n_fam=40, messy=0.0, seed=3, genome_len=6_000)
    fa = str(tmp_path / "g.fa")
    write_fasta(fa, s.ref)
    assert len(ranks.plan_cuts(p, 4, threads=2, slack=SLACK)) == 0
    info4, _, got4, _ = _run(tmp_path, p, fa, "four", 4)
    info1, _, got1, _ = _run(tmp_path, p, fa, "one1", 1)
    assert info4["ranks"] == 1 and not info4["cuts_fallback"]
    assert got4 == got1 and info4["records_in"] == s.raw.n


def test_empty_input(tmp_path):
    """No records: one range, a header-only BAM and empty FASTQ files"""
    from bsseqconsensusreads_amd import records as R
    s, p = _sorted_bam(tmp_path, cfg="C2", n_fam=5, messy=0.0, seed=3, genome_len=6_000)
    hdr, raw = bam.read_bam(p)
    q = str(tmp_path / "empty.bam")
    bam.write_bam(q, hdr, bam.records_to_bam(R.take(raw, np.zeros(0, np.int64))))
    fa = str(tmp_path / "g.fa")
    write_fasta(fa, s.ref)
    info, _, got, _ = _run(tmp_path, q, fa, "empty", 3)
    assert info["ranks"] == 1 and info["records_in"] == 0 and info["records_out"] == 0
    assert got[1] == b"" and got[2] == b""
    assert bam.read_bam(str(tmp_path / "empty.bam"))[1].n == 0


def test_pool_runs_several_files(sorted_input, one_range):  # noqa: F811
    """A RankPool started once runs several calls (its ranks keep their runners), each writing the
    one-range bytes; a failing call leaves the pool usable"""
    s, p, fa, tmp = sorted_input
    with ranks.RankPool([0, 0], runner=STANDIN) as pool:
        for k in range(2):
            info, st, got, _ = _run(tmp, p, fa, "pool%d" % k, 2, pool=pool)
            assert info["ranks"] == 2 and not info["cuts_fallback"] and st["pool_start_s"] == 0.0
            assert got == one_range[2]
        bad = bam.find_cut(p, os.path.getsize(p) // 2, 2, min_span=0, slack=0, guard=0)
        with pytest.raises(ranks.ForeignRecords):
            _run(tmp, p, fa, "poolbad", 2, cuts=[bad], on_foreign="raise", pool=pool)
        info, _, got, _ = _run(tmp, p, fa, "pool2", 2, pool=pool)
        assert got == one_range[2]


@pytest.fixture(scope="module")
def cross_input(tmp_path_factory):
    """Two contigs: templates of some families with their R2 moved onto the second contig (mate on
    another contig), families whose mates are flagged unmapped, and the rest ordinary.  Their keys
    sort at their contig's end, wherever the records lie: every rank spills its share of them and
    the owners of the contigs' ends form their families (phase 2)."""
    from bsseqconsensusreads_amd import records as R
    from bsseqconsensusreads_amd import synth
    from test_stream import _header
    tmp = tmp_path_factory.mktemp("cross")
    s = synth.generate("C2", 1500, seed=11, device="cpu", genome_len=300_000)
    raw = s.raw
    rng = np.random.default_rng(11)
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    c0 = R.NT16_TO_ASCII[codes[int(s.ref.contig_off[0]):int(s.ref.contig_off[0]) + int(s.ref.contig_len[0])]].tobytes()
    c1 = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 40_000).tobytes())
    names = [s.ref.names[0], "chrX2"]
    ref = R.Reference.from_contigs(names, {names[0]: c0, names[1]: c1}, keep_letters=False)
    fam_x = rng.random(int(raw.mi_id.max()) + 1) < 0.06   # families with mates on contig 1
    fam_u = (rng.random(int(raw.mi_id.max()) + 1) < 0.04) & ~fam_x  # mates unmapped
    by_name = {}
    for k in range(raw.n):
        by_name.setdefault(int(raw.name_id[k]), []).append(k)
    for ks in by_name.values():
        if len(ks) != 2 or raw.mi_id[ks[0]] < 0:
            continue
        i, j = (ks[0], ks[1]) if raw.flag[ks[0]] & 64 else (ks[1], ks[0])  # R1, R2
        m = int(raw.mi_id[i])
        if fam_x[m]:
            P = int(rng.integers(1000, 35_000))
            raw.tid[j], raw.pos[j] = 1, P
            raw.next_tid[i], raw.next_pos[i] = 1, P
            raw.next_tid[j], raw.next_pos[j] = 0, raw.pos[i]
            raw.tlen[i] = raw.tlen[j] = 0
        elif fam_u[m]:
            raw.flag[i] |= 8
            raw.flag[j] |= 8
    raw = R.take(raw, np.lexsort((raw.pos, raw.tid)))
    p = str(tmp / "in.bam")
    bam.write_bam(p, _header(ref), bam.records_to_bam(raw), level=1, threads=4)
    fa = str(tmp / "g.fa")
    write_fasta(fa, ref)
    return raw, p, fa, tmp


@pytest.mark.parametrize("n", [2, 3])
def test_cross_contig_and_unmapped_mates(cross_input, n):  # noqa: F811
    """Mates on another contig and unmapped mates: the ranks' output equals the one-range run's
    bytes with no fallback, the cross-key templates going through phase 2"""
    raw, p, fa, tmp = cross_input
    info1, _, ref_bytes, _ = _run(tmp, p, fa, "x1", 1)
    info, st, got, _ = _run(tmp, p, fa, "x%d" % n, n)
    assert info["ranks"] == n and not info["cuts_fallback"]
    assert info["deferred_records"] > 100
    assert info["records_in"] == info1["records_in"] == raw.n
    for a, b in zip(got, ref_bytes):
        assert a == b
    assert not [f for f in os.listdir(tmp) if f.startswith(".")], "pieces left behind"
    if n == 3:  # (and the records are the whole file's, against oracle/)
        assert_bam_matches_oracle(str(tmp / "x3.bam"), p, fa, "ranks, cross-contig mates") > 0


@pytest.fixture(scope="module")
def long_input(tmp_path_factory):
    """Long-span templates (2% of families with mates 20 kb - 2.5 Mb away, one spanning 60% of the
    contig) and mates on a second contig: every far template is deferred by the rank whose core
    holds its records and spliced in at its key."""
    from test_long_span import _long_input
    tmp = tmp_path_factory.mktemp("long")
    raw, p, fa, span = _long_input(tmp, n_fam=2000, cross=0.03)
    return raw, p, fa, tmp


@pytest.mark.parametrize("n", [2, 3])
def test_long_span_ranks_equal_one_range(long_input, n):  # noqa: F811
    """No rank stops on a far record (no fallback), the bytes equal the one-range run's, the records
    equal oracle/ on the whole file, and every rank's buffered bytes stay a few chunks"""
    raw, p, fa, tmp = long_input
    info1, _, ref_bytes, _ = _run(tmp, p, fa, "L1", 1, read_size=16 << 10)
    info, st, got, out = _run(tmp, p, fa, "L%d" % n, n, read_size=16 << 10)
    assert info["ranks"] == n and not info["cuts_fallback"]
    assert info["deferred_records"] > 100
    for a, b in zip(got, ref_bytes):
        assert a == b
    assert max(st["rank_peak_buffered"]) <= 8 * 80_000, st["rank_peak_buffered"]
    assert not [f for f in os.listdir(tmp) if f.startswith(".")], "pieces left behind"
    if n == 3:
        assert_bam_matches_oracle(out, p, fa, "ranks, long-span templates") > 0
