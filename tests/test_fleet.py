"""Multi-GPU streaming step 5 (bsseqconsensusreads_amd/fleet.py) on CPU: one coordinator process
reads the coordinate-sorted BAM once (stream chunks), forms the families, deals the device batches
to two spawned worker processes through shared memory and writes the outputs in input order.  The
workers run tests/fleet_standin.py (oracle/ in the kernels' output layout) in place of the GPU, so
this covers everything but the launch: spawn, the chunk path, the hand-offs, the ordering, the
writer, errors.  tests/test_gpu_fleet.py runs the same path on the GPU against --gpus 1."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, fleet
from bsseqconsensusreads_amd import records as R
from helpers import assert_bam_matches_oracle
from test_stream import _sorted_bam

STANDIN = "fleet_standin:OracleRunner"


def write_fasta(path, ref):
    codes = R.unpack_nibbles(ref.packed, ref.n_nibbles)
    with open(path, "w") as fh:
        for t, name in enumerate(ref.names):
            o, n = int(ref.contig_off[t]), int(ref.contig_len[t])
            fh.write(">%s\n%s\n" % (name, R.NT16_TO_ASCII[codes[o:o + n]].tobytes().decode()))


@pytest.fixture(scope="module")
def sorted_input(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("fleet")
    s, p = _sorted_bam(tmp, cfg="C2", n_fam=1200, messy=0.15, seed=7, genome_len=300_000)
    fa = str(tmp / "g.fa")
    write_fasta(fa, s.ref)
    return s, p, fa, tmp


def _run(tmp, p, fa, tag, devices, **kw):
    out = str(tmp / ("%s.bam" % tag))
    fq = (str(tmp / ("%s_1.fq.gz" % tag)), str(tmp / ("%s_2.fq.gz" % tag)))
    info = fleet.step5_stream_multi(p, fa, out, devices, threads=2, fastq=fq, runner=STANDIN, chunk_bytes=80_000,
                                    slack=2000, batch_bases=40_000, **kw)
    return info, [open(x, "rb").read() for x in (out,) + fq]


def test_two_workers_write_the_bytes_of_one(sorted_input):
    s, p, fa, tmp = sorted_input
    one, b1 = _run(tmp, p, fa, "one", [0])
    two, b2 = _run(tmp, p, fa, "two", [0, 0], inflight=1)
    assert one["chunks"] > 5 and two["batches"] > one["chunks"]  # several chunks, several batches each
    assert b1 == b2
    assert one["records_out"] == two["records_out"] > 0


def test_records_equal_the_whole_file_oracle(sorted_input):
    """the dealt, gathered, reordered consensus is the whole file's consensus: record by record
    (R1, R2 per emitted family, TemplateCoordinate order) against oracle/ on the whole file"""
    s, p, fa, tmp = sorted_input
    info, _ = _run(tmp, p, fa, "cmp", [0, 0, 0])
    assert assert_bam_matches_oracle(str(tmp / "cmp.bam"), p, fa, "3 workers") == info["records_out"]


def test_worker_error_reaches_the_caller(sorted_input, tmp_path):
    """a failing worker fails the step with its message (no hang, no partial success)"""
    s, p, fa, _ = sorted_input
    with pytest.raises(RuntimeError, match="NotImplementedError|no such module|fleet worker"):
        fleet.step5_stream_multi(p, fa, str(tmp_path / "x.bam"), [0, 0], threads=2,
                                 runner="fleet_standin:NoSuchRunner", chunk_bytes=80_000, slack=2000)


def test_worker_failure_mid_stream(sorted_input, tmp_path):
    """a worker failing after some batches: the step raises its message and every process ends"""
    s, p, fa, _ = sorted_input
    with pytest.raises(RuntimeError, match="stand-in failure on batch 3"):
        fleet.step5_stream_multi(p, fa, str(tmp_path / "y.bam"), [0, 0], threads=2,
                                 runner="fleet_standin:FailingRunner", chunk_bytes=80_000, slack=2000,
                                 batch_bases=40_000)


def test_pack_roundtrip():
    pool, views = fleet.SegmentPool("t"), fleet.SegmentViews()
    try:
        a = np.arange(100_000, dtype=np.int64).reshape(1000, 100)
        t = {"a": a, "s": bam.StringTable.from_list([b"x", b"yz"]), "l": [a[:3], a[3:5]], "k": 7}
        tree, segs = fleet.pack(t, pool)
        assert len(segs) == 1
        u = fleet.unpack(tree, views)
        assert np.array_equal(u["a"], a) and u["k"] == 7 and u["s"][1] == b"yz"
        assert np.array_equal(u["l"][1], a[3:5])
        # an array already in one of the pool's segments travels by reference (no second segment)
        name = pool.take(1 << 20)
        img = np.frombuffer(pool.buf(name), np.uint8, count=1 << 20)
        img[:] = 7
        tree2, segs2 = fleet.pack({"img": img[4096:]}, pool)
        assert segs2 == [name] and tree2[1]["img"][1:3] == (name, 4096)
        assert (fleet.unpack(tree2, views)["img"] == 7).all()
        pool.give(segs[0])
        assert pool.take(100) == segs[0]  # reused
        del u
    finally:
        views.close()
        pool.close()


def test_segment_churn_and_forget():
    """prefilled segments count towards `keep` (steady state reuses them, nothing is
    dropped and re-created); a segment the pool does drop is reported through on_drop, and the
    other side's SegmentViews.forget unmaps it; small arrays travel as copies (the queue pickles
    them later, when their segment may already be reused)."""
    dropped = []
    pool = fleet.SegmentPool("c", keep=1, on_drop=dropped.append)
    views = fleet.SegmentViews()
    try:
        pool.prefill(3, 1 << 20).join()
        assert pool.keep == 4 and len(pool.free) == 3
        names = [pool.take(1 << 10) for _ in range(3)]
        for n in names:
            pool.give(n)
        assert dropped == [] and len(pool.free) == 3
        names = [pool.take(1 << 10) for _ in range(3)]
        extra = [pool.take(2 << 20) for _ in range(2)]  # two more than the prefilled ones
        assert not set(extra) & set(names)
        for n in extra + names:
            views.buf(n)
        for n in extra + names:
            pool.give(n)
        assert len(pool.free) == 4 and len(dropped) == 1
        views.forget(dropped[0])
        assert dropped[0] not in views.open and len(views.open) == 4 and dropped[0] not in pool.segs
        views.forget("no-such-segment")
        small = np.frombuffer(pool.buf(pool.free[0]), np.uint8, count=64)
        small[:] = 3
        tree, segs = fleet.pack({"q": small}, pool)
        assert segs == [] and tree[1]["q"][1] is not small
        small[:] = 5
        assert (fleet.unpack(tree)["q"] == 3).all()
    finally:
        views.close()
        pool.close()
