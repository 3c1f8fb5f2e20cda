"""bam.step5_stream's thread pipeline on the CPU (decoder, reader with pooled record buffers,
planner + materialize, GPU stage, builder, writer): the GPU stage's batches are
answered by oracle/ (tests/fleet_standin.OracleRunner, TEST INFRASTRUCTURE ONLY) and pinned pools
by plain host arrays, so every hand-off, buffer rotation and drain runs without a GPU.  The BAM
(with tags) and the FASTQ pair it writes are checked record by record against oracle/ on the
whole file; a failing stage must surface its error."""
import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, device, pipeline
from bsseqconsensusreads_amd import records as R
from fleet_standin import OracleRunner
from helpers import assert_bam_matches_oracle
from test_gpu_stream import _inputs


class _HostPool:
    """device.PinnedPool with host arrays."""

    def images(self, n_slots):
        return np.empty(n_slots // 2 + 64, np.uint8), np.empty(n_slots, np.uint8)

    def reset(self):
        pass


class _Engine:
    device = "cpu"

    def __init__(self):
        self.runner = OracleRunner(0)

    def load_reference(self, ref):
        self.runner.load_reference(ref)

    def close(self):
        pass


@pytest.fixture
def standin(monkeypatch):
    monkeypatch.setattr(device, "PinnedPool", _HostPool)
    orig = pipeline.materialize_ranges

    def materialize_ranges(plan, ranges, images=None):
        fbs = orig(plan, ranges, images)
        for fb in fbs:
            fb._raw = plan.raw  # the stand-in answers a batch from its records
        return fbs

    def run_batches(engine, batches, mode, tags=False, timing=None):
        out = []
        for fb in batches:
            sub = R.take(fb._raw, np.asarray(fb.src, np.int64))
            out.append(pipeline.consensus_from_output(fb, engine.runner.run_batch(fb, mode, tags, sub)))
        return out
    monkeypatch.setattr(pipeline, "materialize_ranges", materialize_ranges)
    monkeypatch.setattr(pipeline, "run_batches", run_batches)
    return _Engine()


def test_stream_pipeline_bam_and_fastq_match_oracle(standin, tmp_path):
    inp, fa = _inputs(tmp_path, "C2", 900, 0.0, 21)
    b = str(tmp_path / "s.bam")
    fq = (str(tmp_path / "r1.fq.gz"), str(tmp_path / "r2.fq.gz"))
    stats = {}
    info = bam.step5_stream(inp, fa, b, engine=standin, threads=2, level=1, fastq=fq, chunk_bytes=60_000,
                            slack=2000, stats=stats)
    assert info["chunks"] > 4 and stats["reader_copy"] > 0
    assert assert_bam_matches_oracle(b, inp, fa, "stream pipeline") == info["records_out"]
    assert open(fq[0], "rb").read()[:2] == b"\x1f\x8b"


def test_stream_pipeline_surfaces_a_stage_error(standin, tmp_path, monkeypatch):
    inp, fa = _inputs(tmp_path, "C2", 600, 0.0, 22)
    calls = {"n": 0}
    orig = bam.duplex_records

    def failing(*a, **k):
        calls["n"] += 1
        if calls["n"] == 3:
            raise RuntimeError("builder failed on purpose")
        return orig(*a, **k)
    monkeypatch.setattr(bam, "duplex_records", failing)
    with pytest.raises(RuntimeError, match="on purpose"):
        bam.step5_stream(inp, fa, str(tmp_path / "x.bam"), engine=standin, threads=2, level=1, chunk_bytes=40_000,
                         slack=2000)
