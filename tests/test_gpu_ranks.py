"""Rank-parallel step 5 on the GPU (bsseqconsensusreads_amd/ranks.py): `cli step5 --gpus N` on a
coordinate-sorted BAM (the default --multi ranks: N spawned rank processes, here all on GPU 0 via
--devices, each decoding, computing and encoding its own key interval of the file) writes a BAM
and FASTQ pair that decompress to the bytes of `--gpus 1`, whose records equal oracle/ on the
whole file (tests/test_gpu_fleet.py).  Only the BGZF blocks at the ranks' seams differ."""
import gzip
import json
import os
import subprocess
import sys

import pytest

from helpers import assert_bam_matches_oracle
from test_gpu_fleet import _cli, cli_input  # noqa: F401 -- (the module fixture)
from test_ranks import cross_input  # noqa: F401 -- (the module fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2, 3])
def test_cli_ranks_equal_one_gpu_and_oracle(cli_input, n):  # noqa: F811
    tmp, inp, fa = cli_input
    one = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "r_one")]
    got = _cli(tmp, inp, fa, "r%d" % n, "--gpus", str(n), "--devices", ",".join(["0"] * n))
    assert [gzip.decompress(b) for b in got] == one
    assert assert_bam_matches_oracle(str(tmp / ("r%d.bam" % n)), inp, fa, "cli --gpus %d ranks" % n) > 0


def test_cli_ranks_report(cli_input):  # noqa: F811
    """The ranks really split the file (no fallback): the info line names 2 ranks"""
    tmp, inp, fa = cli_input
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-m", "bsseqconsensusreads_amd.cli", "step5", "--reference", fa, inp,
                        str(tmp / "rep.bam"), "--threads", "4", "--gpus", "2", "--devices", "0,0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    info = json.loads(p.stderr.strip().splitlines()[-1])
    assert info["ranks"] == 2 and not info["cuts_fallback"]


def test_cli_ranks_cross_contig_mates(cross_input):  # noqa: F811
    """Mates on another contig and unmapped mates on the GPU: the two ranks spill them, form them
    in phase 2 (no fallback), and the output decompresses to the bytes of --gpus 1 and equals
    oracle/ on the whole file"""
    raw, inp, fa, tmp = cross_input
    one = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "x_one")]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-m", "bsseqconsensusreads_amd.cli", "step5", "--reference", fa, inp,
                        str(tmp / "x2.bam"), "--fastq1", str(tmp / "x21.fq.gz"), "--fastq2", str(tmp / "x22.fq.gz"),
                        "--threads", "4", "--batch-bases", "20000", "--chunk-mb", "0",
                        "--gpus", "2", "--devices", "0,0"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    info = json.loads(p.stderr.strip().splitlines()[-1])
    assert info["ranks"] == 2 and not info["cuts_fallback"] and info["deferred_records"] > 100
    got = [gzip.decompress((tmp / ("x2%s" % x)).read_bytes()) for x in (".bam", "1.fq.gz", "2.fq.gz")]
    assert got == one
    assert assert_bam_matches_oracle(str(tmp / "x2.bam"), inp, fa, "cli --gpus 2 ranks, cross-contig") > 0


@pytest.fixture(scope="module")
def long_gpu_input(tmp_path_factory):
    from test_long_span import _long_input
    tmp = tmp_path_factory.mktemp("longgpu")
    raw, p, fa, span = _long_input(tmp, n_fam=2000, cross=0.03)
    return raw, p, fa, tmp


def test_cli_long_span_templates(long_gpu_input):  # noqa: F811
    """Long-span templates (mates 20 kb - 2.5 Mb away, one spanning 60% of the contig) and mates
    on a second contig on the GPU: the one-GPU stream defers them and splices
    their families in (with the GPU BGZF too), two ranks on GPU 0 do the same with no fallback; all
    decompress to the same bytes and equal oracle/ on the whole file"""
    raw, inp, fa, tmp = long_gpu_input
    one = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "L_one")]
    gz = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "L_gz", "--gpu-bgzf", "true")]
    assert gz == one
    assert assert_bam_matches_oracle(str(tmp / "L_one.bam"), inp, fa, "cli one GPU, long-span") > 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-m", "bsseqconsensusreads_amd.cli", "step5", "--reference", fa, inp,
                        str(tmp / "L2.bam"), "--fastq1", str(tmp / "L21.fq.gz"), "--fastq2", str(tmp / "L22.fq.gz"),
                        "--threads", "4", "--batch-bases", "20000", "--chunk-mb", "0",
                        "--gpus", "2", "--devices", "0,0"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    info = json.loads(p.stderr.strip().splitlines()[-1])
    assert info["ranks"] == 2 and not info["cuts_fallback"] and info["deferred_records"] > 100
    got = [gzip.decompress((tmp / ("L2%s" % x)).read_bytes()) for x in (".bam", "1.fq.gz", "2.fq.gz")]
    assert got == one


def test_cli_many_contigs(tmp_path_factory):
    """Seven contigs with mates across them and long-span templates (tests/test_many_contigs.py's
    input) on the GPU: one GPU, and two ranks on GPU 0 whose key intervals each span several
    contigs, decompress to the same bytes, equal to oracle/ on the whole file"""
    from test_many_contigs import _contigs_input
    raw, inp, fa, tmp, cross = _contigs_input(tmp_path_factory.mktemp("contigsgpu"))
    assert cross > 20
    one = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "C_one")]
    assert assert_bam_matches_oracle(str(tmp / "C_one.bam"), inp, fa, "cli one GPU, seven contigs") > 0
    got = [gzip.decompress(b) for b in _cli(tmp, inp, fa, "C_two", "--gpus", "2", "--devices", "0,0")]
    assert got == one
