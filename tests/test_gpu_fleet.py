"""The multi-GPU streaming step on the GPU (bsseqconsensusreads_amd/fleet.py): `cli step5 --gpus 2
--multi fleet` on a coordinate-sorted BAM (one coordinator reading the file once, two spawned GPU workers, here
both on GPU 0 via --devices 0,0) writes the bytes of `--gpus 1` (the one-GPU stream), and those
records equal oracle/ on the whole file, record by record.  The whole-file distributed path
(--stream false: every rank plans, rank 0 gathers and writes) is held to the same bar."""
import os
import subprocess
import sys

import numpy as np
import pytest

from bsseqconsensusreads_amd import bam, synth
from bsseqconsensusreads_amd import records as R
from helpers import assert_bam_matches_oracle
from test_fleet import write_fasta

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cli_input(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("gpufleet")
    s = synth.generate("C2", 1500, seed=23, device="cpu", genome_len=120_000)
    raw = synth.messify(s.raw, frac=0.1, seed=2)
    raw = R.take(raw, np.lexsort((raw.pos, raw.tid)))  # coordinate-sorted, as step 5's input is
    fa = str(tmp / "g.fa")
    write_fasta(fa, s.ref)
    codes_len = int(s.ref.contig_len[0])
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tLB:L1\n" % (
        s.ref.names[0], codes_len), [s.ref.names[0]], np.asarray([codes_len], np.int64))
    inp = str(tmp / "in.bam")
    bam.write_bam(inp, hdr, bam.records_to_bam(raw))
    return tmp, inp, fa


def _cli(tmp, inp, fa, tag, *extra):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "bsseqconsensusreads_amd.cli", "step5", "--reference", fa, inp,
           str(tmp / ("%s.bam" % tag)), "--fastq1", str(tmp / ("%s1.fq.gz" % tag)),
           "--fastq2", str(tmp / ("%s2.fq.gz" % tag)), "--threads", "4", "--batch-bases", "20000",
           "--chunk-mb", "0"] + list(extra)
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    return [(tmp / ("%s%s" % (tag, x))).read_bytes() for x in (".bam", "1.fq.gz", "2.fq.gz")]


def test_cli_fleet_two_gpus_equal_one_and_oracle(cli_input):
    tmp, inp, fa = cli_input
    one = _cli(tmp, inp, fa, "one")
    two = _cli(tmp, inp, fa, "two", "--gpus", "2", "--devices", "0,0", "--multi", "fleet")
    assert one == two
    assert assert_bam_matches_oracle(str(tmp / "two.bam"), inp, fa, "cli --gpus 2") > 0


def test_cli_whole_file_ranks_equal_one_and_oracle(cli_input):
    """--stream false --gpus 2: the torch.distributed ranks path (every rank plans, batches dealt,
    rank 0 gathers) -- same bytes as --gpus 1, same records as oracle/"""
    tmp, inp, fa = cli_input
    one = _cli(tmp, inp, fa, "one_w", "--stream", "false")
    two = _cli(tmp, inp, fa, "two_w", "--stream", "false", "--gpus", "2", "--devices", "0,0")
    assert one == two
    assert assert_bam_matches_oracle(str(tmp / "two_w.bam"), inp, fa, "cli --gpus 2 whole file") > 0


def test_cli_fleet_gpu_bgzf_equals_one_gpu(cli_input):
    """--gpus 2 --gpu-bgzf true: the coordinator's writer deflates on devices[0] (GpuBgzf), the
    same blocks as the one-GPU stream with --gpu-bgzf true, so the files are byte-identical"""
    tmp, inp, fa = cli_input
    one = _cli(tmp, inp, fa, "one_gz", "--gpu-bgzf", "true")
    two = _cli(tmp, inp, fa, "two_gz", "--gpus", "2", "--devices", "0,0", "--gpu-bgzf", "true", "--multi", "fleet")
    assert one == two
    assert assert_bam_matches_oracle(str(tmp / "two_gz.bam"), inp, fa, "cli --gpus 2 --gpu-bgzf") > 0
