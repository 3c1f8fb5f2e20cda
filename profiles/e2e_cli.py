"""CLI wall time on the GPU box (not the bench metric): `python -m
bsseqconsensusreads_amd.cli step5` on a synthetic coordinate-sorted C2 BAM, one process (--gpus 1)
against the rank path (--gpus N --devices 0,..,0: N spawned rank processes on GPU 0), each timed
around the whole command as a user would see it -- interpreter start, imports, HIP start-up, the
ranks' spawn, the run and the assembly.  Alternated, `--reps` times each; the outputs must
decompress to the same bytes.  The input is written first (untimed).
Usage: python profiles/e2e_cli.py [--families N] [--threads T] [--ranks N] [--reps K]"""
import argparse
import gzip
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--families", type=int, default=1_000_000)
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--ranks", type=int, default=2)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--gpu-bgzf", default="true")
a = ap.parse_args()


def prepare(d):
    import torch

    from bsseqconsensusreads_amd import bam, synth
    from bsseqconsensusreads_amd import records as R
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    s = synth.generate("C2", a.families, seed=42, device=dev, genome_len=10_000_000)
    raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    fa = os.path.join(d, "g.fa")
    with open(fa, "wb") as fh:
        fh.write((">%s\n" % s.ref.names[0]).encode() + R.NT16_TO_ASCII[codes].tobytes() + b"\n")
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tSM:s\tLB:L1\n" % (
        s.ref.names[0], len(codes)), [s.ref.names[0]], np.asarray([len(codes)], np.int64))
    inp = os.path.join(d, "in.bam")
    bam.write_bam(inp, hdr, bam.records_to_bam(raw), threads=a.threads)
    return inp, fa, int(raw.n)


def run(d, inp, fa, tag, extra, threads):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    out = [os.path.join(d, "%s.bam" % tag), os.path.join(d, "%s_1.fq.gz" % tag), os.path.join(d, "%s_2.fq.gz" % tag)]
    cmd = [sys.executable, "-m", "bsseqconsensusreads_amd.cli", "step5", "--reference", fa, inp, out[0],
           "--fastq1", out[1], "--fastq2", out[2], "--threads", str(threads), "--gpu-bgzf", a.gpu_bgzf] + extra
    t0 = time.perf_counter()
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    sec = time.perf_counter() - t0
    if p.returncode != 0:
        print(p.stderr[-3000:], file=sys.stderr)
        raise SystemExit("%s failed" % tag)
    info = json.loads(p.stderr.strip().splitlines()[-1])
    return sec, info, out


def main():
    d = tempfile.mkdtemp(prefix="bsdc_e2ecli_")
    t0 = time.perf_counter()
    inp, fa, n_rec = prepare(d)
    prep = time.perf_counter() - t0
    # the fixed cost of a process that touches the GPU: interpreter + torch import + HIP start
    t1 = time.perf_counter()
    subprocess.run([sys.executable, "-c", "import torch; torch.cuda.init(); torch.zeros(1, device='cuda')"], check=True)
    torch_start = time.perf_counter() - t1
    res = {"families": a.families, "records": n_rec, "input_MB": round(os.path.getsize(inp) / 1e6, 1),
           "threads_one_process": a.threads, "threads_per_rank": max(1, a.threads // a.ranks), "ranks": a.ranks, "prep_s": round(prep, 1),
           "torch_hip_start_s": round(torch_start, 3), "one": [], "ranks_s": [], "rank_info": None}
    print("prepared", json.dumps(res), flush=True)
    outs = {}
    devs = ",".join(["0"] * a.ranks)
    for rep in range(a.reps):
        for mode in ("one", "ranks"):
            extra = [] if mode == "one" else ["--gpus", str(a.ranks), "--devices", devs]
            sec, info, out = run(d, inp, fa, "%s%d" % (mode, rep), extra,
                                 a.threads if mode == "one" else max(1, a.threads // a.ranks))
            res["one" if mode == "one" else "ranks_s"].append(round(sec, 3))
            if mode == "ranks":
                res["rank_info"] = info
            outs[mode] = out
            print(mode, rep, round(sec, 3), json.dumps(info)[:400], flush=True)
    same = all(gzip.decompress(open(x, "rb").read()) == gzip.decompress(open(y, "rb").read())
               for x, y in zip(outs["one"], outs["ranks"]))
    res["outputs_identical"] = same
    res["ratio_ranks_over_one"] = round(min(res["ranks_s"]) / min(res["one"]), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
