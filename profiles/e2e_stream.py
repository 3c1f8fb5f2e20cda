"""End-to-end families/s of the file-level step 5 on the GPU box (not the bench metric): a
synthetic coordinate-sorted C2 BAM + FASTA on local disk, then, each in a fresh child process
(so that its peak RSS is its own):
  whole   bam.step5: read the whole BAM, form every family, GPU batches, write the BAM
  stream  bam.step5_stream: bounded chunks, reader / GPU / writer threads overlapped
  stream_fastq  the same, writing the FASTQ pair of the next rule instead of the BAM
  stream_gpubgzf, stream_fastq_gpubgzf  the same with the BGZF deflate on the GPU
  fleet   fleet.step5_stream_multi: this child reads and writes, --workers spawned GPU worker
          processes (all on GPU 0 on a one-GPU box; started before the clock) run the batches
  fleet_gpubgzf  the same with the writer's deflate on GPU 0
  ranks, ranks_gpubgzf  ranks.step5_ranks: --workers rank processes (all on GPU 0 here; a
          RankPool started before the clock), each decoding, computing and writing its own key
          interval with threads / workers host threads
  molecular_stream, molecular_whole  step 1 (bam.molecular_stream / bam.molecular) on the same
          families in GroupReadsByUmi order (a second input, MI runs contiguous; BAM with tags, GPU BGZF)
The BAMs are compared byte for byte.  Usage:
  python profiles/e2e_stream.py [--families N] [--threads T] [--chunk-mb M] [--level L]
                                [--modes stream,stream_fastq,whole,fleet] [--workers W]"""
import argparse
import json
import os
import resource
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def prep(args):
    """The input files (synthetic data generated on the GPU, in this child only)."""
    import numpy as np

    from bsseqconsensusreads_amd import bam, synth
    from bsseqconsensusreads_amd import records as R
    s = synth.generate("C2", args.families, seed=42, device="cuda", genome_len=50_000_000)
    raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))
    codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
    with open(args.fa, "wb") as fh:
        fh.write((">%s\n" % s.ref.names[0]).encode() + R.NT16_TO_ASCII[codes].tobytes() + b"\n")
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tSM:s\tLB:L1\n" % (
        s.ref.names[0], len(codes)), [s.ref.names[0]], np.asarray([len(codes)], np.int64))
    bam.write_bam(args.inp, hdr, bam.records_to_bam(raw), level=args.level, threads=args.threads)
    if args.grouped:  # step 1's input: each MI's /A and /B molecules contiguous
        g = R.take(s.raw, np.lexsort((s.raw.mi_strand, s.raw.mi_id)))
        bam.write_bam(args.grouped, hdr, bam.records_to_bam(g), level=args.level, threads=args.threads)
    print(json.dumps({"records": int(raw.n)}))


def child(args):
    if args.mode == "prep":
        return prep(args)
    import bsseqconsensusreads_amd  # noqa: F401  (first, as in the CLI: its OpenMP wait policy)
    import torch  # noqa: F401  (the GPU runtime, as the CLI loads it)

    from bsseqconsensusreads_amd import bam
    stats = {}
    if args.mode in ("fleet", "fleet_gpubgzf"):  # the coordinator's workers hold the GPU
        from bsseqconsensusreads_amd import fleet
        ts = time.perf_counter()
        fl = fleet.Fleet([0] * args.workers)  # started (spawn, import, HIP init) outside the clock
        if args.mode == "fleet_gpubgzf":  # (the writer's GPU runtime too, as the stream's engine is)
            import torch
            torch.zeros(1, device="cuda:0")
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            info = fleet.step5_stream_multi(args.inp, args.fa, args.out, [0] * args.workers, threads=args.threads,
                                            level=args.level, chunk_bytes=args.chunk_mb << 20, stats=stats,
                                            gpu_bgzf=args.mode == "fleet_gpubgzf", fleet=fl)
            dt = time.perf_counter() - t0
        finally:
            fl.close()
        stats["fleet_start_s"] = round(t0 - ts, 3)
        rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024
        crss = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 1024
        print(json.dumps({"mode": args.mode, "workers": args.workers, "seconds": round(dt, 3),
                          "peak_rss_MiB": round(rss, 1), "worker_peak_rss_MiB": round(crss, 1),
                          "stage_busy_s": stats, **info}))
        return 0
    if args.mode in ("ranks", "ranks_gpubgzf"):  # rank processes, each its own part of the file
        from bsseqconsensusreads_amd import ranks
        ts = time.perf_counter()
        pool = ranks.RankPool([0] * args.workers)  # started (spawn, import, HIP init) outside the clock
        t0 = time.perf_counter()
        try:
            info = ranks.step5_ranks(args.inp, args.fa, args.out, [0] * args.workers,
                                     threads=max(1, args.threads // args.workers), level=args.level,
                                     chunk_bytes=args.chunk_mb << 20, stats=stats,
                                     gpu_bgzf=args.mode == "ranks_gpubgzf", pool=pool)
            dt = time.perf_counter() - t0
        finally:
            pool.close()
        stats["pool_start_s"] = round(t0 - ts, 3)
        crss = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 1024
        print(json.dumps({"mode": args.mode, "ranks": args.workers, "seconds": round(dt, 3),
                          "rank_peak_rss_MiB": round(crss, 1), "stage_busy_s": stats, **info}))
        return 0
    from bsseqconsensusreads_amd.device import Engine
    eng = Engine(0)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    cpu0 = ru0.ru_utime + ru0.ru_stime
    t0 = time.perf_counter()
    if args.mode == "molecular_stream":
        info = bam.molecular_stream(args.grouped, args.out, engine=eng, threads=args.threads, level=args.level,
                                    chunk_bytes=args.chunk_mb << 20, stats=stats, gpu_bgzf=True)
    elif args.mode == "molecular_whole":
        info = bam.molecular(args.grouped, args.out, engine=eng, threads=args.threads, level=args.level)
    elif args.mode == "whole":
        info = bam.step5(args.inp, args.fa, args.out, engine=eng, threads=args.threads, level=args.level)
    elif args.mode in ("stream_fastq", "stream_fastq_gpubgzf"):  # the fused FASTQ emission
        # (main.snake.py:167-177), no BAM; _gpubgzf: its blocks deflated on the GPU
        info = bam.step5_stream(args.inp, args.fa, None, engine=eng, threads=args.threads, level=args.level,
                                fastq=(args.out + ".1.fq.gz", args.out + ".2.fq.gz"),
                                chunk_bytes=args.chunk_mb << 20, stats=stats,
                                gpu_bgzf=args.mode == "stream_fastq_gpubgzf")
    else:  # stream, or stream_gpubgzf: the BAM's blocks deflated on the GPU (bam.GpuBgzf)
        info = bam.step5_stream(args.inp, args.fa, args.out, engine=eng, threads=args.threads, level=args.level,
                                chunk_bytes=args.chunk_mb << 20, stats=stats, gpu_bgzf=args.mode == "stream_gpubgzf")
    dt = time.perf_counter() - t0
    eng.close()
    ru = resource.getrusage(resource.RUSAGE_SELF)
    rss = ru.ru_maxrss / 1024  # MiB
    cpu = ru.ru_utime + ru.ru_stime - cpu0  # host CPU seconds of the run (all threads)
    print(json.dumps({"mode": args.mode, "seconds": round(dt, 3), "peak_rss_MiB": round(rss, 1),
                      "cpu_s": round(cpu, 2), "cores_busy": round(cpu / dt, 2),
                      "stage_busy_s": stats, **info}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--chunk-mb", type=int, default=64)
    ap.add_argument("--level", type=int, default=5)
    ap.add_argument("--mode", default=None)
    ap.add_argument("--modes", default="stream,stream_fastq,whole")
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--inp")
    ap.add_argument("--fa")
    ap.add_argument("--out")
    ap.add_argument("--grouped", default="")
    a = ap.parse_args()
    if a.mode:
        return child(a)
    # this process never touches the GPU: every GPU step runs in a child process
    d = tempfile.mkdtemp(prefix="bsdc_e2es_")
    t0 = time.perf_counter()
    fa, inp = os.path.join(d, "g.fa"), os.path.join(d, "in.bam")
    grouped = os.path.join(d, "grouped.bam") if "molecular" in a.modes else ""
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--mode", "prep", "--inp", inp, "--fa", fa,
                        "--families", str(a.families), "--threads", str(a.threads), "--level", str(a.level),
                        "--grouped", grouped],
                       stdout=subprocess.PIPE, text=True, timeout=900)
    if p.returncode != 0:
        print(p.stdout[-2000:], file=sys.stderr)
        return p.returncode
    n_rec = json.loads(p.stdout.strip().splitlines()[-1])["records"]
    prep = time.perf_counter() - t0
    res = {"families": a.families, "records": n_rec, "input_MB": round(os.path.getsize(inp) / 1e6, 1),
           "host_threads": a.threads, "level": a.level, "chunk_MiB": a.chunk_mb, "prep_s": round(prep, 1)}
    print("prepared", json.dumps(res), flush=True)
    outs = {}
    for mode in a.modes.split(","):
        out = os.path.join(d, mode + ".bam")
        p = subprocess.run([sys.executable, os.path.abspath(__file__), "--mode", mode, "--inp", inp, "--fa", fa,
                            "--out", out, "--threads", str(a.threads), "--chunk-mb", str(a.chunk_mb),
                            "--level", str(a.level), "--workers", str(a.workers), "--grouped", grouped],
                           stdout=subprocess.PIPE, text=True,
                           timeout=900)
        if p.returncode != 0:
            print(p.stdout[-2000:], file=sys.stderr)
            return p.returncode
        r = json.loads(p.stdout.strip().splitlines()[-1])
        r["families_per_s"] = round(a.families / r["seconds"], 1)
        res[mode] = r
        outs[mode] = out
        print(mode, json.dumps(r), flush=True)
    bams = [open(outs[m], "rb").read() for m in outs if m != "stream_fastq" and "gpubgzf" not in m
            and not m.startswith("molecular") and not m.startswith("ranks")]
    if "ranks" in outs and "stream" in outs:  # other BGZF blocks at the rank seams: the bytes inside
        import gzip
        res["ranks_bytes_identical"] = gzip.open(outs["ranks"]).read() == gzip.open(outs["stream"]).read()
    res["outputs_identical"] = all(b == bams[0] for b in bams)
    gz = [open(outs[m], "rb").read() for m in ("stream_gpubgzf", "fleet_gpubgzf") if m in outs]
    if len(gz) == 2:  # the same GPU-deflated blocks from one GPU and from the fleet's writer
        res["gpubgzf_fleet_identical"] = gz[0] == gz[1]
    if "stream_gpubgzf" in outs and "stream" in outs:  # other compressed bytes: compare the records
        sys.path.insert(0, ROOT)
        from bsseqconsensusreads_amd import bam as B
        _, ra = B.read_bam(outs["stream"], a.threads)
        _, rb = B.read_bam(outs["stream_gpubgzf"], a.threads)
        res["gpubgzf_records_identical"] = bool(ra.n == rb.n and (ra.seq == rb.seq).all() and (ra.qual == rb.qual).all()
                                                and (ra.aux.buf == rb.aux.buf).all())
        res["gpubgzf_size_ratio"] = round(os.path.getsize(outs["stream_gpubgzf"]) / os.path.getsize(outs["stream"]), 3)
    if "stream_fastq_gpubgzf" in outs and "stream_fastq" in outs:  # the same FASTQ text
        import gzip
        res["fastq_gpubgzf_text_identical"] = all(
            gzip.open(outs["stream_fastq"] + x).read() == gzip.open(outs["stream_fastq_gpubgzf"] + x).read()
            for x in (".1.fq.gz", ".2.fq.gz"))
    if "molecular_stream" in outs and "molecular_whole" in outs:  # GPU BGZF vs host deflate: the records
        sys.path.insert(0, ROOT)
        from bsseqconsensusreads_amd import bam as B
        _, ra = B.read_bam(outs["molecular_whole"], a.threads)
        _, rb = B.read_bam(outs["molecular_stream"], a.threads)
        res["molecular_records_identical"] = bool(ra.n == rb.n and (ra.seq == rb.seq).all() and (ra.qual == rb.qual).all())
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
