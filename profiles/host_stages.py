"""Host-side stages of the streaming step 5, timed on the CPU alone (no GPU): BGZF decode of a
coordinate-sorted synthetic C2 BAM, family formation (plan), batch materialize, then the output
side (duplex records + BAM/FASTQ encode) on a consensus of the right shape.  The GPU stage is
replaced by a fake consensus (every family emitted, full-length random calls, per-base tag rows),
so this measures what the host does around the kernels, not the kernels.
Usage: python profiles/host_stages.py [--families N] [--threads T] [--fastq]"""
import argparse
import json
import os
import resource
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bsseqconsensusreads_amd import bam, pipeline, synth  # noqa: E402
from bsseqconsensusreads_amd import records as R  # noqa: E402
from bsseqconsensusreads_amd.hostplan import materialize, plan_families  # noqa: E402


def fake_consensus(fb, tags: bool, rng):
    F, stride = fb.n_fam, fb.stride
    seq = rng.integers(0, 4, size=(F, 2, stride), dtype=np.uint8)
    seq = (np.uint8(1) << seq).astype(np.uint8)
    qual = rng.integers(2, 60, size=(F, 2, stride), dtype=np.uint8)
    ln = np.full((F, 2), min(150, stride - 2), np.int32)
    ss = None
    if tags:
        ss = {"len": np.full((F, 4), min(150, stride - 2), np.int32),
              "base": np.repeat(seq, 2, axis=1), "qual": np.repeat(qual, 2, axis=1),
              "depth": np.full((F, 4, stride), 2, np.uint16), "err": np.zeros((F, 4, stride), np.uint16)}
    return pipeline.Consensus(fb.fam_mi.copy(), np.full(F, 7, np.uint8), ln, seq, qual,
                              fb.fam_off.astype(np.int64), fb.src.astype(np.int64), ss)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=200_000)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--chunk-mb", type=int, default=256)
    ap.add_argument("--fastq", action="store_true", help="write the FASTQ pair (no tags) instead of the BAM")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="bsdc_host_")
    s = synth.generate("C2", a.families, seed=42, device="cpu", genome_len=10_000_000)
    raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))
    inp = os.path.join(d, "in.bam")
    names = s.ref.names
    hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tSM:s\tLB:L1\n" % (
        names[0], int(s.ref.n_nibbles)), [names[0]], np.asarray([int(s.ref.n_nibbles)], np.int64))
    bam.write_bam(inp, hdr, bam.records_to_bam(raw), level=5, threads=a.threads)
    T = {"decode": 0.0, "plan": 0.0, "materialize": 0.0, "fake_gpu": 0.0, "records": 0.0, "encode": 0.0}
    rng = np.random.default_rng(1)
    out = os.path.join(d, "out.bam")
    w = None if a.fastq else bam.BamWriter(out, bam.output_header(hdr), 5)
    fq = bam.FastqWriter(out + ".1.fq.gz", out + ".2.fq.gz", 5) if a.fastq else None
    nfam = 0
    C = {k: 0.0 for k in T}  # host CPU seconds per stage (all threads; OpenMP spin-waits included)

    def cpu():
        r = resource.getrusage(resource.RUSAGE_SELF)
        return r.ru_utime + r.ru_stime
    t_all = time.perf_counter()
    it = bam.stream_bam(inp, a.threads, a.chunk_mb << 20)
    while True:
        t0 = time.perf_counter()
        c0 = cpu()
        try:
            h, chunk = next(it)
        except StopIteration:
            break
        t1 = time.perf_counter()
        c1 = cpu()
        plan = plan_families(chunk, "full", s.ref)
        t2 = time.perf_counter()
        c2 = cpu()
        parts = []
        for f0, f1 in pipeline.plan_ranges(plan):
            fb = materialize(plan, f0, f1, 24 * 1024)
            t3 = time.perf_counter()
            parts.append(fake_consensus(fb, not a.fastq, rng))
            T["fake_gpu"] += time.perf_counter() - t3
        cons = pipeline.concat_consensus(parts)
        t4 = time.perf_counter()
        c4 = cpu()
        recs = bam.duplex_records(cons, chunk, "L1", a.threads)
        t5 = time.perf_counter()
        c5 = cpu()
        if w is not None:
            w.add(recs, a.threads)
        if fq is not None:
            fq.add(recs, a.threads)
        t6 = time.perf_counter()
        c6 = cpu()
        C["decode"] += c1 - c0
        C["plan"] += c2 - c1
        C["materialize"] += c4 - c2
        C["records"] += c5 - c4
        C["encode"] += c6 - c5
        T["decode"] += t1 - t0
        T["plan"] += t2 - t1
        T["materialize"] += t4 - t2
        T["records"] += t5 - t4
        T["encode"] += t6 - t5
        nfam += cons.status.shape[0]
    if w is not None:
        w.close(a.threads)
    if fq is not None:
        fq.close(a.threads)
    T["materialize"] -= T["fake_gpu"]
    wall = time.perf_counter() - t_all
    print(json.dumps({"families": a.families, "consensus_families": nfam, "records": int(raw.n), "threads": a.threads,
                      "input_MB": round(os.path.getsize(inp) / 1e6, 1), "seconds": {k: round(v, 3) for k, v in T.items()},
                      "serial_wall_s": round(wall, 3),
                      "cpu_seconds": {k: round(v, 2) for k, v in C.items() if k != "fake_gpu"},
                      "families_per_s_per_stage": {k: round(a.families / v) for k, v in T.items() if v > 0}}))


if __name__ == "__main__":
    main()
