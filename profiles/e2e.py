"""End-to-end timing of the file-level drop-ins on the GPU box (not the bench metric): a synthetic
grouped BAM + FASTA on local disk -> bam.step5 (decode, family formation, upload, fused kernels,
fetch, output records, BAM + FASTQ encode) and bam.molecular, stage by stage.  The BAM and FASTA
are written first (untimed).  Usage: python profiles/e2e.py [--families N] [--threads T]"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bsseqconsensusreads_amd import bam, batch, pipeline, synth  # noqa: E402
from bsseqconsensusreads_amd import records as R  # noqa: E402
from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_VOTE  # noqa: E402
from bsseqconsensusreads_amd.device import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--families", type=int, default=200_000)
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--config", default="C2")
a = ap.parse_args()

d = tempfile.mkdtemp(prefix="bsdc_e2e_")
s = synth.generate(a.config, a.families, seed=42, device=torch.device("cuda", 0), genome_len=10_000_000)
raw = R.take(s.raw, np.lexsort((s.raw.pos, s.raw.tid)))  # coordinate-sorted, as the step-5 input is
codes = R.unpack_nibbles(s.ref.packed, s.ref.n_nibbles)
fa = os.path.join(d, "g.fa")
with open(fa, "wb") as fh:
    fh.write((">%s\n" % s.ref.names[0]).encode())
    fh.write(R.NT16_TO_ASCII[codes].tobytes())
    fh.write(b"\n")
hdr = bam.BamHeader("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:%s\tLN:%d\n@RG\tID:x\tSM:s\tLB:L1\n" % (
    s.ref.names[0], len(codes)), [s.ref.names[0]], np.asarray([len(codes)], np.int64))
inp = os.path.join(d, "in.bam")
bam.write_bam(inp, hdr, bam.records_to_bam(raw), threads=a.threads)
in_mb = os.path.getsize(inp) / 1e6

eng = Engine(0)
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    T[name] = round(time.perf_counter() - t0, 4)
    return time.perf_counter()


for rep in range(2):  # the first pass warms the code paths and the page cache
    T = {}
    t = time.perf_counter()
    t0 = t
    h, r = bam.read_bam(inp, a.threads)
    t = tick("bam_decode", t)
    ref = bam.read_fasta(fa, h)
    eng.load_reference(ref)
    t = tick("fasta+reference_upload", t)
    fb = batch.build_family_batch(r, "full", eng.ref)
    t = tick("family_formation", t)
    db = eng.upload(fb)
    t = tick("upload", t)
    eng.run(db, MODE_CONVERT | MODE_EXTEND | MODE_VOTE)
    t = tick("kernels", t)
    cons = pipeline.consensus_from_output(fb, db.fetch())
    t = tick("fetch", t)
    recs = bam.duplex_records(cons, r, bam.read_name_prefix(h), a.threads)
    t = tick("output_records", t)
    bam.write_bam(os.path.join(d, "out.bam"), bam.output_header(h), recs, 6, a.threads)
    t = tick("bam_encode", t)
    bam.write_fastq(os.path.join(d, "o1.fq.gz"), os.path.join(d, "o2.fq.gz"), recs, 6, a.threads)
    t = tick("fastq_encode", t)
    total = time.perf_counter() - t0
t0 = time.perf_counter()
info = bam.molecular(inp, os.path.join(d, "mol.bam"), eng, threads=a.threads)
mol = time.perf_counter() - t0
print(json.dumps({"config": a.config, "families": a.families, "records": int(r.n), "input_MB": round(in_mb, 1),
                  "host_threads": a.threads, "step5_stage_s": T, "step5_total_s": round(total, 3),
                  "step5_families_per_s": round(a.families / total, 1),
                  "kernel_share": round(T["kernels"] / total, 4),
                  "molecular_total_s": round(mol, 3), "molecular_families_per_s": round(info["families"] / mol, 1)}))
eng.close()
