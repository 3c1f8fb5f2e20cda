"""Step-5 duplex path throughput on MI355X (BASELINE.json metric: duplex families/sec).

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): 1M synthetic WGBS/EM-seq duplex families per
GPU, 2x150 bp, Poisson(4) templates per family split between the strands, generated on the GPU
from a seeded model (no network, no real data).  A "step" is one pass of the fused hot path --
B-strand conversion, gap extension, overlapping-bases consensus, source reads, alignment filter,
single-strand vote, duplex combine -- over every resident batch of the rank (bsdc_run, both
family kernels).  Inputs are in HBM before the timed region; outputs stay in HBM.

Multi-GPU: one process per GPU.  `--gpus N` without a launcher spawns the N ranks itself
(shard.launch, before anything touches the GPU); under torch.distributed.run the environment's
WORLD_SIZE must equal N.  Every rank owns its own families (weak scaling, no data-path
collective); barrier + synchronize around the timed steps; shard.reduce_step takes the MAX time
over ranks and SUMs the family counters (the optional RCCL counter reduction of SURVEY.md 8e);
value = families on all ranks / that time.

C5 (configs[4], 100M families over 2/4/8 GPUs): C2-shaped families, each rank's share (default
12.5M = 100M / 8) generated and uploaded as a stream of bounded batches (--batch-families) that
stay resident; a step runs every batch once.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bsseqconsensusreads_amd import batch as B  # noqa: E402
from bsseqconsensusreads_amd import shard, synth  # noqa: E402
from bsseqconsensusreads_amd._lib import (MODE_CONVERT, MODE_EXTEND, MODE_SKIP_LARGE, MODE_SKIP_SMALL,  # noqa: E402
                                          MODE_TAGS, MODE_VOTE)

METRIC = "duplex families/sec (node) at 1/2/4/8 MI355X; % HBM roofline; speedup vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    "C2": "configs[1]: 1M-family synthetic WGBS grouped BAM, 2x150bp, Poisson(4) family size, one MI355X",
    "C0": "1 template per strand (the pipeline as written), 2x150bp",
    "C1": "configs[0] shape: 3 reads/strand EM-seq families, 2x150bp",
    "C3": "configs[2]: high-depth panel, 20-100 templates/family, short overlapping inserts",
    "C4": "configs[3]: skewed 1-500 family sizes, 30% AB-only",
    "C5": "configs[4]: 100M-family C2-shaped EM-seq set sharded by family batch; per-GPU share as a "
          "stream of resident batches",
}
DEFAULT_FAMILIES = {"C3": 200_000, "C5": 12_500_000}
FULL_MODE = MODE_CONVERT | MODE_EXTEND | MODE_VOTE
# the arithmetic the vote computes in (the data are u8 bases / quals)
DTYPE = ("int64 fixed-point log-likelihood sums (2^-20 nats) + fp32 exp; fp64 read-order sums on near ties; "
         "u8 nt16 bases / phred quals")


def family_input_bytes(fb: B.FamilyBatch) -> np.ndarray:
    """SURVEY.md 8d, input side per family: sum_records(ceil(L/2) + L + 16) + sum_converted ceil((L+2)/2)."""
    L = (fb.rec_lenflag & 0xFFFF).astype(np.int64)
    conv = (fb.rec_link & B.LINK_CONVERT) != 0
    per_rec = (L + 1) // 2 + L + 16 + np.where(conv, (L + 3) // 2, 0)
    sizes = np.diff(fb.fam_off.astype(np.int64))
    fam_of = np.repeat(np.arange(fb.n_fam), sizes)
    return np.bincount(fam_of, weights=per_rec, minlength=fb.n_fam).astype(np.int64)


def family_output_bytes(cons_len: np.ndarray, status: np.ndarray) -> np.ndarray:
    """SURVEY.md 8d, output side per family: sum_{2 ends}(ceil(Lc/2) + Lc)."""
    lc = np.where((status & 1)[:, None] != 0, cons_len, 0).astype(np.int64)
    return ((lc + 1) // 2 + lc).sum(1)


def cpu_baseline(raw, ref, n_fam_sample: int, threads: int):
    """oracle/ (C restatement, OpenMP over families) on the first n_fam_sample families -> families/s."""
    from oracle import oracle
    sub = synth.subset_families(raw, n_fam_sample)
    res = oracle.run(sub, ref, threads=threads)
    return n_fam_sample / res.seconds, res.seconds


class Resident:
    """One device batch kept in HBM for the timed steps, with its host-side accounting."""

    def __init__(self, eng, fb: B.FamilyBatch, tags: bool = False):
        self.db = eng.upload(fb, tags=tags)
        self.in_bytes = family_input_bytes(fb)
        self.small = fb.small_fams.astype(np.int64)
        self.n_large = int(fb.large_fams.shape[0])
        self.n_disp = sum(1 for b in fb.small_buckets if b.shape[0])  # one k_small dispatch per LDS bucket
        # one k_large dispatch per bucket, + the part dispatch and the k_join one of split families
        self.n_disp_large = sum(1 for b in fb.large_buckets if b.shape[0]) + (2 if fb.split_fams.shape[0] else 0)
        self.molecules = int(np.unique(fb.fam_mi).shape[0])
        self.n_fam, self.n_rec, self.n_bases = fb.n_fam, fb.n_rec, fb.n_bases
        self.db.release_host()


def build(args, rank: int, dev, eng):
    """-> (resident batches, the first batch's raw records + reference for the CPU baseline)."""
    if args.config != "C5":
        s = synth.generate(args.config, args.families, seed=args.seed + rank, device=dev)
        eng.load_reference(s.ref)
        return [Resident(eng, B.build_family_batch(s.raw, "full", s.ref), tags=True)], s
    # C5: the rank's share as a stream of batches, each its own seeded chunk of families (the
    # chunk index is part of the seed) on the rank's one genome
    out, first = [], None
    left, i = args.families, 0
    while left > 0:
        n = min(args.batch_families, left)
        s = synth.generate("C2", n, seed=args.seed + 1000 * rank + i, device=dev, reuse=first)
        if first is None:
            eng.load_reference(s.ref)
            first = s
        out.append(Resident(eng, B.build_family_batch(s.raw, "full", s.ref)))
        left -= n
        i += 1
    return out, first


def run(args):
    rank, world, local = shard.env_rank()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = shard.init("nccl", dev)
    from bsseqconsensusreads_amd.device import Engine

    t0 = time.time()
    eng = Engine(local)
    res, s0 = build(args, rank, dev, eng)
    torch.cuda.synchronize()
    setup_s = time.time() - t0

    stream = torch.cuda.current_stream(dev)

    def step(mode=FULL_MODE):
        for r in res:
            eng.run(r.db, mode, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- timed region: K full steps ----
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - w0
    elapsed = max(wall, ev0.elapsed_time(ev1) / 1e3)

    outs = [r.db.fetch_lengths() for r in res]
    emitted = sum(int((st & 1).sum()) for st, _ in outs)
    # the unit is the input family (one MI base = one molecule); TemplateCoordinate order can
    # split a molecule into several consensus families (config.consensus_families_per_gpu)
    molecules = sum(r.molecules for r in res)
    elapsed, (fams_total, emitted_total) = shard.reduce_step(dist, elapsed, [molecules, emitted], dev)

    # ---- roofline of the dominant kernel (small-family kernel), HIP events on its stream ----
    ks = max(5, args.steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(ks):
        step(FULL_MODE | MODE_SKIP_LARGE)
    e1.record(stream)
    torch.cuda.synchronize()
    t_small = e0.elapsed_time(e1) / 1e3 / ks
    t_large = 0.0
    if any(r.n_large for r in res):
        e0.record(stream)
        for _ in range(ks):
            step(FULL_MODE | MODE_SKIP_SMALL)
        e1.record(stream)
        torch.cuda.synchronize()
        t_large = e0.elapsed_time(e1) / 1e3 / ks
    # the drop-in's default BAM output carries fgbio's per-base consensus tags (cli.py, main.snake.py:159):
    # the same resident batches with BSDC_MODE_TAGS, timed after the headline (C5 keeps no tag buffers)
    tags_ms = None
    if args.tags_leg and all(r.db.tags for r in res):
        e0.record(stream)
        for _ in range(ks):
            step(FULL_MODE | MODE_TAGS)
        e1.record(stream)
        torch.cuda.synchronize()
        tags_ms = e0.elapsed_time(e1) / ks
    n_disp = sum(r.n_disp for r in res)
    # the tag leg's extra algorithmic bytes: the single-strand lengths (4 x u16 a family) and, for
    # the emitted families, each set's read -- base, qual, depth, errors: 4 B a column
    tag_extra = 0
    if tags_ms is not None:
        for r in res:
            F = r.db.n_fam
            ssl = r.db.ss_len[:4 * F].cpu().numpy().view(np.uint16).astype(np.int64).reshape(F, 4)
            st = r.db.status[:F].cpu().numpy()
            tag_extra += 8 * F + 4 * int(ssl[(st & 1) != 0].sum())
    bytes_small, bytes_all = 0, 0
    for r, (st, ln) in zip(res, outs):
        per = r.in_bytes + family_output_bytes(ln, st)
        bytes_small += int(per[r.small].sum())
        bytes_all += int(per.sum())
    # the dominant kernel: the one that takes longer per step (k_small on C0-C2, k_large on C3)
    bytes_large = bytes_all - bytes_small
    dom_large = t_large > t_small
    kname = "k_large" if dom_large else "k_small"
    t_dom, b_dom = (t_large, bytes_large) if dom_large else (t_small, bytes_small)
    n_disp_dom = sum(r.n_disp_large for r in res) if dom_large else n_disp
    achieved = b_dom / t_dom / 1e9
    # HBM bytes of one launch set of that kernel (one dispatch per non-empty bucket), from the PMC
    # passes of profiles/collect_pmc.sh on this same workload (FETCH_SIZE x2 + WRITE_SIZE,
    # MI355X_MICROARCH.md HBM section); null when no summary for this config is committed
    traffic = None
    issue = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc) and args.families == DEFAULT_FAMILIES.get(args.config, 1_000_000) and args.seed == 42:
        with open(pmc) as fh:
            kd = json.load(fh).get(kname, {})
        per = kd.get("hbm_bytes_per_dispatch")
        if per is not None:
            traffic = int(per * n_disp_dom)
        # the bound that actually binds: VALU issue.  A wave64 VALU instruction takes 2 cycles of
        # its SIMD (MI355X_MICROARCH.md), 1024 SIMDs at 2.4 GHz; instructions per launch from the
        # same PMC passes (SQ_INSTS_VALU is per wave-instruction)
        valu = kd.get("mean_per_dispatch", {}).get("SQ_INSTS_VALU")
        if valu is not None:
            v_launch = valu * n_disp_dom
            n_k = sum(r.n_large if dom_large else int(r.small.size) for r in res)
            issue = {"valu_insts_per_family": round(v_launch / max(n_k, 1), 1),
                     "valu_issue_floor_ms": round(v_launch * 2 / (1024 * 2.4e9) * 1e3, 4),
                     "valu_issue_frac": round(v_launch * 2 / (1024 * 2.4e9) / t_dom, 4),
                     "pmc_source": os.path.relpath(pmc, ROOT)}

    # the tag leg's HBM bytes per step, from the TAGS=1 PMC passes (profiles/pmc_<config>_tags.json:
    # its k_small<true> and k_large / k_join tag instances), when committed for this workload
    tags_traffic = None
    pmt = os.path.join(ROOT, "profiles", "pmc_%s_tags.json" % args.config)
    if tags_ms is not None and os.path.exists(pmt) and args.families == DEFAULT_FAMILIES.get(args.config, 1_000_000) \
            and args.seed == 42:
        with open(pmt) as fh:
            kt = json.load(fh)
        parts = [(kt.get("k_small_tags", {}).get("hbm_bytes_per_dispatch"), n_disp),
                 (kt.get("k_large_tags", {}).get("hbm_bytes_per_dispatch"), sum(r.n_disp_large for r in res))]
        if all(b is not None or nd == 0 for b, nd in parts):
            tags_traffic = int(sum(b * nd for b, nd in parts if nd))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        # the host's CPU share: OMP_NUM_THREADS / nproc (16 on the GPU box, whose os.cpu_count()
        # shows the whole machine); no further cap
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        n_s = min(args.cpu_sample, int(s0.n_fam))
        v, secs = cpu_baseline(s0.raw, s0.ref, n_s, threads)
        n_1 = min(args.cpu_sample_1core, n_s)
        v1, secs1 = cpu_baseline(s0.raw, s0.ref, n_1, 1) if n_1 > 0 else (None, 0.0)
        cpu = {"value": round(v, 1), "unit": "families/s", "cores": threads, "kind": "port",
               "cores_all": threads, "value_all": round(v, 1),
               "value_1core": round(v1, 1) if v1 is not None else None,
               "sample": "first %d families of the same %s workload through oracle/ (C restatement of tools 1+2 "
                         "and the duplex vote, OpenMP over families) on %d threads, %.1f s; 1 core: first %d "
                         "families, %.1f s" % (n_s, args.config, threads, secs, n_1, secs1)}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(fams_total * args.steps / elapsed, 1),  # every step processes every family
            "unit": "families/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPE,
            "data": "synthetic (seeded EM-seq duplex model generated on the GPU, SURVEY.md 8d)",
            "config": {"workload": args.config + " -- " + WORKLOADS[args.config],
                       "families_per_gpu": molecules, "consensus_families_per_gpu": sum(r.n_fam for r in res),
                       "batches_per_gpu": len(res),
                       "family_order": "fgbio TemplateCoordinate runs of one MI",
                       "records_per_gpu": sum(r.n_rec for r in res), "bases_per_gpu": sum(r.n_bases for r in res),
                       "small_families": sum(int(r.small.size) for r in res),
                       "large_families": sum(r.n_large for r in res), "parallelism": "family-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(t_dom * 1e3, 4),
                         "dispatches_per_launch": n_disp_dom,
                         "avg_dispatch_ms": round(t_dom * 1e3 / max(n_disp_dom, 1), 4),
                         "algorithmic_bytes_per_launch": b_dom,
                         "small_kernel_ms": round(t_small * 1e3, 4),
                         "small_frac": round(bytes_small / t_small / 1e9 / HBM_PEAK_GBS, 4) if t_small > 0 else None,
                         "large_kernel_ms": round(t_large * 1e3, 4),
                         "large_frac": round(bytes_large / t_large / 1e9 / HBM_PEAK_GBS, 4) if t_large > 0 else None,
                         "step_algorithmic_GBps": round(bytes_all / (elapsed / args.steps) / 1e9, 1),
                         "issue": issue},
            "cpu_baseline": cpu,
            "tags_ms_per_step": round(tags_ms, 4) if tags_ms is not None else None,
            "tags_roofline": {"bound": "hbm", "achieved": round((bytes_all + tag_extra) / (tags_ms / 1e3) / 1e9, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round((bytes_all + tag_extra) / (tags_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                              "algorithmic_bytes_per_step": int(bytes_all + tag_extra),
                              "tag_bytes_per_step": int(tag_extra),
                              "traffic": tags_traffic,
                              "vs_headline_ms": round(tags_ms / (elapsed / args.steps * 1e3), 4)}
            if tags_ms is not None else None,
            "tags_families_per_s": round(molecules / (tags_ms / 1e3), 1) if tags_ms else None,
            "families_emitted": int(emitted_total),
            "setup_s": round(setup_s, 1),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--families", type=int, default=None,
                    help="families per GPU (default 1M; C3 200K, whose deep families fill 32-bit image offsets; "
                         "C5 12.5M = 100M / 8)")
    ap.add_argument("--batch-families", type=int, default=1_500_000, help="C5: families per resident batch")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000,
                    help="families for the all-cores CPU baseline (0 = skip)")
    ap.add_argument("--cpu-sample-1core", type=int, default=100_000, help="families for the 1-core CPU baseline")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-tags-leg", dest="tags_leg", action="store_false",
                    help="skip the timed BSDC_MODE_TAGS leg (the PMC passes count the headline kernels only)")
    a = ap.parse_args(argv)
    if a.families is None:
        a.families = DEFAULT_FAMILIES.get(a.config, 1_000_000)
    return a


def main(argv=None) -> int:
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: one spawned process per GPU (this process never touches the GPU)
        return shard.launch(args.gpus, run, (args,))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        return 2
    run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
