"""Step-5 duplex path throughput on MI355X (BASELINE.json metric: duplex families/sec).

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): 1M synthetic WGBS/EM-seq duplex families per
GPU, 2x150 bp, Poisson(4) templates per family split between the strands, generated on the GPU
from a seeded model (no network, no real data).  A "step" is one pass of the fused hot path --
B-strand conversion, gap extension, overlapping-bases consensus, source reads, alignment filter,
single-strand vote, duplex combine -- over the whole resident batch (bsdc_run, both family
kernels).  Inputs are in HBM before the timed region; outputs stay in HBM.

Multi-GPU: one process per GPU (torch.distributed.run), every rank owns its own 1M families
(weak scaling, no data-path collective); barrier + synchronize around the timed steps, max time
over ranks, value = families on all ranks / that time.  One all_reduce of a counter pair rides
along (the optional RCCL counter reduction of SURVEY.md 8e).
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
from bsseqconsensusreads_amd import synth  # noqa: E402
from bsseqconsensusreads_amd._lib import (MODE_CONVERT, MODE_EXTEND, MODE_SKIP_LARGE, MODE_SKIP_SMALL,  # noqa: E402
                                          MODE_VOTE)
from bsseqconsensusreads_amd.device import Engine  # noqa: E402

METRIC = "duplex families/sec (node) at 1/2/4/8 MI355X; % HBM roofline; speedup vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    "C2": "configs[1]: 1M-family synthetic WGBS grouped BAM, 2x150bp, Poisson(4) family size, one MI355X",
    "C0": "1 template per strand (the pipeline as written), 2x150bp",
    "C1": "configs[0] shape: 3 reads/strand EM-seq families, 2x150bp",
    "C3": "configs[2]: high-depth panel, 20-100 templates/family, short overlapping inserts",
    "C4": "configs[3]: skewed 1-500 family sizes, 30% AB-only",
}
FULL_MODE = MODE_CONVERT | MODE_EXTEND | MODE_VOTE


def algorithmic_bytes(fb: B.FamilyBatch, cons_len: np.ndarray, status: np.ndarray, fams: np.ndarray) -> int:
    """B_fam = sum_records(ceil(L/2) + L + 16) + sum_converted ceil((L+2)/2)
    + sum_{2 ends}(ceil(Lc/2) + Lc), summed over `fams`."""
    L = (fb.rec_lenflag & 0xFFFF).astype(np.int64)
    conv = (fb.rec_link & B.LINK_CONVERT) != 0
    per_rec = (L + 1) // 2 + L + 16 + np.where(conv, (L + 3) // 2, 0)
    sizes = np.diff(fb.fam_off.astype(np.int64))
    fam_of = np.repeat(np.arange(fb.n_fam), sizes)
    per_fam = np.bincount(fam_of, weights=per_rec, minlength=fb.n_fam)
    lc = np.where((status & 1)[:, None] != 0, cons_len, 0).astype(np.int64)
    per_fam = per_fam + ((lc + 1) // 2 + lc).sum(1)
    return int(per_fam[fams].sum())


def cpu_baseline(raw, ref, n_fam_sample: int, threads: int):
    """oracle/ (C restatement, OpenMP over families) on the first n_fam_sample families."""
    from oracle import oracle
    sub = synth.subset_families(raw, n_fam_sample)
    res = oracle.run(sub, ref, threads=threads)
    return n_fam_sample / res.seconds, res.seconds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--families", type=int, default=None,
                    help="families per GPU (default 1M; C3 200K, whose deep families fill 32-bit image offsets)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="families for the CPU baseline (0 = skip)")
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    t0 = time.time()
    if args.families is None:
        args.families = 200_000 if args.config == "C3" else 1_000_000
    s = synth.generate(args.config, args.families, seed=args.seed + rank, device=dev)
    fb = B.build_family_batch(s.raw, "full", s.ref)
    eng = Engine(local)
    eng.load_reference(s.ref)
    db = eng.upload(fb)
    torch.cuda.synchronize()
    setup_s = time.time() - t0

    stream = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        eng.run(db, FULL_MODE, stream)
    torch.cuda.synchronize()

    # ---- timed region: K full steps ----
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        eng.run(db, FULL_MODE, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - w0
    elapsed = max(wall, ev0.elapsed_time(ev1) / 1e3)

    out = db.fetch()
    emitted = int((out["status"] & 1).sum())
    tot = torch.tensor([elapsed, 0.0], dtype=torch.float64, device=dev)
    # the unit is the input family (one MI base = one molecule); TemplateCoordinate order can
    # split a molecule into several consensus families (config.consensus_families_per_gpu)
    molecules = int(np.unique(fb.fam_mi).shape[0])
    cnt = torch.tensor([molecules, emitted], dtype=torch.int64, device=dev)
    if dist is not None:
        dist.all_reduce(tot, op=dist.ReduceOp.MAX)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    elapsed = float(tot[0])
    fams_total = int(cnt[0])

    # ---- roofline of the dominant kernel (small-family kernel), HIP events on its stream ----
    small = fb.small_fams.astype(np.int64)
    large = fb.large_fams[:, 0].astype(np.int64)
    ks = max(5, args.steps)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(ks):
        eng.run(db, FULL_MODE | MODE_SKIP_LARGE, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    t_small = e0.elapsed_time(e1) / 1e3 / ks
    t_large = 0.0
    if large.size:
        e0.record(stream)
        for _ in range(ks):
            eng.run(db, FULL_MODE | MODE_SKIP_SMALL, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        t_large = e0.elapsed_time(e1) / 1e3 / ks
    n_disp = sum(1 for b in fb.small_buckets if b.shape[0])  # one k_small dispatch per non-empty LDS bucket
    bytes_small = algorithmic_bytes(fb, out["len"], out["status"], small)
    bytes_all = algorithmic_bytes(fb, out["len"], out["status"], np.arange(fb.n_fam))
    achieved = bytes_small / t_small / 1e9
    # HBM bytes of one k_small launch set (one dispatch per non-empty LDS bucket), from the PMC
    # passes of profiles/collect_pmc.sh on this same workload (FETCH_SIZE x2 + WRITE_SIZE,
    # MI355X_MICROARCH.md HBM section); null when no summary for this config is committed
    traffic = None
    issue = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc) and args.families == 1_000_000 and args.seed == 42:
        with open(pmc) as fh:
            ks = json.load(fh).get("k_small", {})
        per = ks.get("hbm_bytes_per_dispatch")
        if per is not None:
            traffic = int(per * n_disp)
        # the bound that actually binds: VALU issue.  A wave64 VALU instruction takes 2 cycles of
        # its SIMD (MI355X_MICROARCH.md), 1024 SIMDs at 2.4 GHz; instructions per launch from the
        # same PMC passes (SQ_INSTS_VALU is per wave-instruction)
        valu = ks.get("mean_per_dispatch", {}).get("SQ_INSTS_VALU")
        if valu is not None:
            v_launch = valu * n_disp
            issue = {"valu_insts_per_family": round(v_launch / max(int(small.size), 1), 1),
                     "valu_issue_floor_ms": round(v_launch * 2 / (1024 * 2.4e9) * 1e3, 4),
                     "valu_issue_frac": round(v_launch * 2 / (1024 * 2.4e9) / t_small, 4)}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        threads = min(threads, 16)
        n_s = min(args.cpu_sample, args.families)
        v, secs = cpu_baseline(s.raw, s.ref, n_s, threads)
        cpu = {"value": round(v, 1), "unit": "families/s", "cores": threads, "kind": "port",
               "sample": "first %d families of the same %s workload through oracle/ (C restatement of tools 1+2 and "
                         "the duplex vote, OpenMP over families), %.1f s" % (n_s, args.config, secs)}

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
            "dtype": "u8",
            "data": "synthetic (seeded EM-seq duplex model generated on the GPU, SURVEY.md 8d)",
            "config": {"workload": args.config + " -- " + WORKLOADS[args.config],
                       "families_per_gpu": molecules, "consensus_families_per_gpu": int(fb.n_fam),
                       "family_order": "fgbio TemplateCoordinate runs of one MI", "records_per_gpu": int(fb.n_rec),
                       "bases_per_gpu": int(fb.n_bases), "small_families": int(small.size),
                       "large_families": int(large.size), "parallelism": "family-sharded x%d" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_small", "kernel_ms": round(t_small * 1e3, 4),
                         "dispatches_per_launch": n_disp,
                         "avg_dispatch_ms": round(t_small * 1e3 / max(n_disp, 1), 4),
                         "algorithmic_bytes_per_launch": bytes_small,
                         "large_kernel_ms": round(t_large * 1e3, 4),
                         "step_algorithmic_GBps": round(bytes_all / (elapsed / args.steps) / 1e9, 1),
                         "issue": issue},
            "cpu_baseline": cpu,
            "families_emitted": int(cnt[1]),
            "setup_s": round(setup_s, 1),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
