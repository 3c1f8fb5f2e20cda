"""k_small staging ceiling on C2's real family images.

Builds profiles/probe_stage.hip (profiles/_build/libprobe.so, built here beforehand with
`python profiles/probe_stage.py --build`), then on the GPU box: generates C2 (1M families, seed 42),
uploads the batch, runs the real k_small once (for the consensus lengths the output writes use),
and times, per launch set (one dispatch per small bucket, spread over 4 streams as bsdc_run does):
  k_small full, k_small stopped after staging (BSDC_MODE_STOP 1), and the probe forms
  0 launch only / 1 today's staging / 2 all LDS-DMA, packed / 3 two families per wave, the second's
  DMA in flight while the first is written out.
For each: ms, the bytes it moves (list entries, metadata, image, windows, outputs), GB/s and the
fraction of 8 TB/s, and the algorithmic bytes rate for comparison.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "profiles", "probe_stage.hip")
LIB = os.path.join(ROOT, "profiles", "_build", "libprobe.so")


class ProbeArgs(C.Structure):
    _fields_ = [("fams", C.c_void_p), ("nfams", C.c_int64), ("arena", C.c_int32), ("ref_chunks", C.c_int32),
                ("rec", C.c_void_p), ("rec_win", C.c_void_p), ("cig_info", C.c_void_p), ("seq", C.c_void_p),
                ("qual", C.c_void_p), ("ref", C.c_void_p), ("olen", C.c_void_p), ("stride", C.c_int32),
                ("out_seq", C.c_void_p), ("out_qual", C.c_void_p), ("status", C.c_void_p), ("sink", C.c_void_p)]


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-o", LIB, SRC],
                   check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--families", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    sys.path.insert(0, ROOT)
    from bsseqconsensusreads_amd import batch as B, synth
    from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_SKIP_LARGE, MODE_VOTE
    from bsseqconsensusreads_amd.device import Engine
    sys.path.insert(0, os.path.join(ROOT))
    import bench

    dev = torch.device("cuda", 0)
    s = synth.generate("C2", a.families, seed=42, device=dev)
    fb = B.build_family_batch(s.raw, "full", s.ref)
    eng = Engine(0)
    eng.load_reference(s.ref)
    db = eng.upload(fb)
    st = torch.cuda.current_stream()
    full = MODE_CONVERT | MODE_EXTEND | MODE_VOTE | MODE_SKIP_LARGE
    eng.run(db, full, st)
    torch.cuda.synchronize()
    status, lens = db.fetch_lengths()
    olen = torch.from_numpy(np.ascontiguousarray(lens.astype(np.uint16)).view(np.uint8)).to(dev)
    ref_t = torch.from_numpy(np.concatenate([np.ascontiguousarray(s.ref.packed).view(np.uint8),
                                             np.full(1024, 0xFF, np.uint8)])).to(dev)
    out_seq = torch.zeros(max(fb.n_fam * fb.stride, 16), dtype=torch.uint8, device=dev)
    out_qual = torch.zeros(max(2 * fb.n_fam * fb.stride, 16), dtype=torch.uint8, device=dev)
    out_st = torch.zeros(max(fb.n_fam, 1), dtype=torch.uint8, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    lib = C.CDLL(LIB)
    lib.probe_run.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    lib.probe_run.restype = C.c_int
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    rcn = B.ref_chunks(fb.max_len)

    # ---- bytes per family (the small families only) ----
    small = fb.small_fams.astype(np.int64)
    sizes = np.diff(fb.fam_off.astype(np.int64))
    ent = fb.fam_entry.astype(np.int64)
    img = (ent[:, 2] >> 8) * 32
    conv = (fb.rec_link & B.LINK_CONVERT) != 0
    fam_of = np.repeat(np.arange(fb.n_fam), sizes)
    nconv = np.bincount(fam_of, weights=conv, minlength=fb.n_fam).astype(np.int64)
    lc = np.where((status & 1)[:, None] != 0, lens, 0).astype(np.int64)
    out_b = ((lc + 1) // 2 + lc).sum(1)
    moved = 16 + sizes * 28 + img + img // 2 + nconv * rcn * 16 + out_b + 5
    algo = bench.family_input_bytes(fb) + out_b
    bytes_moved = int(moved[small].sum())
    bytes_algo = int(algo[small].sum())

    # ---- launch sets ----
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    buckets, off = [], 0
    fams_t = db.t["small_fams"]
    for q, bl in enumerate(fb.small_buckets):
        n = int(bl.shape[0])
        if n:
            args = ProbeArgs(fams=C.c_void_p(fams_t.data_ptr() + 16 * off), nfams=n, arena=int(fb.small_arenas[q]),
                             ref_chunks=rcn, rec=p(db.t["rec"]), rec_win=p(db.t["rec_win"]), cig_info=p(db.t["cig_info"]),
                             seq=p(db.t["seq"]), qual=p(db.t["qual"]), ref=p(ref_t), olen=p(olen), stride=fb.stride,
                             out_seq=p(out_seq), out_qual=p(out_qual), status=p(out_st), sink=p(sink))
            buckets.append(args)
        off += n

    def probe_set(form):
        ev = torch.cuda.Event()
        ev.record(st)
        for i, args in enumerate(buckets):
            ss = streams[i % 4]
            ss.wait_event(ev)
            rc = lib.probe_run(form, C.byref(args), C.c_void_p(ss.cuda_stream))
            assert rc == 0, rc
        for ss in streams:
            e = torch.cuda.Event()
            e.record(ss)
            st.wait_event(e)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    res = {}
    res["k_small_full"] = timed(lambda: eng.run(db, full, st))
    res["k_small_stop_staging"] = timed(lambda: eng.run(db, full | (1 << 8), st))
    res["k_small_launch_only"] = timed(lambda: eng.run(db, full | (15 << 8), st))
    for form, name in ((0, "probe0_launch"), (1, "probe1_today"), (2, "probe2_dma_packed"), (3, "probe3_dma_2fpw")):
        res[name] = timed(lambda f=form: probe_set(f))
    # the output bytes the probes wrote equal the real run's (lengths); spot-check the status byte
    torch.cuda.synchronize()
    assert int(out_st[torch.from_numpy(small).to(dev)].min()) == 1
    line = {"families": a.families, "small_families": int(small.size), "buckets": [int(b.shape[0]) for b in fb.small_buckets],
            "arenas": [int(x) for x in fb.small_arenas], "bytes_moved_per_set": bytes_moved,
            "bytes_algorithmic_per_set": bytes_algo, "ms": {k: round(v, 4) for k, v in res.items()},
            "GBps_moved": {k: round(bytes_moved / (v / 1e3) / 1e9, 1) for k, v in res.items()},
            "frac_moved_of_8TBps": {k: round(bytes_moved / (v / 1e3) / 1e9 / 8000.0, 4) for k, v in res.items()},
            "GBps_algorithmic": {k: round(bytes_algo / (v / 1e3) / 1e9, 1) for k, v in res.items()}}
    print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
