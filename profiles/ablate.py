"""Profiling aid: time one family kernel stopped after each phase (BSDC_MODE_STOP_SHIFT).
Usage on the GPU box: python profiles/ablate.py [--config C2] [--families N] [--kernel small|large]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bsseqconsensusreads_amd import batch as B, synth  # noqa: E402
from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_VOTE, MODE_SKIP_LARGE, MODE_SKIP_SMALL  # noqa: E402
from bsseqconsensusreads_amd.device import Engine  # noqa: E402

# (name, stop code): the kernel returns after the named phase
PHASES = [("launch", 15), ("tables", 14), ("staging", 1), ("convert", 2), ("extend", 3), ("overlap", 4), ("srcreads+lists", 5),
          ("vote-preamble", 6), ("vote-main", 7), ("vote-queue", 8), ("full", 0)]
LARGE_PHASES = [("launch", 15), ("tables", 14), ("staging", 1), ("convert", 2), ("extend", 3), ("overlap-wild", 11),
                ("overlap-templates", 12), ("overlap", 4), ("srcreads", 10), ("filter+lists", 5), ("vote-sums", 6), ("vote", 7),
                ("full", 0)]

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--families", type=int, default=None)
ap.add_argument("--kernel", default="small", choices=("small", "large"))
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
if a.families is None:
    a.families = 200_000 if a.config == "C3" else 1_000_000
skip = MODE_SKIP_LARGE if a.kernel == "small" else MODE_SKIP_SMALL
dev = torch.device("cuda", 0)
s = synth.generate(a.config, a.families, seed=42, device=dev)
fb = B.build_family_batch(s.raw, "full", s.ref)
eng = Engine(0)
eng.load_reference(s.ref)
db = eng.upload(fb)
st = torch.cuda.current_stream()
out = {}
for name, code in (PHASES if a.kernel == "small" else LARGE_PHASES):
    mode = MODE_CONVERT | MODE_EXTEND | MODE_VOTE | skip | (code << 8)
    for _ in range(2):
        eng.run(db, mode, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        eng.run(db, mode, st)
    e1.record(st)
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) / a.reps, 4)
print(json.dumps({"config": a.config, "kernel": a.kernel, "small_families": int(fb.small_fams.shape[0]),
                  "large_families": int(fb.large_fams.shape[0]), "ms_after_phase": out}))
