"""PC-sampling target: one C2 batch (200K families) through the fused step, 30 times."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bsseqconsensusreads_amd import batch as B, synth  # noqa: E402
from bsseqconsensusreads_amd._lib import MODE_CONVERT, MODE_EXTEND, MODE_VOTE  # noqa: E402
from bsseqconsensusreads_amd.device import Engine  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
s = synth.generate(cfg, n, seed=42, device="cuda")
fb = B.build_family_batch(s.raw, "full", s.ref)
eng = Engine(0)
eng.load_reference(s.ref)
db = eng.upload(fb)
for _ in range(30):
    eng.run(db, MODE_CONVERT | MODE_EXTEND | MODE_VOTE)
torch.cuda.synchronize()
print("done", fb.n_fam)
