"""C3 k_large arena model: the LDS arena of every large
C3 family under the verdict's layout changes, restated from ArenaLayout (include/bsdc_layout.h) in
numpy, per LDS class (5, 4, 3, 2, 1 workgroups per CU, HBM).  "today" must reproduce the batch's
actual bucket counts.  CPU only: python profiles/c3_arena_model.py > profiles/r06/c3_arena_model.log"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bsseqconsensusreads_amd import batch as B  # noqa: E402
from bsseqconsensusreads_amd import synth  # noqa: E402

s = synth.generate("C3", 20000, seed=42, device="cpu", genome_len=10_000_000)
fb = B.build_family_batch(s.raw, "full", s.ref)
large = fb.large_fams.astype(np.int64) if fb.large_fams.size else np.zeros((0, 4), np.int64)
print("families", fb.n_fam, "large", large.shape[0], "max_len", fb.max_len)
n = large[:, 2]
slot = large[:, 3]  # image entries: a byte of qual + a base each
ssw = (fb.max_len + 2 + 15) // 16 * 16


def arena(n, slot, meta_b, vote_b, nib):
    """ArenaLayout.total with meta_b bytes of record metadata, vote_b bytes per vote column (the
    second wave part's sums, ORs, counts), bases as bytes or nibbles (no complex cigars in C3)."""
    img_bytes = slot * 3 // 2 if nib else 2 * slot
    meta = np.maximum((n * meta_b + 15) // 16 * 16 + (2 * n + 15) // 16 * 16, vote_b * ssw)
    return meta + (n * 8 + 15) // 16 * 16 + 8 * ssw + (img_bytes + 15) // 16 * 16


caps = B.LARGE_BUCKETS
print("caps", caps)
print("actual buckets", [int(b.shape[0]) for b in fb.large_buckets], "arenas", fb.large_arenas)
for name, mb, vb, nib in (("today", 48, 44, False), ("meta24", 24, 44, False), ("meta24+vote28", 24, 28, False),
                          ("nibble", 48, 44, True), ("nibble+meta24+vote28", 24, 28, True)):
    a = arena(n, slot, mb, vb, nib)
    q = np.percentile(a, [50, 90])
    cls = np.searchsorted(np.array(caps), a)
    print("%-22s p50 %6.0f p90 %6.0f   per class (5,4,3,2,1,HBM): %s" % (name, q[0], q[1],
                                                                         np.bincount(cls, minlength=6).tolist()))
