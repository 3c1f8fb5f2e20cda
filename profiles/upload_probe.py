"""Where a batch's upload time goes (device.DeviceBatch), step 5 against step 1's molecular runs
on the same synthetic molecules: host arrays, their copies, the output allocations."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/profiles/", 1)[0])
from bsseqconsensusreads_amd import batch as B, pipeline, synth  # noqa: E402
from bsseqconsensusreads_amd import records as R  # noqa: E402
from bsseqconsensusreads_amd.device import Engine  # noqa: E402

eng = Engine(0)
s = synth.generate("C2", 30000, seed=3, device="cpu", genome_len=2_000_000)
eng.load_reference(s.ref)
g = R.take(s.raw, np.lexsort((s.raw.mi_strand, s.raw.mi_id)))
rm = pipeline.molecular_records(g)
for name, plan in (("step5", pipeline.plan_families(s.raw, "full", s.ref)),
                   ("molecular", pipeline.plan_families(rm, "vote", family_order="mi-group"))):
    (a, b), = pipeline.plan_ranges(plan, None)
    fb = pipeline.materialize(plan, a, b, images=eng.stage_images)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = fb.device_arrays()
        t1 = time.perf_counter()
        sizes = {k: (np.asarray(v).nbytes, bool(torch.from_numpy(np.ascontiguousarray(v).view(np.uint8)).is_pinned()))
                 for k, v in d.items()}
        t2 = time.perf_counter()
        db = eng.upload(fb, tags=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(name, "F", fb.n_fam, "R", fb.n_rec, "device_arrays %.1f ms, upload %.1f ms" % ((t1 - t0) * 1e3, (t3 - t2) * 1e3),
              flush=True)
    big = sorted(sizes.items(), key=lambda x: -x[1][0])[:8]
    print("  largest arrays (bytes, pinned):", big, flush=True)
