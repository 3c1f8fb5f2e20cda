"""Debug: the failing molecular C1 column (GPU vs oracle/)."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from bsseqconsensusreads_amd import pipeline, synth
from bsseqconsensusreads_amd import records as R
from bsseqconsensusreads_amd.device import Engine
from oracle import oracle

s = synth.generate("C1", 300, seed=21, device="cpu", genome_len=200_000)
raw = R.take(s.raw, np.lexsort((s.raw.mi_strand, s.raw.mi_id)))
eng = Engine(0)
for tags in (False, True):
    cons, rm = pipeline.run_molecular(eng, raw, tags=tags)
    ref = oracle.run(rm, s.ref, run_tools=False, family_order="mi-group", min_consensus_base_quality=0, keep_sources=True)
    L = ref.cons_len
    bad = []
    for f in range(len(ref.status)):
        for e in range(2):
            n = int(L[f, e])
            d = np.nonzero(cons.seq[f, e, :n] != ref.cons_seq[f, e, :n])[0]
            for c in d:
                bad.append((f, e, int(c)))
    print("tags", tags, "bad columns", len(bad), bad[:10])
    if bad:
        f, e, c = bad[0]
        print("gpu", cons.seq[f, e, c], cons.qual[f, e, c], "oracle", ref.cons_seq[f, e, c], ref.cons_qual[f, e, c])
        src = ref.sources
        cnt = src["count"]
        # reads of family f, set e (X = set 0 for end 0)
        start = int(cnt[:f].sum())
        o = start + int(cnt[f, :e].sum())
        lens = src["len"]
        boff = int(lens[:o].sum())
        for i in range(int(cnt[f, e])):
            li = int(lens[o + i])
            if c < li:
                print(" read", i, "len", li, "base", src["base"][boff + c], "qual", src["qual"][boff + c])
            boff += li
        if tags:
            print(" gpu ss", cons.ss["base"][f, e, c], cons.ss["qual"][f, e, c], cons.ss["depth"][f, e, c],
                  "oracle ss", ref.ss["base"][f, e, c], ref.ss["qual"][f, e, c], ref.ss["depth"][f, e, c])
