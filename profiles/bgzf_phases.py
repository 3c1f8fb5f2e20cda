"""Per-phase time of the GPU BGZF kernel (csrc/bsdc_bgzf.hip built with -DBSDC_BGZF_PHASES into
profiles/_build/libbsdc_phases.so by profiles/bgzf_phases.sh): thread 0's wall clock at the end of
load, A (candidates), A2 (chains), B (parse), C (codes), D (bit counts), E (bits) for every block of one launch
of MAX_BLOCKS blocks over step-5 output bytes; mean microseconds per phase and block.
Usage (GPU box, after the build): BSDC_LIB_PATH=profiles/_build/libbsdc_phases.so python profiles/bgzf_phases.py"""
import ctypes
import json
import os
import struct
import sys
import tempfile
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    from bsseqconsensusreads_amd import bam, synth
    from oracle import oracle
    from test_bam import _cons_of, _header
    s = synth.generate("C2", 4000, seed=5, device="cpu", genome_len=1_000_000)
    res = oracle.run(s.raw, s.ref)
    recs = bam.duplex_records(_cons_of(res), s.raw, "x")
    p = os.path.join(tempfile.mkdtemp(prefix="bsdc_bgzfp_"), "u.bam")
    bam.write_bam(p, bam.output_header(_header(s.ref)), recs, level=0)
    raw, data, o = open(p, "rb").read(), [], 0
    while o < len(raw):
        bs = struct.unpack_from("<H", raw, o + 16)[0] + 1
        data.append(zlib.decompress(raw[o + 18:o + bs - 8], -15))
        o += bs
    one = b"".join(data)
    g = bam.GpuBgzf(0)
    nblk = g.MAX_BLOCKS
    n = nblk * 65280
    buf = np.frombuffer((one * (n // len(one) + 1))[:n], np.uint8).copy()
    din = torch.from_numpy(buf).to("cuda")
    sz = torch.empty(nblk, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    lib = g.lib
    lib.bsdc_bgzf_phases.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    out = {}
    for rep in range(2):
        if lib.bsdc_bgzf_deflate(din.data_ptr(), n, 0, nblk, g.scratch.data_ptr(), sz.data_ptr(), st.cuda_stream):
            raise RuntimeError("deflate")
        torch.cuda.synchronize()
    ph = np.zeros(8192 * 8, np.uint64)
    lib.bsdc_bgzf_phases(ph.ctypes.data, ph.size)
    ph = ph.reshape(8192, 8)[:nblk, :8].astype(np.int64)
    d = np.diff(ph, axis=1) / 100.0  # 100 MHz -> microseconds
    names = ["load", "A_candidates", "A2_chains", "B_parse", "C_codes", "D_bitcount", "E_bits"]
    out = {"blocks": nblk, "us_per_block_mean": {k: round(float(d[:, i].mean()), 1) for i, k in enumerate(names)},
           "us_per_block_total": round(float((ph[:, 7] - ph[:, 0]).mean()) / 100.0, 1),
           "launch_span_ms": round(float(ph[:, 7].max() - ph[:, 0].min()) / 1e5, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
