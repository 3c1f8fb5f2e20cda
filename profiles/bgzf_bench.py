"""GPU BGZF encoder throughput (bam.GpuBgzf, csrc/bsdc_bgzf.hip) on step-5 output bytes: the
uncompressed BAM of an oracle run, tiled to --mb MB, compressed block by block; times of the
host->device copy, the kernels and the copy back (HIP events on the encoder's stream), the ratio,
and the host's libdeflate level 5 on the same bytes for comparison.
Usage (GPU box): python profiles/bgzf_bench.py [--mb 430] [--families 4000]"""
import argparse
import json
import os
import struct
import sys
import tempfile
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=430)
    ap.add_argument("--families", type=int, default=4000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from bsseqconsensusreads_amd import bam, synth
    from oracle import oracle
    from test_bam import _cons_of, _header
    s = synth.generate("C2", a.families, seed=5, device="cpu", genome_len=1_000_000)
    res = oracle.run(s.raw, s.ref)
    recs = bam.duplex_records(_cons_of(res), s.raw, "x")
    p = os.path.join(tempfile.mkdtemp(prefix="bsdc_bgzfb_"), "u.bam")
    bam.write_bam(p, bam.output_header(_header(s.ref)), recs, level=0)
    raw, data, o = open(p, "rb").read(), [], 0
    while o < len(raw):
        bs = struct.unpack_from("<H", raw, o + 16)[0] + 1
        data.append(zlib.decompress(raw[o + 18:o + bs - 8], -15))
        o += bs
    one = b"".join(data)
    reps = (a.mb << 20) // len(one) + 1
    buf = np.frombuffer((one * reps)[:(a.mb << 20) // 65280 * 65280], np.uint8).copy()
    n = buf.shape[0]
    g = bam.GpuBgzf(0)
    g.compress(buf.ctypes.data, n)  # warm-up (allocations, code)
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        packed, sizes = g.compress(buf.ctypes.data, n)
        ts.append(time.perf_counter() - t0)
    # the kernels alone on device-resident bytes
    din = torch.from_numpy(buf).to("cuda")
    nblk = n // 65280
    sz = torch.empty(nblk, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for b0 in range(0, nblk, g.MAX_BLOCKS):
        nb = min(g.MAX_BLOCKS, nblk - b0)
        g.lib.bsdc_bgzf_deflate(din.data_ptr(), n, b0, nb, g.scratch.data_ptr(), sz.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1)
    out_bytes = int(sizes.astype(np.int64).sum())
    import ctypes
    L = ctypes.CDLL("libdeflate.so.0")
    L.libdeflate_alloc_compressor.restype = ctypes.c_void_p
    L.libdeflate_alloc_compressor.argtypes = [ctypes.c_int]
    L.libdeflate_deflate_compress.restype = ctypes.c_size_t
    L.libdeflate_deflate_compress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_size_t]
    c = L.libdeflate_alloc_compressor(5)
    dst = np.zeros(70000, np.uint8)
    nb5 = min(nblk, 400)
    t0 = time.perf_counter()
    cs = sum(L.libdeflate_deflate_compress(c, buf.ctypes.data + b * 65280, 65280, dst.ctypes.data, 70000) for b in range(nb5))
    l5 = time.perf_counter() - t0
    print(json.dumps({"MB": round(n / 1e6, 1), "blocks": nblk, "compress_s": [round(x, 4) for x in ts],
                      "end_to_end_GBps": round(n / min(ts) / 1e9, 2), "kernel_ms": round(k_ms, 2),
                      "kernel_GBps": round(n / (k_ms / 1e3) / 1e9, 2), "ratio_gpu": round(n / out_bytes, 3),
                      "libdeflate5_MBps_1thread": round(nb5 * 65280 / l5 / 1e6, 1),
                      "ratio_libdeflate5": round(nb5 * 65280 / cs, 3)}))


if __name__ == "__main__":
    main()
