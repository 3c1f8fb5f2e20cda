"""The BAM writer's deflate cost on the real step-5 output shape: 20K C2 families through oracle/
(consensus + fgbio's per-base tags), the output records encoded uncompressed (level 0), then every
64 KiB block compressed with the system libdeflate at each level (one thread): MB/s and ratio.
Usage: python profiles/deflate_levels.py [--families N]"""
import argparse
import ctypes
import json
import os
import struct
import sys
import tempfile
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=20_000)
    a = ap.parse_args()
    from bsseqconsensusreads_amd import bam, synth
    from oracle import oracle
    from test_bam import _cons_of, _header
    s = synth.generate("C2", a.families, seed=42, device="cpu", genome_len=2_000_000)
    res = oracle.run(s.raw, s.ref)
    p = os.path.join(tempfile.mkdtemp(prefix="bsdc_defl_"), "out.bam")
    bam.write_bam(p, bam.output_header(_header(s.ref)), bam.duplex_records(_cons_of(res), s.raw, "x"), level=0)
    data = open(p, "rb").read()
    blocks, o = [], 0
    while o + 18 < len(data):
        xlen = struct.unpack_from("<H", data, o + 10)[0]
        bsize = struct.unpack_from("<H", data, o + 16)[0] + 1
        blocks.append(zlib.decompress(data[o + 12 + xlen:o + bsize - 8], -15))
        o += bsize
    blocks = [b for b in blocks if len(b) > 1000]
    total = sum(len(b) for b in blocks)
    L = ctypes.CDLL("libdeflate.so.0")
    L.libdeflate_alloc_compressor.restype = ctypes.c_void_p
    L.libdeflate_alloc_compressor.argtypes = [ctypes.c_int]
    L.libdeflate_deflate_compress.restype = ctypes.c_size_t
    L.libdeflate_deflate_compress.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_size_t]
    dst = ctypes.create_string_buffer(70000)
    out = {"families": a.families, "uncompressed_MB": round(total / 1e6, 2),
           "bytes_per_family": round(total / a.families, 1), "levels": {}}
    for lvl in (1, 3, 5, 6):
        c = L.libdeflate_alloc_compressor(lvl)
        t0 = time.perf_counter()
        cs = sum(L.libdeflate_deflate_compress(c, b, len(b), dst, 70000) for b in blocks)
        dt = time.perf_counter() - t0
        out["levels"][lvl] = {"MB_per_s_1thread": round(total / 1e6 / dt, 1), "ratio": round(total / cs, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
