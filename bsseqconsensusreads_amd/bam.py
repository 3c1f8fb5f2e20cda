"""The file-level step-5 drop-in: BAM in -> duplex consensus BAM out.

The reference's step 5 is four Snakemake rules over files (main.snake.py:121-164): tool 1 and
tool 2 read and write BAM through pysam, fgbio SortBam writes the TemplateCoordinate-sorted BAM,
and CallDuplexConsensusReads writes the unmapped consensus pairs.  Here one call reads the input
BAM (libbsdc_io: BGZF inflated and records parsed in parallel, include/bsdc_io.h), runs the fused
device path (pipeline.run_step5: tools 1+2, TemplateCoordinate families, vote, duplex), builds
fgbio's output records and writes them (libbsdc_io: BGZF deflated in
parallel).

Output records (fgbio DuplexConsensusCaller as restated; PARITY UNPINNED -- fgbio is not
vendored): an unmapped pair per emitted family, R1 flag 77 and R2 flag 141, name
``<prefix>:<MI base>``, tags RG:Z:A, MI:Z:<MI base>, RX:Z:<consensus UMI> (when the inputs carry
RX), then fgbio's consensus tags when the consensus was called with tags=True (the default of
the file-level calls, as fgbio's --output-per-base-tags defaults to true): per read cD cM cE,
aD aM aE, bD bM bE; per base ad ae ac aq, bd be bc bq (molecular: cD cM cE, cd ce), encoded by
libbsdc_io (bsdc_consensus_tags) from the single-strand reads the kernels write.  The consumer of
this file (SamToFastq, main.snake.py:167-177) reads name, flag, SEQ and QUAL only.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import records as R

IO_LIB_PATH = os.environ.get("BSDC_IO_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                 "libbsdc_io.so")
BSDC_IO_ABI_VERSION = 12
_P = C.c_void_p


class _Sizes(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n_rec", "n_bases", "n_cigar", "n_mc", "aux_bytes", "n_names", "name_bytes",
                                         "n_mi", "mi_bytes", "header_bytes")] + \
               [("n_ref", C.c_int32), ("ref_name_bytes", C.c_int64)]


class _Arrays(C.Structure):
    _fields_ = [(k, _P) for k in (
        "flag", "tid", "pos", "mapq", "l_seq", "seq_off", "seq", "qual", "cig_off", "n_cig", "cigar", "next_tid",
        "next_pos", "tlen", "name_id", "name_off", "name_buf", "mi_id", "mi_strand", "mi_off", "mi_buf", "mc_off",
        "mc_n", "mc_cigar", "la", "rd", "aux_off", "aux", "header", "ref_len", "ref_name_off", "ref_name_buf")]


class _Records(C.Structure):
    _fields_ = [("n_rec", C.c_int64)] + [(k, _P) for k in (
        "flag", "tid", "pos", "mapq", "next_tid", "next_pos", "tlen", "name_off", "name_buf", "cig_off", "cigar",
        "seq_off", "seq", "qual", "aux_off", "aux", "aux2_off", "aux2")]


_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(IO_LIB_PATH):
        raise RuntimeError("%s is missing: run __graft_entry__.build()" % IO_LIB_PATH)
    lib = C.CDLL(IO_LIB_PATH)  # (OMP_WAIT_POLICY: see the package __init__)
    lib.bsdc_io_abi_version.restype = C.c_int32
    lib.bsdc_io_last_error.restype = C.c_char_p
    lib.bsdc_bam_read.argtypes = [C.c_char_p, C.c_int32, C.POINTER(_P)]
    lib.bsdc_bam_read.restype = C.c_int32
    lib.bsdc_bam_sizes_of.argtypes = [_P, C.POINTER(_Sizes)]
    lib.bsdc_bam_copy.argtypes = [_P, C.POINTER(_Arrays)]
    lib.bsdc_bam_copy.restype = C.c_int32
    lib.bsdc_bam_free.argtypes = [_P]
    lib.bsdc_bam_stream_open.argtypes = [C.c_char_p, C.c_int32, C.c_int64, C.POINTER(_P)]
    lib.bsdc_bam_stream_open.restype = C.c_int32
    lib.bsdc_bam_stream_next.argtypes = [_P, C.c_int64, C.c_int64, C.POINTER(_P)]
    lib.bsdc_bam_stream_next.restype = C.c_int32
    lib.bsdc_bam_stream_next_raw.argtypes = [_P, C.c_int64, C.c_int64, C.POINTER(_P)]
    lib.bsdc_bam_stream_next_raw.restype = C.c_int32
    lib.bsdc_bam_stream_next_runs.argtypes = [_P, C.c_int64, C.POINTER(_P)]
    lib.bsdc_bam_stream_next_runs.restype = C.c_int32
    lib.bsdc_bam_parse.argtypes = [_P, C.c_int32]
    lib.bsdc_bam_parse.restype = C.c_int32
    lib.bsdc_bam_stream_close.argtypes = [_P]
    lib.bsdc_bam_stream_recycle.argtypes = [_P, _P]
    lib.bsdc_bam_stream_recycle.restype = None
    lib.bsdc_bam_stream_header.argtypes = [_P, C.POINTER(_P)]
    lib.bsdc_bam_stream_header.restype = C.c_int32
    lib.bsdc_bam_writer_open.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int32, _P, _P, _P, C.c_int32,
                                         C.POINTER(_P)]
    lib.bsdc_bam_writer_open.restype = C.c_int32
    lib.bsdc_bam_writer_add.argtypes = [_P, C.POINTER(_Records), C.c_int32]
    lib.bsdc_bam_writer_add.restype = C.c_int32
    lib.bsdc_bam_writer_encode.argtypes = [_P, C.POINTER(_Records), C.c_int32, C.POINTER(C.c_void_p)]
    lib.bsdc_bam_writer_encode.restype = C.c_int64
    lib.bsdc_bam_writer_take.argtypes = [_P, C.c_int64, _P, _P, C.c_int32]
    lib.bsdc_bam_writer_take.restype = C.c_int32
    lib.bsdc_bam_writer_put.argtypes = [_P, C.c_int64, _P, _P, _P, _P, C.c_int32]
    lib.bsdc_bam_writer_put.restype = C.c_int32
    lib.bsdc_fastq_writer_encode.argtypes = [_P, C.POINTER(_Records), C.c_int32, _P]
    lib.bsdc_fastq_writer_encode.restype = C.c_int32
    lib.bsdc_fastq_writer_take.argtypes = [_P, C.c_int32, C.c_int64, _P, _P, C.c_int32]
    lib.bsdc_fastq_writer_take.restype = C.c_int32
    lib.bsdc_fastq_writer_put.argtypes = [_P, C.c_int32, C.c_int64, _P, _P, _P, _P, C.c_int32]
    lib.bsdc_fastq_writer_put.restype = C.c_int32
    lib.bsdc_bam_writer_close.argtypes = [_P, C.c_int32]
    lib.bsdc_bam_writer_close.restype = C.c_int32
    lib.bsdc_fastq_writer_open.argtypes = [C.c_char_p, C.c_char_p, C.c_int32, C.POINTER(_P)]
    lib.bsdc_fastq_writer_open.restype = C.c_int32
    lib.bsdc_fastq_writer_add.argtypes = [_P, C.POINTER(_Records), C.c_int32]
    lib.bsdc_fastq_writer_add.restype = C.c_int32
    lib.bsdc_fastq_writer_close.argtypes = [_P, C.c_int32]
    lib.bsdc_fastq_writer_close.restype = C.c_int32
    lib.bsdc_bam_write.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.c_int32, _P, _P, _P, C.POINTER(_Records),
                                   C.c_int32, C.c_int32]
    lib.bsdc_bam_write.restype = C.c_int32
    lib.bsdc_rx_consensus.argtypes = [C.c_int64, _P, _P, _P, _P, _P, _P, _P, C.c_int32]
    lib.bsdc_rx_consensus.restype = C.c_int64
    lib.bsdc_fastq_write.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(_Records), C.c_int32, C.c_int32]
    lib.bsdc_fastq_write.restype = C.c_int32
    lib.bsdc_family_image.argtypes = [C.c_int64, _P, _P, _P, _P, _P, C.c_int64, _P, _P, C.c_int32]
    lib.bsdc_family_image.restype = C.c_int32
    lib.bsdc_consensus_tags.argtypes = [C.c_int64, _P, _P, _P, C.c_int32, C.c_int32, _P, _P, _P, _P, _P, _P, _P,
                                        _P, _P, C.c_int32]
    lib.bsdc_consensus_tags.restype = C.c_int64
    lib.bsdc_table_concat.argtypes = [C.c_int64, C.c_int32, C.POINTER(_P), C.POINTER(_P), _P, _P, _P, C.c_int32]
    lib.bsdc_table_concat.restype = C.c_int64
    lib.bsdc_table_rank.argtypes = [C.c_int64, _P, _P, _P, C.c_int32]
    lib.bsdc_table_rank.restype = None
    lib.bsdc_table_take.argtypes = [C.c_int64, _P, _P, _P, _P, _P, C.c_int32]
    lib.bsdc_table_take.restype = C.c_int64
    lib.bsdc_unpack_nibbles.argtypes = [C.c_int64, _P, _P, C.c_int32]
    lib.bsdc_unpack_nibbles.restype = None
    lib.bsdc_rows_gather.argtypes = [C.c_int64, _P, _P, C.c_int64, _P, _P, _P, C.c_int32]
    lib.bsdc_rows_gather.restype = None
    lib.bsdc_bam_find_cut.argtypes = [C.c_char_p, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                      _P]
    lib.bsdc_bam_find_cut.restype = C.c_int32
    lib.bsdc_bam_stream_open_range.argtypes = [C.c_char_p, C.c_int32, C.c_int64, C.c_int64, C.c_int64, C.c_int64,
                                               C.c_int64, C.POINTER(_P)]
    lib.bsdc_bam_stream_open_range.restype = C.c_int32
    lib.bsdc_bam_stream_set_owner.argtypes = [_P, C.c_int32, _P, C.c_int32, C.c_int64, C.c_int32]
    lib.bsdc_bam_stream_set_owner.restype = C.c_int32
    lib.bsdc_bam_stream_spill.argtypes = [_P, _P]
    lib.bsdc_bam_stream_spill.restype = C.c_int64
    lib.bsdc_bam_stream_set_defer.argtypes = [_P, C.c_int64]
    lib.bsdc_bam_stream_set_defer.restype = C.c_int32
    lib.bsdc_bam_stream_splices.argtypes = [_P, _P]
    lib.bsdc_bam_stream_splices.restype = C.c_int64
    lib.bsdc_bam_rec_keys.argtypes = [_P, _P]
    lib.bsdc_bam_rec_keys.restype = C.c_int32
    lib.bsdc_spill_sort.argtypes = [_P, C.c_int64, _P, _P]
    lib.bsdc_spill_sort.restype = C.c_int64
    lib.bsdc_bam_writer_flush.argtypes = [_P, C.c_int32]
    lib.bsdc_bam_writer_flush.restype = C.c_int32
    lib.bsdc_bam_writer_tell.argtypes = [_P]
    lib.bsdc_bam_writer_tell.restype = C.c_int64
    lib.bsdc_bam_writer_raw.argtypes = [_P, _P, C.c_int64, C.c_int32]
    lib.bsdc_bam_writer_raw.restype = C.c_int32
    lib.bsdc_fastq_writer_flush.argtypes = [_P, C.c_int32]
    lib.bsdc_fastq_writer_flush.restype = C.c_int32
    lib.bsdc_fastq_writer_tell.argtypes = [_P, _P]
    lib.bsdc_fastq_writer_tell.restype = None
    lib.bsdc_bam_stream_range_stats.argtypes = [_P, _P]
    lib.bsdc_bam_stream_range_stats.restype = None
    lib.bsdc_bam_writer_fragment.argtypes = [_P, C.c_int32]
    lib.bsdc_bam_writer_fragment.restype = C.c_int32
    lib.bsdc_fastq_writer_fragment.argtypes = [_P]
    lib.bsdc_fastq_writer_fragment.restype = C.c_int32
    if lib.bsdc_io_abi_version() != BSDC_IO_ABI_VERSION:
        raise RuntimeError("libbsdc_io ABI %d != %d" % (lib.bsdc_io_abi_version(), BSDC_IO_ABI_VERSION))
    _lib = lib
    return lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


class StringTable:
    """Strings packed in one buffer (``buf[off[i]:off[i+1]]``); indexing gives bytes (or str)."""

    def __init__(self, buf: np.ndarray, off: np.ndarray, as_str: bool = False):
        self.buf = np.ascontiguousarray(buf, np.uint8)
        self.off = np.ascontiguousarray(off, np.int64)
        self.as_str = as_str

    def __len__(self):
        return int(self.off.shape[0]) - 1

    def __getitem__(self, i):
        b = self.buf[int(self.off[i]):int(self.off[i + 1])].tobytes()
        return b.decode() if self.as_str else b

    @staticmethod
    def from_list(items) -> "StringTable":
        bs = [x if isinstance(x, bytes) else str(x).encode() for x in items]
        off = np.zeros(len(bs) + 1, np.int64)
        if bs:
            off[1:] = np.cumsum([len(x) for x in bs])
        return StringTable(np.frombuffer(b"".join(bs), np.uint8) if bs else np.zeros(0, np.uint8), off,
                           as_str=bool(items) and isinstance(items[0], str))

    def lex_key(self, ids: np.ndarray) -> np.ndarray:
        """A key per id ordering the ids as their strings sort in byte order (vectorised)."""
        ids = np.asarray(ids, np.int64)
        if ids.shape[0] == 0:
            return np.zeros(0, np.int64)
        u, inv = np.unique(ids, return_inverse=True)
        lens = self.off[u + 1] - self.off[u]
        w = max(int(lens.max()), 1)
        j = np.arange(w)[None, :]
        idx = self.off[u][:, None] + j
        m = np.where(j < lens[:, None], self.buf[np.minimum(idx, max(self.buf.shape[0] - 1, 0))], 0).astype(np.uint8)
        fixed = np.ascontiguousarray(m).view("S%d" % w).reshape(-1)
        _, rk = np.unique(fixed, return_inverse=True)
        return rk.astype(np.int64)[inv]


@dataclass
class BamHeader:
    text: str
    ref_names: List[str]
    ref_lens: np.ndarray

    def read_groups(self) -> List[dict]:
        out = []
        for line in self.text.splitlines():
            if line.startswith("@RG"):
                out.append(dict(f.split(":", 1) for f in line.split("\t")[1:] if ":" in f))
        return out


class BufferPool:
    """Host byte buffers handed from one stream chunk's decoded records to a later chunk's
    (bam.step5_stream): a fresh array of a few hundred MB costs its page faults and the kernel's
    zeroing on every chunk.  take() the smallest free buffer that fits (or a new one), give() it
    back once nothing refers to the arrays carved from it."""

    def __init__(self, keep: int = 6):
        import threading
        self.free: list = []
        self.keep = keep
        self.lock = threading.Lock()

    def take(self, nbytes: int) -> np.ndarray:
        with self.lock:
            fit = [i for i, b in enumerate(self.free) if b.size >= nbytes]
            if fit:
                return self.free.pop(min(fit, key=lambda i: self.free[i].size))
        return np.empty(max(int(nbytes * 1.15), 1), np.uint8)

    def give(self, buf: Optional[np.ndarray]):
        if buf is None:
            return
        with self.lock:
            self.free.append(buf)
            if len(self.free) > self.keep:  # drop the smallest (by position: arrays do not compare)
                del self.free[min(range(len(self.free)), key=lambda i: self.free[i].size)]


def _decode(lib, h, what: str, pool: Optional[BufferPool] = None):
    """A bsdc_bam handle (whole file or stream chunk) -> (BamHeader, RawRecords); frees nothing.
    With `pool`, the record arrays are carved from one pooled buffer (bsdc_bam_copy writes every
    element), kept as RawRecords._pool_buf for the caller to give back."""
    s = _Sizes()
    lib.bsdc_bam_sizes_of(h, C.byref(s))
    n = s.n_rec
    specs = []

    def z(k, dt):
        specs.append((max(int(k), 1), np.dtype(dt)))
        return len(specs) - 1
    A = dict(flag=z(n, np.uint16), tid=z(n, np.int32), pos=z(n, np.int32), mapq=z(n, np.uint8),
             l_seq=z(n, np.int32), seq_off=z(n, np.int64), seq=z(s.n_bases, np.uint8), qual=z(s.n_bases, np.uint8),
             cig_off=z(n, np.int64), n_cig=z(n, np.int32), cigar=z(s.n_cigar, np.uint32),
             next_tid=z(n, np.int32), next_pos=z(n, np.int32), tlen=z(n, np.int32), name_id=z(n, np.int32),
             name_off=z(s.n_names + 1, np.int64), name_buf=z(s.name_bytes, np.uint8), mi_id=z(n, np.int32),
             mi_strand=z(n, np.int8), mi_off=z(s.n_mi + 1, np.int64), mi_buf=z(s.mi_bytes, np.uint8),
             mc_off=z(n, np.int64), mc_n=z(n, np.int32), mc_cigar=z(s.n_mc, np.uint32), la=z(n, np.int32),
             rd=z(n, np.int32), aux_off=z(n + 1, np.int64), aux=z(s.aux_bytes, np.uint8),
             header=z(s.header_bytes, np.uint8), ref_len=z(s.n_ref, np.int64),
             ref_name_off=z(s.n_ref + 1, np.int64), ref_name_buf=z(s.ref_name_bytes, np.uint8))
    buf = None
    if pool is None:
        arrs = [np.zeros(k, dt) for k, dt in specs]
    else:
        sizes = [(k * dt.itemsize + 63) & ~63 for k, dt in specs]
        buf = pool.take(sum(sizes))
        arrs, o = [], 0
        for (k, dt), nb in zip(specs, sizes):
            arrs.append(buf[o:o + k * dt.itemsize].view(dt))
            o += nb
    A = {key: arrs[i] for key, i in A.items()}
    a = _Arrays(**{k: _ptr(v) for k, v in A.items()})
    if lib.bsdc_bam_copy(h, C.byref(a)) != 0:
        raise OSError("%s: %s" % (what, lib.bsdc_io_last_error().decode()))
    names_tab = StringTable(A["ref_name_buf"][:s.ref_name_bytes], A["ref_name_off"][:s.n_ref + 1], as_str=True)
    header = BamHeader(A["header"][:s.header_bytes].tobytes().decode(errors="replace"),
                       [names_tab[i] for i in range(s.n_ref)], A["ref_len"][:s.n_ref].copy())
    raw = R.RawRecords(
        flag=A["flag"][:n], tid=A["tid"][:n], pos=A["pos"][:n], mapq=A["mapq"][:n], l_seq=A["l_seq"][:n],
        seq_off=A["seq_off"][:n], seq=A["seq"][:s.n_bases], qual=A["qual"][:s.n_bases], cig_off=A["cig_off"][:n],
        n_cig=A["n_cig"][:n], cigar=A["cigar"][:s.n_cigar], next_tid=A["next_tid"][:n], next_pos=A["next_pos"][:n],
        tlen=A["tlen"][:n], name_id=A["name_id"][:n],
        names=StringTable(A["name_buf"][:s.name_bytes], A["name_off"][:s.n_names + 1]),
        mi_id=A["mi_id"][:n], mi_strand=A["mi_strand"][:n],
        mi_names=StringTable(A["mi_buf"][:s.mi_bytes], A["mi_off"][:s.n_mi + 1], as_str=True),
        mc_off=A["mc_off"][:n], mc_n=A["mc_n"][:n], mc_cigar=A["mc_cigar"][:s.n_mc],
        aux=StringTable(A["aux"][:s.aux_bytes], A["aux_off"][:n + 1]), la_tag=A["la"][:n], rd_tag=A["rd"][:n])
    raw._pool_buf = buf
    return header, raw


def read_bam(path: str, threads: int = 0):
    """BAM file -> (BamHeader, records.RawRecords) with MI / MC / LA / RD decoded and the other
    aux bytes kept (``raw.aux`` is a StringTable of per-record aux blocks)."""
    lib = _load()
    h = _P()
    rc = lib.bsdc_bam_read(path.encode(), int(threads), C.byref(h))
    if rc != 0:
        raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
    try:
        return _decode(lib, h, path)
    finally:
        lib.bsdc_bam_free(h)


DEFAULT_CHUNK_BYTES = 64 << 20  # uncompressed record bytes per stream chunk (about 0.23M records)
DEFAULT_SLACK = 10_000           # positions: > any template's span (fragment + clips)
# a template whose mate lies further than this (or on another contig, unmapped or absent) is
# deferred: it leaves the stream for the spill, whose families are spliced in at their keys
# (bsdc_bam_stream_set_defer); half the slack, so that no rank window misses a near template's end
DEFAULT_DEFER_SPAN = DEFAULT_SLACK // 2
DEFER_MARGIN = 12  # kDeferMargin (csrc/bsdc_io.cpp): 3 x kKeyDelta


def read_bam_header(path: str) -> BamHeader:
    """The header of a BAM (its first BGZF blocks only)."""
    lib = _load()
    st = _P()
    if lib.bsdc_bam_stream_open(path.encode(), 1, 1 << 20, C.byref(st)) != 0:
        raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
    try:
        h = _P()
        lib.bsdc_bam_stream_header(st, C.byref(h))
        try:
            return _decode(lib, h, path)[0]
        finally:
            lib.bsdc_bam_free(h)
    finally:
        lib.bsdc_bam_stream_close(st)


class StreamChunk:
    """A chunk cut from a BAM stream but not yet decoded (bsdc_bam_stream_next_raw).  decode()
    parses it and copies it out (any thread: the stream meanwhile cuts the next chunk); discard()
    drops it.  Either returns its buffer to the stream; exactly one of them must be called."""

    def __init__(self, lib, st, h, path: str):
        self._lib, self._st, self._h, self._path = lib, st, h, path
        self.keys = False      # decode() also fills RawRecords.tc_key (bsdc_bam_rec_keys)
        self.splices = None    # int64 [k, 2]: deferred keys to cut this chunk's output before
        self.spill = b""       # spill entries (bsdc_bam_stream_spill) since the chunk before

    def decode(self, threads: int = 0, timing: Optional[dict] = None, pool: Optional[BufferPool] = None):
        """-> (BamHeader, RawRecords); `timing`: seconds added under "parse" (records, tags,
        interning) and "copy" (the arrays copied out); `pool`: see _decode."""
        import time
        lib, h = self._lib, self._h
        self._h = None
        try:
            t0 = time.perf_counter()
            if lib.bsdc_bam_parse(h, int(threads)) != 0:
                raise OSError("%s: %s" % (self._path, lib.bsdc_io_last_error().decode()))
            t1 = time.perf_counter()
            out = _decode(lib, h, self._path, pool)
            if self.keys:  # the records' coarse TemplateCoordinate keys (splicing deferred families)
                kk = np.zeros(2 * max(out[1].n, 1), np.int64)
                if lib.bsdc_bam_rec_keys(h, _ptr(kk)) != 0:
                    raise OSError("%s: %s" % (self._path, lib.bsdc_io_last_error().decode()))
                out[1].tc_key = kk[:2 * out[1].n].reshape(-1, 2)
            if timing is not None:
                timing["parse"] = timing.get("parse", 0.0) + t1 - t0
                timing["copy"] = timing.get("copy", 0.0) + time.perf_counter() - t1
            return out
        finally:
            lib.bsdc_bam_stream_recycle(self._st, h)

    def discard(self):
        if self._h is not None:
            h, self._h = self._h, None
            self._lib.bsdc_bam_stream_recycle(self._st, h)


KEY_GUARD = 16  # positions of key gap on each side of a rank boundary (> 2 x kKeyDelta of the tools' jitter)


def find_cut(path: str, start: int, threads: int = 0, min_span: Optional[int] = None, slack: int = DEFAULT_SLACK,
             guard: int = KEY_GUARD, max_bytes: int = 256 << 20):
    """A rank boundary of a coordinate-sorted BAM after file offset `start` (bsdc_bam_find_cut), or
    None: a dict with `key` (the boundary X, 2 ints), `coord` (contig << 32 | x), `start` (block,
    offset) of the first record at or past x - slack, `end` the same at or past x + slack, and
    `slack`."""
    lib = _load()
    out = np.zeros(8, np.int64)
    ms = 2 * slack if min_span is None else min_span
    if lib.bsdc_bam_find_cut(path.encode(), int(threads), int(start), int(ms), int(slack), int(guard), int(max_bytes),
                             _ptr(out)) != 0:
        raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
    if not out[7]:
        return None
    return {"start": (int(out[0]), int(out[1])), "end": (int(out[2]), int(out[3])), "key": (int(out[4]), int(out[5])),
            "coord": int(out[6]), "slack": int(slack)}


OWN_STOP_FOREIGN = 1  # include/bsdc_io.h BSDC_OWN_*


def _stream_spill(lib, st) -> bytes:
    """The stream's spill entries since the last call (bsdc_bam_stream_spill: per record an int64
    coordinate, an int64 file sequence number, the block_size-prefixed record)."""
    n = int(lib.bsdc_bam_stream_spill(st, None))
    if n == 0:
        return b""
    buf = np.empty(n, np.uint8)
    lib.bsdc_bam_stream_spill(st, _ptr(buf))
    return buf.tobytes()


def _stream_splices(lib, st) -> np.ndarray:
    """The deferred keys the last chunk reported (bsdc_bam_stream_splices) -> int64 [k, 2]."""
    n = int(lib.bsdc_bam_stream_splices(st, None))
    out = np.zeros((max(n, 1), 2), np.int64)
    if n:
        lib.bsdc_bam_stream_splices(st, _ptr(out))
    return out[:n]


def spill_sorted_records(data: bytes):
    """Spill entries (_stream_spill, possibly several streams' concatenated) -> (their records in
    file order -- sorted by (coordinate, sequence), the stable order of the input for equal pairs
    (bsdc_spill_sort) --, their count)."""
    if not data:
        return b"", 0
    lib = _load()
    a = np.frombuffer(data, np.uint8)
    cnt = np.zeros(1, np.int64)
    n = int(lib.bsdc_spill_sort(_ptr(a), a.shape[0], None, _ptr(cnt)))
    if n < 0:
        raise ValueError("spill: %s" % lib.bsdc_io_last_error().decode())
    out = np.empty(max(n, 1), np.uint8)
    lib.bsdc_spill_sort(_ptr(a), a.shape[0], _ptr(out), None)
    return out[:n].tobytes(), int(cnt[0])


def stream_chunks(path: str, threads: int = 0, chunk_bytes: int = DEFAULT_CHUNK_BYTES, slack: int = DEFAULT_SLACK,
                  read_size: int = 8 << 20, runs: bool = False, rng=None, stats: Optional[dict] = None, owner=None,
                  defer: int = 0, keys: bool = False):
    """The chunks of a coordinate-sorted BAM in bounded memory, undecoded (StreamChunk): cut where no
    template or MI family straddles two chunks (include/bsdc_io.h, bsdc_bam_stream_next_raw).  The
    stream itself is freed once it is exhausted and every chunk has been decoded or discarded.
    runs: a GroupReadsByUmi-ordered BAM (step 1's input) cut between runs of one MI value instead
    (bsdc_bam_stream_next_runs; any record order, no `slack`).  rng: (start block, offset in it,
    end block, offset in it) -- the records of that range only (start block -1: from the first
    record, end block -1: to the end; bsdc_bam_stream_open_range); `stats` then receives the range
    statistics (bsdc_bam_stream_range_stats: n, c0, dropped, foreign) once the stream is exhausted.
    owner: (rank, boundaries[, flags]) -- keep the records whose key lies in the rank's interval
    between the boundaries (find_cut dicts; bsdc_bam_stream_set_owner); flags (OWN_*):
    OWN_STOP_FOREIGN -- a foreign record raises OSError("... foreign record ...").
    defer: the span past which a template is deferred (bsdc_bam_stream_set_defer; 0 = off): each
    chunk then carries its `spill` entries and its `splices` (the deferred keys its output is cut
    before), and its records decode with their keys (RawRecords.tc_key); once exhausted, `stats`
    receives the rest as "spill_tail" and "splices_tail".  keys: the records decode with their keys
    in any case."""
    lib = _load()
    st = _P()
    if rng is None:
        rc = lib.bsdc_bam_stream_open(path.encode(), int(threads), int(read_size), C.byref(st))
    else:
        rc = lib.bsdc_bam_stream_open_range(path.encode(), int(threads), int(read_size), *[int(x) for x in rng],
                                            C.byref(st))
    if rc != 0:
        raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
    try:
        if owner is not None:
            rank, cuts = owner[:2]
            flags = int(owner[2]) if len(owner) > 2 else 0  # OWN_* (True: OWN_STOP_FOREIGN)
            bd = np.array([[c["key"][0], c["key"][1], c["coord"]] for c in cuts], np.int64).reshape(-1)
            wsl = min(c["slack"] for c in cuts) if cuts else 0  # (the windows' own margin)
            if lib.bsdc_bam_stream_set_owner(st, int(rank), _ptr(bd) if len(bd) else None, len(cuts), int(wsl),
                                             flags) != 0:
                raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
        if defer and lib.bsdc_bam_stream_set_defer(st, int(defer)) != 0:
            raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
        while True:
            h = _P()
            if runs:
                rc = lib.bsdc_bam_stream_next_runs(st, int(chunk_bytes), C.byref(h))
            else:
                rc = lib.bsdc_bam_stream_next_raw(st, int(chunk_bytes), int(slack), C.byref(h))
            if rc != 0:
                raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))
            if not h:
                if stats is not None:
                    v = np.zeros(7, np.int64)
                    lib.bsdc_bam_stream_range_stats(st, _ptr(v))
                    stats.update(n=int(v[0]), c0=int(v[1]), dropped=int(v[2]), foreign=int(v[3]), spilled=int(v[4]),
                                 deferred=int(v[5]), peak_buffered=int(v[6]), spill_tail=_stream_spill(lib, st),
                                 splices_tail=_stream_splices(lib, st))
                return
            ch = StreamChunk(lib, st, h, path)
            ch.keys = bool(defer) or keys
            if defer:
                ch.spill = _stream_spill(lib, st)
                ch.splices = _stream_splices(lib, st)
            yield ch
    finally:
        lib.bsdc_bam_stream_close(st)


def stream_bam(path: str, threads: int = 0, chunk_bytes: int = DEFAULT_CHUNK_BYTES, slack: int = DEFAULT_SLACK,
               read_size: int = 8 << 20):
    """Chunks of a coordinate-sorted BAM in bounded memory: yields (BamHeader, RawRecords) per chunk,
    cut where no template or MI family straddles two chunks (include/bsdc_io.h,
    bsdc_bam_stream_next); names and MI ids are chunk-local."""
    for c in stream_chunks(path, threads, chunk_bytes, slack, read_size):
        yield c.decode(threads)


def _aux_table(raw: R.RawRecords) -> StringTable:
    if isinstance(raw.aux, StringTable):
        return raw.aux
    if raw.aux is None:
        return StringTable(np.zeros(0, np.uint8), np.zeros(raw.n + 1, np.int64))
    return StringTable.from_list(list(raw.aux))


@dataclass
class OutRecordsBam:
    """Records to write, structure-of-arrays (the bsdc_bam_records layout)."""

    flag: np.ndarray
    tid: np.ndarray
    pos: np.ndarray
    mapq: np.ndarray
    next_tid: np.ndarray
    next_pos: np.ndarray
    tlen: np.ndarray
    names: StringTable
    cig_off: np.ndarray     # [n + 1]
    cigar: np.ndarray
    seq_off: np.ndarray     # [n + 1]
    seq: np.ndarray         # nt16 codes
    qual: np.ndarray
    aux: StringTable
    aux2: Optional[StringTable] = None  # more aux bytes written after aux (the consensus tags)

    @property
    def n(self) -> int:
        return int(self.flag.shape[0])


def _ascii_int(x: np.ndarray):
    """Non-negative ints -> their decimal ASCII, packed: (buf, off)."""
    x = np.asarray(x, np.int64)
    d = np.ones_like(x)
    for k in range(1, 19):
        d += x >= 10 ** k
    off = np.zeros(x.shape[0] + 1, np.int64)
    off[1:] = np.cumsum(d)
    pos = np.arange(int(off[-1]), dtype=np.int64)
    rec = np.repeat(np.arange(x.shape[0]), d)
    p = pos - off[rec]                       # digit index from the left
    buf = (48 + (x[rec] // (10 ** (d[rec] - 1 - p))) % 10).astype(np.uint8)
    return buf, off


def _concat_fields(parts, n):
    """Per-record byte fields (each (buf, off) or a constant bytes) -> one packed StringTable
    (libbsdc_io bsdc_table_concat: parallel copies, no per-byte index arrays)."""
    lib = _load()
    k = len(parts)
    offs = (_P * k)()
    bufs = (_P * k)()
    clen = np.zeros(k, np.int64)
    keep = []
    for j, p in enumerate(parts):
        if isinstance(p, bytes):
            b = np.frombuffer(p if p else b"\0", np.uint8).copy()
            keep.append(b)
            offs[j], bufs[j], clen[j] = None, _ptr(b), len(p)
        else:
            pb = np.ascontiguousarray(p[0], np.uint8)
            po = np.ascontiguousarray(p[1], np.int64)
            if pb.size == 0:
                pb = np.zeros(1, np.uint8)
            keep += [pb, po]
            offs[j], bufs[j] = _ptr(po), _ptr(pb)
    off = np.zeros(n + 1, np.int64)
    total = lib.bsdc_table_concat(int(n), k, offs, bufs, _ptr(clen), _ptr(off), None, 0)
    buf = np.empty(max(int(total), 1), np.uint8)
    lib.bsdc_table_concat(int(n), k, offs, bufs, _ptr(clen), _ptr(off), _ptr(buf), 0)
    return StringTable(buf[:int(total)], off)


def table_ranks(t: StringTable) -> np.ndarray:
    """Byte-order rank of every entry of a packed table (equal entries share a rank; libbsdc_io)."""
    lib = _load()
    n = len(t)
    rank = np.zeros(max(n, 1), np.int64)
    if n:
        buf = np.ascontiguousarray(t.buf, np.uint8) if t.buf.size else np.zeros(1, np.uint8)
        lib.bsdc_table_rank(n, _ptr(np.ascontiguousarray(t.off, np.int64)), _ptr(buf), _ptr(rank), 0)
    return rank[:n]


def unpack_nibbles(packed: np.ndarray, threads: int = 0) -> np.ndarray:
    """Packed nt16 bytes (high nibble first) -> one code per byte, same leading shape, last axis x2
    (libbsdc_io, parallel)."""
    a = np.ascontiguousarray(packed, np.uint8)
    out = np.empty(a.shape[:-1] + (2 * a.shape[-1],), np.uint8)
    if a.size:
        _load().bsdc_unpack_nibbles(int(a.size), _ptr(a), _ptr(out), int(threads))
    return out


def _take_table(t: StringTable, idx: np.ndarray) -> StringTable:
    """Entries idx[0], idx[1], ... of a packed table (libbsdc_io bsdc_table_take)."""
    lib = _load()
    idx = np.ascontiguousarray(idx, np.int64)
    n = int(idx.shape[0])
    src_off = np.ascontiguousarray(t.off, np.int64)
    src = np.ascontiguousarray(t.buf, np.uint8) if t.buf.size else np.zeros(1, np.uint8)
    off = np.zeros(n + 1, np.int64)
    total = lib.bsdc_table_take(n, _ptr(idx), _ptr(src_off), _ptr(src), _ptr(off), None, 0)
    buf = np.empty(max(int(total), 1), np.uint8)
    lib.bsdc_table_take(n, _ptr(idx), _ptr(src_off), _ptr(src), _ptr(off), _ptr(buf), 0)
    return StringTable(buf[:int(total)], off)


def take_records(recs: "OutRecordsBam", idx: np.ndarray) -> "OutRecordsBam":
    """Records idx[0], idx[1], ... of an OutRecordsBam (a contiguous range for the streaming writer)."""
    idx = np.asarray(idx, np.int64)

    def ragged(off, vals):
        ln = (off[1:] - off[:-1])[idx]
        o = np.zeros(idx.shape[0] + 1, np.int64)
        o[1:] = np.cumsum(ln)
        src = np.repeat(off[:-1][idx] - o[:-1], ln) + np.arange(int(o[-1]), dtype=np.int64)
        return o, vals[src]
    co, cig = ragged(recs.cig_off, recs.cigar)
    so, seq = ragged(recs.seq_off, recs.seq)
    _, qual = ragged(recs.seq_off, recs.qual)
    return OutRecordsBam(flag=recs.flag[idx], tid=recs.tid[idx], pos=recs.pos[idx], mapq=recs.mapq[idx],
                         next_tid=recs.next_tid[idx], next_pos=recs.next_pos[idx], tlen=recs.tlen[idx],
                         names=_take_table(recs.names, idx), cig_off=co, cigar=cig, seq_off=so, seq=seq, qual=qual,
                         aux=_take_table(recs.aux, idx),
                         aux2=_take_table(recs.aux2, idx) if recs.aux2 is not None else None)


def _synthetic_fields(raw: R.RawRecords):
    """Vectorised MI / MC aux and QNAMEs of a synthetic stream (decimal lazy names, one-op MC)."""
    n = raw.n
    mi_pre = getattr(raw.mi_names, "prefix", None)
    nm_pre = getattr(raw.names, "prefix", None)
    if mi_pre is None or nm_pre is None or (raw.mc_n > 1).any() or (raw.mi_id < 0).any() or (raw.mi_strand < 0).any():
        return None
    mi = _ascii_int(raw.mi_id)
    sfx = (np.frombuffer(b"AB", np.uint8)[raw.mi_strand.astype(np.int64)], np.arange(n + 1, dtype=np.int64))
    has_mc = raw.mc_off >= 0
    mcv = raw.mc_cigar[np.where(has_mc, raw.mc_off, 0)] if raw.mc_cigar.shape[0] else np.zeros(n, np.uint32)
    if not has_mc.all():
        return None
    mcl = _ascii_int(mcv >> 4)
    mco = (np.frombuffer(R.CIGAR_OPS.encode(), np.uint8)[(mcv & 0xF).astype(np.int64)], np.arange(n + 1, dtype=np.int64))
    aux = _concat_fields([b"MIZ" + mi_pre.encode(), mi, b"/", sfx, b"\0MCZ", mcl, mco, b"\0"], n)
    names = _concat_fields([nm_pre.encode(), _ascii_int(raw.name_id)], n)
    return aux, names


def records_to_bam(raw: R.RawRecords) -> OutRecordsBam:
    """A RawRecords stream as records to write: its own aux bytes, or for synthetic streams
    (no aux) the MI (with the /A|/B strand) and MC tags rebuilt from the decoded fields."""
    n = raw.n
    syn = _synthetic_fields(raw) if raw.aux is None and n else None
    if raw.aux is not None:
        aux = _aux_table(raw)
    elif syn is not None:
        aux = syn[0]
    else:
        parts = []
        for k in range(n):
            t = []
            if raw.mi_id[k] >= 0:
                sfx = {0: "/A", 1: "/B"}.get(int(raw.mi_strand[k]), "")
                t.append(("MI", "Z", "%s%s" % (raw.mi_names[int(raw.mi_id[k])], sfx)))
            if raw.mc_off[k] >= 0:
                mc = raw.mc_cigar[raw.mc_off[k]:raw.mc_off[k] + raw.mc_n[k]]
                t.append(("MC", "Z", R.cigar_string([int(x) for x in mc])))
            parts.append(R.encode_aux(t))
        aux = StringTable.from_list(parts)
    cig_off = np.zeros(n + 1, np.int64)
    cig_off[:n] = raw.cig_off
    cig_off[n] = int(raw.cig_off[-1] + raw.n_cig[-1]) if n else 0
    seq_off = np.zeros(n + 1, np.int64)
    seq_off[:n] = raw.seq_off
    seq_off[n] = int(raw.seq_off[-1] + raw.l_seq[-1]) if n else 0
    if syn is not None:
        tab = syn[1]
    else:
        names = raw.names
        tab = StringTable.from_list([names[int(i)] for i in raw.name_id.astype(np.int64)])
    return OutRecordsBam(raw.flag, raw.tid, raw.pos, raw.mapq, raw.next_tid, raw.next_pos, raw.tlen, tab, cig_off,
                         raw.cigar, seq_off, raw.seq, raw.qual, aux)


def _records_struct(recs: OutRecordsBam, keep: list) -> _Records:
    def c(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dt)
        keep.append(a)
        return _ptr(a)
    return _Records(recs.n, c(recs.flag, np.uint16), c(recs.tid, np.int32), c(recs.pos, np.int32),
                    c(recs.mapq, np.uint8), c(recs.next_tid, np.int32), c(recs.next_pos, np.int32),
                    c(recs.tlen, np.int32), c(recs.names.off, np.int64), c(recs.names.buf, np.uint8),
                    c(recs.cig_off, np.int64), c(recs.cigar, np.uint32), c(recs.seq_off, np.int64),
                    c(recs.seq, np.uint8), c(recs.qual, np.uint8), c(recs.aux.off, np.int64),
                    c(recs.aux.buf, np.uint8),
                    c(recs.aux2.off, np.int64) if recs.aux2 is not None else None,
                    c(recs.aux2.buf, np.uint8) if recs.aux2 is not None else None)


def family_image(src_off, length, dst_off, seq, qual, n_slots: int, packed: np.ndarray, qual_out: np.ndarray,
                 threads: int = 0):
    """batch.build_family_batch's image: record r's bases / quals at src_off[r] -> nibble / byte
    dst_off[r] + 1 of `packed` / `qual_out` (zeroed by the caller; libbsdc_io)."""
    lib = _load()
    so = np.ascontiguousarray(src_off, np.int64)
    ln = np.ascontiguousarray(length, np.int64)
    do = np.ascontiguousarray(dst_off, np.int64)
    sq = np.ascontiguousarray(seq, np.uint8)
    ql = np.ascontiguousarray(qual, np.uint8)
    if packed.shape[0] * 2 < n_slots or qual_out.shape[0] < n_slots or not (packed.flags.c_contiguous and
                                                                           qual_out.flags.c_contiguous):
        raise ValueError("family image outputs too small")
    if so.shape[0] and (int((so + ln).max()) > sq.shape[0] or int((so + ln).max()) > ql.shape[0]):
        raise ValueError("family image: record past the end of seq / qual")
    rc = lib.bsdc_family_image(so.shape[0], _ptr(so), _ptr(ln), _ptr(do), _ptr(sq), _ptr(ql), int(n_slots),
                               _ptr(packed), _ptr(qual_out), int(threads))
    if rc != 0:
        raise ValueError(lib.bsdc_io_last_error().decode())


def write_fastq(path1: str, path2: str, recs: OutRecordsBam, level: int = 6, threads: int = 0):
    """Paired gzip FASTQ of `recs` as picard SamToFastq F=path1 F2=path2 writes it (the rule after
    step 5, main.snake.py:167-177): '@name/1' / '@name/2', SEQ, '+', QUAL+33 (libbsdc_io)."""
    lib = _load()
    keep = []
    r = _records_struct(recs, keep)
    rc = lib.bsdc_fastq_write(path1.encode(), path2.encode(), C.byref(r), int(level), int(threads))
    if rc != 0:
        raise ValueError("%s, %s: %s" % (path1, path2, lib.bsdc_io_last_error().decode()))


def write_bam(path: str, header: BamHeader, recs: OutRecordsBam, level: int = 6, threads: int = 0):
    lib = _load()
    rn = StringTable.from_list([x.encode() for x in header.ref_names])
    keep = []

    def c(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dt)
        keep.append(a)
        return _ptr(a)
    r = _records_struct(recs, keep)
    text = header.text.encode()
    rc = lib.bsdc_bam_write(path.encode(), text, len(text), len(header.ref_names), c(rn.off, np.int64),
                            c(rn.buf, np.uint8), c(np.asarray(header.ref_lens, np.int64), np.int64), C.byref(r),
                            int(level), int(threads))
    if rc != 0:
        raise OSError("%s: %s" % (path, lib.bsdc_io_last_error().decode()))


class GpuBgzf:
    """BGZF compression of a BAM writer's whole blocks on one GPU (libbsdc bsdc_bgzf_*,
    csrc/bsdc_bgzf.hip): the encoded bytes go to HBM from a pinned staging slot, one workgroup
    deflates each 65280-byte block, the blocks come back packed; the writer fills their CRC32 /
    ISIZE and writes them.  Its own HIP stream, so it overlaps the consensus kernels; submit()
    returns at once, so the writer encodes the next records while the GPU compresses these."""

    MAX_BLOCKS = 1024  # blocks per kernel launch (the scratch: bsdc_bgzf_scratch_bytes of these)

    def __init__(self, device):
        import torch

        from . import _lib
        self.torch = torch
        self.lib = _lib.load()
        self.dev = torch.device(device)
        self.stream = torch.cuda.Stream(self.dev)
        self.scratch = torch.empty(int(self.lib.bsdc_bgzf_scratch_bytes(self.MAX_BLOCKS)), dtype=torch.uint8,
                                   device=self.dev)
        self.buf = {}  # grown on demand: device din / out / sizes, pinned sizes_h / out_h / raw0 / raw1
        self.slot = 0
        self.job = None  # the submitted, unfinished (nblk, event)
        self.blocks = 0
        self.bytes_in = 0
        self.bytes_out = 0

    def _buf(self, name, n, dtype=None, pinned=False):
        torch = self.torch
        t = self.buf.get(name)
        if t is None or t.numel() < n:
            n = max(int(n * 1.25), 1)
            t = (torch.empty(n, dtype=dtype or torch.uint8, pin_memory=True) if pinned else
                 torch.empty(n, dtype=dtype or torch.uint8, device=self.dev))
            self.buf[name] = t
        return t

    def staging(self, nbytes: int):
        """the next pinned staging slot (two alternate: one may still feed the last submit)."""
        self.slot ^= 1
        return self._buf("raw%d" % self.slot, nbytes, pinned=True)

    def submit(self, raw, nblk: int):
        """launch the compression of nblk blocks from the pinned slot `raw` (staging()); one job in
        flight: finish() the last one first."""
        torch = self.torch
        if self.job is not None:
            raise RuntimeError("GpuBgzf.submit with a job in flight")
        n = nblk * 65280
        din = self._buf("din", n)
        out = self._buf("out", nblk * 65536)
        sizes = self._buf("sizes", nblk, torch.int32)
        sizes_h = self._buf("sizes_h", nblk, torch.int32, pinned=True)
        st = self.stream.cuda_stream
        with torch.cuda.stream(self.stream):
            din[:n].copy_(raw[:n], non_blocking=True)
            for b0 in range(0, nblk, self.MAX_BLOCKS):
                nb = min(self.MAX_BLOCKS, nblk - b0)
                if self.lib.bsdc_bgzf_deflate(din.data_ptr(), n, b0, nb, self.scratch.data_ptr(), sizes.data_ptr(),
                                              st) != 0:
                    raise RuntimeError("bsdc_bgzf_deflate failed")
                if self.lib.bsdc_bgzf_pack(self.scratch.data_ptr(), sizes.data_ptr(), b0, nb, out.data_ptr(), st) != 0:
                    raise RuntimeError("bsdc_bgzf_pack failed")
            sizes_h[:nblk].copy_(sizes[:nblk], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.job = (nblk, ev)

    def finish(self):
        """wait for the submitted job -> (packed blocks: a pinned view valid until the next finish,
        sizes int32[nblk])."""
        nblk, ev = self.job
        self.job = None
        ev.synchronize()
        sizes_h = self.buf["sizes_h"][:nblk].numpy().copy()
        total = int(np.maximum(sizes_h, 0).sum(dtype=np.int64))
        out_h = self._buf("out_h", max(total, 1), pinned=True)
        if total:
            with self.torch.cuda.stream(self.stream):
                out_h[:total].copy_(self.buf["out"][:total], non_blocking=True)
            self.stream.synchronize()
        self.blocks += nblk
        self.bytes_in += nblk * 65280
        self.bytes_out += total
        return out_h.numpy(), sizes_h

    def compress(self, data_ptr: int, nbytes: int):
        """host bytes [data_ptr, +nbytes) (whole blocks) -> (packed blocks, sizes int32[nblk])."""
        nblk = nbytes // 65280
        host = np.ctypeslib.as_array(C.cast(data_ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))
        raw = self.staging(nbytes)
        raw.numpy()[:nbytes] = host
        self.submit(raw, nblk)
        packed, sizes = self.finish()
        return packed[:int(np.maximum(sizes, 0).sum())].copy(), sizes


class BamWriter:
    """Streaming BAM writer (bsdc_bam_writer): header at open, records added in order, the same
    bytes as write_bam of all the records at once -- or, with `gpu` (a GpuBgzf), every whole block
    deflated on the GPU (valid BGZF, other compressed bytes), one add's blocks compressing while
    the next add encodes."""

    def __init__(self, path: str, header: BamHeader, level: int = 6, gpu: Optional["GpuBgzf"] = None,
                 fragment: Optional[str] = None):
        """fragment: "first" (header, no EOF block) or "next" (neither) -- one rank's piece of a
        BAM that ranks.assemble concatenates."""
        self.lib = _load()
        self.path = path
        self.gpu = gpu
        self.pending = None  # (nblk, crc, raw) submitted to the GPU, not yet written
        rn = StringTable.from_list([x.encode() for x in header.ref_names])
        keep = []

        def c(x, dt):
            a = np.ascontiguousarray(x, dtype=dt)
            if a.size == 0:
                a = np.zeros(1, dt)
            keep.append(a)
            return _ptr(a)
        text = header.text.encode()
        self.h = _P()
        rc = self.lib.bsdc_bam_writer_open(path.encode(), text, len(text), len(header.ref_names), c(rn.off, np.int64),
                                           c(rn.buf, np.uint8), c(np.asarray(header.ref_lens, np.int64), np.int64),
                                           int(level), C.byref(self.h))
        if rc != 0:
            raise OSError("%s: %s" % (path, self.lib.bsdc_io_last_error().decode()))
        if fragment is not None and self.lib.bsdc_bam_writer_fragment(self.h, int(fragment == "first")) != 0:
            raise self._err()

    def _err(self):
        return OSError("%s: %s" % (self.path, self.lib.bsdc_io_last_error().decode()))

    def _drain(self, threads: int):
        if self.pending is None:
            return
        nblk, crc, raw = self.pending
        self.pending = None
        packed, sizes = self.gpu.finish()
        if self.lib.bsdc_bam_writer_put(self.h, nblk, _ptr(packed), _ptr(sizes), _ptr(crc), raw.data_ptr(),
                                        int(threads)) != 0:
            raise self._err()

    def add(self, recs: OutRecordsBam, threads: int = 0):
        keep = []
        r = _records_struct(recs, keep)
        if self.gpu is None:
            if self.lib.bsdc_bam_writer_add(self.h, C.byref(r), int(threads)) != 0:
                raise self._err()
            return
        data = C.c_void_p()
        nbytes = self.lib.bsdc_bam_writer_encode(self.h, C.byref(r), int(threads), C.byref(data))
        if nbytes < 0:
            raise self._err()
        nblk = int(nbytes) // 65280
        job = None
        if nblk:
            raw = self.gpu.staging(int(nbytes))
            crc = np.empty(nblk, np.uint32)
            if self.lib.bsdc_bam_writer_take(self.h, nblk, raw.data_ptr(), _ptr(crc), int(threads)) != 0:
                raise self._err()
            job = (nblk, crc, raw)
        self._drain(threads)
        if job is not None:
            self.gpu.submit(job[2], nblk)
            self.pending = job

    def flush(self, threads: int = 0) -> int:
        """Everything added so far written as whole BGZF blocks; -> the file's length, a point
        where it may be cut (ranks.py splices other pieces in there)."""
        self._drain(threads)
        if self.lib.bsdc_bam_writer_flush(self.h, int(threads)) != 0:
            raise self._err()
        return int(self.lib.bsdc_bam_writer_tell(self.h))

    def add_raw(self, data: bytes, threads: int = 0):
        """Raw BAM records (block_size-prefixed), as a stream chunk holds them (host deflate)."""
        if data:
            buf = np.frombuffer(data, np.uint8)
            if self.lib.bsdc_bam_writer_raw(self.h, _ptr(buf), buf.shape[0], int(threads)) != 0:
                raise self._err()

    def close(self, threads: int = 0):
        if self.h:
            try:
                self._drain(threads)
            finally:
                h, self.h = self.h, _P()
                if self.lib.bsdc_bam_writer_close(h, int(threads)) != 0:
                    raise self._err()


def close_quietly(*writers):
    """Best-effort close of writers a failed step leaves open (BamWriter / FastqWriter / None):
    finishes their in-flight GPU BGZF job and releases the C writer's FILE and buffers, swallowing
    secondary errors (the step raises its first error anyway; the partial output is garbage)."""
    for w in writers:
        if w is None:
            continue
        try:
            w.close()
        except Exception:  # noqa: BLE001
            pass


class FastqWriter:
    """Streaming paired-FASTQ writer (bsdc_fastq_writer): the bytes write_fastq writes for all the
    records at once; every add holds whole pairs.  With `gpu` (a GpuBgzf), the whole blocks of
    both files are deflated on the GPU in one job (valid BGZF-framed gzip, other compressed
    bytes), one add's blocks compressing while the next add encodes."""

    def __init__(self, path1: str, path2: str, level: int = 6, gpu: Optional["GpuBgzf"] = None,
                 fragment: bool = False):
        self.lib = _load()
        self.path = path1
        self.gpu = gpu
        self.pending = None  # (nblk per file, crc per file, raw) submitted to the GPU, not yet written
        self.h = _P()
        if self.lib.bsdc_fastq_writer_open(path1.encode(), path2.encode(), int(level), C.byref(self.h)) != 0:
            raise OSError("%s: %s" % (path1, self.lib.bsdc_io_last_error().decode()))
        if fragment and self.lib.bsdc_fastq_writer_fragment(self.h) != 0:  # (no EOF blocks: ranks.assemble)
            raise self._err()

    def _err(self):
        return OSError("%s: %s" % (self.path, self.lib.bsdc_io_last_error().decode()))

    def _drain(self, threads: int):
        if self.pending is None:
            return
        nb, crcs, raw = self.pending
        self.pending = None
        packed, sizes = self.gpu.finish()
        n0 = nb[0]
        o1 = int(np.maximum(sizes[:n0], 0).sum(dtype=np.int64))  # file 2's blocks follow file 1's
        for d, (lo, po, ro) in enumerate(((0, 0, 0), (n0, o1, n0 * 65280))):
            if nb[d] == 0:
                continue
            sz = np.ascontiguousarray(sizes[lo:lo + nb[d]])
            if self.lib.bsdc_fastq_writer_put(self.h, d, nb[d], packed.ctypes.data + po, _ptr(sz), _ptr(crcs[d]),
                                              raw.data_ptr() + ro, int(threads)) != 0:
                raise self._err()

    def add(self, recs: OutRecordsBam, threads: int = 0):
        keep = []
        r = _records_struct(recs, keep)
        if self.gpu is None:
            if self.lib.bsdc_fastq_writer_add(self.h, C.byref(r), int(threads)) != 0:
                raise self._err()
            return
        whole = np.zeros(2, np.int64)
        if self.lib.bsdc_fastq_writer_encode(self.h, C.byref(r), int(threads), _ptr(whole)) != 0:
            raise self._err()
        nb = [int(whole[0]) // 65280, int(whole[1]) // 65280]
        job = None
        if nb[0] + nb[1]:
            raw = self.gpu.staging((nb[0] + nb[1]) * 65280)
            crcs = [np.empty(max(k, 1), np.uint32) for k in nb]
            for d in range(2):
                if nb[d] and self.lib.bsdc_fastq_writer_take(self.h, d, nb[d], raw.data_ptr() + (nb[0] * 65280 if d else 0),
                                                             _ptr(crcs[d]), int(threads)) != 0:
                    raise self._err()
            job = (nb, crcs, raw)
        self._drain(threads)
        if job is not None:
            self.gpu.submit(job[2], nb[0] + nb[1])
            self.pending = job

    def flush(self, threads: int = 0):
        """Everything added so far written as whole BGZF blocks; -> (length of file 1, of file 2)."""
        self._drain(threads)
        if self.lib.bsdc_fastq_writer_flush(self.h, int(threads)) != 0:
            raise self._err()
        out = np.zeros(2, np.int64)
        self.lib.bsdc_fastq_writer_tell(self.h, _ptr(out))
        return int(out[0]), int(out[1])

    def close(self, threads: int = 0):
        if self.h:
            try:
                self._drain(threads)
            finally:
                h, self.h = self.h, _P()
                if self.lib.bsdc_fastq_writer_close(h, int(threads)) != 0:
                    raise self._err()


def read_fasta(path: str, header: BamHeader) -> R.Reference:
    """FASTA -> the packed reference in the BAM header's tid order (contigs the FASTA lacks are
    absent: tool 1 then converts against N, tools/1.convert_AG_to_CT.py:103-117)."""
    data = np.fromfile(path, dtype=np.uint8)
    starts = np.nonzero(data == ord(">"))[0]
    starts = starts[(starts == 0) | (data[np.maximum(starts - 1, 0)] == ord("\n"))]
    contigs = {}
    for i, s0 in enumerate(starts):
        e = int(starts[i + 1]) if i + 1 < len(starts) else data.shape[0]
        nl = s0 + int(np.argmax(data[s0:e] == ord("\n"))) if (data[s0:e] == ord("\n")).any() else e
        name = data[s0 + 1:nl].tobytes().decode().split()[0]
        body = data[nl:e]
        body = body[(body != ord("\n")) & (body != ord("\r"))]
        contigs[name] = body.tobytes()
    return R.Reference.from_contigs(header.ref_names, {k: v for k, v in contigs.items()}, keep_letters=False,
                                    header_lengths=list(header.ref_lens))


def read_name_prefix(header: BamHeader) -> str:
    """fgbio's default consensus read-name prefix (restated, parity unpinned): the input read
    groups' libraries (or IDs), distinct, sorted, joined by '|'."""
    ids = sorted({rg.get("LB", rg.get("ID", "")) for rg in header.read_groups()})
    return "|".join(ids)


def output_header(header: BamHeader) -> BamHeader:
    """fgbio's consensus header (restated): unsorted/query-grouped, the input's @SQ lines, one
    read group A carrying the input's sample and library when they are unique."""
    rgs = header.read_groups()
    rg = ["@RG", "ID:A"]
    for key in ("SM", "LB"):
        vals = sorted({g[key] for g in rgs if key in g})
        if len(vals) == 1:
            rg.append("%s:%s" % (key, vals[0]))
    lines = ["@HD\tVN:1.6\tSO:unsorted\tGO:query"]
    lines += [ln for ln in header.text.splitlines() if ln.startswith("@SQ")]
    lines += ["\t".join(rg), "@PG\tID:bsseqconsensusreads_amd\tPN:bsseqconsensusreads_amd\tCL:step5"]
    return BamHeader("\n".join(lines) + "\n", list(header.ref_names), np.asarray(header.ref_lens, np.int64))


def consensus_tags(cons, em: np.ndarray, molecular: bool = False, threads: int = 0,
                   pool: Optional["BufferPool"] = None) -> StringTable:
    """fgbio's consensus tags (aux bytes) of the output records R1, R2 of families `em`, from the
    single-strand reads in cons.ss (libbsdc_io bsdc_consensus_tags).  Duplex: a record's 'a'
    strand is its AB read (AB-R1 for R1, AB-R2 for R2), or the only strand present; 'b' its BA read
    when both are present.  Molecular: set 0 for R1, set 1 for R2.  With `pool`, the bytes land in
    a pooled buffer (kept as the table's _pool_buf for the caller to give back): the tags are
    ≈1.8 KB a record, and fresh pages for them cost as much as writing them."""
    lib = _load()
    ss = cons.ss
    F = em.shape[0]
    n = 2 * F
    em2 = np.repeat(em.astype(np.int64), 2)
    end = np.tile(np.asarray([0, 1], np.int64), F)
    if molecular:
        row_a = 4 * em2 + end
        row_b = np.full(n, -1, np.int64)
    else:
        sa, sb = end, 3 - end                      # R1: sets 0 / 3, R2: sets 1 / 2
        la = ss["len"][em2, sa] > 0
        lb = ss["len"][em2, sb] > 0
        row_a = 4 * em2 + np.where(la, sa, sb)
        row_b = np.where(la & lb, 4 * em2 + sb, -1)
    out_len = np.ascontiguousarray(cons.length[em].reshape(-1), np.int32)
    stride = int(ss["base"].shape[2])
    c = lambda a, dt: np.ascontiguousarray(a, dt).reshape(-1)
    base, qual = c(ss["base"], np.uint8), c(ss["qual"], np.uint8)
    wide, wdepth, werr = ss.get("wide"), ss.get("wdepth"), ss.get("werr")
    if np.asarray(ss["depth"]).dtype != np.uint8:  # u16 statistics (oracle/): bytes + wide rows
        d16, e16 = np.asarray(ss["depth"]), np.asarray(ss["err"])
        big = (d16.reshape(d16.shape[0], -1).max(axis=1, initial=0) > 255) | \
              (e16.reshape(e16.shape[0], -1).max(axis=1, initial=0) > 255)
        wide = np.where(big, np.cumsum(big) - 1, -1).astype(np.int32)
        wdepth, werr = d16[big].astype(np.uint16), e16[big].astype(np.uint16)
        depth, err = c(np.minimum(d16, 255), np.uint8), c(np.minimum(e16, 255), np.uint8)
    else:
        depth, err = c(ss["depth"], np.uint8), c(ss["err"], np.uint8)
    has_wide = wide is not None and wdepth is not None and wdepth.shape[0] > 0
    if has_wide:
        wide = np.ascontiguousarray(wide, np.int32)
        wdepth, werr = c(wdepth[:, :, :stride], np.uint16), c(werr[:, :, :stride], np.uint16)
    row_a, row_b = np.ascontiguousarray(row_a), np.ascontiguousarray(row_b)
    off = np.zeros(n + 1, np.int64)
    args = (n, _ptr(row_a), _ptr(row_b), _ptr(out_len), 1 if molecular else 0, stride, _ptr(base), _ptr(qual),
            _ptr(depth), _ptr(err), _ptr(wide) if has_wide else None, _ptr(wdepth) if has_wide else None,
            _ptr(werr) if has_wide else None, _ptr(off))
    total = lib.bsdc_consensus_tags(*args, None, int(threads))
    buf = pool.take(max(int(total), 1)) if pool is not None else np.empty(max(int(total), 1), np.uint8)
    lib.bsdc_consensus_tags(*args, _ptr(buf), int(threads))
    tab = StringTable(buf[:int(total)], off)
    tab._pool_buf = buf if pool is not None else None
    return tab


def duplex_records(cons, raw: R.RawRecords, prefix: str, threads: int = 0, molecular: bool = False,
                   pool: Optional["BufferPool"] = None) -> OutRecordsBam:
    """fgbio duplex output records for the emitted families of `cons`
    (pipeline.Consensus, family order): R1 then R2 per family; fgbio's consensus tags appended
    when cons.ss holds the single-strand reads (``molecular``: CallMolecularConsensusReads' set).
    `pool`: the tags' buffer comes from it (consensus_tags)."""
    lib = _load()
    em = np.nonzero((cons.status & 1) != 0)[0]
    F = em.shape[0]
    n = 2 * F
    # consensus UMI per family from its records' RX (libbsdc_io)
    aux = _aux_table(raw)
    fro = np.ascontiguousarray(cons.fam_rec_off, np.int64)
    fsrc = np.ascontiguousarray(cons.fam_src, np.int64)
    strand = np.ascontiguousarray(raw.mi_strand, np.int8)
    nf_all = int(fro.shape[0]) - 1
    width = lib.bsdc_rx_consensus(nf_all, _ptr(fro), _ptr(fsrc), _ptr(strand), _ptr(aux.off),
                                  _ptr(aux.buf if aux.buf.size else np.zeros(1, np.uint8)), None, None, int(threads))
    rx = np.zeros(max(nf_all * max(width, 1), 1), np.uint8)
    rx_len = np.zeros(max(nf_all, 1), np.int32)
    if width > 0:
        lib.bsdc_rx_consensus(nf_all, _ptr(fro), _ptr(fsrc), _ptr(strand), _ptr(aux.off), _ptr(aux.buf), _ptr(rx),
                              _ptr(rx_len), int(threads))
    # names "prefix:MI" and aux RG/MI/RX, both mates of a family alike (packed tables, no per-family
    # Python objects for the byte work)
    mi_ids = cons.fam_mi[em].astype(np.int64)
    if isinstance(raw.mi_names, StringTable):  # decoded BAM: a packed table already
        mt = _take_table(raw.mi_names, mi_ids)
    else:
        uniq, inv = np.unique(mi_ids, return_inverse=True)
        mt = _take_table(StringTable.from_list([(lambda m: m if isinstance(m, bytes) else m.encode())(
            raw.mi_names[int(i)]) for i in uniq]), inv)
    mi = (mt.buf, mt.off)
    if width > 0:
        rl = rx_len[em].astype(np.int64)
        has = rl > 0
        rxb = rx.reshape(-1, width)[em] if F else np.zeros((0, max(width, 1)), np.uint8)
        rxv = (rxb[np.arange(width)[None, :] < rl[:, None]], np.concatenate([[0], np.cumsum(rl)]).astype(np.int64))
        tag = (np.repeat(np.frombuffer(b"RXZ", np.uint8)[None, :], F, 0)[has].reshape(-1),
               np.concatenate([[0], np.cumsum(np.where(has, 3, 0))]).astype(np.int64))
        nul = (np.zeros(int(has.sum()), np.uint8), np.concatenate([[0], np.cumsum(has)]).astype(np.int64))
        fam_aux = _concat_fields([b"RGZA\0MIZ", mi, b"\0", tag, rxv, nul], F)
    else:
        fam_aux = _concat_fields([b"RGZA\0MIZ", mi, b"\0"], F)
    fam_names = _concat_fields([prefix.encode() + b":", mi], F)
    two = np.repeat(np.arange(F, dtype=np.int64), 2)
    names_t, auxs_t = _take_table(fam_names, two), _take_table(fam_aux, two)
    tg = consensus_tags(cons, em, molecular, threads, pool) if getattr(cons, "ss", None) is not None else None
    L = np.ascontiguousarray(cons.length[em].reshape(-1), np.int32)  # R1, R2, R1, R2 ...
    seq_off = np.zeros(n + 1, np.int64)
    seq_off[1:] = np.cumsum(L)
    stride = cons.seq.shape[2]
    rows = np.ascontiguousarray(np.repeat(em.astype(np.int64), 2) * 2 + np.tile(np.asarray([0, 1], np.int64), F))
    total = int(seq_off[-1])
    seq = np.empty(max(total, 1), np.uint8)[:total]
    qual = np.empty(max(total, 1), np.uint8)[:total]
    for src, dst in ((cons.seq, seq), (cons.qual, qual)):  # the (family, end) rows, in record order
        src = np.ascontiguousarray(src, np.uint8)
        if n:
            lib.bsdc_rows_gather(n, _ptr(rows), _ptr(L), int(stride), _ptr(src), _ptr(seq_off), _ptr(dst), int(threads))
    return OutRecordsBam(
        flag=np.tile(np.asarray([77, 141], np.uint16), F), tid=np.full(n, -1, np.int32), pos=np.full(n, -1, np.int32),
        mapq=np.zeros(n, np.uint8), next_tid=np.full(n, -1, np.int32), next_pos=np.full(n, -1, np.int32),
        tlen=np.zeros(n, np.int32), names=names_t, cig_off=np.zeros(n + 1, np.int64),
        cigar=np.zeros(0, np.uint32), seq_off=seq_off, seq=seq, qual=qual, aux=auxs_t, aux2=tg)


def consensus_sharded(eng, raw: R.RawRecords, tags: bool, batch_bases: Optional[int] = None, dist=None):
    """pipeline.run_step5 over the ranks of `dist` (None = this process alone): every rank forms
    the same family plan, runs the batches shard.deal gives it on its own GPU, and rank 0 gets the
    consensus of all batches in plan order (shard.gather_in_order; other ranks get None).  A plan
    whose tool-2 extension partners straddle families runs on rank 0 alone (pipeline.run_step5's
    two-launch fallback)."""
    from . import pipeline, shard
    if dist is None or dist.get_world_size() == 1:
        return pipeline.run_step5(eng, raw, tags=tags, batch_bases=batch_bases)[0]
    rank, world = dist.get_rank(), dist.get_world_size()
    plan = pipeline.plan_families(raw, "full", eng.ref)
    if plan.split_ext:
        return pipeline.run_step5(eng, raw, tags=tags, batch_bases=batch_bases)[0] if rank == 0 else None
    ranges = pipeline.plan_ranges(plan, batch_bases)
    mine_idx = shard.deal(ranges, world, rank)
    parts = pipeline.run_ranges(eng, plan, [ranges[i] for i in mine_idx],
                                pipeline.MODE_CONVERT | pipeline.MODE_EXTEND | pipeline.MODE_VOTE, tags)
    got = shard.gather_in_order(dist, dict(zip(mine_idx, parts)), len(ranges))
    return pipeline.concat_consensus(got) if rank == 0 else None


def step5(in_bam: str, fasta: str, out_bam: Optional[str], engine=None, prefix: Optional[str] = None, threads: int = 0,
          level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True, batch_bases: Optional[int] = None,
          dist=None) -> dict:
    """Rules convert_Bstrain .. callduplex (main.snake.py:121-164) as one call on files; with
    `fastq`, also the following consensusduplex_to_fq rule (main.snake.py:167-177) straight from
    the consensus records (out_bam may then be None: no BAM round trip).  The stream runs as
    bounded device batches (batch_bases, pipeline.DEFAULT_BATCH_BASES); with `dist` the batches
    are shared by the ranks (one GPU each) and rank 0 writes the files."""
    from .device import Engine
    header, raw = read_bam(in_bam, threads)
    ref = read_fasta(fasta, header)
    own = engine is None
    eng = Engine(0) if own else engine
    try:
        eng.load_reference(ref)
        cons = consensus_sharded(eng, raw, tags and out_bam is not None, batch_bases, dist)
    finally:
        if own:
            eng.close()
    if cons is None:  # not rank 0
        return {"records_in": raw.n}
    recs = duplex_records(cons, raw, read_name_prefix(header) if prefix is None else prefix, threads)
    if out_bam is not None:
        write_bam(out_bam, output_header(header), recs, level, threads)
    if fastq is not None:
        write_fastq(fastq[0], fastq[1], recs, level, threads)
    return {"records_in": raw.n, "families": int(cons.status.shape[0]),
            "families_emitted": int(((cons.status & 1) != 0).sum()), "records_out": recs.n}


def step5_stream(in_bam: str, fasta: str, out_bam: Optional[str], engine=None, prefix: Optional[str] = None,
                 threads: int = 0, level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True,
                 chunk_bytes: int = DEFAULT_CHUNK_BYTES, slack: int = DEFAULT_SLACK,
                 batch_bases: Optional[int] = None, stats: Optional[dict] = None, gpu_bgzf: bool = False,
                 defer: Optional[int] = None, read_size: int = 8 << 20) -> dict:
    """step5 in bounded memory, pipelined (_stream_step); defer: the span past which a template is
    deferred (default DEFAULT_DEFER_SPAN; 0 = off); read_size: compressed bytes per refill."""
    return _public(_stream_step(in_bam, fasta, out_bam, engine, prefix, threads, level, fastq, tags, chunk_bytes,
                                slack, batch_bases, stats, gpu_bgzf, None, defer=defer, read_size=read_size))


def molecular_stream(in_bam: str, out_bam: Optional[str], engine=None, prefix: Optional[str] = None, threads: int = 0,
                     level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True,
                     chunk_bytes: int = DEFAULT_CHUNK_BYTES, batch_bases: Optional[int] = None,
                     stats: Optional[dict] = None, gpu_bgzf: bool = False, min_consensus_base_quality: int = 0) -> dict:
    """Rule call_consensus_reads_molecular (main.snake.py:46-55) in bounded memory: the same
    pipeline as step5_stream over a GroupReadsByUmi-ordered input cut between MI runs
    (stream_chunks(runs=True)); each chunk's runs are its consensus families (pipeline.molecular_records,
    the vote alone, --min-consensus-base-quality applied).  The output is byte-identical to
    molecular()'s whole-file path: no run straddles two chunks.  The reference's rule needs -Xmx100g
    (main.snake.py:54, README.md:83); this holds about six chunks."""
    return _public(_stream_step(in_bam, None, out_bam, engine, prefix, threads, level, fastq, tags, chunk_bytes,
                                DEFAULT_SLACK, batch_bases, stats, gpu_bgzf, int(min_consensus_base_quality)))


def _public(info: dict) -> dict:
    """The stream's info as the CLI prints it (JSON): the spliced keys become their count"""
    sp = info.pop("splices", None)
    info["spliced_families"] = 0 if sp is None else int(len(sp))
    return info


MINKEY = -(1 << 62)  # sort key of the pieces before every family (the header, a first range's start)


def _family_cuts(cons, raw, plan, splices, strict: bool, start: int = 0):
    """Output record indices where a chunk's BAM / FASTQ output is cut before each splice key, in
    order: (record index, key) per key used.  A family's key is its first record's coarse key
    (RawRecords.tc_key).  strict (the main stream): before the first family whose key exceeds the
    splice (no family lies within kDeferMargin of one); else (the spill's pass): before the first
    family whose key reaches the splice minus kDeferMargin (a deferred template's two records may
    estimate its key a few positions apart).  splices[start:] are tried; a key no family of the
    chunk reaches is left (-> cuts, the index of the first key left)."""
    F = int(cons.status.shape[0])
    if F == 0 or splices.shape[0] <= start:
        return [], start
    first = plan.order[plan.fam_off[:-1]]
    k0, k1 = raw.tc_key[first, 0], raw.tc_key[first, 1]
    em = np.zeros(F + 1, np.int64)
    em[1:] = np.cumsum((cons.status & 1) != 0)
    out, lo, j = [], 0, start
    while j < splices.shape[0]:
        s0, s1 = int(splices[j, 0]), int(splices[j, 1]) - (0 if strict else DEFER_MARGIN)
        hit = (k0 > s0) | ((k0 == s0) & ((k1 > s1) if strict else (k1 >= s1)))
        hit[:lo] = False
        if not hit.any():
            if not strict:  # (the pass's later chunks take it)
                break
            f = F
        else:
            f = int(np.argmax(hit))
        lo = max(lo, f)
        out.append((2 * int(em[lo]), (int(splices[j, 0]), int(splices[j, 1]))))
        j += 1
    return out, j


def _region_cuts(cons, raw, plan, prev: list) -> list:
    """Output record indices where a chunk's output is cut before the first family of each new key
    contig pair (a family's key: its first record's coarse key), keyed (pair, MINKEY); prev[0] =
    the pair of the family before the chunk (at first: that of the range's first piece's key)."""
    first = plan.order[plan.fam_off[:-1]]
    k0 = raw.tc_key[first, 0]
    em = np.zeros(k0.shape[0] + 1, np.int64)
    em[1:] = np.cumsum((cons.status & 1) != 0)
    before = np.empty_like(k0)
    before[0] = k0[0] if prev[0] is None else prev[0]
    before[1:] = k0[:-1]
    prev[0] = int(k0[-1])
    return [(2 * int(em[f]), (int(k0[f]), MINKEY)) for f in np.nonzero(k0 != before)[0]]


def _slice_records(recs: "OutRecordsBam", a: int, b: int) -> "OutRecordsBam":
    """Records a..b-1 as views (the encoders index the ragged fields by absolute offsets)."""
    return OutRecordsBam(flag=recs.flag[a:b], tid=recs.tid[a:b], pos=recs.pos[a:b], mapq=recs.mapq[a:b],
                         next_tid=recs.next_tid[a:b], next_pos=recs.next_pos[a:b], tlen=recs.tlen[a:b],
                         names=StringTable(recs.names.buf, recs.names.off[a:b + 1]), cig_off=recs.cig_off[a:b + 1],
                         cigar=recs.cigar, seq_off=recs.seq_off[a:b + 1], seq=recs.seq, qual=recs.qual,
                         aux=StringTable(recs.aux.buf, recs.aux.off[a:b + 1]),
                         aux2=StringTable(recs.aux2.buf, recs.aux2.off[a:b + 1]) if recs.aux2 is not None else None)


def pieces_of(marks, paths, phase: int, rank: int) -> list:
    """One output's pieces between its marks (_stream_step): (sort key, phase, rank, index, paths,
    starts, ends), ends of the last piece = the files' sizes."""
    out = []
    size = [os.path.getsize(x) if x else 0 for x in paths]
    for i, (offs, key) in enumerate(marks):
        end = list(marks[i + 1][0]) if i + 1 < len(marks) else size
        out.append((tuple(key), phase, rank, i, list(paths), list(offs), end))
    return out


def assemble(dst: str, pieces, k: int):
    """Output file k (0 the BAM, 1 / 2 the FASTQ pair) from the pieces in sort-key order, then one
    BGZF EOF block; written aside and renamed over dst."""
    tmp = dst + ".asm"
    with open(tmp, "wb") as out:
        for p in sorted(pieces, key=lambda x: (x[0], x[1], x[2], x[3])):
            path, a, b = p[4][k], p[5][k], p[6][k]
            if path is None or b <= a:
                continue
            with open(path, "rb") as f:
                f.seek(a)
                left = b - a
                while left > 0:
                    buf = f.read(min(left, 1 << 24))
                    if not buf:
                        raise RuntimeError("%s: short piece" % path)
                    out.write(buf)
                    left -= len(buf)
        out.write(EOF_BLOCK)
    os.replace(tmp, dst)


EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def write_spill_bam(dst: str, header: "BamHeader", spills: Sequence[str], level: int = 1, threads: int = 0) -> int:
    """The spill files' records (bsdc_bam_stream_spill entries) in file order as a BAM -> records."""
    data = b"".join(open(x, "rb").read() for x in spills if x and os.path.exists(x))
    recs, n = spill_sorted_records(data)
    del data
    w = BamWriter(dst, header, level)
    try:
        w.add_raw(recs, threads)
    finally:
        w.close(threads)
    return n


def _stream_step(in_bam: str, fasta: Optional[str], out_bam: Optional[str], engine, prefix: Optional[str],
                 threads: int, level: int, fastq: Optional[Tuple[str, str]], tags: bool, chunk_bytes: int, slack: int,
                 batch_bases: Optional[int], stats: Optional[dict], gpu_bgzf: bool,
                 molecular: Optional[int], rng=None, fragment: Optional[str] = None, runner=None,
                 range_stats: Optional[dict] = None, owner=None, spill: Optional[str] = None,
                 marks: Optional[list] = None, defer: Optional[int] = None, late_splices=None,
                 first_key=None, read_size: int = 8 << 20, regions: bool = False) -> dict:
    """step5 (molecular None) or step 1 (molecular = its --min-consensus-base-quality) in bounded
    memory, pipelined: a decoder thread cuts the next chunk of the
    coordinate-sorted input (stream_bam: inflate, split where no template or MI family straddles),
    a reader thread parses the chunk before, a planner thread forms the families of the one before
    that (C++ plan) and materializes its batches into pinned memory; this thread uploads a chunk's
    batches and runs them on the GPU; a builder thread builds
    the output records of the chunk before and a writer thread appends them to the BAM
    (BamWriter).  Peak host memory is about six chunks, whatever the file size.  The output is
    byte-identical to step5's (tests/test_stream.py): every chunk's TemplateCoordinate keys sort
    before the next chunk's, so the chunks' families in order are the whole file's.  gpu_bgzf: the
    BAM's and the FASTQ pair's blocks are deflated on the engine's GPU (GpuBgzf; the same records,
    other compressed bytes, files ≈4% larger).
    Deferred templates (step 5; defer = the span, default DEFAULT_DEFER_SPAN, 0 = off): a template
    whose other end lies far away or on another contig (bsdc_bam_stream_set_defer) would hold every
    family after its key in memory until the stream reaches that end.  Its records go to a spill
    file instead (with every family that may interleave with it), and the output is cut, at every
    deferred key, into pieces (marks).  At the end a second pass runs the spill's records (in file
    order, their own BAM; memory as their count) with the same keys (late_splices: each cut before
    the first family that reaches the key), and the pieces of both are assembled in key order: the
    same records as the whole file's.  Without deferred templates the output is written in place,
    as it always was.
    rank-parallel use (ranks.py): rng = the record range of the input to run (stream_chunks),
    range_stats its statistics once read, fragment = "first" / "next" (the output pieces a rank
    writes: BamWriter, FastqWriter), runner = a fleet-style runner (run_batch / run_chunk; the CPU
    stand-in of the tests) instead of an Engine, owner = the rank's key interval (stream_chunks),
    spill = the file the deferred records go to, marks = a list that receives the output's cut
    points ((BAM offset, FASTQ offsets x 2), sort key of the piece that starts there): ranks.py
    runs the second pass and the assembly; first_key = the sort key of the rank's first piece;
    regions (the ranks' passes) = also cut before the first family of every new key contig pair
    (a piece keyed (pair, MINKEY)): a rank does not register cross keys (bsdc_io.cpp), so the
    deferred families of a contig's cross keys go between those pieces."""
    import queue
    import threading
    import time

    from . import pipeline
    own = engine is None and runner is None
    # (a rank's engine may still be loading: ranks._LazyEngine; torch is imported with it)
    lazy = bool(getattr(engine, "lazy", False))
    if runner is None:
        if own:
            from .device import Engine
        eng = Engine(0) if own else engine
    else:
        eng = None
        if gpu_bgzf or molecular is not None:
            raise ValueError("a runner stream: step 5 with host deflate only")
    chunks: "queue.Queue" = queue.Queue(maxsize=1)
    outs: "queue.Queue" = queue.Queue(maxsize=1)
    err: list = []
    info = {"records_in": 0, "families": 0, "families_emitted": 0, "records_out": 0, "chunks": 0,
            "spilled_bytes": 0, "deferred_families": 0, "splices": []}
    # deferral (step 5): the spill file and the output's pieces
    dspan = 0 if molecular is not None else (DEFAULT_DEFER_SPAN if defer is None else int(defer))
    late = None if late_splices is None else np.asarray(late_splices, np.int64).reshape(-1, 2)
    lj = [0]  # (the spill's pass: the first deferred key not yet cut at)
    rk_prev = [None]  # (regions: the key contig pair of the last family written; set with k_first)
    tie = 0 if late is not None else 1  # (a spill piece sorts before the stream's piece of its key)
    solo = marks is None and late is None  # this call runs the spill's pass and the assembly itself
    mk = [] if marks is None else marks
    frag = "first" if (solo and dspan) else fragment
    # (the spill pass's first piece, before its first key, is empty: after the header in any case)
    k_first = tuple(first_key) if first_key is not None else (MINKEY, 0, 2 if late is not None else 1)
    rk_prev[0] = int(k_first[0])  # (a range whose first family lies in a later contig pair: cut before it)
    out0 = out_bam if out_bam is not None else fastq[0]
    spill_path = spill if spill is not None else \
        (os.path.join(os.path.dirname(os.path.abspath(out0)), ".%s.%d.%x.spill" % (os.path.basename(out0), os.getpid(),
                                                                                  id(info))) if dspan else None)
    splices_tail: list = []
    T = {"decode": 0.0, "plan": 0.0, "materialize": 0.0, "gpu": 0.0, "records": 0.0, "encode": 0.0,
         "gpu_wait": 0.0, "writer_wait": 0.0}
    G: dict = {}  # the GPU stage's host steps (pipeline.run_batches timing)
    R_: dict = {}  # the reader's steps (StreamChunk.decode timing)
    bufs = BufferPool()  # a chunk's record arrays, given back once its output is written
    first = {}
    stop = threading.Event()  # set on any failure: the decoder and planner stop at their next chunk

    raws: "queue.Queue" = queue.Queue(maxsize=1)

    def decoder():  # cuts the next chunk (inflate, split, family-complete selection) while the
        # reader thread parses the one before
        it = sw = None
        rs = range_stats if range_stats is not None else {}
        try:
            if dspan:
                sw = open(spill_path, "wb")
            it = stream_chunks(in_bam, threads, chunk_bytes, slack, read_size, runs=molecular is not None, rng=rng,
                               stats=rs, owner=owner, defer=dspan, keys=late is not None)
            while not stop.is_set():
                t0 = time.perf_counter()
                nxt = next(it, None)
                T["decode"] += time.perf_counter() - t0
                if nxt is None:
                    break
                if sw is not None and nxt.spill:
                    sw.write(nxt.spill)
                    info["spilled_bytes"] += len(nxt.spill)
                raws.put(nxt)
            if not stop.is_set():
                info["deferred_families"] = int(rs.get("deferred", 0))
                info["peak_buffered"] = int(rs.get("peak_buffered", 0))
            if sw is not None and not stop.is_set():
                tail = rs.pop("spill_tail", b"")
                sw.write(tail)
                info["spilled_bytes"] += len(tail)
                splices_tail.append(rs.pop("splices_tail", np.zeros((0, 2), np.int64)))
        except BaseException as e:  # noqa: BLE001 -- handed to the main thread
            err.append(e)
            stop.set()
        finally:
            if sw is not None:
                sw.close()
            if it is not None:
                it.close()  # (the stream is freed once every chunk is back)
            raws.put(None)

    parsed: "queue.Queue" = queue.Queue(maxsize=1)

    def reader():  # parses a chunk's records while the planner forms the families of the one before
        try:
            while True:
                ch = raws.get()
                if ch is None:
                    break
                if stop.is_set():
                    ch.discard()
                    continue  # drain to the decoder's None without parsing
                raw = ch.decode(threads, R_, bufs)[1]
                raw._splices = ch.splices  # (the deferred keys this chunk's output is cut before)
                parsed.put(raw)
        except BaseException as e:  # noqa: BLE001 -- handed to the main thread
            err.append(e)
            stop.set()
            while True:  # let the decoder finish
                ch = raws.get()
                if ch is None:
                    break
                ch.discard()
        finally:
            parsed.put(None)

    # the planner materializes chunk k's batches into pool k % 3: chunk k - 3 is done on the GPU
    # by then (the planner handed chunk k - 1 over only after the GPU stage took chunk k - 2).  A
    # loading engine's first chunks materialize into plain host arrays, the pools come with it
    def new_pools():
        from .device import PinnedPool
        return [PinnedPool() for _ in range(3)]
    pools = None if runner is not None else ([] if lazy else new_pools())

    def planner():  # forms a chunk's families and materializes its batches ahead of the GPU stage
        try:
            k = 0
            while True:
                raw = parsed.get()
                if raw is None:
                    break
                if stop.is_set():
                    continue  # drain to the reader's None without planning
                t0 = time.perf_counter()
                buf = raw._pool_buf
                if molecular is None:
                    plan = pipeline.plan_families(raw, "full", first["ref"])
                else:  # step 1: the chunk's MI runs are the families, the vote alone
                    raw = pipeline.molecular_records(raw)
                    plan = pipeline.plan_families(raw, "vote", family_order="mi-group")
                raw._pool_buf = buf
                t1 = time.perf_counter()
                fbs = None
                if not plan.split_ext:
                    images = None
                    if pools is not None and not pools and eng.ready():
                        pools.extend(new_pools())
                    if pools:
                        pool = pools[k % 3]
                        k += 1
                        pool.reset()
                        images = pool.images
                    fbs = pipeline.materialize_ranges(plan, pipeline.plan_ranges(plan, batch_bases), images)
                T["plan"] += t1 - t0
                T["materialize"] += time.perf_counter() - t1
                chunks.put((raw, plan, fbs))
        except BaseException as e:  # noqa: BLE001 -- handed to the main thread
            err.append(e)
            stop.set()
            while parsed.get() is not None:  # let the reader finish
                pass
        finally:
            chunks.put(None)

    recq: "queue.Queue" = queue.Queue(maxsize=1)  # built records -> encoder

    def builder():  # the output records of a chunk, while the encoder compresses the one before
        try:
            while True:
                t0 = time.perf_counter()
                item = outs.get()
                T["writer_wait"] += time.perf_counter() - t0
                if item is None:
                    break
                cons, raw, cuts = item
                t0 = time.perf_counter()
                recs = duplex_records(cons, raw, first["prefix"], threads, molecular=molecular is not None, pool=bufs)
                T["records"] += time.perf_counter() - t0
                back = [raw._pool_buf, getattr(recs.aux2, "_pool_buf", None)]
                del item, cons, raw
                recq.put((recs, back, cuts))
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            stop.set()
            while outs.get() is not None:  # drain so the main thread never blocks
                pass
        finally:
            recq.put(None)

    def writer():
        w = fq = None
        try:
            gz = GpuBgzf(eng.device) if gpu_bgzf and out_bam is not None else None
            gzf = GpuBgzf(eng.device) if gpu_bgzf and fastq is not None else None  # (one job in flight each)
            w = BamWriter(out_bam, output_header(first["header"]), level, gz, frag) if out_bam is not None else None
            fq = FastqWriter(fastq[0], fastq[1], level, gzf, frag is not None) if fastq is not None else None

            def cut(key):  # everything so far leaves as whole blocks; a piece with this key starts here
                bo = w.flush(threads) if w is not None else 0
                fo = fq.flush(threads) if fq is not None else (0, 0)
                mk.append(((bo, fo[0], fo[1]), key))
            mk.append(((0, 0, 0), k_first))  # (a first piece holds the header, if any)
            while True:
                item = recq.get()
                if item is None:
                    break
                recs, back, cuts = item
                t1 = time.perf_counter()
                a = 0
                for idx, key in cuts + [(recs.n, None)]:
                    part = recs if (a == 0 and idx == recs.n) else _slice_records(recs, a, idx)
                    if idx > a:
                        if w is not None:
                            w.add(part, threads)
                        if fq is not None:
                            fq.add(part, threads)
                    if key is not None:
                        cut((key[0], key[1], tie))
                    a = idx
                info["records_out"] += recs.n
                T["encode"] += time.perf_counter() - t1
                del item, recs
                for buf in back:  # (the chunk's records are written; nothing refers to their arrays)
                    bufs.give(buf)
            if w is not None:
                w.close(threads)
            if fq is not None:
                fq.close(threads)
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            stop.set()
            close_quietly(w, fq)
            while recq.get() is not None:  # drain so the builder never blocks
                pass

    # the header and the reference come first: the plan of a chunk needs the reference
    hdr0 = read_bam_header(in_bam)
    first["header"] = hdr0
    ref = read_fasta(fasta, hdr0) if molecular is None else None  # (step 1 converts nothing)
    first["ref"] = ref
    first["prefix"] = read_name_prefix(hdr0) if prefix is None else prefix
    import contextlib
    flags = contextlib.nullcontext() if molecular is None else eng.flags(min_consensus_base_quality=molecular)
    try:
        flags.__enter__()
    except BaseException:
        if own:
            eng.close()
        raise
    try:
        if ref is not None:
            (runner if runner is not None else eng).load_reference(ref)
        td = threading.Thread(target=decoder, daemon=True)
        tr = threading.Thread(target=reader, daemon=True)
        tp = threading.Thread(target=planner, daemon=True)
        tb = threading.Thread(target=builder, daemon=True)
        tw = threading.Thread(target=writer, daemon=True)
        td.start()
        tr.start()
        tp.start()
        tb.start()
        tw.start()
        mode = pipeline.MODE_CONVERT | pipeline.MODE_EXTEND | pipeline.MODE_VOTE if molecular is None else pipeline.MODE_VOTE
        drained = False
        try:
            while True:
                t0 = time.perf_counter()
                item = chunks.get()
                T["gpu_wait"] += time.perf_counter() - t0
                if item is None:
                    drained = True
                    break
                if stop.is_set():  # another stage failed: stop working, drain below
                    break
                raw, plan, fbs = item
                t0 = time.perf_counter()
                tg = tags and out_bam is not None  # the FASTQ pair carries no tags
                if runner is not None:
                    if fbs is None:
                        cons = runner.run_chunk(raw, tg, batch_bases)
                    else:
                        parts = []
                        for fb in fbs:
                            sub = R.take(raw, fb.src) if getattr(runner, "needs_raw", False) else None
                            parts.append(pipeline.consensus_from_output(fb, runner.run_batch(fb, mode, tg, sub)))
                        cons = pipeline.concat_consensus(parts)
                        del fbs, parts
                elif fbs is None:
                    cons = pipeline.run_step5(eng, raw, tags=tg, batch_bases=batch_bases)[0]
                else:
                    cons = pipeline.concat_consensus(pipeline.run_batches(eng, fbs, mode, tg, G))
                    del fbs
                T["gpu"] += time.perf_counter() - t0
                info["records_in"] += raw.n
                info["families"] += int(cons.status.shape[0])
                info["families_emitted"] += int(((cons.status & 1) != 0).sum())
                info["chunks"] += 1
                cuts = []
                if late is not None:  # the spill's pass: cut before the families of each deferred key
                    cuts, lj[0] = _family_cuts(cons, raw, plan, late, False, lj[0])
                elif getattr(raw, "_splices", None) is not None and raw._splices.shape[0]:
                    cuts, _ = _family_cuts(cons, raw, plan, raw._splices, True)
                    info["splices"].append(raw._splices)
                if regions and cons.status.shape[0]:
                    cuts = sorted(cuts + _region_cuts(cons, raw, plan, rk_prev))
                outs.put((cons, raw, cuts))
        except BaseException:
            stop.set()
            raise
        finally:
            if not drained:  # let the planner finish (it stops planning once `stop` is set)
                stop.set()
                while chunks.get() is not None:
                    pass
            outs.put(None)
            tb.join()
            tw.join()
            tp.join()
            tr.join()
            td.join()
        if not err:
            info["splices"] = np.concatenate(info["splices"] + splices_tail + [np.zeros((0, 2), np.int64)]) \
                if dspan else np.zeros((0, 2), np.int64)
            if solo and dspan:  # the deferred templates' pass and the assembly (or just the EOF blocks)
                _finish_deferred(in_bam, fasta, out_bam, fastq, eng if runner is None else None, runner, first["prefix"],
                                 threads, level, tags, chunk_bytes, slack, batch_bases, gpu_bgzf, mk, spill_path, info)
    finally:
        flags.__exit__(None, None, None)
        if own:
            eng.close()
        if solo and spill_path is not None and os.path.exists(spill_path):
            os.unlink(spill_path)
    if err:
        raise err[0]
    if stats is not None:
        stats.update({k: round(v, 4) for k, v in T.items()})
        stats.update({"gpu_" + k: round(v, 4) for k, v in G.items()})
        stats.update({"reader_" + k: round(v, 4) for k, v in R_.items()})
    return info


def _finish_deferred(in_bam, fasta, out_bam, fastq, eng, runner, prefix, threads, level, tags, chunk_bytes, slack,
                     batch_bases, gpu_bgzf, marks, spill_path, info):
    """One process's deferred templates: with none, the EOF blocks the fragment-mode writers left
    out; else the spill's records as their own BAM through the stream (no deferral; cut at every
    deferred key), then the pieces of both outputs assembled in key order."""
    paths = [out_bam, fastq[0] if fastq else None, fastq[1] if fastq else None]
    if info["splices"].shape[0] == 0 and info["spilled_bytes"] == 0:
        for x in paths:
            if x is not None:
                with open(x, "ab") as f:
                    f.write(EOF_BLOCK)
        return
    base = spill_path + ".p2"
    sb = base + ".bam"
    p2 = [base + ".out.bam" if out_bam is not None else None,
          base + ".1.fq.gz" if fastq else None, base + ".2.fq.gz" if fastq else None]
    try:
        info["deferred_records"] = write_spill_bam(sb, read_bam_header(in_bam), [spill_path], 1, threads)
        mk2: list = []
        inf2 = _stream_step(sb, fasta, p2[0], eng, prefix, threads, level, (p2[1], p2[2]) if fastq else None, tags,
                            chunk_bytes, slack, batch_bases, None, gpu_bgzf, None, fragment="next",
                            runner=runner, marks=mk2, defer=0, late_splices=info["splices"])
        for k in ("records_in", "families", "families_emitted", "records_out"):
            info[k] += inf2[k]
        pieces = pieces_of(marks, paths, 0, 0) + pieces_of(mk2, p2, 1, 0)
        for k in range(3):
            if paths[k] is not None:
                assemble(paths[k], pieces, k)
    finally:
        for x in [sb] + p2:
            if x is not None and os.path.exists(x):
                os.unlink(x)


def molecular(in_bam: str, out_bam: Optional[str], engine=None, prefix: Optional[str] = None, threads: int = 0,
              level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True,
              min_consensus_base_quality: int = 0) -> dict:
    """Rule call_consensus_reads_molecular (main.snake.py:46-55, fgbio CallMolecularConsensusReads)
    on files; with `fastq`, also consensus_to_fq_unfiltered (main.snake.py:58-67)."""
    from . import pipeline
    from .device import Engine
    header, raw = read_bam(in_bam, threads)
    own = engine is None
    eng = Engine(0) if own else engine
    try:
        cons, rm = pipeline.run_molecular(eng, raw, tags=tags and out_bam is not None,
                                          min_consensus_base_quality=min_consensus_base_quality)
    finally:
        if own:
            eng.close()
    recs = duplex_records(cons, rm, read_name_prefix(header) if prefix is None else prefix, threads, molecular=True)
    if out_bam is not None:
        write_bam(out_bam, output_header(header), recs, level, threads)
    if fastq is not None:
        write_fastq(fastq[0], fastq[1], recs, level, threads)
    return {"records_in": raw.n, "families": int(cons.status.shape[0]),
            "families_emitted": int(((cons.status & 1) != 0).sum()), "records_out": recs.n}
