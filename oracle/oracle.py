"""ctypes wrapper of the CPU restatement (oracle/bsdc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  The product path (bsseqconsensusreads_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BSDC_ORACLE_LIB: an alternative build of the same restatement (the sanitizer run, tests/sanitize/)
LIB = os.environ.get("BSDC_ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")

NT16 = "=ACMGRSVTWYHKDBN"
_NT16_ASCII = np.frombuffer(NT16.encode(), dtype=np.uint8)
_ASCII_NT16 = np.full(256, 15, np.uint8)
for _i, _c in enumerate(NT16):
    _ASCII_NT16[ord(_c)] = _i
    _ASCII_NT16[ord(_c.lower())] = _i
_ASCII_NT16[ord("U")] = _ASCII_NT16[ord("u")] = 8


class _Records(C.Structure):
    _fields_ = [("n", C.c_int64)] + [(k, C.c_void_p) for k in (
        "flag", "tid", "pos", "l_seq", "seq_off", "seq", "qual", "cig_off", "n_cig", "cigar", "mi_id",
        "mi_strand", "name_id", "next_tid", "next_pos", "tlen", "mc_off", "mc_n", "mc_cigar", "mi_lex", "name_lex",
        "lib_id")]


class _Reference(C.Structure):
    _fields_ = [("n_contig", C.c_int32), ("off", C.c_void_p), ("len", C.c_void_p), ("seq", C.c_void_p)]


class _Params(C.Structure):
    _fields_ = [("error_rate_pre_umi", C.c_double), ("error_rate_post_umi", C.c_double),
                ("min_input_base_quality", C.c_int32), ("consensus_call_overlapping_bases", C.c_int32),
                ("run_tools", C.c_int32), ("n_threads", C.c_int32), ("family_order", C.c_int32),
                ("keep_sources", C.c_int32), ("min_consensus_base_quality", C.c_int32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        lib.orc_run.restype = C.c_void_p
        lib.orc_run.argtypes = [C.POINTER(_Records), C.POINTER(_Reference), C.POINTER(_Params)]
        lib.orc_last_error.restype = C.c_char_p
        lib.orc_free.argtypes = [C.c_void_p]
        for fn in ("orc_n_records", "orc_total_bases", "orc_total_cigar"):
            getattr(lib, fn).restype = C.c_int64
            getattr(lib, fn).argtypes = [C.c_void_p, C.c_int]
        lib.orc_get_records.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 9
        lib.orc_n_families.restype = C.c_int64
        lib.orc_n_families.argtypes = [C.c_void_p]
        lib.orc_get_families.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.orc_max_cons_len.restype = C.c_int32
        lib.orc_max_cons_len.argtypes = [C.c_void_p]
        lib.orc_get_consensus.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 6
        lib.orc_get_ss.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 5
        lib.orc_tables.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_void_p]
        lib.orc_tables_fp64.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_void_p]
        lib.orc_det_expf.restype = C.c_float
        lib.orc_det_expf.argtypes = [C.c_float]
        lib.orc_sources_size.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        lib.orc_get_sources.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        lib.orc_check_agree.restype = C.c_int64
        lib.orc_check_agree.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        lib.bgzf_ref_block.restype = C.c_int
        lib.bgzf_ref_block.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        _lib = lib
    return _lib


class OracleError(RuntimeError):
    pass


@dataclass
class OracleRecords:
    src: np.ndarray
    pos: np.ndarray
    l_seq: np.ndarray
    seq_off: np.ndarray
    seq: np.ndarray   # nt16 codes
    qual: np.ndarray
    n_cig: np.ndarray
    cig_off: np.ndarray
    cigar: np.ndarray
    rd: np.ndarray
    la: np.ndarray

    def record(self, k: int):
        o, l = int(self.seq_off[k]), int(self.l_seq[k])
        c, m = int(self.cig_off[k]), int(self.n_cig[k])
        return dict(src=int(self.src[k]), pos=int(self.pos[k]), seq=self.seq[o:o + l], qual=self.qual[o:o + l],
                    cigar=self.cigar[c:c + m], rd=int(self.rd[k]), la=int(self.la[k]))


@dataclass
class OracleResult:
    tool1: OracleRecords
    tool2: OracleRecords
    fam_mi: np.ndarray
    status: np.ndarray      # 1 = consensus pair emitted
    cons_len: np.ndarray    # [F, 2]
    cons_seq: np.ndarray    # [F, 2, stride] nt16 codes
    cons_qual: np.ndarray   # [F, 2, stride]
    n_reads: np.ndarray
    seconds: float = 0.0    # wall time of orc_run alone
    fam_rec_off: np.ndarray = None  # [F + 1] family membership: fam_src[fam_rec_off[f]:fam_rec_off[f+1]]
    fam_src: np.ndarray = None      # input record index of each family record (family order)
    # single-strand reads per family and set (0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2) with the
    # consensus-tag column statistics: "len" [F, 4], "base" (nt16) / "qual" / "depth" / "err" [F, 4, stride]
    ss: dict = None
    # keep_sources=True: the source reads each set's vote saw -- "count" [F, 4] reads per (family,
    # set), then per read in family / set order "len", and flat "base" (nt16) / "qual" arrays
    sources: dict = None


def _ptr(a):
    return a.ctypes.data


def lex_ranks(strings, ids) -> np.ndarray:
    """rank[id] = byte-order rank of strings[id] over the ids in use (equal strings share a rank)."""
    ids = np.asarray(ids, np.int64)
    if hasattr(strings, "lex_key"):  # synthetic / decoded name tables order their own ids
        u = np.unique(ids[ids >= 0])
        rank = np.zeros(max(int(u[-1]) + 1 if u.shape[0] else 1, 1), np.int32)
        if u.shape[0]:
            _, rk = np.unique(strings.lex_key(u), return_inverse=True)
            rank[u] = rk
        return rank
    used = sorted(set(int(i) for i in np.unique(ids[ids >= 0])))
    rank = np.zeros(max(used[-1] + 1 if used else 1, 1), np.int32)
    b = {i: (strings[i] if isinstance(strings[i], bytes) else strings[i].encode()) for i in used}
    r, prev = -1, None
    for i in sorted(used, key=lambda i: b[i]):
        if prev is None or b[i] != prev:
            r += 1
            prev = b[i]
        rank[i] = r
    return rank


def run(raw, ref, pre=45.0, post=30.0, overlap=True, run_tools=True, threads=0,
        family_order="template-coordinate", keep_sources=False, min_consensus_base_quality=2) -> OracleResult:
    """raw: bsseqconsensusreads_amd.records.RawRecords; ref: records.Reference.
    family_order: "template-coordinate" (fgbio SortBam + consecutive-MI grouping) or "mi-group"
    (tool 2's first-seen MI groups).  min_consensus_base_quality: single-strand calls below it
    become (N, 2) -- 2 for step 5's duplex caller, 0 for step 1 (main.snake.py:54)."""
    lib = load()
    keep = []

    def arr(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        if a.size == 0:
            a = np.zeros(1, dt)
        keep.append(a)
        return _ptr(a)

    rr = _Records()
    rr.n = raw.n
    rr.flag = arr(raw.flag, np.uint16)
    rr.tid = arr(raw.tid, np.int32)
    rr.pos = arr(raw.pos, np.int32)
    rr.l_seq = arr(raw.l_seq, np.int32)
    rr.seq_off = arr(raw.seq_off, np.int64)
    rr.seq = arr(_NT16_ASCII[raw.seq], np.uint8)
    rr.qual = arr(raw.qual, np.uint8)
    rr.cig_off = arr(raw.cig_off, np.int64)
    rr.n_cig = arr(raw.n_cig, np.int32)
    rr.cigar = arr(raw.cigar, np.uint32)
    rr.mi_id = arr(raw.mi_id, np.int32)
    rr.mi_strand = arr(raw.mi_strand, np.int8)
    rr.name_id = arr(raw.name_id, np.int32)
    rr.next_tid = arr(raw.next_tid, np.int32)
    rr.next_pos = arr(raw.next_pos, np.int32)
    rr.tlen = arr(raw.tlen, np.int32)
    rr.mc_off = arr(raw.mc_off, np.int64)
    rr.mc_n = arr(raw.mc_n, np.int32)
    rr.mc_cigar = arr(raw.mc_cigar, np.uint32)
    rr.mi_lex = arr(lex_ranks(raw.mi_names, raw.mi_id), np.int32)
    rr.name_lex = arr(lex_ranks(raw.names, raw.name_id), np.int32)
    rr.lib_id = None

    # reference letters: the FASTA's own when kept, else the nt16 letters
    offs, lens, parts, o = [], [], [], 0
    for t, name in enumerate(ref.names):
        if ref.contig_off[t] < 0:
            offs.append(-1)
            lens.append(0)
            continue
        if name in ref.letters:
            b = np.frombuffer(ref.letters[name], dtype=np.uint8)
        else:
            co, cl = int(ref.contig_off[t]), int(ref.contig_len[t])
            lo, hi = co // 2, (co + cl + 1) // 2 + 1
            pk = ref.packed[lo:hi]
            codes = np.empty(2 * pk.shape[0], np.uint8)
            codes[0::2] = pk >> 4
            codes[1::2] = pk & 0xF
            codes = codes[co - 2 * lo: co - 2 * lo + cl]
            b = _NT16_ASCII[codes]
        offs.append(o)
        lens.append(len(b))
        parts.append(b)
        o += len(b)
    rf = _Reference()
    rf.n_contig = len(ref.names)
    rf.off = arr(np.asarray(offs, np.int64), np.int64)
    rf.len = arr(np.asarray(lens, np.int64), np.int64)
    rf.seq = arr(np.concatenate(parts) if parts else np.zeros(1, np.uint8), np.uint8)

    if family_order not in ("template-coordinate", "mi-group"):
        raise ValueError(family_order)
    p = _Params(pre, post, 0, int(overlap), int(run_tools), int(threads), int(family_order == "template-coordinate"),
                int(keep_sources), int(min_consensus_base_quality))
    t0 = time.perf_counter()
    h = lib.orc_run(C.byref(rr), C.byref(rf), C.byref(p))
    seconds = time.perf_counter() - t0
    if not h:
        raise OracleError(lib.orc_last_error().decode())
    try:
        outs = []
        for which in (1, 2):
            n = lib.orc_n_records(h, which)
            nb = lib.orc_total_bases(h, which)
            nc = lib.orc_total_cigar(h, which)
            src = np.zeros(max(n, 1), np.int64)
            pos = np.zeros(max(n, 1), np.int32)
            l_seq = np.zeros(max(n, 1), np.int32)
            seq = np.zeros(max(nb, 1), np.uint8)
            qual = np.zeros(max(nb, 1), np.uint8)
            n_cig = np.zeros(max(n, 1), np.int32)
            cig = np.zeros(max(nc, 1), np.uint32)
            rd = np.zeros(max(n, 1), np.int32)
            la = np.zeros(max(n, 1), np.int32)
            lib.orc_get_records(h, which, _ptr(src), _ptr(pos), _ptr(l_seq), _ptr(seq), _ptr(qual), _ptr(n_cig),
                                _ptr(cig), _ptr(rd), _ptr(la))
            so = np.zeros(n, np.int64)
            if n:
                so[1:] = np.cumsum(l_seq[:n])[:-1]
            co = np.zeros(n, np.int64)
            if n:
                co[1:] = np.cumsum(n_cig[:n])[:-1]
            outs.append(OracleRecords(src[:n], pos[:n], l_seq[:n], so, _ASCII_NT16[seq[:nb]], qual[:nb], n_cig[:n],
                                      co, cig[:nc], rd[:n], la[:n]))
        F = lib.orc_n_families(h)
        stride = max(int(lib.orc_max_cons_len(h)), 1)
        mi = np.zeros(max(F, 1), np.int32)
        st = np.zeros(max(F, 1), np.int32)
        ln = np.zeros(max(2 * F, 1), np.int32)
        bs = np.zeros(max(2 * F * stride, 1), np.uint8)
        qs = np.zeros(max(2 * F * stride, 1), np.uint8)
        nr = np.zeros(max(F, 1), np.int32)
        lib.orc_get_consensus(h, stride, _ptr(mi), _ptr(st), _ptr(ln), _ptr(bs), _ptr(qs), _ptr(nr))
        fro = np.zeros(F + 1, np.int64)
        fsrc = np.zeros(max(lib.orc_n_records(h, 2), 1), np.int64)
        lib.orc_get_families(h, _ptr(fro), _ptr(fsrc))
        sl = np.zeros(max(4 * F, 1), np.int32)
        sb = np.zeros(max(4 * F * stride, 1), np.uint8)
        sq = np.zeros(max(4 * F * stride, 1), np.uint8)
        sd = np.zeros(max(4 * F * stride, 1), np.int32)
        se = np.zeros(max(4 * F * stride, 1), np.int32)
        lib.orc_get_ss(h, stride, _ptr(sl), _ptr(sb), _ptr(sq), _ptr(sd), _ptr(se))
        sources = None
        if keep_sources:
            nrd, nbs = C.c_int64(0), C.c_int64(0)
            lib.orc_sources_size(h, C.byref(nrd), C.byref(nbs))
            cnt = np.zeros(max(4 * F, 1), np.int32)
            sln = np.zeros(max(nrd.value, 1), np.int32)
            sbs = np.zeros(max(nbs.value, 1), np.uint8)
            sqs = np.zeros(max(nbs.value, 1), np.uint8)
            lib.orc_get_sources(h, _ptr(cnt), _ptr(sln), _ptr(sbs), _ptr(sqs))
            sources = {"count": cnt[:4 * F].reshape(F, 4), "len": sln[:nrd.value],
                       "base": _ASCII_NT16[sbs[:nbs.value]], "qual": sqs[:nbs.value]}
        n4 = 4 * F * stride
        ss = {"len": sl[:4 * F].reshape(F, 4), "base": _ASCII_NT16[sb[:n4]].reshape(F, 4, stride),
              "qual": sq[:n4].reshape(F, 4, stride), "depth": sd[:n4].reshape(F, 4, stride),
              "err": se[:n4].reshape(F, 4, stride)}
        return OracleResult(outs[0], outs[1], mi[:F], st[:F], ln[:2 * F].reshape(F, 2),
                            _ASCII_NT16[bs[:2 * F * stride]].reshape(F, 2, stride) if F else np.zeros((0, 2, stride), np.uint8),
                            qs[:2 * F * stride].reshape(F, 2, stride), nr[:F], seconds, fro, fsrc[:int(fro[-1])], ss,
                            sources)
    finally:
        lib.orc_free(h)


def tables(pre=45.0, post=30.0):
    lib = load()
    lr = np.zeros(256, np.int64)
    thr = np.zeros(94, np.float32)
    lib.orc_tables(pre, post, _ptr(lr), _ptr(thr))
    return lr, thr


def tables_fp64(pre=45.0, post=30.0):
    """fgbio's per-read log-space terms (ln P(correct), ln P(error) / 3 per phred) in double precision:
    what the near-tie decision sums read by read."""
    lnc = np.zeros(256, np.float64)
    lne3 = np.zeros(256, np.float64)
    load().orc_tables_fp64(pre, post, _ptr(lnc), _ptr(lne3))
    return lnc, lne3


def det_expf(x: float) -> float:
    return float(load().orc_det_expf(x))


def check_agree_tables(qlo, dthr, thr, dmax) -> int:
    """First D where libbsdc's agreement tables disagree with this restatement, or -1."""
    qlo = np.ascontiguousarray(qlo, np.uint8)
    dthr = np.ascontiguousarray(dthr, np.int32)
    thr = np.ascontiguousarray(thr, np.float32)
    return int(load().orc_check_agree(_ptr(qlo), _ptr(dthr), _ptr(thr), int(dmax)))


def bgzf_block(data: bytes) -> bytes:
    """One BGZF block of `data` (<= 65280 bytes) by the restatement of the GPU encoder
    (bgzf_ref.c), CRC32 and ISIZE included; b"" when it would not fit (stored by the writer)."""
    lib = load()
    src = np.frombuffer(bytes(data) + b"\0" * 8, np.uint8)
    out = np.zeros(65536, np.uint8)
    n = lib.bgzf_ref_block(src.ctypes.data, len(data), out.ctypes.data)
    return out[:n].tobytes()


class _HostSlot:
    """a host byte buffer with the data_ptr() a pinned torch tensor has."""

    def __init__(self, n: int):
        self.a = np.zeros(max(n, 1), np.uint8)

    def data_ptr(self) -> int:
        return self.a.ctypes.data


class BgzfStandIn:
    """bam.GpuBgzf's interface on the CPU with bgzf_block: the BAM writer's GPU-compressed path
    (encode, take into a staging slot, submit / finish, CRC / ISIZE filled by the writer)
    exercised without a GPU."""

    def __init__(self):
        self.blocks = 0
        self.slots = [None, None]
        self.slot = 0
        self.job = None

    def staging(self, nbytes: int):
        self.slot ^= 1
        if self.slots[self.slot] is None or self.slots[self.slot].a.size < nbytes:
            self.slots[self.slot] = _HostSlot(nbytes)
        return self.slots[self.slot]

    def submit(self, raw, nblk: int):
        assert self.job is None
        self.job = self.compress(raw.data_ptr(), nblk * 65280)

    def finish(self):
        job, self.job = self.job, None
        return job

    def compress(self, data_ptr: int, nbytes: int):
        host = np.ctypeslib.as_array(C.cast(data_ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))
        parts, sizes = [], []
        for b in range(nbytes // 65280):
            blk = bgzf_block(host[b * 65280:(b + 1) * 65280].tobytes())
            if len(blk) and b % 7 == 3:  # every 7th block as if it did not fit: the writer deflates it
                blk = b""
            parts.append(blk)
            sizes.append(len(blk))
        self.blocks += len(sizes)
        packed = np.frombuffer(b"".join(parts) or b"\0", np.uint8).copy()
        return packed, np.asarray(sizes, np.int32)
