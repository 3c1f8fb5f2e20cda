"""ctypes binding of the C++ family formation (include/bsdc_host.h, csrc/bsdc_host.cpp, built into
libbsdc_io.so): batch.plan_families / batch.materialize for the step-5 modes ('full' and 'vote').

The numpy statements in batch.py (plan_families_py / materialize_py) stay as the restatement the
C++ is tested against (tests/test_host_plan.py) and as the path of the tool-only modes ('convert',
'extend') the file-level tools use.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import records as R

_P = C.c_void_p
PLAN_FULL, PLAN_VOTE = 0, 1
EMISSING_MI = -61
SMALL_BUCKETS_N, LARGE_BUCKETS_N = 8, 6  # BSDC_SMALL_BUCKETS, BSDC_LARGE_BUCKETS


class _Records(C.Structure):
    _fields_ = [("n", C.c_int64)] + [(k, _P) for k in (
        "flag", "tid", "pos", "l_seq", "seq_off", "seq", "qual", "cig_off", "n_cig", "cigar", "next_tid", "next_pos",
        "tlen", "name_id", "mi_id", "mi_strand", "mc_off", "mc_n", "mc_cigar", "mi_rank", "name_rank")]


class _Reference(C.Structure):
    _fields_ = [("n_contig", C.c_int64), ("contig_off", _P), ("contig_len", _P), ("packed", _P)]


class _PlanArrays(C.Structure):
    _fields_ = [(k, _P) for k in ("order", "fam_off", "fam_mi", "t2_rank", "fam_split", "conv", "ext_right", "ext_left",
                                  "rd_in", "partner_raw", "sL", "L", "kfirst", "kn")]


class _PlanView(C.Structure):
    _fields_ = [("n_fam", C.c_int64)] + [(k, _P) for k in (
        "order", "fam_off", "conv", "ext_right", "ext_left", "rd_in", "partner_raw", "sL", "L", "kfirst", "kn")]


class _BatchSizes(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n_rec", "n_fam", "n_slots", "n_bases", "n_cigar_max")] + \
               [("max_len", C.c_int32)]


class _BatchArrays(C.Structure):
    _fields_ = [(k, _P) for k in ("seq", "qual", "rec", "rec_win", "rt", "cig_off", "cig_info", "cigar", "src",
                                  "fam_off", "fam_entry", "need_l", "img", "cls", "large_caps")]


_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    from .bam import _load as load_io
    lib = load_io()
    if not hasattr(lib, "bsdc_plan_families"):
        raise RuntimeError("libbsdc_io.so lacks the host family formation (bsdc_host.cpp): run __graft_entry__.build()")
    lib.bsdc_plan_families.argtypes = [C.POINTER(_Records), C.POINTER(_Reference), C.c_int32, C.c_int32, C.c_int32,
                                       C.POINTER(_P)]
    lib.bsdc_plan_families.restype = C.c_int32
    lib.bsdc_plan_sizes.argtypes = [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.bsdc_plan_copy.argtypes = [_P, C.POINTER(_PlanArrays)]
    lib.bsdc_plan_free.argtypes = [_P]
    lib.bsdc_materialize_prepare.argtypes = [C.POINTER(_Records), C.POINTER(_Reference), C.POINTER(_PlanView), C.c_int64,
                                             C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.POINTER(_P),
                                             C.POINTER(_BatchSizes)]
    lib.bsdc_materialize_prepare.restype = C.c_int32
    lib.bsdc_materialize_fill.argtypes = [_P, C.POINTER(_BatchArrays), C.POINTER(C.c_int64)]
    lib.bsdc_materialize_fill.restype = C.c_int32
    lib.bsdc_batch_free.argtypes = [_P]
    lib.bsdc_host_last_error.restype = C.c_char_p
    lib.bsdc_host_error_record.restype = C.c_int64
    lib.bsdc_split_count.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p,
                                     C.c_int32]
    lib.bsdc_split_count.restype = C.c_int64
    lib.bsdc_split_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_int32]
    lib.bsdc_split_fill.restype = None
    lib.bsdc_split_move.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                    C.c_int32]
    lib.bsdc_split_move.restype = None
    _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_P)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class _RecordsView:
    """RawRecords as the C struct, holding the contiguous arrays alive."""

    def __init__(self, raw: R.RawRecords, with_ranks: bool):
        from .batch import lex_rank
        self.keep = []

        def k(a, dt):
            a = _c(a, dt)
            self.keep.append(a)
            return _p(a)

        s = _Records()
        s.n = raw.n
        s.flag = k(raw.flag, np.uint16)
        for f, dt in (("tid", np.int32), ("pos", np.int32), ("l_seq", np.int32), ("seq_off", np.int64),
                      ("seq", np.uint8), ("qual", np.uint8), ("cig_off", np.int64), ("n_cig", np.int32),
                      ("cigar", np.uint32), ("next_tid", np.int32), ("next_pos", np.int32), ("tlen", np.int32),
                      ("name_id", np.int32), ("mi_id", np.int32), ("mi_strand", np.int8), ("mc_off", np.int64),
                      ("mc_n", np.int32), ("mc_cigar", np.uint32)):
            a = getattr(raw, f)
            if a.shape[0] == 0:  # a valid pointer for empty stores
                a = np.zeros(1, dt)
            setattr(s, f, k(a, dt))
        if with_ranks and raw.n:
            s.mi_rank = k(lex_rank(raw.mi_names, np.maximum(raw.mi_id, 0)), np.int64)
            s.name_rank = k(lex_rank(raw.names, raw.name_id), np.int64)
        self.s = s


def _ref_struct(ref: Optional[R.Reference], keep: list):
    if ref is None:
        return None
    s = _Reference()
    s.n_contig = len(ref.names)
    for f, a in (("contig_off", _c(ref.contig_off, np.int64)), ("contig_len", _c(ref.contig_len, np.int64)),
                 ("packed", _c(ref.packed if ref.packed.shape[0] else np.zeros(1, np.uint8), np.uint8))):
        keep.append(a)
        setattr(s, f, _p(a))
    return s


def _err(lib):
    return lib.bsdc_host_last_error().decode(errors="replace")


def plan_families(raw: R.RawRecords, mode: str = "full", ref: Optional[R.Reference] = None,
                  family_order: str = "template-coordinate", n_threads: int = 0):
    """batch.plan_families in C++ (modes 'full' / 'vote')."""
    from .batch import FamilyPlan, MissingMITag
    if mode not in ("full", "vote"):
        raise ValueError("native plan: mode 'full' or 'vote', not %r" % mode)
    if family_order not in ("template-coordinate", "mi-group"):
        raise ValueError(family_order)
    lib = _load()
    tc = family_order == "template-coordinate"
    rv = _RecordsView(raw, with_ranks=tc)
    keep = []
    rs = _ref_struct(ref, keep)
    h = _P()
    rc = lib.bsdc_plan_families(C.byref(rv.s), C.byref(rs) if rs is not None else None,
                                PLAN_FULL if mode == "full" else PLAN_VOTE, int(tc), int(n_threads), C.byref(h))
    if rc == EMISSING_MI:
        k = int(lib.bsdc_host_error_record())
        raise MissingMITag("%s does not have MI tag." % raw.qname(k).decode())
    if rc != 0:
        raise ValueError(_err(lib))
    try:
        nr, nf = C.c_int64(), C.c_int64()
        lib.bsdc_plan_sizes(h, C.byref(nr), C.byref(nf))
        nr, nf, n = nr.value, nf.value, raw.n
        out = dict(order=np.empty(nr, np.int64), fam_off=np.empty(nf + 1, np.int64), fam_mi=np.empty(nf, np.int32),
                   t2_rank=np.empty(nr, np.int64), fam_split=np.empty(nf, np.uint8), conv=np.empty(n, np.uint8),
                   ext_right=np.empty(n, np.uint8), ext_left=np.empty(n, np.uint8), rd_in=np.empty(n, np.uint8),
                   partner_raw=np.empty(n, np.int64), sL=np.empty(n, np.int64), L=np.empty(n, np.int64),
                   kfirst=np.empty(n, np.int64), kn=np.empty(n, np.int64))
        pa = _PlanArrays(**{k: _p(v) for k, v in out.items()})
        lib.bsdc_plan_copy(h, C.byref(pa))
    finally:
        lib.bsdc_plan_free(h)
    for k in ("fam_split", "conv", "ext_right", "ext_left", "rd_in"):
        out[k] = out[k].view(bool)
    return FamilyPlan(raw=raw, mode=mode, ref=ref, **out)


def materialize(plan, f0: int, f1: int, small_cap: int, n_threads: int = 0, images=None):
    """batch.materialize in C++ (plans of modes 'full' / 'vote').  images(n_slots) -> (seq, qual):
    caller-owned uint8 arrays of at least n_slots / 2 and n_slots bytes for the family images
    (e.g. pinned staging buffers, Engine.stage_images); the fill writes every byte of them."""
    from . import batch as B
    if plan.mode not in ("full", "vote"):
        raise ValueError("native materialize: mode 'full' or 'vote', not %r" % plan.mode)
    lib = _load()
    raw = plan.raw
    rv = _RecordsView(raw, with_ranks=False)
    keep = []
    rs = _ref_struct(plan.ref, keep)
    pvk = {}
    for f, dt in (("order", np.int64), ("fam_off", np.int64), ("conv", np.uint8), ("ext_right", np.uint8),
                  ("ext_left", np.uint8), ("rd_in", np.uint8), ("partner_raw", np.int64), ("sL", np.int64),
                  ("L", np.int64), ("kfirst", np.int64), ("kn", np.int64)):
        a = getattr(plan, f)
        a = _c(a.view(np.uint8) if a.dtype == bool else a, dt)
        if a.shape[0] == 0:
            a = np.zeros(1, dt)
        pvk[f] = a
    pv = _PlanView(n_fam=plan.n_fam, **{k: _p(v) for k, v in pvk.items()})
    h = _P()
    sz = _BatchSizes()
    rc = lib.bsdc_materialize_prepare(C.byref(rv.s), C.byref(rs) if rs is not None else None, C.byref(pv), int(f0),
                                      int(f1), int(plan.mode == "full"), int(small_cap), int(n_threads), C.byref(h),
                                      C.byref(sz))
    if rc != 0:
        raise ValueError(_err(lib))
    try:
        nr, nf, n_slots = sz.n_rec, sz.n_fam, sz.n_slots
        if images is not None:
            seq_img, qual_img = images(n_slots)
            seq_img, qual_img = seq_img[:n_slots // 2], qual_img[:n_slots]
        else:
            seq_img, qual_img = np.empty(n_slots // 2, np.uint8), np.empty(n_slots, np.uint8)
        a = dict(seq=seq_img, qual=qual_img,
                 rec=np.empty((nr, 4), np.uint32), rec_win=np.empty((nr, 2), np.uint32), rt=np.empty(4 * nr, np.int32),
                 cig_off=np.empty(nr, np.uint32), cig_info=np.empty(nr, np.uint32),
                 cigar=np.empty(max(sz.n_cigar_max, 1), np.uint32), src=np.empty(nr, np.int64),
                 fam_off=np.empty(nf + 1, np.uint32), fam_entry=np.empty((nf, 4), np.uint32),
                 need_l=np.empty(nf, np.int64), img=np.empty(nf, np.int64), cls=np.empty(nf, np.int8))
        caps = np.asarray(B.LARGE_BUCKETS, np.int64)
        ba = _BatchArrays(large_caps=_p(caps), **{k: _p(v) for k, v in a.items()})
        nc = C.c_int64()
        rc = lib.bsdc_materialize_fill(h, C.byref(ba), C.byref(nc))
        if rc != 0:
            raise ValueError(_err(lib))
    finally:
        lib.bsdc_batch_free(h)
    nc = nc.value
    cls = a["cls"].astype(np.int64)
    img = a["img"]
    fam_off = a["fam_off"]
    fam_sizes = np.diff(fam_off.astype(np.int64))
    nsb = B.SMALL_BUCKETS
    buckets, arenas = [], []
    capped = False
    for q, cap in enumerate(nsb):  # the same bucket walk as batch.materialize_py
        if capped:
            buckets.append(np.zeros(0, np.uint32))
            arenas.append(16)
            continue
        cap = min(cap, small_cap)
        buckets.append(np.nonzero(cls == q)[0].astype(np.uint32))
        arenas.append(int(cap))
        capped = cap == small_cap
    lbuckets, larenas = [], []
    for q in range(LARGE_BUCKETS_N):
        lf = np.nonzero(cls == SMALL_BUCKETS_N + q)[0]
        lf = lf[np.argsort(-img[lf], kind="stable")]  # largest image first (batch.py)
        e = np.zeros((lf.shape[0], 4), np.int64)
        e[:, 0] = lf
        e[:, 1] = fam_off[lf]
        e[:, 2] = fam_sizes[lf]
        e[:, 3] = img[lf]
        lbuckets.append(e.astype(np.uint32))
        if q < LARGE_BUCKETS_N - 1:
            larenas.append(int(B.LARGE_BUCKETS[q]))
        else:
            larenas.append(int(B.round16(a["need_l"][lf].max())) if lf.shape[0] else 16)
    rec = a["rec"]
    order = a["src"]
    r0, r1 = int(plan.fam_off[f0]), int(plan.fam_off[f1])
    return B.FamilyBatch(
        fam_off=fam_off, rec_off=rec[:, 0].copy(), fam_entry=a["fam_entry"], rec_pos=rec[:, 1].view(np.int32).copy(),
        rec_lenflag=rec[:, 2].copy(), rec_tid=raw.tid[order].astype(np.int32), rec_link=rec[:, 3].copy(),
        rec_win=a["rec_win"], cig_off=a["cig_off"], cig_info=a["cig_info"],
        cigar=a["cigar"][:nc] if nc else np.zeros(1, np.uint32), rt=a["rt"], seq=a["seq"], qual=a["qual"],
        small_buckets=buckets, small_arenas=arenas, large_buckets=lbuckets, large_arenas=larenas,
        max_len=int(sz.max_len), src=order, fam_mi=plan.fam_mi[f0:f1].astype(np.int32), n_bases=int(sz.n_bases),
        n_slots=int(n_slots), t2_rank=plan.t2_rank[r0:r1], split_ext=bool(plan.fam_split[f0:f1].any()))


def enabled() -> bool:
    """The C++ family formation is the default; BSDC_HOST_PLAN=numpy selects the numpy statement."""
    return os.environ.get("BSDC_HOST_PLAN", "native") != "numpy"
