"""Device side of the step: family batches in HBM (torch tensors as plumbing), libbsdc launches.

The Engine owns one libbsdc context per GPU.  ``upload`` copies a FamilyBatch into HBM once;
``run`` enqueues the kernels on the current torch stream (so torch events time exactly them) and
``fetch`` brings the consensus (and the optional stage dump) back to the host.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from dataclasses import dataclass, replace
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib
from .batch import FamilyBatch, wide_rows
from .records import Reference


@dataclass
class ConsensusParams:
    """fgbio CallDuplexConsensusReads options, defaults from main.snake.py:163.
    min_consensus_base_quality: single-strand calls below it become (N, 2).  The duplex caller
    passes no such flag; fgbio's single-strand caller inside it masks below PhredScore.MinValue = 2
    (DESIGN.md 3.5).  Step 1 passes --min-consensus-base-quality=0 (main.snake.py:54):
    MOLECULAR_PARAMS."""

    error_rate_pre_umi: float = 45.0
    error_rate_post_umi: float = 30.0
    min_input_base_quality: int = 0
    consensus_call_overlapping_bases: bool = True
    min_reads: int = 0
    min_consensus_base_quality: int = 2

    def c_struct(self):
        return _lib.Params(self.error_rate_pre_umi, self.error_rate_post_umi, self.min_input_base_quality,
                           int(self.consensus_call_overlapping_bases), self.min_reads,
                           self.min_consensus_base_quality)


# fgbio CallMolecularConsensusReads as rule call_consensus_reads_molecular runs it (main.snake.py:54):
# --error-rate-pre-umi=45 --error-rate-post-umi=30 --min-input-base-quality=0
# --min-consensus-base-quality=0 --consensus-call-overlapping-bases=true (--min-reads=1: a column
# without an A/C/G/T read is a no-call, as in the duplex caller's single-strand caller)
MOLECULAR_PARAMS = ConsensusParams(min_consensus_base_quality=0)


def _dptr(t: torch.Tensor) -> int:
    return int(t.data_ptr())


class DeviceBatch:
    """A FamilyBatch resident in HBM plus its output buffers."""

    def __init__(self, fb: FamilyBatch, device: torch.device, dump: bool = False, tags: bool = False):
        self.fb = fb
        self.n_fam, self.n_rec = fb.n_fam, fb.n_rec
        self.device = device
        self.t: Dict[str, torch.Tensor] = {}
        for k, v in fb.device_arrays().items():
            a = np.ascontiguousarray(v)
            if a.size == 0:
                a = np.zeros(1, dtype=a.dtype)
            # torch has no uint32/uint16 arithmetic we need; move raw bytes.  Pinned sources (the
            # engine's staging images) copy asynchronously on the stream; the engine double-buffers
            # them, and the batch before is fetched (stream synchronized) before a buffer is refilled
            h = torch.from_numpy(a.view(np.uint8))
            self.t[k] = h.to(device, non_blocking=h.is_pinned())
        F, Rn = fb.n_fam, fb.n_rec
        self.stride = fb.stride
        self.status = torch.zeros(max(F, 1), dtype=torch.uint8, device=device)
        self.len = torch.zeros(max(2 * F, 1), dtype=torch.int16, device=device)
        self.seq = torch.zeros(max(F * self.stride, 16), dtype=torch.uint8, device=device)
        self.qual = torch.zeros(max(2 * F * self.stride, 16), dtype=torch.uint8, device=device)
        self.dump = dump
        if dump:
            cap = fb.n_slots + 16
            self.dump_pos = torch.zeros(max(Rn, 1), dtype=torch.int32, device=device)
            self.dump_len = torch.zeros(max(Rn, 1), dtype=torch.int16, device=device)
            self.dump_tags = torch.zeros(max(Rn, 1), dtype=torch.uint8, device=device)
            self.dump_seq = torch.zeros(cap, dtype=torch.uint8, device=device)
            self.dump_qual = torch.zeros(cap, dtype=torch.uint8, device=device)
        self.tags = tags
        if tags:  # single-strand reads + column statistics (BSDC_MODE_TAGS), rows (family, set)
            nss = max(4 * F * self.stride, 16)
            self.ss_len = torch.zeros(max(4 * F, 1), dtype=torch.int16, device=device)
            self.ss_base = torch.zeros(nss, dtype=torch.uint8, device=device)
            self.ss_qual = torch.zeros(nss, dtype=torch.uint8, device=device)
            self.ss_depth = torch.zeros(nss, dtype=torch.uint8, device=device)
            self.ss_err = torch.zeros(nss, dtype=torch.uint8, device=device)
            # families whose depths may pass a byte get exact u16 rows too (include/bsdc.h ss_wide)
            self.ss_wide, self.n_wide = wide_rows(fb.fam_off)
            if self.n_wide:
                nw = 4 * self.n_wide * self.stride
                self.t["ss_wide"] = torch.from_numpy(self.ss_wide.view(np.uint8)).to(device)
                self.ss_wdepth = torch.zeros(nw, dtype=torch.int16, device=device)
                self.ss_werr = torch.zeros(nw, dtype=torch.int16, device=device)
        # HBM scratch: arenas of the large buckets beyond the LDS budget, one region per bucket (the
        # bucket dispatches run concurrently on the library's side streams), the split families'
        # fallback arenas and their parts' sums (FamilyBatch.scratch_layout; + slack: dword reads
        # may run a few bytes past the last arena, their bytes masked).  Every byte a kernel reads
        # there it wrote first: no zero fill
        need, _, poff = fb.scratch_layout()
        self.scratch = torch.empty(need, dtype=torch.uint8, device=device) if need else None
        self._b = _lib.FamilyBatchC()
        b = self._b
        b.n_rec, b.n_fam = Rn, F
        for k in ("fam_off", "rec", "rec_win", "cig_off", "cig_info", "cigar", "rt", "seq", "qual",
                  "small_fams", "large_fams", "split_parts", "split_part_recs", "split_fams"):
            setattr(b, k, _dptr(self.t[k]))
        b.n_split_parts, b.n_split_fams = int(fb.split_parts.shape[0]), int(fb.split_fams.shape[0])
        b.split_part_arena, b.split_partial_off = int(fb.split_part_arena), int(poff)
        for q in range(_lib.SMALL_BUCKETS):
            b.n_small[q] = int(fb.small_buckets[q].shape[0])
            b.small_arena[q] = int(fb.small_arenas[q])
        for q in range(_lib.LARGE_BUCKETS):
            b.n_large[q] = int(fb.large_buckets[q].shape[0])
            b.large_arena[q] = int(fb.large_arenas[q])
        b.max_len = fb.max_len
        self._o = _lib.ConsensusC()
        o = self._o
        o.stride = self.stride
        o.status, o.len, o.seq, o.qual = _dptr(self.status), _dptr(self.len), _dptr(self.seq), _dptr(self.qual)
        if dump:
            o.dump_pos, o.dump_len, o.dump_tags = _dptr(self.dump_pos), _dptr(self.dump_len), _dptr(self.dump_tags)
            o.dump_seq, o.dump_qual = _dptr(self.dump_seq), _dptr(self.dump_qual)
        o.scratch = _dptr(self.scratch) if self.scratch is not None else None
        if tags:
            o.ss_len, o.ss_base, o.ss_qual = _dptr(self.ss_len), _dptr(self.ss_base), _dptr(self.ss_qual)
            o.ss_depth, o.ss_err = _dptr(self.ss_depth), _dptr(self.ss_err)
            if self.n_wide:
                o.ss_wide = _dptr(self.t["ss_wide"])
                o.ss_wdepth, o.ss_werr = _dptr(self.ss_wdepth), _dptr(self.ss_werr)

    def release_host(self):
        """Drop the host copy of the batch (the device copy stays resident)."""
        self.fb = None

    def fetch_lengths(self):
        """-> (status [F], len [F, 2]): the small outputs only (bench bookkeeping)."""
        F = self.n_fam
        return (self.status[:F].cpu().numpy(),
                self.len[:2 * F].cpu().numpy().view(np.uint16).astype(np.int32).reshape(F, 2))

    def fetch(self, alloc=None):
        """-> dict of numpy arrays (consensus and, if dumped, the post-tool records).  The copies
        are queued together on the current stream into pinned host memory (torch's caching host
        allocator), then one synchronize.  With alloc(nbytes) -> uint8 array (a fleet worker's
        shared segment) the outputs land in that buffer instead, so they leave the worker by name."""
        F = self.n_fam
        t = {"status": self.status[:F], "len": self.len[:2 * F], "seq": self.seq[:F * self.stride],
             "qual": self.qual[:2 * F * self.stride]}
        n = 4 * F * self.stride
        if self.tags:
            t.update(ss_len=self.ss_len[:4 * F], ss_base=self.ss_base[:n], ss_qual=self.ss_qual[:n],
                     ss_depth=self.ss_depth[:n], ss_err=self.ss_err[:n])
            if self.n_wide:
                t.update(ss_wdepth=self.ss_wdepth, ss_werr=self.ss_werr)
        Rn = self.n_rec
        if self.dump:
            t.update(dump_pos=self.dump_pos[:Rn], dump_len=self.dump_len[:Rn], dump_tags=self.dump_tags[:Rn],
                     dump_seq=self.dump_seq, dump_qual=self.dump_qual)
        if alloc is None:
            h = {k: v.to("cpu", non_blocking=True) for k, v in t.items()}
            torch.cuda.current_stream(self.device).synchronize()
            a = {k: v.numpy() for k, v in h.items()}
        else:
            sizes = {k: (v.numel() * v.element_size() + 255) // 256 * 256 for k, v in t.items()}
            buf = alloc(max(1, sum(sizes.values())))
            a, o = {}, 0
            for k, v in t.items():
                nb = v.numel() * v.element_size()
                dst = torch.from_numpy(buf[o:o + nb]).view(v.dtype)
                dst.copy_(v)
                a[k] = dst.numpy()
                o += sizes[k]
            torch.cuda.current_stream(self.device).synchronize()
        out = {
            "status": a["status"],
            "len": a["len"].view(np.uint16).astype(np.int32).reshape(F, 2),
            "seq": a["seq"].reshape(F, 2, self.stride // 2),
            "qual": a["qual"].reshape(F, 2, self.stride),
            "stride": self.stride,
        }
        if self.tags:
            out["ss_len"] = a["ss_len"].view(np.uint16).astype(np.int32).reshape(F, 4)
            out["ss_base"] = a["ss_base"].reshape(F, 4, self.stride)
            out["ss_qual"] = a["ss_qual"].reshape(F, 4, self.stride)
            out["ss_depth"] = a["ss_depth"].reshape(F, 4, self.stride)
            out["ss_err"] = a["ss_err"].reshape(F, 4, self.stride)
            out["ss_wide"] = self.ss_wide
            W = self.n_wide
            out["ss_wdepth"] = a["ss_wdepth"].view(np.uint16).reshape(W, 4, self.stride) if W else \
                np.zeros((0, 4, self.stride), np.uint16)
            out["ss_werr"] = a["ss_werr"].view(np.uint16).reshape(W, 4, self.stride) if W else \
                np.zeros((0, 4, self.stride), np.uint16)
        if self.dump:
            out["dump_pos"] = a["dump_pos"]
            out["dump_len"] = a["dump_len"].view(np.uint16).astype(np.int32)
            out["dump_tags"] = a["dump_tags"]
            out["dump_seq"] = a["dump_seq"]
            out["dump_qual"] = a["dump_qual"]
        return out


class PinnedPool:
    """A pinned host arena for the family images of one chunk's batches (materialize's `images`,
    bump-allocated): the streaming step materializes a whole chunk ahead of the GPU stage into
    one pool, the batches upload asynchronously from it, and the pool is reset for a later chunk
    once every upload from it is done (bam.step5_stream keeps three in rotation)."""

    SEGMENT = 64 << 20

    def __init__(self):
        self.segs = []  # pinned uint8 tensors; the last one is being filled
        self.used = 0  # bytes of the last segment handed out
        self.total = 0  # bytes handed out since the reset

    def images(self, n_slots: int):
        nq = n_slots
        ns = n_slots // 2 + 64
        need = (ns + 255) // 256 * 256 + nq
        if not self.segs or self.used + need > self.segs[-1].numel():
            self.segs.append(torch.empty(max(need, self.SEGMENT), dtype=torch.uint8, pin_memory=True))
            self.used = 0
        seg = self.segs[-1]
        a = self.used
        b = a + (ns + 255) // 256 * 256
        self.used = (b + nq + 255) // 256 * 256
        self.total += need
        return seg[a:a + ns].numpy(), seg[b:b + nq].numpy()

    def reset(self):
        """every batch materialized from the pool has been uploaded: hand its bytes out again
        (a pool that spilled over several segments becomes one that holds the largest chunk)."""
        if len(self.segs) > 1:
            size = int(max(self.total, sum(t.numel() for t in self.segs)) * 1.25)
            self.segs = [torch.empty(size, dtype=torch.uint8, pin_memory=True)]
        self.used = 0
        self.total = 0


class Engine:
    """One libbsdc context on one GPU."""

    def __init__(self, device_index: int = 0, params: Optional[ConsensusParams] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU: the bsdc product path runs on MI355X only (no CPU fallback)")
        self.lib = _lib.load()
        self.device_index = device_index
        self.device = torch.device("cuda", device_index)
        self.params = params or ConsensusParams()
        self._stage = [None, None]  # pinned family-image staging buffers (stage_images)
        self._stage_i = 0
        p = self.params.c_struct()
        h = C.c_void_p()
        rc = self.lib.bsdc_ctx_create(device_index, C.byref(p), C.byref(h))
        if rc != 0:
            raise RuntimeError("bsdc_ctx_create failed (%d)" % rc)
        self.ctx = h
        self.ref: Optional[Reference] = None

    def set_params(self, params: ConsensusParams):
        """Replace the context's flags (bsdc_ctx_set_params); later launches use them."""
        p = params.c_struct()
        self._check(self.lib.bsdc_ctx_set_params(self.ctx, C.byref(p)), "bsdc_ctx_set_params")
        self.params = params

    @contextlib.contextmanager
    def flags(self, **changes):
        """`with engine.flags(min_consensus_base_quality=0): ...` -- the engine runs with these
        flags inside the block and its own afterwards (one context serving step 1 and step 5)."""
        old = self.params
        if all(getattr(old, k) == v for k, v in changes.items()):
            yield self
            return
        self.set_params(replace(old, **changes))
        try:
            yield self
        finally:
            self.set_params(old)

    def stage_images(self, n_slots: int):
        """Pinned host arrays (seq, qual) for the next batch's family images (materialize's
        `images`), alternating between two buffer pairs that grow on demand: a batch's images
        upload asynchronously while the next one is filled (pipeline.run_ranges)."""
        i = self._stage_i
        self._stage_i ^= 1
        st = self._stage[i]
        if st is None or st[1].numel() < n_slots:
            cap = int(n_slots * 1.25) + 4096
            st = (torch.empty(cap // 2 + 64, dtype=torch.uint8, pin_memory=True),
                  torch.empty(cap, dtype=torch.uint8, pin_memory=True))
            self._stage[i] = st
        return st[0].numpy(), st[1].numpy()

    def close(self):
        if self.ctx:
            self.lib.bsdc_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError("%s failed (%d): %s" % (what, rc, self.lib.bsdc_last_error(self.ctx).decode()))

    def load_reference(self, ref: Reference):
        packed = np.ascontiguousarray(ref.packed)
        off = np.ascontiguousarray(ref.contig_off, dtype=np.int64)
        ln = np.ascontiguousarray(ref.contig_len, dtype=np.int64)
        rc = self.lib.bsdc_load_reference(self.ctx, packed.ctypes.data, ref.n_nibbles, off.ctypes.data,
                                          ln.ctypes.data, len(ref.names))
        self._check(rc, "bsdc_load_reference")
        self.ref = ref

    def upload(self, fb: FamilyBatch, dump: bool = False, tags: bool = False) -> DeviceBatch:
        with torch.cuda.device(self.device):
            return DeviceBatch(fb, self.device, dump, tags)

    def run(self, db: DeviceBatch, mode: int, stream: Optional[torch.cuda.Stream] = None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = self.lib.bsdc_run(self.ctx, C.byref(db._b), C.byref(db._o), mode, C.c_void_p(s.cuda_stream))
        self._check(rc, "bsdc_run")

    def tables(self):
        lr = np.zeros(256, np.int64)
        thr = np.zeros(94, np.float32)
        self._check(self.lib.bsdc_get_tables(self.ctx, lr.ctypes.data, thr.ctypes.data), "bsdc_get_tables")
        return lr, thr
