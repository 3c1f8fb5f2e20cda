"""Host-side family formation: RawRecords -> the device family batch (include/bsdc.h).

Everything here is record bookkeeping that needs no base or quality value -- which records the two
tools keep, soft-clip stripping, MI grouping, the 4-record pairing plan and the template mates --
so the kernel only ever sees records that reach the vote:

* tool 1 dispatch (tools/1.convert_AG_to_CT.py:70-80): flags {0,99,147} pass, {1,83,163} are
  converted unless their cigar has I, D or H, every other flag is dropped;
* tool 2 (tools/2.extend_gap.py:155-186): hard-clipped records dropped (:160-161), soft clips
  stripped (:168-176, identical to tool 1's own strip at :81-83), a missing/empty MI raises
  (:179-180), groups keyed by MI.split('/')[0] in first-seen order; groups of exactly four
  (:114-115) pair (99,163) and (83,147) and are emitted in the order 163, 99, 83, 147 with any
  other flag dropped (:123-138);
* family formation for the vote: one family per tool-2 group (DESIGN.md section 3.7 on how this
  relates to fgbio's TemplateCoordinate grouping).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _lib
from . import records as R

LINK_MATE_NONE = 0xFFFF
LINK_AB = 1 << 16
LINK_BA = 1 << 17
LINK_COMPLEX = 1 << 18
LINK_RT = 1 << 19
LINK_CONVERT = 1 << 20
LINK_EXT_RIGHT = 1 << 21
LINK_EXT_LEFT = 1 << 22
LINK_PARTNER_SHIFT = 23
LINK_RD_IN = 1 << 25
LINK_USABLE = 1 << 26

MODE_CONVERT, MODE_EXTEND, MODE_VOTE, MODE_DUMP = 1, 2, 4, 8

# small families run one per wavefront with their arena in LDS, in buckets of these arena sizes
SMALL_BUCKETS = (3072, 4096, 5120, 6144, 8192, 12288, 16384, 24576)  # BSDC_SMALL_BUCKETS classes
SMALL_ARENA_CAP = 24576  # the largest small-family arena (profiles/r05/README.md: small-arena cap A/B)
# route_small_cap: a batch whose small families are mostly ones with arenas above MID_ARENA_CAP
# sends those to k_large (SMALL_ROUTE = False: never)
MID_ARENA_CAP = 16384
SMALL_ROUTE = True
LDS_TABLES = 1024 + 1024 + 384 + 2048 + 192  # kTabBytes (csrc/bsdc_kernels.hip)
# large families run one per 256-thread workgroup, in buckets of these LDS arena sizes; the last
# bucket (anything larger) keeps its arenas in HBM scratch
LARGE_LDS_MAX = 158912  # BSDC_LARGE_LDS_MAX: 160 KB - the tables - the kernel's other LDS
# the largest arena that still fits k = 5, 4, 3, 2, 1 workgroups per CU (5 is the VGPR limit)
LARGE_BUCKETS = tuple((160 * 1024 // k - LDS_TABLES - 256) // 16 * 16 for k in (5, 4, 3, 2, 1))  # + 1 scratch bucket
assert LARGE_BUCKETS[-1] == LARGE_LDS_MAX
# k_large part mode (include/bsdc.h split_parts): the families of the 1-per-CU class and of the
# HBM-scratch bucket are cut into parts whose arena fits the 5-per-CU class (profiles/r04/ab_g,
# ab_h: smaller parts keep more workgroups in flight; cutting the 2-per-CU class too loses);
# PART_CAP = 0 turns it off
PART_CAP = LARGE_BUCKETS[0]
MAX_PART_REC = 254  # a part's per-set sums stay int32 and its read counts fit a byte
# the first large bucket whose families are cut into parts: 4 = the 1-per-CU class and the
# HBM-scratch bucket (profiles/r05/README.md: split-from A/B)
SPLIT_FROM = len(LARGE_BUCKETS) - 1


def round16(x):
    return (np.asarray(x, dtype=np.int64) + 15) & ~np.int64(15)


def ref_chunks(max_len):
    """16-B chunks that cover one converted record's packed reference window (mirror of the kernel)."""
    return (15 + (int(max_len) + 4) // 2 + 15) // 16


def small_arena_bytes(n, img, nconv, complex_ops, max_len):
    """Mirror of SmallLayout (csrc/bsdc_kernels.hip) / bsdc_small_arena_bytes: the image, the
    descriptors, lc[4], then the largest of the phase-local regions sharing one span."""
    n = np.asarray(n, dtype=np.int64)
    ws = 32 * ref_chunks(max_len)
    cops = np.asarray(complex_ops, dtype=np.int64)
    ow = int(round16(int(max_len) + 2))
    R = 2 * np.asarray(img, dtype=np.int64) + round16(4 * n) + 16 + round16(n)
    e_ref = R + np.asarray(nconv, dtype=np.int64) * ws
    simp = R + round16(16 * n) + round16(n) + 2 * round16(2 * n)
    e_f = simp + np.where(cops > 0, round16(4 * (cops + 4 * n)) + 256, 0)  # (+ filter_group's scratch)
    e_v = R + 8 * ow
    return np.maximum(np.maximum(e_ref, e_f), e_v)


def large_arena_bytes(n, slot_bytes, max_len, complex_ops):
    """Mirror of ArenaLayout (csrc/bsdc_kernels.hip) / bsdc_family_arena_bytes."""
    n = np.asarray(n, dtype=np.int64)
    ssw = round16(np.asarray(max_len, dtype=np.int64) + 2)
    # RecMeta per record + the converted-record list, or (vote) the second wave part's column sums,
    # ORs and read counts: 44 B per column (bsdc_layout::kVoteRegionPerCol)
    total = np.maximum(round16(n * 48) + round16(2 * n), 44 * ssw) + round16(n * 8) + 8 * ssw
    cops = np.asarray(complex_ops, dtype=np.int64)
    total = total + np.where(cops > 0, round16(4 * (cops + 4 * n)) + 512, 0)  # (+ filter_group's scratch, X and Y)
    total = total + round16(np.asarray(slot_bytes, dtype=np.int64))
    return total


class MissingMITag(ValueError):
    pass


@dataclass
class FamilyBatch:
    # ---- device arrays (include/bsdc.h bsdc_family_batch) ----
    fam_off: np.ndarray      # u32 [F+1]
    rec_off: np.ndarray      # u32 [R] slot start (nibble index into seq == byte index into qual)
    rec_pos: np.ndarray      # i32
    rec_lenflag: np.ndarray  # u32
    rec_tid: np.ndarray      # i32 (host only)
    rec_link: np.ndarray     # u32
    rec_win: np.ndarray      # u32 [R, 2] converted records: reference window start nibble, valid nibbles
    cig_off: np.ndarray      # u32
    cig_info: np.ndarray     # u32
    cigar: np.ndarray        # u32
    rt: np.ndarray           # i32 [4R]
    seq: np.ndarray          # u8 packed nt16, slot layout
    qual: np.ndarray         # u8, slot layout
    small_buckets: List[np.ndarray]  # 4 lists of family ids (u32), one per LDS arena size
    small_arenas: List[int]
    large_buckets: List[np.ndarray]  # BSDC_LARGE_BUCKETS lists of entries u32 [n, 4]: family, first record, n_rec, image bytes
    large_arenas: List[int]
    fam_entry: np.ndarray    # u32 [F, 4] small-kernel list entry of each family
    max_len: int
    # ---- host bookkeeping ----
    src: np.ndarray          # i64 [R] input record index
    fam_mi: np.ndarray       # i32 [F] MI id of each family
    n_bases: int
    n_slots: int
    t2_rank: np.ndarray      # i64 [R] tool-2 output position of each batch record
    split_ext: bool          # a tool-2 extension partner sits in another family (see build_family_batch)
    # ---- k_large part mode (split_hbm_bucket; include/bsdc.h) ----
    split_parts: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.uint32))  # u32 [P, 4]
    split_part_recs: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.uint32))  # u32 [PR, 4]
    split_fams: np.ndarray = field(default_factory=lambda: np.zeros((0, 8), np.uint32))   # u32 [S, 8], arena offsets relative
    split_part_arena: int = 16

    @property
    def n_rec(self) -> int:
        return int(self.rec_off.shape[0])

    @property
    def n_fam(self) -> int:
        return int(self.fam_off.shape[0]) - 1

    @property
    def stride(self) -> int:
        return int(round16(self.max_len + 2))

    @property
    def small_fams(self) -> np.ndarray:
        return np.concatenate(self.small_buckets).astype(np.uint32)

    @property
    def large_fams(self) -> np.ndarray:
        """u32 [n_large, 4] list entries of every large bucket, in order."""
        return np.concatenate(self.large_buckets).astype(np.uint32).reshape(-1, 4)

    def scratch_layout(self):
        """HBM scratch of the batch (bsdc_consensus.scratch): the arenas of the large buckets beyond
        the LDS budget, the split families' fallback arenas, the parts' sums.  -> (total bytes, split
        arena base, partial sums offset)."""
        hbm = sum(int(b.shape[0]) * a for b, a in zip(self.large_buckets, self.large_arenas)
                  if b.shape[0] and a > LARGE_LDS_MAX)
        base = int(round16(hbm))
        sf = self.split_fams
        arenas = int(sf[:, 7].astype(np.int64).sum()) if sf.shape[0] else 0
        poff = int(round16(base + arenas))
        npart = int(self.split_parts.shape[0])
        psz = int(round16(32 * npart)) + npart * 4 * self.stride * 24 if npart else 0
        total = poff + psz
        return (total + 256 if total else 0), base, poff

    def device_arrays(self):
        rec = np.stack([self.rec_off, self.rec_pos.view(np.uint32), self.rec_lenflag, self.rec_link], axis=1)
        d = {"fam_off": self.fam_off, "rec": np.ascontiguousarray(rec, dtype=np.uint32),
             "rec_win": np.ascontiguousarray(self.rec_win, dtype=np.uint32)}
        for k in ("cig_off", "cig_info", "cigar", "rt", "seq", "qual", "large_fams"):
            d[k] = getattr(self, k)
        d["small_fams"] = np.ascontiguousarray(self.fam_entry[self.small_fams.astype(np.int64)]).reshape(-1) \
            if self.small_fams.shape[0] else np.zeros(4, np.uint32)
        d["split_parts"] = np.ascontiguousarray(self.split_parts, np.uint32).reshape(-1)
        d["split_part_recs"] = np.ascontiguousarray(self.split_part_recs, np.uint32).reshape(-1)
        sf = np.array(self.split_fams, np.uint32).reshape(-1, 8)
        if sf.shape[0]:  # fallback arena offsets: scratch-absolute, in 16-byte units
            sf[:, 6] += np.uint32(self.scratch_layout()[1] // 16)
        d["split_fams"] = sf.reshape(-1)
        return d


def _per_record_ops(raw: R.RawRecords):
    n = raw.n
    rec = np.repeat(np.arange(n, dtype=np.int64), raw.n_cig)
    ops = (raw.cigar & 0xF).astype(np.int64)
    lens = (raw.cigar >> 4).astype(np.int64)
    j = np.arange(ops.shape[0], dtype=np.int64) - raw.cig_off[rec] if ops.shape[0] else np.zeros(0, np.int64)
    return rec, ops, lens, j


def _has_op(rec, ops, n, op):
    return np.bincount(rec[ops == op], minlength=n)[:n] > 0


def tool1_plan(raw: R.RawRecords):
    """tools/1.convert_AG_to_CT.py:70-80 -> (pass_through, convert) masks."""
    n = raw.n
    rec, ops, _, _ = _per_record_ops(raw)
    f = raw.flag.astype(np.int64)
    idh = _has_op(rec, ops, n, R.OP_I) | _has_op(rec, ops, n, R.OP_D) | _has_op(rec, ops, n, R.OP_H)
    pas = np.isin(f, (0, 99, 147))
    conv = np.isin(f, (1, 83, 163)) & ~idh
    return pas, conv


def _softclip_strip(raw: R.RawRecords):
    """remove_softclips (tools/2.extend_gap.py:30-52): (lead S, trailing S, first kept op, kept op count)."""
    n = raw.n
    nc = raw.n_cig.astype(np.int64)
    has = nc > 0
    co = raw.cig_off.astype(np.int64)
    first = np.where(has, raw.cigar[np.minimum(co, max(raw.cigar.shape[0] - 1, 0))] if raw.cigar.shape[0] else 0, 0)
    first = np.asarray(first, dtype=np.int64)
    fS = has & ((first & 0xF) == R.OP_S)
    sL = np.where(fS, first >> 4, 0)
    rem = nc - fS
    lasti = co + nc - 1
    last = np.where(has, raw.cigar[np.clip(lasti, 0, max(raw.cigar.shape[0] - 1, 0))] if raw.cigar.shape[0] else 0, 0)
    last = np.asarray(last, dtype=np.int64)
    lS = (rem > 0) & ((last & 0xF) == R.OP_S)
    sR = np.where(lS, last >> 4, 0)
    l0 = raw.l_seq.astype(np.int64)
    a = np.maximum(l0 - sL, 0)
    L = np.where(sR > 0, np.maximum(a - sR, 0), a)
    kfirst = fS.astype(np.int64)
    kn = rem - lS
    return sL, L, kfirst, kn


def _clips_reflen(cig: np.ndarray, off: np.ndarray, cnt: np.ndarray):
    """Per record of a cigar store (ops at cig[off : off + cnt], cnt <= 0 = none): leading S/H
    length, trailing S/H length, reference-consuming length."""
    n = cnt.shape[0]
    cnt = np.where(cnt > 0, cnt, 0).astype(np.int64)
    one = cnt == 1
    if one.any():  # one-op cigars (the common 150M) without the per-op expansion
        lead, trail, reflen = np.zeros(n, np.int64), np.zeros(n, np.int64), np.zeros(n, np.int64)
        c1 = cig[np.where(one, off, 0).astype(np.int64)]
        op1, ln1 = (c1 & 0xF).astype(np.int64), (c1 >> 4).astype(np.int64)
        reflen[one] = np.where(np.isin(op1, R.REF_CONSUMING), ln1, 0)[one]
        lead[one] = np.where(np.isin(op1, (R.OP_S, R.OP_H)), ln1, 0)[one]  # a lone clip leads
        many = np.nonzero(cnt > 1)[0]
        if many.shape[0]:
            lm_, tm_, rm_ = _clips_reflen(cig, np.asarray(off)[many], cnt[many])
            lead[many], trail[many], reflen[many] = lm_, tm_, rm_
        return lead, trail, reflen
    tot = int(cnt.sum())
    if tot == 0:
        z = np.zeros(n, np.int64)
        return z, z.copy(), z.copy()
    rec = np.repeat(np.arange(n, dtype=np.int64), cnt)
    start = np.cumsum(cnt) - cnt
    j = np.arange(tot, dtype=np.int64) - start[rec]
    c = cig[np.repeat(np.where(cnt > 0, off, 0).astype(np.int64), cnt) + j]
    op = (c & 0xF).astype(np.int64)
    ln = (c >> 4).astype(np.int64)
    clip = np.isin(op, (R.OP_S, R.OP_H))
    refc = np.isin(op, R.REF_CONSUMING)
    reflen = np.bincount(rec[refc], weights=ln[refc], minlength=n)[:n].astype(np.int64)
    nc = np.cumsum(~clip)                       # non-clip ops up to and including this one
    upto = nc - np.where(start > 0, nc[np.maximum(start - 1, 0)], 0)[rec]
    before = upto - (~clip)
    after = np.bincount(rec[~clip], minlength=n)[:n][rec] - upto
    lm = clip & (before == 0)
    tm = clip & (after == 0) & ~lm
    lead = np.bincount(rec[lm], weights=ln[lm], minlength=n)[:n].astype(np.int64)
    trail = np.bincount(rec[tm], weights=ln[tm], minlength=n)[:n].astype(np.int64)
    return lead, trail, reflen


def _mc_clips_reflen(raw: R.RawRecords, idx: np.ndarray):
    """MC cigars of records `idx`: (leading S/H length, trailing S/H length, reference length); a
    clip op counts as leading when no non-clip op precedes it and as trailing when none follows
    (an all-clip MC counts as both -- fgbio's mate-end arithmetic on an unusable mate)."""
    idx = np.asarray(idx, np.int64)
    m = idx.shape[0]
    cnt = np.where(raw.mc_off[idx] >= 0, raw.mc_n[idx], 0).astype(np.int64)
    tot = int(cnt.sum())
    z = np.zeros(m, np.int64)
    if tot == 0:
        return z, z.copy(), z.copy()
    rec = np.repeat(np.arange(m, dtype=np.int64), cnt)
    first = np.cumsum(cnt) - cnt
    j = np.arange(tot, dtype=np.int64) - first[rec]
    c = raw.mc_cigar[np.repeat(np.where(cnt > 0, raw.mc_off[idx], 0), cnt) + j]
    op = (c & 0xF).astype(np.int64)
    ln = (c >> 4).astype(np.int64)
    refm = np.isin(op, R.REF_CONSUMING)
    mref = np.bincount(rec[refm], weights=ln[refm], minlength=m)[:m].astype(np.int64)
    clip = np.isin(op, (R.OP_S, R.OP_H))
    ncum = np.cumsum(~clip)
    base = np.where(first > 0, ncum[np.maximum(first - 1, 0)], 0)
    upto = ncum - base[rec]                       # non-clip ops up to and including this one
    before = upto - (~clip)
    after = np.bincount(rec[~clip], minlength=m)[:m][rec] - upto
    lm = clip & (before == 0)
    tm = clip & (after == 0)
    lead = np.bincount(rec[lm], weights=ln[lm], minlength=m)[:m].astype(np.int64)
    trail = np.bincount(rec[tm], weights=ln[tm], minlength=m)[:m].astype(np.int64)
    return lead, trail, mref


def mate_unclipped(raw: R.RawRecords):
    """Mate unclipped (start, end) from PNEXT and the MC tag (stale after tools 1/2); PNEXT alone
    without MC."""
    lead, trail, mref = _clips_reflen(raw.mc_cigar, raw.mc_off, np.where(raw.mc_off >= 0, raw.mc_n, 0))
    np_ = raw.next_pos.astype(np.int64)
    has = raw.mc_off >= 0
    return np.where(has, np_ - lead, np_), np.where(has, np_ + mref - 1 + trail, np_)


def predict_rd(raw: R.RawRecords, ref: R.Reference, sel: np.ndarray, sL: np.ndarray, L: np.ndarray) -> np.ndarray:
    """Tool 1's RD (tools/1.convert_AG_to_CT.py:157-170) of converted records `sel`, from the input
    bases and the reference alone: the last output base is C iff the last input base (the seed
    ref[0] for an empty read) is C with ref = C G at (L', L'+1) -- the rule at :134-150 with no next
    base -- and RD = that C before a reference G."""
    sel = np.asarray(sel, np.int64)
    if sel.shape[0] == 0:
        return np.zeros(0, bool)
    tid = raw.tid[sel].astype(np.int64)
    np0 = np.maximum(raw.pos[sel].astype(np.int64) - 1, 0)
    nt = len(ref.names)
    okt = (tid >= 0) & (tid < nt)
    ti = np.clip(tid, 0, max(nt - 1, 0))
    coff = np.where(okt, ref.contig_off[ti], -1) if nt else np.full(sel.shape[0], -1)
    clen = np.where(okt, ref.contig_len[ti], 0) if nt else np.zeros(sel.shape[0], np.int64)
    Ls = L[sel].astype(np.int64)
    Lp = Ls + 1
    avail = np.where(coff >= 0, np.clip(clen - np0, 0, Lp + 1), 0)

    def refnib(i):
        ok = i < avail
        idx = np.where(ok, coff + np0 + i, 0)
        b = ref.packed[np.minimum(idx >> 1, max(ref.packed.shape[0] - 1, 0))] if ref.packed.shape[0] else np.zeros_like(idx)
        nib = np.where(idx & 1, b & 0xF, b >> 4)
        return np.where(ok, nib, 15)

    lastpos = raw.seq_off[sel] + sL[sel] + Ls - 1
    last = np.where(Ls > 0, raw.seq[np.clip(lastpos, 0, max(raw.seq.shape[0] - 1, 0))], refnib(np.zeros_like(Ls)))
    return (last == 2) & (refnib(Lp - 1) == 2) & (refnib(Lp) == 4)


def lex_rank(strings, ids: np.ndarray) -> np.ndarray:
    """A key per element of ids that orders them as strings[id] sort in byte order."""
    ids = np.asarray(ids, np.int64)
    from .bam import StringTable, table_ranks
    if isinstance(strings, StringTable):  # a decoded BAM's packed table: ranked in C++
        return table_ranks(strings)[ids] if ids.shape[0] else np.zeros(0, np.int64)
    if hasattr(strings, "lex_key"):  # synthetic names: computed, not materialised
        return strings.lex_key(ids)
    if ids.shape[0] == 0:
        return np.zeros(0, np.int64)
    u, inv = np.unique(ids, return_inverse=True)
    a = np.array([strings[int(i)] if isinstance(strings[int(i)], bytes) else strings[int(i)].encode() for i in u],
                 dtype=object).astype(bytes)
    _, rk = np.unique(a, return_inverse=True)
    return rk.astype(np.int64)[inv]


def template_coordinate_order(raw: R.RawRecords, recs: np.ndarray, us: np.ndarray, ue: np.ndarray,
                              mate_us: np.ndarray, mate_ue: np.ndarray) -> np.ndarray:
    """fgbio SortBam -s TemplateCoordinate (main.snake.py:152; SURVEY.md 8a row 7, parity
    unpinned) of records `recs` (raw indices) whose current unclipped ends are us / ue: the
    stable permutation by (tid, mate tid, unclipped 5' pos, mate unclipped 5' pos, strands,
    library, MI base, name, upper-of-pair), the template's lower end first.  Mate fields are the
    input's (stale), one library."""
    fl = raw.flag[recs].astype(np.int64)
    neg = (fl & 16) != 0
    t1 = raw.tid[recs].astype(np.int64)
    p1 = np.where(neg, ue, us)
    paired = ((fl & 1) != 0) & ((fl & 8) == 0)
    big = np.int64(np.iinfo(np.int32).max)
    n2 = paired & ((fl & 32) != 0)
    t2 = np.where(paired, raw.next_tid[recs].astype(np.int64), big)
    p2 = np.where(paired, np.where(n2, mate_ue[recs], mate_us[recs]), big)
    lower = (t1 < t2) | ((t1 == t2) & ((p1 < p2) | ((p1 == p2) & (neg <= n2))))
    T1, T2 = np.where(lower, t1, t2), np.where(lower, t2, t1)
    P1, P2 = np.where(lower, p1, p2), np.where(lower, p2, p1)
    N1, N2 = np.where(lower, neg, n2), np.where(lower, n2, neg)
    mi = lex_rank(raw.mi_names, raw.mi_id[recs])
    nm = lex_rank(raw.names, raw.name_id[recs])
    return np.lexsort((np.arange(recs.shape[0]), ~lower, nm, mi, N2, N1, P2, P1, T2, T1))


@dataclass
class FamilyPlan:
    """Family formation over a whole record stream, before any per-record device array exists:
    which records reach the kernels, in which order, grouped into which families, and the tool-1 /
    tool-2 roles.  ``materialize`` turns any contiguous family range of it into a device batch, so a
    stream larger than one batch (32-bit slot offsets, HBM budget) runs as a sequence of batches
    whose concatenated output equals the one-batch output."""

    raw: R.RawRecords
    mode: str
    ref: Optional[R.Reference]
    order: np.ndarray        # i64 [R] input record of each plan record, family order
    fam_off: np.ndarray      # i64 [F + 1]
    fam_mi: np.ndarray       # i32 [F]
    t2_rank: np.ndarray      # i64 [R] tool-2 output position of each plan record
    conv: np.ndarray         # bool [n] per input record: tool 1 converts it (this launch)
    ext_right: np.ndarray    # bool [n] tool 2 prepends its partner's first base
    ext_left: np.ndarray     # bool [n] tool 2 appends its partner's last base (if RD)
    partner_raw: np.ndarray  # i64 [n] tool-2 extension partner, -1 = none
    rd_in: np.ndarray        # bool [n] RD of an already converted input
    sL: np.ndarray           # i64 [n] leading soft clip stripped
    L: np.ndarray            # i64 [n] length after the strip
    kfirst: np.ndarray       # i64 [n] first kept cigar op
    kn: np.ndarray           # i64 [n] kept cigar ops
    fam_split: np.ndarray    # bool [F] a record's tool-2 extension partner is outside its family

    @property
    def n_fam(self) -> int:
        return int(self.fam_off.shape[0]) - 1

    @property
    def split_ext(self) -> bool:
        return bool(self.fam_split.any())

    def fam_bases(self) -> np.ndarray:
        """Bases per family (the size measure shard.plan_batches balances)."""
        if self.order.shape[0] == 0:
            return np.zeros(self.n_fam, np.int64)
        cs = np.concatenate([[0], np.cumsum(self.L[self.order] + 2)])
        return cs[self.fam_off[1:]] - cs[self.fam_off[:-1]]


def build_family_batch(raw: R.RawRecords, mode: str = "full", ref: Optional[R.Reference] = None,
                       small_cap: Optional[int] = None, family_order: str = "template-coordinate") -> FamilyBatch:
    """mode: 'full' (raw step-5 input: tools 1+2 then the vote), 'convert' (tool 1 alone: one
    family per converted record), 'extend' (tool-1 output: tool 2 alone), 'vote' (tool-2 output).
    family_order ('full' / 'vote'): 'template-coordinate' -- the vote's families are the runs of one
    MI base in fgbio TemplateCoordinate order of the tool-2 records (SortBam, main.snake.py:152,
    then the duplex caller's grouping), records in that order; 'mi-group' -- tool 2's MI groups.
    The whole stream as one batch: materialize(plan_families(...))."""
    plan = plan_families(raw, mode, ref, family_order)
    return materialize(plan, 0, plan.n_fam, small_cap)


def plan_families(raw: R.RawRecords, mode: str = "full", ref: Optional[R.Reference] = None,
                  family_order: str = "template-coordinate") -> FamilyPlan:
    """Family formation of build_family_batch (see there), without the device arrays: the C++
    statement (hostplan, csrc/bsdc_host.cpp) for the step-5 modes, this module's numpy statement
    (plan_families_py) for the tool-only modes or with BSDC_HOST_PLAN=numpy."""
    from . import hostplan
    if mode in ("full", "vote") and hostplan.enabled():
        return hostplan.plan_families(raw, mode, ref, family_order)
    return plan_families_py(raw, mode, ref, family_order)


def plan_families_py(raw: R.RawRecords, mode: str = "full", ref: Optional[R.Reference] = None,
                     family_order: str = "template-coordinate") -> FamilyPlan:
    """The numpy statement of plan_families (every mode)."""
    if family_order not in ("template-coordinate", "mi-group"):
        raise ValueError(family_order)
    n = raw.n
    f = raw.flag.astype(np.int64)
    rec, ops, lens, jop = _per_record_ops(raw)
    hasH = _has_op(rec, ops, n, R.OP_H)

    if mode in ("full", "convert"):
        pas, conv = tool1_plan(raw)
        keep1 = pas | conv
    else:
        conv = np.zeros(n, bool)
        keep1 = np.ones(n, bool)
    if mode == "convert":
        keep2 = conv
    elif mode in ("full", "extend"):
        keep2 = keep1 & ~hasH
    else:
        keep2 = keep1

    if mode != "convert":
        miss = keep2 & (raw.mi_id < 0)
        if miss.any():
            k = int(np.nonzero(miss)[0][0])
            raise MissingMITag("%s does not have MI tag." % raw.qname(k).decode())

    sL, L, kfirst, kn = _softclip_strip(raw)
    if mode == "vote":  # tool-2 output has no clips left; keep records as they are
        sL = np.zeros(n, np.int64)
        L = raw.l_seq.astype(np.int64)
        kfirst = np.zeros(n, np.int64)
        kn = raw.n_cig.astype(np.int64)

    idx2 = np.nonzero(keep2)[0].astype(np.int64)
    ext_right = np.zeros(n, bool)
    ext_left = np.zeros(n, bool)
    partner_raw = np.full(n, -1, np.int64)  # tool-2 extension partner (input record index)
    rd_in = np.zeros(n, bool)

    if mode == "convert":
        order = idx2
        fam_sizes = np.ones(idx2.shape[0], np.int64)
        fam_mi = np.full(idx2.shape[0], -1, np.int32)
    else:
        keys = raw.mi_id[idx2].astype(np.int64)
        if idx2.shape[0]:
            uniq, first, inv = np.unique(keys, return_index=True, return_inverse=True)
            rank = np.empty(uniq.shape[0], np.int64)
            rank[np.argsort(first, kind="stable")] = np.arange(uniq.shape[0])
            grp = rank[inv]
            perm = np.argsort(grp, kind="stable")
            members = idx2[perm]
            gsz = np.bincount(grp, minlength=uniq.shape[0])
            fam_mi = uniq[np.argsort(rank)].astype(np.int32)
        else:
            members = idx2
            gsz = np.zeros(0, np.int64)
            fam_mi = np.zeros(0, np.int32)
        goff = np.zeros(gsz.shape[0] + 1, np.int64)
        goff[1:] = np.cumsum(gsz)
        keep_rec = np.ones(members.shape[0], bool)
        out_members = members.copy()
        fam_sizes = gsz.copy()
        if mode in ("full", "extend"):
            g4 = np.nonzero(gsz == 4)[0]
            if g4.shape[0]:
                base = goff[g4]
                M = members[base[:, None] + np.arange(4)[None, :]]
                Fl = f[M]
                slot = np.full(Fl.shape, 4, np.int64)
                for s, fl in enumerate((99, 163, 83, 147)):
                    slot[Fl == fl] = s
                key = slot * 4 + np.arange(4)[None, :]
                ordr = np.argsort(key, axis=1, kind="stable")
                outm = np.take_along_axis(M, ordr, axis=1)
                outs = np.take_along_axis(slot, ordr, axis=1)
                cnt = np.stack([(slot == s).sum(1) for s in range(4)], axis=1)
                start = np.zeros_like(cnt)
                start[:, 1:] = np.cumsum(cnt, axis=1)[:, :-1]
                rows = np.arange(g4.shape[0])
                # pair (99, 163): left = the 163 record, right = the 99 record; swapped in the
                # output (tools/2.extend_gap.py:124-126 assigns process_read_pair's (left, right))
                p1 = (cnt[:, 0] > 0) & (cnt[:, 1] > 0)
                start = np.minimum(start, 3)  # only read where the pair exists
                a_pos, b_pos = start[:, 0], start[:, 1]
                a_rec = outm[rows, a_pos]
                b_rec = outm[rows, b_pos]
                outm[rows[p1], a_pos[p1]] = b_rec[p1]
                outm[rows[p1], b_pos[p1]] = a_rec[p1]
                # pair (83, 147): left = 83, right = 147
                p2 = (cnt[:, 2] > 0) & (cnt[:, 3] > 0)
                c_pos, d_pos = start[:, 2], start[:, 3]
                c_rec = outm[rows, c_pos]
                d_rec = outm[rows, d_pos]
                # LA / RD of the left (converted) record
                if mode == "full":
                    la_b = np.ones(g4.shape[0], bool)
                    la_c = np.ones(g4.shape[0], bool)
                else:
                    la = raw.la_tag if raw.la_tag is not None else np.full(n, -1, np.int32)
                    rd = raw.rd_tag if raw.rd_tag is not None else np.full(n, -1, np.int32)
                    for pm, lrec in ((p1, b_rec), (p2, c_rec)):
                        bad = pm & ((la[lrec] < 0) | (rd[lrec] < 0))
                        if bad.any():
                            k = int(lrec[np.nonzero(bad)[0][0]])
                            raise KeyError("%s: tag 'LA'/'RD' not present" % raw.qname(k).decode())
                    la_b = la[b_rec] == 1
                    la_c = la[c_rec] == 1
                    rd_in[b_rec[p1]] = rd[b_rec[p1]] == 1
                    rd_in[c_rec[p2]] = rd[c_rec[p2]] == 1
                # number of kept records per group and their local positions
                nkeep = (outs < 4).sum(1)
                # roles; local indices are positions within the group's output list
                q = p1 & la_b
                ext_right[a_rec[q]] = True
                partner_raw[a_rec[q]] = b_rec[q]
                ext_left[b_rec[p1]] = True
                partner_raw[b_rec[p1]] = a_rec[p1]
                q = p2 & la_c
                ext_right[d_rec[q]] = True
                partner_raw[d_rec[q]] = c_rec[q]
                ext_left[c_rec[p2]] = True
                partner_raw[c_rec[p2]] = d_rec[p2]
                # write back the new order; dropped flags go to the tail and are masked out
                out_members[base[:, None] + np.arange(4)[None, :]] = outm
                kr = np.arange(4)[None, :] < nkeep[:, None]
                keep_rec[base[:, None] + np.arange(4)[None, :]] = kr
                fam_sizes[g4] = nkeep
        order = out_members[keep_rec]
    t2_rank = np.arange(order.shape[0], dtype=np.int64)  # tool-2 output position of each batch record
    if mode in ("full", "vote") and family_order == "template-coordinate" and order.shape[0]:
        # the tool-2 records' current unclipped ends: tools 1/2 move pos and grow the cigar by the
        # prepended / appended base (clips are stripped); tool 1's RD is predicted from the input
        lead, trail, rref = _clips_reflen(raw.cigar, raw.cig_off, raw.n_cig)
        pos0 = raw.pos[order].astype(np.int64)
        if mode == "full":
            cv = conv[order]
            rdp = np.zeros(order.shape[0], bool)
            if cv.any():
                if ref is None:
                    raise ValueError("converting records needs the reference")
                rdp[cv] = predict_rd(raw, ref, order[cv], sL, L)
            er, el = ext_right[order], ext_left[order]
            pos1 = np.where(cv, np.maximum(pos0 - 1, 0), np.where(er, pos0 - 1, pos0))
            rl1 = rref[order] + cv.astype(np.int64) - (cv & rdp) + er.astype(np.int64) + (el & rdp)
            us, ue = pos1, pos1 + rl1 - 1
        else:
            us, ue = pos0 - lead[order], pos0 + rref[order] - 1 + trail[order]
        mus, mue = mate_unclipped(raw)
        perm = template_coordinate_order(raw, order, us, ue, mus, mue)
        order = order[perm]
        t2_rank = perm
        mi = raw.mi_id[order]
        brk = np.ones(order.shape[0], bool)
        brk[1:] = mi[1:] != mi[:-1]
        starts = np.nonzero(brk)[0]
        fam_sizes = np.diff(np.append(starts, order.shape[0])).astype(np.int64)
        fam_mi = mi[starts].astype(np.int32)
    nr = int(order.shape[0])
    nf = int(fam_sizes.shape[0])
    fam_off = np.zeros(nf + 1, np.int64)
    fam_off[1:] = np.cumsum(fam_sizes)
    # extension partners must share the record's family for the fused launch; a partner in another
    # family (a TemplateCoordinate run that splits a tool-2 4-group between the two pairs' reads)
    # marks both families
    fam_split = np.zeros(nf, bool)
    if nr:
        fam_of = np.repeat(np.arange(nf, dtype=np.int64), fam_sizes)
        inv = np.full(n, -1, np.int64)
        inv[order] = np.arange(nr, dtype=np.int64)
        has_p = (ext_right | ext_left)[order]
        pb = inv[np.where(has_p, partner_raw[order], 0)]
        pfam = np.where(pb >= 0, fam_of[np.maximum(pb, 0)], -1)
        pl = pb - fam_off[fam_of]
        bad = has_p & ((pb < 0) | (pfam != fam_of) | (pl > 3))
        fam_split[fam_of[bad]] = True
    return FamilyPlan(raw=raw, mode=mode, ref=ref, order=order.astype(np.int64), fam_off=fam_off,
                      fam_mi=np.asarray(fam_mi, np.int32), t2_rank=np.asarray(t2_rank, np.int64), conv=conv,
                      ext_right=ext_right, ext_left=ext_left, partner_raw=partner_raw, rd_in=rd_in, sL=sL, L=L,
                      kfirst=kfirst, kn=kn, fam_split=fam_split)


def route_small_cap(plan: FamilyPlan, f0: int, f1: int, cap: int = SMALL_ARENA_CAP, mid: int = MID_ARENA_CAP,
                    sample: int = 2048) -> int:
    """The small-arena cap for plan families [f0, f1): `mid` when more than half of the records of
    the small families (<= 64 records, arena <= cap) are in families whose arena exceeds `mid`,
    else `cap`.  k_small runs such families 6 waves per CU at most (LDS), k_large's 5-per-CU class
    at half their cost: C3 (deep families) 9.00 -> 8.54 ms per step; where they are a minority (C4)
    moving them lengthens the large leg more than it shortens the small one (profiles/r05/README.md).
    Estimated on up to `sample` evenly spaced families, with the arena of SmallLayout for no complex
    cigar (small_arena_bytes; the exact one is the C++ plan's)."""
    nf = f1 - f0
    if not SMALL_ROUTE or cap <= mid or nf <= 0:
        return cap
    pick = np.unique(np.linspace(f0, f1 - 1, min(nf, sample)).astype(np.int64))
    a, b = plan.fam_off[pick].astype(np.int64), plan.fam_off[pick + 1].astype(np.int64)
    sizes = b - a
    if not sizes.sum():
        return cap
    fam_of = np.repeat(np.arange(pick.shape[0]), sizes)
    recs = plan.order[np.repeat(a - np.cumsum(sizes) + sizes, sizes) + np.arange(int(sizes.sum()))]
    L = plan.L[recs].astype(np.int64)
    cap4 = (L + 2 + 3) & ~np.int64(3)
    img = (np.bincount(fam_of, weights=cap4, minlength=pick.shape[0]).astype(np.int64) + 31) & ~np.int64(31)
    nconv = np.bincount(fam_of, weights=plan.conv[recs].astype(np.int64), minlength=pick.shape[0]).astype(np.int64)
    need = small_arena_bytes(sizes, img, nconv, np.zeros_like(sizes), int(L.max()))
    small = (sizes <= 64) & (need <= cap)
    return mid if 2 * int(sizes[small & (need > mid)].sum()) > int(sizes[small].sum()) else cap


def materialize(plan: FamilyPlan, f0: int, f1: int, small_cap: Optional[int] = None, images=None) -> FamilyBatch:
    """The device batch of plan families [f0, f1) (family ids renumbered from 0): C++ (hostplan)
    for the step-5 modes, materialize_py otherwise; then the HBM bucket's families cut into parts
    (split_hbm_bucket).  small_cap: the largest small-family arena (None: route_small_cap).
    images: see hostplan.materialize."""
    from . import hostplan
    if small_cap is None:
        small_cap = route_small_cap(plan, f0, f1)
    if plan.mode in ("full", "vote") and hostplan.enabled():
        return split_hbm_bucket(hostplan.materialize(plan, f0, f1, small_cap, images=images))
    return split_hbm_bucket(materialize_py(plan, f0, f1, small_cap))


def split_hbm_bucket(fb: FamilyBatch, part_cap: Optional[int] = None, threads: int = 0) -> FamilyBatch:
    """k_large's part mode (include/bsdc.h): the families of the large buckets from SPLIT_FROM on
    (the 1-per-CU class and the HBM-scratch one) that can be cut between templates (no complex
    cigar, no tool-2 role) become parts of at most part_cap LDS bytes, run in LDS, and one join
    workgroup per family; the rest stay in their buckets.  In place."""
    from . import hostplan
    cap = PART_CAP if part_cap is None else int(part_cap)
    lo = min(max(SPLIT_FROM, 0), len(fb.large_buckets) - 1)
    sizes = [int(np.asarray(b).reshape(-1, 4).shape[0]) for b in fb.large_buckets[lo:]]
    ents = np.concatenate([np.asarray(b, np.uint32).reshape(-1, 4) for b in fb.large_buckets[lo:]]) \
        if sum(sizes) else np.zeros((0, 4), np.uint32)
    if cap <= 0 or ents.shape[0] == 0:
        return fb
    cap = cap // 16 * 16
    lib = hostplan._load()
    rec = np.ascontiguousarray(np.stack([fb.rec_off, fb.rec_pos.view(np.uint32), fb.rec_lenflag, fb.rec_link], axis=1),
                               np.uint32)
    k = ents.shape[0]
    nparts = np.zeros(k, np.int32)
    nrecs = np.zeros(k, np.int64)
    tot = int(lib.bsdc_split_count(rec.ctypes.data, ents.ctypes.data, k, cap, MAX_PART_REC, nparts.ctypes.data,
                                   nrecs.ctypes.data, int(threads)))
    if tot == 0:
        return fb
    first = np.zeros(k, np.int64)
    first[1:] = np.cumsum(nparts[:-1], dtype=np.int64)
    first_rec = np.zeros(k, np.int64)
    first_rec[1:] = np.cumsum(nrecs[:-1])
    parts = np.zeros((tot, 4), np.uint32)
    part_recs = np.zeros((int(nrecs.sum()), 4), np.uint32)
    lib.bsdc_split_fill(rec.ctypes.data, ents.ctypes.data, k, cap, MAX_PART_REC, first.ctypes.data, first_rec.ctypes.data,
                        parts.ctypes.data, part_recs.ctypes.data, int(threads))
    cut = nparts > 0
    ce = ents[cut].astype(np.int64)
    # the fallback arena of each cut family (ArenaLayout of the whole family, no complex cigars)
    L = (fb.rec_lenflag & 0xFFFF).astype(np.int64)
    mlf = np.asarray([int(L[a:a + m].max()) for a, m in zip(ce[:, 1], ce[:, 2])], np.int64)
    need = round16(large_arena_bytes(ce[:, 2], 2 * ce[:, 3], mlf, np.zeros(ce.shape[0], np.int64)))
    sf = np.zeros((ce.shape[0], 8), np.int64)
    sf[:, :4] = ce
    sf[:, 4] = first[cut]
    sf[:, 5] = nparts[cut]
    off = np.zeros(ce.shape[0], np.int64)
    off[1:] = np.cumsum(need[:-1])
    sf[:, 6] = off // 16
    sf[:, 7] = need
    parts[:, 2] |= (np.repeat(np.arange(ce.shape[0], dtype=np.int64), nparts[cut]) << 8).astype(np.uint32)  # | split family
    fb.split_parts = parts
    fb.split_part_recs = part_recs
    fb.split_fams = sf.astype(np.uint32)
    fb.split_part_arena = cap
    # each cut family's image re-laid out part after part (contiguous parts stage in 16-B chunks)
    assert fb.rec_off.dtype == np.uint32 and fb.rec_off.flags.c_contiguous
    assert fb.seq.flags.c_contiguous and fb.qual.flags.c_contiguous
    lib.bsdc_split_move(fb.seq.ctypes.data, fb.qual.ctypes.data, fb.rec_off.ctypes.data, fb.split_fams.ctypes.data,
                        int(fb.split_fams.shape[0]), parts.ctypes.data, part_recs.ctypes.data, int(threads))
    keep = ~cut
    tail, o = [], 0
    for k in sizes:  # the families left whole stay in their buckets
        tail.append(ents[o:o + k][keep[o:o + k]])
        o += k
    fb.large_buckets = list(fb.large_buckets[:lo]) + tail
    return fb


def materialize_py(plan: FamilyPlan, f0: int, f1: int, small_cap: int = SMALL_ARENA_CAP) -> FamilyBatch:
    """The numpy statement of materialize (every mode)."""
    raw, mode, ref = plan.raw, plan.mode, plan.ref
    n = raw.n
    f = raw.flag.astype(np.int64)
    conv, ext_right, ext_left, partner_raw, rd_in = plan.conv, plan.ext_right, plan.ext_left, plan.partner_raw, plan.rd_in
    sL, L, kfirst, kn = plan.sL, plan.L, plan.kfirst, plan.kn
    r0, r1 = int(plan.fam_off[f0]), int(plan.fam_off[f1])
    order = plan.order[r0:r1]
    fam_sizes = np.diff(plan.fam_off[f0:f1 + 1])
    fam_mi = plan.fam_mi[f0:f1]
    t2_rank = plan.t2_rank[r0:r1]
    nr = int(order.shape[0])
    nf = int(fam_sizes.shape[0])
    fam_off = np.zeros(nf + 1, np.int64)
    fam_off[1:] = np.cumsum(fam_sizes)
    fam_of = np.repeat(np.arange(nf, dtype=np.int64), fam_sizes)
    local = np.arange(nr, dtype=np.int64) - fam_off[fam_of]
    # extension partners as family-local indices (a partner outside the family -- plan.fam_split --
    # makes the fused launch invalid; the caller then runs the tools and the vote apart)
    has_p = (ext_right | ext_left)[order]
    pl = np.zeros(nr, np.int64)
    if has_p.any():
        srt = np.argsort(order, kind="stable")
        so = order[srt]
        want = partner_raw[order[has_p]]
        k = np.minimum(np.searchsorted(so, want), nr - 1)
        found = so[k] == want
        plh = np.where(found, srt[k], -1) - fam_off[fam_of[has_p]]
        pl[has_p] = np.where(found & (plh >= 0) & (plh <= 3), plh, 0)
    split_ext = bool(plan.fam_split[f0:f1].any())

    # ---- per batch record ----
    Lb = L[order]
    if nr and Lb.max() > 0xFFFF - 8:
        raise ValueError("record longer than 65527 bases")
    # HBM layout: record slots of cap4 = round4(L+2) (prepend / append room, dword aligned), the
    # record's bases at slot+1; every family image starts on a 32-nibble boundary
    cap4 = (Lb + 2 + 3) & ~np.int64(3)
    span = np.bincount(fam_of, weights=cap4, minlength=nf)[:nf].astype(np.int64) if nr else np.zeros(nf, np.int64)
    img = (span + 31) & ~np.int64(31)
    fam_base = np.zeros(nf + 1, np.int64)
    fam_base[1:] = np.cumsum(img)
    within = np.zeros(nr, np.int64)
    if nr:
        cs = np.cumsum(cap4) - cap4
        within = cs - cs[fam_off[fam_of]]
    rec_off = fam_base[fam_of] + within if nr else np.zeros(0, np.int64)
    n_slots = int(fam_base[-1]) + 64
    if n_slots >= 1 << 32:
        raise ValueError("batch too large for 32-bit offsets; split it")
    total = int(Lb.sum()) if nr else 0
    seq = np.zeros(n_slots // 2, np.uint8)
    qual = np.zeros(n_slots, np.uint8)
    shift = raw.seq_off[order] + sL[order]
    if nr:
        from .bam import family_image  # libbsdc_io: per-record copies, OpenMP over records
        family_image(shift, Lb, rec_off, raw.seq, raw.qual, n_slots, seq, qual)

    # stripped cigars, complex records
    nops = kn[order]
    cfirst = raw.cig_off[order] + kfirst[order]
    opid = np.repeat(cfirst - np.concatenate([[0], np.cumsum(nops)[:-1]]) if nr else np.zeros(0, np.int64), nops) \
        + np.arange(int(nops.sum()) if nr else 0, dtype=np.int64)
    sc = raw.cigar[opid] if opid.shape[0] else np.zeros(0, np.uint32)
    sc_rec = np.repeat(np.arange(nr, dtype=np.int64), nops)
    sc_op = (sc & 0xF).astype(np.int64)
    sc_len = (sc >> 4).astype(np.int64)
    not_m = ~np.isin(sc_op, (R.OP_M, R.OP_EQ, R.OP_X))
    complex_ = np.bincount(sc_rec[not_m], minlength=nr)[:nr] > 0 if nr else np.zeros(0, bool)
    refc = np.isin(sc_op, R.REF_CONSUMING)
    reflen = np.bincount(sc_rec[refc], weights=sc_len[refc], minlength=nr)[:nr].astype(np.int64) if nr else np.zeros(0, np.int64)
    if mode == "vote":
        reflen = np.where(complex_, reflen, Lb)
    # compact cigar array holding only complex records' ops
    keep_op = complex_[sc_rec] if nr else np.zeros(0, bool)
    cigar_c = sc[keep_op].astype(np.uint32)
    cnt_c = np.where(complex_, nops, 0)
    cig_off = np.zeros(nr, np.int64)
    if nr:
        cig_off[1:] = np.cumsum(cnt_c)[:-1]
    if complex_.any() and (nops[complex_].max() > 0xFFFF or reflen[complex_].max() > 0xFFFF):
        raise ValueError("cigar too long")
    cig_info = np.where(complex_, nops | (reflen << 16), 0).astype(np.uint32)

    # link word
    fo = f[order]
    tid = raw.tid[order].astype(np.int64)
    strand = raw.mi_strand[order].astype(np.int64)
    usable = ((fo & 1) != 0) & ((fo & 0x900) == 0) & (strand >= 0)
    link = np.full(nr, LINK_MATE_NONE, np.int64)
    # template mates: first usable R1 of a name -> first usable R2 of the name, within a family;
    # only mates that can overlap (both mapped, one contig) are linked
    name = raw.name_id[order].astype(np.int64)
    key = fam_of * (int(name.max()) + 1 if nr else 1) + name
    r1 = usable & ((fo & 0x40) != 0)
    r2 = usable & ((fo & 0x80) != 0)
    i1 = np.nonzero(r1)[0]
    i2 = np.nonzero(r2)[0]
    if i1.shape[0] and i2.shape[0]:
        u1, f1 = np.unique(key[i1], return_index=True)
        u2, f2 = np.unique(key[i2], return_index=True)
        _, ia, ib = np.intersect1d(u1, u2, assume_unique=True, return_indices=True)
        a = i1[f1[ia]]
        b = i2[f2[ib]]
        ok = (tid[a] == tid[b]) & ((fo[a] & 4) == 0) & ((fo[b] & 4) == 0)
        link[a[ok]] = local[b[ok]]
    link |= np.where(strand == 0, LINK_AB, 0) | np.where(strand == 1, LINK_BA, 0)
    link |= np.where(complex_, LINK_COMPLEX, 0)
    link |= np.where(conv[order], LINK_CONVERT, 0)
    link |= np.where(ext_right[order], LINK_EXT_RIGHT, 0)
    link |= np.where(ext_left[order], LINK_EXT_LEFT, 0)
    link |= np.where(has_p, pl << LINK_PARTNER_SHIFT, 0)
    link |= np.where(rd_in[order], LINK_RD_IN, 0)
    link |= np.where(usable, LINK_USABLE, 0)

    # tool-1 reference window of converted records: nibbles [max(pos-1,0), +L+2) of the contig,
    # N past the contig end or for a contig the FASTA lacks (tools/1.convert_AG_to_CT.py:103-117)
    rec_win = np.zeros((nr, 2), np.int64)
    convb = conv[order]
    if convb.any():
        if ref is None:
            raise ValueError("converting records needs the reference")
        np0 = np.maximum(raw.pos[order].astype(np.int64) - 1, 0)
        okt = (tid >= 0) & (tid < len(ref.names))
        coff = np.where(okt, ref.contig_off[np.clip(tid, 0, max(len(ref.names) - 1, 0))], -1) if len(ref.names) else np.full(nr, -1)
        clen = np.where(okt, ref.contig_len[np.clip(tid, 0, max(len(ref.names) - 1, 0))], 0) if len(ref.names) else np.zeros(nr, np.int64)
        present = coff >= 0
        rec_win[:, 0] = np.where(convb & present, coff + np0, 0)
        rec_win[:, 1] = np.where(convb & present, np.clip(clen - np0, 0, Lb + 2), 0)
        if rec_win[:, 0].max() >= 1 << 32:
            raise ValueError("reference too large for 32-bit nibble offsets")

    # read-through candidates (stale mate fields, MC tag)
    rt = np.zeros((nr, 4), np.int64)
    has_mc = raw.mc_off[order] >= 0
    base_rt = usable & ((fo & 0xC) == 0) & (raw.next_tid[order] == raw.tid[order]) & has_mc
    if base_rt.any():
        lead, trail, mref = _mc_clips_reflen(raw, order)
        np_ = raw.next_pos[order].astype(np.int64)
        mate_us = np_ - lead
        mate_ue = np_ + mref - 1 + trail
        pos = raw.pos[order].astype(np.int64)
        rl = np.where(complex_, reflen, Lb)
        neg = (fo & 16) != 0
        cand = base_rt & np.where(neg, pos - 2 < mate_us, pos + rl - 1 + 2 > mate_ue)
        link |= np.where(cand, LINK_RT, 0)
        rt[:, 0] = np_
        rt[:, 1] = raw.tlen[order]
        rt[:, 2] = mate_us
        rt[:, 3] = mate_ue
        rt[~cand] = 0

    # ---- family classes: small (one wavefront, LDS) by arena bucket, or large (one workgroup) ----
    max_len = int(Lb.max()) if nr else 0
    max_len_f = np.zeros(nf, np.int64)
    if nr:
        np.maximum.at(max_len_f, fam_of, Lb)
    cops = np.bincount(fam_of, weights=cnt_c, minlength=nf)[:nf].astype(np.int64) if nr else np.zeros(nf, np.int64)
    nconv = np.bincount(fam_of, weights=convb.astype(np.int64), minlength=nf)[:nf].astype(np.int64) if nr else np.zeros(nf, np.int64)
    need_s = small_arena_bytes(fam_sizes, img, nconv, cops, max_len)
    need_l = large_arena_bytes(fam_sizes, 2 * img, max_len_f, cops)
    small = (fam_sizes <= 64) & (need_s <= small_cap) & (img // 32 < (1 << 24))
    buckets, arenas = [], []
    lo = -1
    for cap in SMALL_BUCKETS:
        if cap > small_cap:
            cap = small_cap
        sel = small & (need_s > lo) & (need_s <= cap)
        buckets.append(np.nonzero(sel)[0].astype(np.uint32))
        arenas.append(int(cap))
        lo = cap
        if cap == small_cap:
            break
    while len(buckets) < len(SMALL_BUCKETS):
        buckets.append(np.zeros(0, np.uint32))
        arenas.append(16)
    # large-family list entries: family, first record, n, image bytes (the image starts at the first slot)
    lbuckets, larenas = [], []
    lo = -1
    for cap in LARGE_BUCKETS + (None,):
        sel = ~small & (need_l > lo) if cap is None else ~small & (need_l > lo) & (need_l <= cap)
        lf = np.nonzero(sel)[0]
        # the largest images first: a class's dispatch lasts until its longest workgroup ends, so
        # the longest start first and the short ones fill in around them
        lf = lf[np.argsort(-img[lf], kind="stable")]
        e = np.zeros((lf.shape[0], 4), np.int64)
        e[:, 0] = lf
        e[:, 1] = fam_off[lf]
        e[:, 2] = fam_sizes[lf]
        e[:, 3] = img[lf]
        lbuckets.append(e.astype(np.uint32))
        larenas.append(int(cap) if cap is not None else (int(round16(need_l[lf].max())) if lf.shape[0] else 16))
        lo = cap if cap is not None else lo

    # small-family list entries: family, first record, n | (image / 32) << 8, image base
    ent = np.zeros((nf, 4), np.int64)
    ent[:, 0] = np.arange(nf)
    ent[:, 1] = fam_off[:-1]
    ent[:, 2] = fam_sizes | ((img // 32) << 8)
    ent[:, 3] = fam_base[:-1]
    return FamilyBatch(
        fam_off=fam_off.astype(np.uint32), rec_off=rec_off.astype(np.uint32), fam_entry=ent.astype(np.uint32),
        rec_pos=raw.pos[order].astype(np.int32),
        rec_lenflag=(Lb | (fo << 16)).astype(np.uint32), rec_tid=raw.tid[order].astype(np.int32),
        rec_link=link.astype(np.uint32), rec_win=rec_win.astype(np.uint32),
        cig_off=cig_off.astype(np.uint32), cig_info=cig_info,
        cigar=cigar_c if cigar_c.shape[0] else np.zeros(1, np.uint32),
        rt=rt.reshape(-1).astype(np.int32), seq=seq, qual=qual,
        small_buckets=buckets, small_arenas=arenas, large_buckets=lbuckets, large_arenas=larenas,
        max_len=max_len, src=order.astype(np.int64), fam_mi=fam_mi.astype(np.int32),
        n_bases=total, n_slots=n_slots, t2_rank=t2_rank, split_ext=split_ext)


WIDE_MIN_RECORDS = 256  # a family of this many records may have a depth past a byte (include/bsdc.h ss_wide)


def wide_rows(fam_off) -> "tuple[np.ndarray, int]":
    """Per family its wide row (-1: none) -- the families of WIDE_MIN_RECORDS records or more,
    numbered in order -- and their count."""
    n = np.diff(np.asarray(fam_off, np.int64))
    w = n >= WIDE_MIN_RECORDS
    rows = np.where(w, np.cumsum(w) - 1, -1).astype(np.int32)
    return rows, int(w.sum())


def ss_stats16(ss: dict):
    """(depth, err) [F, 4, stride] u16 of a consensus' single-strand reads: the bytes the kernels
    write, with the exact values of the families that have wide rows (device.fetch's ss_wide)."""
    d = np.asarray(ss["depth"]).astype(np.uint16)
    e = np.asarray(ss["err"]).astype(np.uint16)
    wide = ss.get("wide")
    if wide is not None:
        f = np.nonzero(np.asarray(wide) >= 0)[0]
        if f.size:
            w = np.asarray(wide)[f]
            st = d.shape[2]
            d[f] = ss["wdepth"][w][:, :, :st]
            e[f] = ss["werr"][w][:, :, :st]
    return d, e
