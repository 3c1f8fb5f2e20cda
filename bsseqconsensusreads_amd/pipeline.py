"""The step-5 path as the reference's stages see it, on top of the Engine.

* ``run_tool1``  -- tools/1.convert_AG_to_CT.py semantics: input order, pass-through records
  unchanged, converted records replaced, every other record dropped.
* ``run_tool2``  -- tools/2.extend_gap.py semantics on tool-1 output (RD/LA tags from the input).
* ``run_step5``  -- convert_Bstrain -> extend -> groupsort_convert -> callduplex in one device pass;
  returns the consensus pair per family and, on request, the tool-2 records (parity dump).
* ``run_duplex`` -- callduplex alone on already converted + extended records.
* ``run_molecular`` -- pipeline step 1, fgbio CallMolecularConsensusReads (main.snake.py:46-55):
  the same single-strand vote over raw MI groups, one consensus pair (R1, R2) per MI.

A record stream of any size runs as a sequence of device batches: the host forms every family
once (batch.plan_families), cuts the family list into contiguous ranges of about `batch_bases`
bases (shard.plan_batches; never inside a family), and each range goes through one launch.  The
concatenated output equals the one-batch output (tests/test_gpu_batches.py).  With several GPUs
the ranges are dealt round-robin to ranks and gathered back in order (shard.deal / gather_in_order).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import TYPE_CHECKING, List, Optional

import numpy as np

from . import records as R
from . import shard
from .batch import FamilyBatch, FamilyPlan, build_family_batch, materialize, plan_families
from ._lib import MODE_CONVERT, MODE_DUMP, MODE_EXTEND, MODE_TAGS, MODE_VOTE

if TYPE_CHECKING:  # (torch loads with the engine, not with the host planning: ranks.py overlaps the two)
    from .device import Engine


@dataclass
class OutRecords:
    """Output records of a tool stage; everything not listed is the input record's (``src``)."""

    src: np.ndarray      # i64 input record index
    pos: np.ndarray
    l_seq: np.ndarray
    seq_off: np.ndarray
    seq: np.ndarray      # nt16 codes
    qual: np.ndarray
    n_cig: np.ndarray
    cig_off: np.ndarray
    cigar: np.ndarray
    rd: np.ndarray       # -1 = tag untouched by this stage
    la: np.ndarray

    @property
    def n(self):
        return int(self.src.shape[0])

    def record(self, k: int):
        o, l = int(self.seq_off[k]), int(self.l_seq[k])
        c, m = int(self.cig_off[k]), int(self.n_cig[k])
        return dict(src=int(self.src[k]), pos=int(self.pos[k]), seq=self.seq[o:o + l], qual=self.qual[o:o + l],
                    cigar=self.cigar[c:c + m], rd=int(self.rd[k]), la=int(self.la[k]))


@dataclass
class Consensus:
    fam_mi: np.ndarray     # i32 MI id per family (RawRecords.mi_names index)
    status: np.ndarray     # u8 bit0 emitted, bit1 AB used, bit2 BA used
    length: np.ndarray     # [F, 2]
    seq: np.ndarray        # [F, 2, stride] nt16 codes
    qual: np.ndarray       # [F, 2, stride]
    fam_rec_off: np.ndarray = None  # [F + 1] family membership: fam_src[fam_rec_off[f]:fam_rec_off[f+1]]
    fam_src: np.ndarray = None      # input record index of each family record (family order)
    # with tags=True: the four single-strand consensus reads per family and their column
    # statistics (BSDC_MODE_TAGS), sets s = 0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2: "len" [F, 4],
    # "base" (nt16) / "qual" / "depth" / "err" [F, 4, stride] (depth and err bytes, saturated; the
    # exact u16 rows of the families of more than 255 records in "wdepth" / "werr" [W, 4, stride],
    # row "wide"[f], -1 none; batch.ss_stats16 merges them)
    ss: Optional[dict] = None


def _stripped_cigar(raw: R.RawRecords, k: int, strip: bool) -> List[int]:
    ops = [int(x) for x in raw.record_cigar(k)]
    if strip:
        if ops and (ops[0] & 0xF) == R.OP_S:
            ops = ops[1:]
        if ops and (ops[-1] & 0xF) == R.OP_S:
            ops = ops[:-1]
    return ops


def _records_from_dump(raw: R.RawRecords, fb: FamilyBatch, out: dict, strip: bool) -> OutRecords:
    """The stage dump as tool-2 output records, in tool-2 output order (the batch may hold them in
    TemplateCoordinate order)."""
    n = fb.n_rec
    bo = np.argsort(fb.t2_rank, kind="stable")  # batch record of each tool-2 output position
    lens = out["dump_len"][:n].astype(np.int64)[bo]
    seq_off = np.zeros(n, np.int64)
    if n:
        seq_off[1:] = np.cumsum(lens)[:-1]
    d = fb.rec_off.astype(np.int64)[bo]
    idx = np.repeat(d - seq_off, lens) + np.arange(int(lens.sum()), dtype=np.int64)
    seq = out["dump_seq"][idx]
    qual = out["dump_qual"][idx]
    tags = out["dump_tags"][:n][bo]
    src = fb.src[bo]
    cig, ncig = [], []
    rd = np.full(n, -1, np.int32)
    la = np.full(n, -1, np.int32)
    for b in range(n):
        k = int(src[b])
        ops = _stripped_cigar(raw, k, strip)
        t = int(tags[b])
        if t & 2:  # converted in this launch: [(M,1)] + cigar, RD trims the last op
            ops = [(1 << 4)] + ops
            if t & 1:
                last = ops[-1]
                if (last >> 4) > 1:
                    ops[-1] = last - (1 << 4)
                else:
                    ops.pop()
            rd[b] = t & 1
            la[b] = 1
        elif t & 4:
            ops = [(1 << 4)] + ops
        if t & 8:
            ops = ops + [(1 << 4)]
        cig.extend(ops)
        ncig.append(len(ops))
    n_cig = np.asarray(ncig, np.int32)
    cig_off = np.zeros(n, np.int64)
    if n:
        cig_off[1:] = np.cumsum(n_cig)[:-1]
    return OutRecords(src.copy(), out["dump_pos"][:n].astype(np.int32)[bo], lens.astype(np.int32), seq_off, seq, qual,
                      n_cig, cig_off, np.asarray(cig, np.uint32), rd, la)


def raw_from_records(raw: R.RawRecords, t: OutRecords) -> R.RawRecords:
    """Tool-2 output records as a RawRecords stream (mate fields, MI, name and MC from the input
    record: the tools leave them stale), for callduplex alone."""
    src = t.src.astype(np.int64)
    mcn = np.where(raw.mc_off[src] >= 0, raw.mc_n[src], 0).astype(np.int64)
    mc_off = np.where(mcn > 0, np.cumsum(mcn) - mcn, -1)
    mcj = np.repeat(np.where(mcn > 0, raw.mc_off[src], 0), mcn) + \
        (np.arange(int(mcn.sum())) - np.repeat(np.cumsum(mcn) - mcn, mcn))
    return R.RawRecords(
        flag=raw.flag[src], tid=raw.tid[src], pos=t.pos.astype(np.int32), mapq=raw.mapq[src],
        l_seq=t.l_seq.astype(np.int32), seq_off=t.seq_off.astype(np.int64), seq=t.seq, qual=t.qual,
        cig_off=t.cig_off.astype(np.int64), n_cig=t.n_cig.astype(np.int32), cigar=t.cigar,
        next_tid=raw.next_tid[src], next_pos=raw.next_pos[src], tlen=raw.tlen[src],
        name_id=raw.name_id[src], names=raw.names, mi_id=raw.mi_id[src], mi_strand=raw.mi_strand[src],
        mi_names=raw.mi_names, mc_off=np.where(raw.mc_off[src] >= 0, mc_off, -1).astype(np.int64),
        mc_n=raw.mc_n[src], mc_cigar=raw.mc_cigar[mcj] if mcj.shape[0] else np.zeros(0, np.uint32),
        la_tag=t.la.astype(np.int32), rd_tag=t.rd.astype(np.int32))


def _concat_records(parts: List[OutRecords], order: np.ndarray) -> OutRecords:
    """Merge record sets and put them in `order` of src."""
    src = np.concatenate([p.src for p in parts])
    where = {int(s): (pi, k) for pi, p in enumerate(parts) for k, s in enumerate(p.src)}
    pos, l_seq, seqs, quals, ncig, cigs, rd, la = [], [], [], [], [], [], [], []
    for s in order:
        pi, k = where[int(s)]
        r = parts[pi].record(k)
        pos.append(r["pos"])
        l_seq.append(len(r["seq"]))
        seqs.append(r["seq"])
        quals.append(r["qual"])
        ncig.append(len(r["cigar"]))
        cigs.append(r["cigar"])
        rd.append(r["rd"])
        la.append(r["la"])
    l_seq = np.asarray(l_seq, np.int32)
    so = np.zeros(len(order), np.int64)
    if len(order):
        so[1:] = np.cumsum(l_seq)[:-1]
    ncig = np.asarray(ncig, np.int32)
    co = np.zeros(len(order), np.int64)
    if len(order):
        co[1:] = np.cumsum(ncig)[:-1]
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return OutRecords(np.asarray(order, np.int64), np.asarray(pos, np.int32), l_seq, so, cat(seqs, np.uint8),
                      cat(quals, np.uint8), ncig, co, cat(cigs, np.uint32), np.asarray(rd, np.int32),
                      np.asarray(la, np.int32))


def _passthrough(raw: R.RawRecords, idx: np.ndarray) -> OutRecords:
    parts_seq = [raw.record_seq(int(k)) for k in idx]
    parts_q = [raw.record_qual(int(k)) for k in idx]
    parts_c = [raw.record_cigar(int(k)) for k in idx]
    l = np.asarray([len(x) for x in parts_seq], np.int32)
    so = np.zeros(len(idx), np.int64)
    if len(idx):
        so[1:] = np.cumsum(l)[:-1]
    nc = np.asarray([len(x) for x in parts_c], np.int32)
    co = np.zeros(len(idx), np.int64)
    if len(idx):
        co[1:] = np.cumsum(nc)[:-1]
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
    return OutRecords(np.asarray(idx, np.int64), raw.pos[idx].astype(np.int32), l, so, cat(parts_seq, np.uint8),
                      cat(parts_q, np.uint8), nc, co, cat(parts_c, np.uint32), np.full(len(idx), -1, np.int32),
                      np.full(len(idx), -1, np.int32))


def run_tool1(engine: Engine, raw: R.RawRecords) -> OutRecords:
    """tools/1.convert_AG_to_CT.py:67-186 over a record stream (reference must be loaded)."""
    from .batch import tool1_plan
    pas, conv = tool1_plan(raw)
    fb = build_family_batch(raw, "convert", engine.ref)
    db = engine.upload(fb, dump=True)
    engine.run(db, MODE_CONVERT | MODE_DUMP)
    out = db.fetch()
    converted = _records_from_dump(raw, fb, out, strip=True)
    passed = _passthrough(raw, np.nonzero(pas)[0])
    order = np.nonzero(pas | conv)[0]
    return _concat_records([passed, converted], order)


def run_tool2(engine: Engine, raw: R.RawRecords) -> OutRecords:
    """tools/2.extend_gap.py:145-190 on tool-1 output (LA / RD tags in the input)."""
    fb = build_family_batch(raw, "extend")
    db = engine.upload(fb, dump=True)
    engine.run(db, MODE_EXTEND | MODE_DUMP)
    return _records_from_dump(raw, fb, db.fetch(), strip=True)


def consensus_from_output(fb: FamilyBatch, out: dict) -> Consensus:
    F = fb.n_fam
    stride = out["stride"]
    from .bam import unpack_nibbles
    seq = unpack_nibbles(out["seq"].reshape(F, 2, stride // 2))
    ss = None
    if "ss_len" in out:
        ss = {"len": out["ss_len"], "base": out["ss_base"], "qual": out["ss_qual"], "depth": out["ss_depth"],
              "err": out["ss_err"], "wide": out["ss_wide"], "wdepth": out["ss_wdepth"], "werr": out["ss_werr"]}
    return Consensus(fb.fam_mi.copy(), out["status"], out["len"], seq, out["qual"], fb.fam_off.astype(np.int64),
                     fb.src.astype(np.int64), ss)


# Device batch budget: bases (+2 per record, the tools' prepend / append room) per launch.  2^31
# keeps a batch's slot offsets inside 32 bits (include/bsdc.h) with room for the 32-entry family
# alignment; a C2 batch of that size is ~1.7M families, ~5 GB of HBM with its outputs.
DEFAULT_BATCH_BASES = 1 << 31


def plan_ranges(plan: FamilyPlan, batch_bases: Optional[int] = None):
    """Contiguous family ranges [a, b) of about batch_bases bases each (shard.plan_batches)."""
    return shard.plan_batches(plan.fam_bases(), DEFAULT_BATCH_BASES if batch_bases is None else batch_bases)


def run_ranges(engine: Engine, plan: FamilyPlan, ranges, mode: int, tags: bool = False,
               timing: Optional[dict] = None) -> List[Consensus]:
    """Plan family ranges through the kernels, one launch each, output per range in range order.
    The host builds range i + 1 while the kernels of range i run.  `timing`: seconds added per
    host step (materialize, upload, fetch = wait + copy out, unpack)."""
    import time
    T = timing if timing is not None else {}
    parts: List[Consensus] = []
    prev = None

    def out(fb, db):
        t0 = time.perf_counter()
        o = db.fetch()
        t1 = time.perf_counter()
        parts.append(consensus_from_output(fb, o))
        T["fetch"] = T.get("fetch", 0.0) + t1 - t0
        T["unpack"] = T.get("unpack", 0.0) + time.perf_counter() - t1
    for a, b in ranges:
        t0 = time.perf_counter()
        fb = materialize(plan, a, b, images=engine.stage_images)
        t1 = time.perf_counter()
        db = engine.upload(fb, tags=tags)
        engine.run(db, mode | (MODE_TAGS if tags else 0))
        T["materialize"] = T.get("materialize", 0.0) + t1 - t0
        T["upload"] = T.get("upload", 0.0) + time.perf_counter() - t1
        if prev is not None:
            out(*prev)
        prev = (fb, db)
    if prev is not None:
        out(*prev)
    return parts


def materialize_ranges(plan: FamilyPlan, ranges, images=None) -> List[FamilyBatch]:
    """The device batches of plan family ranges (batch.materialize each), for run_batches; `images`
    e.g. a PinnedPool's, so that they upload asynchronously."""
    return [materialize(plan, a, b, images=images) for a, b in ranges]


def run_batches(engine: Engine, batches, mode: int, tags: bool = False,
                timing: Optional[dict] = None) -> List[Consensus]:
    """Materialized batches through the kernels, one launch each, output per batch in order; a
    batch uploads and launches before the one before it is fetched.  `timing` as run_ranges."""
    import time
    T = timing if timing is not None else {}
    parts: List[Consensus] = []
    prev = None

    def out(fb, db):
        t0 = time.perf_counter()
        o = db.fetch()
        t1 = time.perf_counter()
        parts.append(consensus_from_output(fb, o))
        T["fetch"] = T.get("fetch", 0.0) + t1 - t0
        T["unpack"] = T.get("unpack", 0.0) + time.perf_counter() - t1
    for fb in batches:
        t0 = time.perf_counter()
        db = engine.upload(fb, tags=tags)
        engine.run(db, mode | (MODE_TAGS if tags else 0))
        T["upload"] = T.get("upload", 0.0) + time.perf_counter() - t0
        if prev is not None:
            out(*prev)
        prev = (fb, db)
    if prev is not None:
        out(*prev)
    return parts


def concat_consensus(parts: List[Consensus]) -> Consensus:
    """Consensus of consecutive family ranges -> one Consensus in range order (strides padded to
    the widest)."""
    if len(parts) == 1:
        return parts[0]
    if not parts:
        z = np.zeros(0, np.int32)
        return Consensus(z, np.zeros(0, np.uint8), np.zeros((0, 2), np.int32), np.zeros((0, 2, 16), np.uint8),
                         np.zeros((0, 2, 16), np.uint8), np.zeros(1, np.int64), np.zeros(0, np.int64))
    stride = max(int(p.seq.shape[2]) for p in parts)

    def pad(a):
        return np.pad(a, [(0, 0)] * (a.ndim - 1) + [(0, stride - a.shape[-1])])
    offs = [0]
    for p in parts:
        offs.append(offs[-1] + int(p.fam_rec_off[-1]))
    fro = np.concatenate([np.asarray(p.fam_rec_off[:-1], np.int64) + o for p, o in zip(parts, offs)] + [[offs[-1]]])
    ss = None
    if all(p.ss is not None for p in parts):
        ss = {"len": np.concatenate([p.ss["len"] for p in parts])}
        for k in ("base", "qual", "depth", "err"):
            ss[k] = np.concatenate([pad(p.ss[k]) for p in parts])
        if any(p.ss.get("wide") is not None for p in parts):  # wide rows renumbered part after part
            wides, w0 = [], 0
            for p in parts:
                F = p.ss["len"].shape[0]
                w = p.ss.get("wide")
                w = np.full(F, -1, np.int32) if w is None else np.asarray(w, np.int32)
                wides.append(np.where(w >= 0, w + w0, -1).astype(np.int32))
                w0 += 0 if p.ss.get("wdepth") is None else int(p.ss["wdepth"].shape[0])
            ss["wide"] = np.concatenate(wides)
            for k in ("wdepth", "werr"):
                ss[k] = np.concatenate([pad(p.ss[k]) for p in parts if p.ss.get(k) is not None])
    return Consensus(np.concatenate([p.fam_mi for p in parts]), np.concatenate([p.status for p in parts]),
                     np.concatenate([p.length for p in parts]), np.concatenate([pad(p.seq) for p in parts]),
                     np.concatenate([pad(p.qual) for p in parts]), fro.astype(np.int64),
                     np.concatenate([np.asarray(p.fam_src, np.int64) for p in parts]), ss)


def _tools_batched(engine: Engine, raw: R.RawRecords, batch_bases: Optional[int]) -> OutRecords:
    """Tools 1 + 2 over tool-2 MI groups, batch by batch, as tool-2 output records in order."""
    plan = plan_families(raw, "full", engine.ref, family_order="mi-group")
    parts = []
    for a, b in plan_ranges(plan, batch_bases):
        fb = materialize(plan, a, b)
        db = engine.upload(fb, dump=True)
        engine.run(db, MODE_CONVERT | MODE_EXTEND | MODE_DUMP)
        parts.append(_records_from_dump(raw, fb, db.fetch(), strip=True))
    return _cat_records(parts)


def _cat_records(parts: List[OutRecords]) -> OutRecords:
    if len(parts) == 1:
        return parts[0]
    if not parts:
        e = np.zeros(0, np.int64)
        return OutRecords(e, e.astype(np.int32), e.astype(np.int32), e, np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                          e.astype(np.int32), e, np.zeros(0, np.uint32), e.astype(np.int32), e.astype(np.int32))
    so, co = [], []
    bs, cs = 0, 0
    for p in parts:
        so.append(p.seq_off + bs)
        co.append(p.cig_off + cs)
        bs += int(p.seq.shape[0])
        cs += int(p.cigar.shape[0])
    cat = np.concatenate
    return OutRecords(cat([p.src for p in parts]), cat([p.pos for p in parts]), cat([p.l_seq for p in parts]),
                      cat(so), cat([p.seq for p in parts]), cat([p.qual for p in parts]),
                      cat([p.n_cig for p in parts]), cat(co), cat([p.cigar for p in parts]),
                      cat([p.rd for p in parts]), cat([p.la for p in parts]))


def run_step5(engine: Engine, raw: R.RawRecords, dump: bool = False, tags: bool = False,
              batch_bases: Optional[int] = None):
    """Rules convert_Bstrain .. callduplex (main.snake.py:121-164) -> (Consensus, tool-2 records or None).
    tags: also the single-strand reads and column statistics of fgbio's consensus tags (Consensus.ss).
    batch_bases: device batch budget (DEFAULT_BATCH_BASES); dump (the tool-2 records, parity
    tests) needs the stream in one batch."""
    plan = plan_families(raw, "full", engine.ref)
    if plan.split_ext:
        # a TemplateCoordinate family lacks a record's tool-2 extension partner: run the tools as
        # their own launches (tool-2 MI groups), then callduplex on their records
        t2 = _tools_batched(engine, raw, batch_bases)
        cons = run_duplex(engine, raw_from_records(raw, t2), tags, batch_bases)
        cons.fam_src = t2.src[cons.fam_src]  # raw2 record k is tool-2 record k
        return cons, (t2 if dump else None)
    mode = MODE_CONVERT | MODE_EXTEND | MODE_VOTE
    if dump:
        fb = materialize(plan, 0, plan.n_fam)
        db = engine.upload(fb, dump=True, tags=tags)
        engine.run(db, mode | MODE_DUMP | (MODE_TAGS if tags else 0))
        out = db.fetch()
        return consensus_from_output(fb, out), _records_from_dump(raw, fb, out, strip=True)
    return concat_consensus(run_ranges(engine, plan, plan_ranges(plan, batch_bases), mode, tags)), None


def run_duplex(engine: Engine, raw: R.RawRecords, tags: bool = False, batch_bases: Optional[int] = None) -> Consensus:
    """callduplex alone (main.snake.py:155-164) on converted + extended records."""
    plan = plan_families(raw, "vote")
    return concat_consensus(run_ranges(engine, plan, plan_ranges(plan, batch_bases), MODE_VOTE, tags))


def molecular_records(raw: R.RawRecords) -> R.RawRecords:
    """The input of CallMolecularConsensusReads (main.snake.py:46-55) as records the vote reads:
    fgbio groups consecutive records of one MI tag (GroupReadsByUmi output order), the /A and /B
    molecules of a duplex apart.  Each run becomes its own MI id with the full tag as its name, and
    every record is marked strand A, so the kernel's X set is the run's R1s and Y its R2s with no
    BA side: the duplex combine passes the two single-strand consensus reads through unchanged."""
    n = raw.n
    key = raw.mi_id.astype(np.int64) * 4 + (raw.mi_strand.astype(np.int64) + 1)
    brk = np.ones(n, bool)
    if n:
        brk[1:] = key[1:] != key[:-1]
    run = np.cumsum(brk) - 1
    starts = np.nonzero(brk)[0]
    from .bam import StringTable
    if isinstance(raw.mi_names, StringTable):  # a decoded BAM: the run names as one packed table
        names = _run_names(raw.mi_names, raw.mi_id[starts], raw.mi_strand[starts])
    else:
        suffix = {0: "/A", 1: "/B", -1: ""}
        names = [raw.mi_names[int(raw.mi_id[k])] + suffix[int(raw.mi_strand[k])] if raw.mi_id[k] >= 0 else ""
                 for k in starts]
    mi_id = np.where(raw.mi_id >= 0, run, -1).astype(np.int32)
    mi_strand = np.where(raw.mi_id >= 0, 0, -1).astype(np.int8)
    return dataclasses.replace(raw, mi_id=mi_id, mi_strand=mi_strand, mi_names=names)


def _run_names(tab, ids: np.ndarray, strands: np.ndarray):
    """StringTable of tab[ids[k]] + "/A" (strand 0) / "/B" (strand 1) / "" (no strand), "" for
    ids[k] < 0: molecular_records' run names, vectorised (one Python string per run cost as much as
    planning the chunk)."""
    from .bam import StringTable
    ids = np.asarray(ids, np.int64)
    strands = np.asarray(strands, np.int64)
    n = int(ids.shape[0])
    ok = ids >= 0
    cid = np.where(ok, ids, 0)
    src_len = np.where(ok, tab.off[cid + 1] - tab.off[cid], 0) if n else np.zeros(0, np.int64)
    sfx = ok & (strands >= 0)
    lens = src_len + 2 * sfx
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    buf = np.empty(int(off[-1]), np.uint8)
    tot = int(src_len.sum())
    if tot:
        k = np.repeat(np.arange(n, dtype=np.int64), src_len)
        j = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(src_len) - src_len, src_len)
        buf[off[k] + j] = tab.buf[tab.off[cid[k]] + j]
    at = off[:-1][sfx] + src_len[sfx]
    buf[at] = ord("/")
    buf[at + 1] = np.where(strands[sfx] == 0, ord("A"), ord("B")).astype(np.uint8)
    return StringTable(buf, off, as_str=True)


def run_molecular(engine: Engine, raw: R.RawRecords, tags: bool = False,
                  min_consensus_base_quality: int = 0):
    """fgbio CallMolecularConsensusReads with the step-1 flags (main.snake.py:54: pre 45, post 30,
    min-reads 1, min-consensus-base-quality 0, overlapping bases on) -> (Consensus over the runs,
    the run records).  Consensus family f is MI run f; its R1 / R2 are the single-strand consensus
    of the run's R1s / R2s.  The engine runs with min_consensus_base_quality for this call only."""
    rm = molecular_records(raw)
    plan = plan_families(rm, "vote", family_order="mi-group")
    with engine.flags(min_consensus_base_quality=min_consensus_base_quality):
        return concat_consensus(run_ranges(engine, plan, plan_ranges(plan), MODE_VOTE, tags)), rm
