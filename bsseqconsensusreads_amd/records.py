"""Decoded record streams and the reference genome, as numpy structure-of-arrays.

``RawRecords`` is what a BAM decoder hands to the step (one entry per alignment record, input
order); it is the common input of the product path (``batch.build_family_batch`` -> libbsdc) and of
the CPU restatement under ``oracle/``.  Bases are nt16 codes (``=ACMGRSVTWYHKDBN``), one per byte,
exactly what BAM stores two to a byte; quals are raw phred bytes.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

NT16 = "=ACMGRSVTWYHKDBN"
NT16_A, NT16_C, NT16_G, NT16_T, NT16_N = 1, 2, 4, 8, 15

# htslib seq_nt16_table: letters of either case map to their code, anything else to N (15)
ASCII_TO_NT16 = np.full(256, 15, dtype=np.uint8)
for _i, _c in enumerate(NT16):
    ASCII_TO_NT16[ord(_c)] = _i
    ASCII_TO_NT16[ord(_c.lower())] = _i
ASCII_TO_NT16[ord("U")] = ASCII_TO_NT16[ord("u")] = 8
NT16_TO_ASCII = np.frombuffer(NT16.encode(), dtype=np.uint8).copy()

CIGAR_OPS = "MIDNSHP=X"
OP_M, OP_I, OP_D, OP_N, OP_S, OP_H, OP_P, OP_EQ, OP_X = range(9)
REF_CONSUMING = (OP_M, OP_D, OP_N, OP_EQ, OP_X)


def encode_seq(s: str) -> np.ndarray:
    return ASCII_TO_NT16[np.frombuffer(s.encode(), dtype=np.uint8)]


def decode_seq(codes: np.ndarray) -> str:
    return NT16_TO_ASCII[np.asarray(codes, dtype=np.uint8)].tobytes().decode()


def parse_cigar_string(s: str) -> List[int]:
    ops, num = [], 0
    for ch in s:
        if ch.isdigit():
            num = num * 10 + ord(ch) - 48
        else:
            ops.append((num << 4) | CIGAR_OPS.index(ch))
            num = 0
    return ops


def cigar_string(ops: Sequence[int]) -> str:
    return "".join("%d%s" % (c >> 4, CIGAR_OPS[c & 0xF]) for c in ops) or "*"


# ------------------------------------------------------------------------------------------
# BAM aux fields
# ------------------------------------------------------------------------------------------
_AUX_FIXED = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}
_AUX_FMT = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I", "f": "<f"}


def parse_aux(buf: bytes) -> List[tuple]:
    """BAM aux bytes -> [(tag, type, value)] in file order."""
    out, i, n = [], 0, len(buf)
    while i + 3 <= n:
        tag = buf[i:i + 2].decode()
        t = chr(buf[i + 2])
        i += 3
        if t == "A":
            out.append((tag, t, chr(buf[i])))
            i += 1
        elif t in _AUX_FMT:
            w = _AUX_FIXED[t]
            out.append((tag, t, struct.unpack(_AUX_FMT[t], buf[i:i + w])[0]))
            i += w
        elif t in "ZH":
            j = buf.index(b"\0", i)
            out.append((tag, t, buf[i:j].decode()))
            i = j + 1
        elif t == "B":
            sub = chr(buf[i])
            cnt = struct.unpack("<i", buf[i + 1:i + 5])[0]
            w = _AUX_FIXED[sub]
            vals = list(struct.unpack("<%d%s" % (cnt, _AUX_FMT[sub][1]), buf[i + 5:i + 5 + w * cnt]))
            out.append((tag, "B" + sub, vals))
            i += 5 + w * cnt
        else:
            raise ValueError("bad aux type %r" % t)
    return out


def encode_aux(tags: Sequence[tuple]) -> bytes:
    out = bytearray()
    for tag, t, v in tags:
        if t in ("i", "I", "c", "C", "s", "S") and t not in _AUX_FMT:
            raise ValueError(t)
        if t == "A":
            out += tag.encode() + b"A" + v.encode()[:1]
        elif t in _AUX_FMT:
            out += tag.encode() + t.encode() + struct.pack(_AUX_FMT[t], v)
        elif t in ("Z", "H"):
            out += tag.encode() + t.encode() + str(v).encode() + b"\0"
        elif t.startswith("B"):
            sub = t[1]
            out += tag.encode() + b"B" + sub.encode() + struct.pack("<i", len(v))
            out += struct.pack("<%d%s" % (len(v), _AUX_FMT[sub][1]), *v)
        else:
            raise ValueError("bad aux type %r" % t)
    return bytes(out)


def aux_get(buf: bytes, tag: str):
    for t, _, v in parse_aux(buf):
        if t == tag:
            return v
    return None


# ------------------------------------------------------------------------------------------
@dataclass
class RawRecords:
    """Decoded alignment records, input order (structure of arrays)."""

    flag: np.ndarray          # u16
    tid: np.ndarray           # i32
    pos: np.ndarray           # i32, 0-based
    mapq: np.ndarray          # u8
    l_seq: np.ndarray         # i32
    seq_off: np.ndarray       # i64, into seq and qual
    seq: np.ndarray           # u8 nt16 codes
    qual: np.ndarray          # u8 raw phred
    cig_off: np.ndarray       # i64
    n_cig: np.ndarray         # i32
    cigar: np.ndarray         # u32
    next_tid: np.ndarray      # i32
    next_pos: np.ndarray      # i32
    tlen: np.ndarray          # i32
    name_id: np.ndarray       # i32
    names: List[bytes]        # QNAME per name id
    mi_id: np.ndarray         # i32, MI with the /A,/B suffix removed; -1 = no (or empty) MI tag
    mi_strand: np.ndarray     # i8, 0 = /A, 1 = /B, -1 = neither
    mi_names: List[str]       # MI base per mi id
    mc_off: np.ndarray        # i64, -1 = no MC tag
    mc_n: np.ndarray          # i32
    mc_cigar: np.ndarray      # u32
    aux: Optional[List[bytes]] = None  # raw aux bytes per record (None for synthetic data)
    la_tag: Optional[np.ndarray] = None  # i32 LA / RD tags when present (-1 absent), for tool-2-only input
    rd_tag: Optional[np.ndarray] = None

    @property
    def n(self) -> int:
        return int(self.flag.shape[0])

    def record_seq(self, k: int) -> np.ndarray:
        o = int(self.seq_off[k])
        return self.seq[o:o + int(self.l_seq[k])]

    def record_qual(self, k: int) -> np.ndarray:
        o = int(self.seq_off[k])
        return self.qual[o:o + int(self.l_seq[k])]

    def record_cigar(self, k: int) -> np.ndarray:
        o = int(self.cig_off[k])
        return self.cigar[o:o + int(self.n_cig[k])]

    def qname(self, k: int) -> bytes:
        return self.names[int(self.name_id[k])]


def _mi_split(mi: Optional[str]):
    """tools/2.extend_gap.py:164-166 key (MI.split('/')[0]) and fgbio's strand suffix."""
    if not mi:
        return None, -1
    key = mi.split("/")[0]
    strand = -1
    if mi.endswith("/A"):
        strand = 0
    elif mi.endswith("/B"):
        strand = 1
    return key, strand


class _Builder:
    """Accumulates records one at a time (fixtures, the BAM decoder)."""

    def __init__(self):
        self.cols: Dict[str, list] = {k: [] for k in (
            "flag", "tid", "pos", "mapq", "l_seq", "next_tid", "next_pos", "tlen", "name_id",
            "mi_id", "mi_strand", "mc_off", "mc_n", "la", "rd")}
        self.seq: List[np.ndarray] = []
        self.qual: List[np.ndarray] = []
        self.cig: List[List[int]] = []
        self.mc: List[int] = []
        self.aux: List[bytes] = []
        self.name_ids: Dict[bytes, int] = {}
        self.names: List[bytes] = []
        self.mi_ids: Dict[str, int] = {}
        self.mi_names: List[str] = []

    def add(self, name: bytes, flag: int, tid: int, pos: int, mapq: int, cigar: List[int],
            seq: np.ndarray, qual: np.ndarray, next_tid: int, next_pos: int, tlen: int, aux: bytes,
            tags: Optional[List[tuple]] = None):
        c = self.cols
        if tags is None:
            tags = parse_aux(aux)
        tagd = {t: v for t, _, v in tags}
        nid = self.name_ids.setdefault(name, len(self.names))
        if nid == len(self.names):
            self.names.append(name)
        key, strand = _mi_split(tagd.get("MI"))
        if key is None:
            mid = -1
        else:
            mid = self.mi_ids.setdefault(key, len(self.mi_names))
            if mid == len(self.mi_names):
                self.mi_names.append(key)
        mc = tagd.get("MC")
        if mc is not None and mc != "*":
            ops = parse_cigar_string(mc)
            c["mc_off"].append(len(self.mc))
            c["mc_n"].append(len(ops))
            self.mc.extend(ops)
        else:
            c["mc_off"].append(-1)
            c["mc_n"].append(0)
        c["flag"].append(flag)
        c["tid"].append(tid)
        c["pos"].append(pos)
        c["mapq"].append(mapq)
        c["l_seq"].append(len(seq))
        c["next_tid"].append(next_tid)
        c["next_pos"].append(next_pos)
        c["tlen"].append(tlen)
        c["name_id"].append(nid)
        c["mi_id"].append(mid)
        c["mi_strand"].append(strand)
        c["la"].append(int(tagd["LA"]) if "LA" in tagd else -1)
        c["rd"].append(int(tagd["RD"]) if "RD" in tagd else -1)
        self.seq.append(np.asarray(seq, dtype=np.uint8))
        self.qual.append(np.asarray(qual, dtype=np.uint8))
        self.cig.append(list(cigar))
        self.aux.append(aux)

    def finish(self) -> RawRecords:
        c = self.cols
        n = len(c["flag"])
        l_seq = np.asarray(c["l_seq"], dtype=np.int32)
        seq_off = np.zeros(n, dtype=np.int64)
        if n:
            seq_off[1:] = np.cumsum(l_seq, dtype=np.int64)[:-1]
        n_cig = np.asarray([len(x) for x in self.cig], dtype=np.int32)
        cig_off = np.zeros(n, dtype=np.int64)
        if n:
            cig_off[1:] = np.cumsum(n_cig, dtype=np.int64)[:-1]
        cat = lambda xs: np.concatenate(xs).astype(np.uint8) if xs else np.zeros(0, np.uint8)
        return RawRecords(
            flag=np.asarray(c["flag"], dtype=np.uint16), tid=np.asarray(c["tid"], dtype=np.int32),
            pos=np.asarray(c["pos"], dtype=np.int32), mapq=np.asarray(c["mapq"], dtype=np.uint8),
            l_seq=l_seq, seq_off=seq_off, seq=cat(self.seq), qual=cat(self.qual),
            cig_off=cig_off, n_cig=n_cig,
            cigar=np.asarray([o for x in self.cig for o in x], dtype=np.uint32),
            next_tid=np.asarray(c["next_tid"], dtype=np.int32), next_pos=np.asarray(c["next_pos"], dtype=np.int32),
            tlen=np.asarray(c["tlen"], dtype=np.int32), name_id=np.asarray(c["name_id"], dtype=np.int32),
            names=self.names, mi_id=np.asarray(c["mi_id"], dtype=np.int32),
            mi_strand=np.asarray(c["mi_strand"], dtype=np.int8), mi_names=self.mi_names,
            mc_off=np.asarray(c["mc_off"], dtype=np.int64), mc_n=np.asarray(c["mc_n"], dtype=np.int32),
            mc_cigar=np.asarray(self.mc, dtype=np.uint32), aux=self.aux,
            la_tag=np.asarray(c["la"], dtype=np.int32), rd_tag=np.asarray(c["rd"], dtype=np.int32))


def _gather_ranges(off: np.ndarray, ln: np.ndarray):
    """Concatenated index ranges [off[k], off[k] + ln[k]) and the new per-record offsets."""
    ln = ln.astype(np.int64)
    new_off = np.zeros(ln.shape[0], np.int64)
    if ln.shape[0]:
        new_off[1:] = np.cumsum(ln)[:-1]
    idx = np.repeat(off.astype(np.int64) - new_off, ln) + np.arange(int(ln.sum()), dtype=np.int64)
    return idx, new_off


def take(raw: RawRecords, idx: np.ndarray) -> RawRecords:
    """Records idx[0], idx[1], ... of `raw` as a new stream (name / MI tables shared)."""
    idx = np.asarray(idx, np.int64)
    si, so = _gather_ranges(raw.seq_off[idx], raw.l_seq[idx])
    ci, co = _gather_ranges(raw.cig_off[idx], raw.n_cig[idx])
    has_mc = raw.mc_off[idx] >= 0
    mi_, mo = _gather_ranges(np.where(has_mc, raw.mc_off[idx], 0), np.where(has_mc, raw.mc_n[idx], 0))
    sub = lambda a: None if a is None else a[idx]  # noqa: E731
    return RawRecords(
        flag=raw.flag[idx], tid=raw.tid[idx], pos=raw.pos[idx], mapq=raw.mapq[idx], l_seq=raw.l_seq[idx],
        seq_off=so, seq=raw.seq[si], qual=raw.qual[si], cig_off=co, n_cig=raw.n_cig[idx], cigar=raw.cigar[ci],
        next_tid=raw.next_tid[idx], next_pos=raw.next_pos[idx], tlen=raw.tlen[idx], name_id=raw.name_id[idx],
        names=raw.names, mi_id=raw.mi_id[idx], mi_strand=raw.mi_strand[idx], mi_names=raw.mi_names,
        mc_off=np.where(has_mc, mo, -1), mc_n=raw.mc_n[idx], mc_cigar=raw.mc_cigar[mi_],
        aux=None if raw.aux is None else [raw.aux[int(k)] for k in idx], la_tag=sub(raw.la_tag),
        rd_tag=sub(raw.rd_tag))


def records_from_dicts(recs: Sequence[dict]) -> RawRecords:
    """Fixture records ({name, flag, tid, pos, cigar, seq, qual, tags, ...}) -> RawRecords."""
    b = _Builder()
    for r in recs:
        cig = [(l << 4) | op for op, l in r["cigar"]]
        seq = encode_seq(r["seq"]) if r["seq"] else np.zeros(0, np.uint8)
        if r.get("qual") is None:
            qual = np.full(len(seq), 0xFF, np.uint8)
        else:
            qual = np.frombuffer(r["qual"].encode(), dtype=np.uint8) - 33
        tags = [tuple(t) for t in r.get("tags", [])]
        b.add(r["name"].encode(), r["flag"], r["tid"], r["pos"], r.get("mapq", 60), cig, seq, qual,
              r.get("next_tid", -1), r.get("next_pos", -1), r.get("tlen", 0), encode_aux(tags), tags)
    return b.finish()


# ------------------------------------------------------------------------------------------
@dataclass
class Reference:
    """Reference genome packed as nt16 nibbles (two per byte, high first), indexed by header tid."""

    names: List[str]              # header contig names (tid order)
    lengths: np.ndarray           # i64 header lengths
    contig_off: np.ndarray        # i64 nibble offset of each contig, -1 = not in the FASTA
    contig_len: np.ndarray        # i64 FASTA length (0 when absent)
    packed: np.ndarray            # u8
    n_nibbles: int
    letters: Dict[str, bytes] = field(default_factory=dict)  # raw FASTA letters (oracle / tests)

    @staticmethod
    def from_contigs(header_names: Sequence[str], contigs: Dict[str, str], keep_letters: bool = True,
                     header_lengths: Optional[Sequence[int]] = None) -> "Reference":
        offs, lens, parts, letters = [], [], [], {}
        o = 0
        for name in header_names:
            s = contigs.get(name)
            if s is None:
                offs.append(-1)
                lens.append(0)
                continue
            b = s.encode() if isinstance(s, str) else bytes(s)
            codes = ASCII_TO_NT16[np.frombuffer(b, dtype=np.uint8)]
            offs.append(o)
            lens.append(len(codes))
            parts.append(codes)
            o += len(codes)
            if keep_letters:
                letters[name] = b
        codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        packed = pack_nibbles(codes)
        hl = np.asarray(header_lengths if header_lengths is not None else lens, dtype=np.int64)
        return Reference(list(header_names), hl, np.asarray(offs, np.int64), np.asarray(lens, np.int64),
                         packed, int(len(codes)), letters)

    @staticmethod
    def from_codes(header_names: Sequence[str], codes_per_contig: Sequence[np.ndarray]) -> "Reference":
        """Reference from nt16 code arrays (synthetic genomes); no letters kept."""
        offs, lens, o = [], [], 0
        for c in codes_per_contig:
            offs.append(o)
            lens.append(len(c))
            o += len(c)
        codes = np.concatenate(list(codes_per_contig)) if len(codes_per_contig) else np.zeros(0, np.uint8)
        return Reference(list(header_names), np.asarray(lens, np.int64), np.asarray(offs, np.int64),
                         np.asarray(lens, np.int64), pack_nibbles(codes), int(len(codes)), {})


def pack_nibbles(codes: np.ndarray) -> np.ndarray:
    """nt16 codes -> BAM packing (two per byte, high nibble first)."""
    codes = np.asarray(codes, dtype=np.uint8)
    n = codes.shape[0]
    if n % 2:
        codes = np.concatenate([codes, np.zeros(1, np.uint8)])
    return ((codes[0::2] << 4) | codes[1::2]).astype(np.uint8)


def unpack_nibbles(packed: np.ndarray, n: int) -> np.ndarray:
    packed = np.asarray(packed, dtype=np.uint8)
    out = np.empty(2 * packed.shape[0], dtype=np.uint8)
    out[0::2] = packed >> 4
    out[1::2] = packed & 0xF
    return out[:n]
