"""Seeded synthetic step-5 input: EM-seq duplex families on a random genome.

Genome: iid bases at 41 % GC.  Methylation is a property of the molecule: CpG cytosines are
methylated with p = 0.75, other cytosines with p = 0.005, decided by a hash of (family, position)
so both strands and every PCR copy of a family agree.  The AB strand is sequenced as 99/147 (top,
C->T) or 83/163 (bottom, G->A) with probability 1/2 and BA takes the other orientation.  Reads are
2 x 150 bp, fragments N(300, 80) clipped to [160, 600] (C3: N(200, 30)), qualities drawn from
Q37 / Q25 / Q12 bins with a tail that decays along the read, errors at each base's own quality.
Records come out grouped by family, position-ordered inside a family, with MI k/A | k/B and MC.

Family-size models (templates per family):
  C0  1 AB + 1 BA (the pipeline as written)      C1  3 + 3
  C2  Poisson(4) total, zero redrawn, split Binomial(T, 1/2)
  C3  U[20, 100] total, split Binomial             C4  Zipf on [1, 500], 30 % AB-only
The generator runs in torch (GPU when present), then hands numpy RawRecords to the host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from . import records as R

CONFIGS = ("C0", "C1", "C2", "C3", "C4")


def _hash_u01(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Deterministic uniform [0,1) from two int64 tensors (splitmix-style mix in 62-bit space)."""
    x = (a * 0x9E3779B1 + b * 0x85EBCA77 + 0x27D4EB2F) & 0x3FFFFFFFFFFFFFFF
    x = ((x ^ (x >> 31)) * 0x2545F4914F6CDD1D) & 0x3FFFFFFFFFFFFFFF
    x = x ^ (x >> 29)
    return (x & 0xFFFFFF).to(torch.float32) / float(1 << 24)


def make_genome(length: int, gen: torch.Generator, device) -> torch.Tensor:
    u = torch.rand(length, generator=gen, device=device)
    codes = torch.full((length,), 8, dtype=torch.uint8, device=device)  # T
    codes[u < 0.705] = 4  # G
    codes[u < 0.5] = 2    # C
    codes[u < 0.295] = 1  # A
    return codes


def family_sizes(cfg: str, n_fam: int, gen: torch.Generator, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """-> (AB templates, BA templates) per family."""
    if cfg == "C0":
        a = torch.ones(n_fam, dtype=torch.int64, device=device)
        return a, a.clone()
    if cfg == "C1":
        a = torch.full((n_fam,), 3, dtype=torch.int64, device=device)
        return a, a.clone()
    if cfg == "C2":
        lam = torch.full((n_fam,), 4.0, device=device)
        t = torch.poisson(lam, generator=gen).to(torch.int64)
        for _ in range(20):
            z = t == 0
            if not bool(z.any()):
                break
            t[z] = torch.poisson(lam[z], generator=gen).to(torch.int64)
        t = t.clamp_min(1)
    elif cfg == "C3":
        t = torch.randint(20, 101, (n_fam,), generator=gen, device=device)
    elif cfg == "C4":
        u = torch.rand(n_fam, generator=gen, device=device).clamp_min(1e-9)
        t = torch.floor(1.0 / u).clamp(1, 500).to(torch.int64)
    else:
        raise ValueError(cfg)
    a = torch.binomial(t.to(torch.float32), torch.full((n_fam,), 0.5, device=device), generator=gen).to(torch.int64)
    if cfg == "C4":
        ab_only = torch.rand(n_fam, generator=gen, device=device) < 0.3
        a = torch.where(ab_only, t, a)
    return a, t - a


@dataclass
class SynthSet:
    raw: R.RawRecords
    ref: R.Reference
    cfg: str
    n_fam: int
    genome: Optional[torch.Tensor] = None  # nt16 codes on the generating device (reusable by later chunks)


def generate(cfg: str = "C2", n_fam: int = 1000, seed: int = 42, device=None, genome_len: int = 10_000_000,
             read_len: int = 150, chunk: int = 1 << 22, frag: Optional[Tuple[float, float, int]] = None,
             reuse: Optional["SynthSet"] = None, long_frac: float = 0.0, long_span: Tuple[int, int] = (20_000, 5_000_000),
             long_giant: bool = False) -> SynthSet:
    """frag = (mean, sd, min) overrides the fragment-length model (tests use short inserts to
    exercise read-through trimming; the configs keep the survey's model).  reuse: draw the
    families on that set's genome (one reference for a stream of chunks).  long_frac: that
    fraction of families get a long-span template pair -- fragments log-uniform in long_span
    (capped at half the genome), the mates that far apart on one contig (discordant pairs of
    whole-genome data); long_giant: family 0's fragment spans 60 % of the genome.  The other
    families are drawn as without them."""
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    L = read_len
    if reuse is not None and reuse.genome is not None:
        genome = reuse.genome.to(device)
        genome_len = int(genome.shape[0])
    else:
        genome = make_genome(genome_len, gen, device)
    na, nb = family_sizes(cfg, n_fam, gen, device)
    fam_ab_top = torch.rand(n_fam, generator=gen, device=device) < 0.5
    if frag is not None:
        fl = torch.normal(float(frag[0]), float(frag[1]), (n_fam,), generator=gen, device=device)
        fl = fl.round().clamp(int(frag[2]), 600).to(torch.int64)
    else:
        if cfg == "C3":
            fl = torch.normal(200.0, 30.0, (n_fam,), generator=gen, device=device)
        else:
            fl = torch.normal(300.0, 80.0, (n_fam,), generator=gen, device=device)
        fl = fl.round().clamp(160, 600).to(torch.int64)
        fl = torch.clamp(fl, min=L + 2)
    s = (torch.rand(n_fam, generator=gen, device=device) * (genome_len - 1400)).to(torch.int64) + 700
    if long_frac > 0 or long_giant:
        import math
        lf = torch.rand(n_fam, generator=gen, device=device) < long_frac
        lo, hi = math.log(long_span[0]), math.log(max(long_span[0] + 1, min(long_span[1], genome_len // 2)))
        u = torch.rand(n_fam, generator=gen, device=device)
        big = torch.exp(lo + u * (hi - lo)).to(torch.int64)
        if long_giant:
            lf[0] = True
            big[0] = genome_len * 6 // 10
        fl = torch.where(lf, big, fl)
        sl = (torch.rand(n_fam, generator=gen, device=device) * (genome_len - fl - 1400).clamp_min(1)).to(torch.int64) + 700
        s = torch.where(lf, sl, s)
    e = s + fl

    # templates: family-major, AB templates first
    nt = na + nb
    T = int(nt.sum())
    tfam = torch.repeat_interleave(torch.arange(n_fam, device=device), nt)
    tstart = torch.cumsum(nt, 0) - nt
    within = torch.arange(T, device=device) - tstart[tfam]
    tstrand = (within >= na[tfam]).to(torch.int64)             # 0 = A, 1 = B
    ttop = fam_ab_top[tfam] ^ (tstrand == 1)                   # AB top -> BA bottom
    # records: 2 per template; R = 2 T
    rt = torch.repeat_interleave(torch.arange(T, device=device), 2)
    is_r1 = (torch.arange(2 * T, device=device) % 2) == 0
    top = ttop[rt]
    fam = tfam[rt]
    # top: R1 99 fwd at s, R2 147 rev at e-L; bottom: R1 83 rev at e-L, R2 163 fwd at s
    fwd = torch.where(top, is_r1, ~is_r1)
    pos = torch.where(fwd, s[fam], e[fam] - L)
    flag = torch.where(top, torch.where(is_r1, 99, 147), torch.where(is_r1, 83, 163)).to(torch.int64)
    mate_pos = torch.where(fwd, e[fam] - L, s[fam])
    tlen = torch.where(fwd, fl[fam], -fl[fam])
    nrec = 2 * T

    # order within family: by position, R1 first on ties (coordinate-sorted-like)
    key = fam * (1 << 40) + pos * 2 + (~is_r1).to(torch.int64)
    order = torch.argsort(key)
    rt, fam, pos, flag, mate_pos, tlen, top, is_r1 = (x[order] for x in (rt, fam, pos, flag, mate_pos, tlen, top, is_r1))
    strand = tstrand[rt]

    seq = torch.empty(nrec * L, dtype=torch.uint8, device=device)
    qual = torch.empty(nrec * L, dtype=torch.uint8, device=device)
    ar = torch.arange(L, device=device)
    qvals = torch.tensor([37, 25, 12, 2], dtype=torch.uint8, device=device)
    for c0 in range(0, nrec, max(1, chunk // L)):
        c1 = min(nrec, c0 + max(1, chunk // L))
        p = pos[c0:c1, None] + ar[None, :]                     # ref positions
        ref = genome[p]
        nxt = genome[(p + 1).clamp_max(genome_len - 1)]
        prv = genome[(p - 1).clamp_min(0)]
        f = fam[c0:c1, None].expand_as(p)
        tp = top[c0:c1, None].expand_as(p)
        # methylation keyed by the C of the site (top: p, bottom: p-1 for a CpG G)
        cpg_top = (ref == 2) & (nxt == 4)
        cpg_bot = (ref == 4) & (prv == 2)
        site = torch.where(tp, p, torch.where(cpg_bot, p - 1, p))
        u = _hash_u01(f, site)
        pm = torch.where(torch.where(tp, cpg_top, cpg_bot), 0.75, 0.005)
        meth = u < pm
        b = ref.clone()
        b = torch.where(tp & (ref == 2) & ~meth, torch.full_like(b, 8), b)     # top: unmethylated C -> T
        b = torch.where(~tp & (ref == 4) & ~meth, torch.full_like(b, 1), b)    # bottom: unmethylated G -> A
        # qualities: bins with a tail decaying along the read
        rr = torch.rand(p.shape, generator=gen, device=device)
        frac = (ar[None, :].to(torch.float32) / L)
        p37 = 0.88 - 0.25 * frac
        p25 = p37 + 0.08 + 0.1 * frac
        qi = torch.where(rr < p37, 0, torch.where(rr < p25, 1, torch.where(rr < 0.999, 2, 3)))
        q = qvals[qi]
        # sequencing errors at the base's own quality; Q2 bases become N
        err = torch.rand(p.shape, generator=gen, device=device) < torch.pow(10.0, -q.to(torch.float32) / 10.0)
        alt = torch.tensor([1, 2, 4, 8], dtype=torch.uint8, device=device)[
            torch.randint(0, 4, p.shape, generator=gen, device=device)]
        alt = torch.where(alt == b, torch.where(b == 1, torch.full_like(b, 8), torch.full_like(b, 1)), alt)
        b = torch.where(err, alt, b)
        b = torch.where(q == 2, torch.full_like(b, 15), b)
        seq[c0 * L:c1 * L] = b.reshape(-1)
        qual[c0 * L:c1 * L] = q.reshape(-1)

    to = lambda x, dt: x.to("cpu").numpy().astype(dt)
    n = nrec
    raw = R.RawRecords(
        flag=to(flag, np.uint16), tid=np.zeros(n, np.int32), pos=to(pos, np.int32),
        mapq=np.full(n, 60, np.uint8), l_seq=np.full(n, L, np.int32),
        seq_off=np.arange(n, dtype=np.int64) * L, seq=to(seq, np.uint8), qual=to(qual, np.uint8),
        cig_off=np.arange(n, dtype=np.int64), n_cig=np.ones(n, np.int32),
        cigar=np.full(n, (L << 4) | 0, np.uint32), next_tid=np.zeros(n, np.int32),
        next_pos=to(mate_pos, np.int32), tlen=to(tlen, np.int32), name_id=to(rt, np.int32),
        names=_LazyNames("t"), mi_id=to(fam, np.int32), mi_strand=to(strand, np.int8),
        mi_names=_LazyNames(""), mc_off=np.arange(n, dtype=np.int64), mc_n=np.ones(n, np.int32),
        mc_cigar=np.full(n, (L << 4) | 0, np.uint32), aux=None, la_tag=None, rd_tag=None)
    ref = reuse.ref if reuse is not None else R.Reference.from_codes(["chrS"], [genome.to("cpu").numpy()])
    return SynthSet(raw, ref, cfg, n_fam, genome)


class _LazyNames:
    """names[i] without materialising millions of Python objects."""

    def __init__(self, prefix: str):
        self.prefix = prefix

    def __getitem__(self, i):
        s = "%s%d" % (self.prefix, i)
        return s.encode() if self.prefix else s

    def __len__(self):
        return 1 << 62

    def lex_key(self, ids: np.ndarray) -> np.ndarray:
        """int64 keys that order ids as their strings sort in byte order (one prefix, decimal
        digits): the digits left-aligned to 10 places, then the digit count (a prefix first)."""
        x = np.asarray(ids, np.int64)
        d = np.ones_like(x)
        for k in range(1, 11):
            d += x >= 10 ** k
        return (x * 10 ** (10 - d)) * 16 + d


def messify(raw: R.RawRecords, frac: float = 0.1, seed: int = 1) -> R.RawRecords:
    """Sprinkle the edge cases the tools handle differently: soft clips, I/D/N ops, hard clips,
    extra N bases, a few odd flags.  Small inputs only (per-record Python)."""
    rng = np.random.default_rng(seed)
    b = R._Builder()
    for k in range(raw.n):
        seq = raw.record_seq(k).copy()
        qual = raw.record_qual(k).copy()
        cig = [int(x) for x in raw.record_cigar(k)]
        flag = int(raw.flag[k])
        pos = int(raw.pos[k])
        L = len(seq)
        r = rng.random()
        if r < frac:
            kind = rng.integers(0, 7)
            if kind == 0:  # leading soft clip (clipped bases were not aligned: pos moves right)
                a = int(rng.integers(1, 10))
                cig = [(a << 4) | R.OP_S, ((L - a) << 4) | R.OP_M]
                pos += a
            elif kind == 1:
                a = int(rng.integers(1, 10))
                cig = [((L - a) << 4) | R.OP_M, (a << 4) | R.OP_S]
            elif kind == 2:  # insertion
                a = int(rng.integers(20, L - 20))
                cig = [(a << 4) | R.OP_M, (2 << 4) | R.OP_I, ((L - a - 2) << 4) | R.OP_M]
            elif kind == 3:  # deletion
                a = int(rng.integers(20, L - 20))
                cig = [(a << 4) | R.OP_M, (3 << 4) | R.OP_D, ((L - a) << 4) | R.OP_M]
            elif kind == 4:  # hard clip
                cig = [(5 << 4) | R.OP_H] + cig
            elif kind == 5:  # a run of N
                a = int(rng.integers(0, L - 5))
                seq[a:a + 5] = 15
                qual[a:a + 5] = 2
            else:  # trailing Ns
                seq[L - 3:] = 15
                qual[L - 3:] = 2
        tags = [("MI", "Z", "%s/%s" % (raw.mi_id[k], "A" if raw.mi_strand[k] == 0 else "B")),
                ("MC", "Z", "%dM" % L), ("RX", "Z", "ACGT-TGCA")]
        b.add(("t%d" % raw.name_id[k]).encode(), flag, int(raw.tid[k]), pos, 60, cig, seq, qual,
              int(raw.next_tid[k]), int(raw.next_pos[k]), int(raw.tlen[k]), R.encode_aux(tags), tags)
    return b.finish()


def subset_families(raw: R.RawRecords, n_fam: int) -> R.RawRecords:
    """The records of families 0..n_fam-1 of a generate() stream (records are family-major)."""
    k = int(np.searchsorted(raw.mi_id, n_fam, side="left"))
    so, co, mo = int(raw.seq_off[k]) if k < raw.n else raw.seq.shape[0], \
        int(raw.cig_off[k]) if k < raw.n else raw.cigar.shape[0], int(raw.mc_off[k]) if k < raw.n else raw.mc_cigar.shape[0]
    return R.RawRecords(
        flag=raw.flag[:k], tid=raw.tid[:k], pos=raw.pos[:k], mapq=raw.mapq[:k], l_seq=raw.l_seq[:k],
        seq_off=raw.seq_off[:k], seq=raw.seq[:so], qual=raw.qual[:so], cig_off=raw.cig_off[:k], n_cig=raw.n_cig[:k],
        cigar=raw.cigar[:co], next_tid=raw.next_tid[:k], next_pos=raw.next_pos[:k], tlen=raw.tlen[:k],
        name_id=raw.name_id[:k], names=raw.names, mi_id=raw.mi_id[:k], mi_strand=raw.mi_strand[:k],
        mi_names=raw.mi_names, mc_off=raw.mc_off[:k], mc_n=raw.mc_n[:k], mc_cigar=raw.mc_cigar[:mo])
