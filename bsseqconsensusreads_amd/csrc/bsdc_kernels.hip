// bsdc_kernels.hip -- gfx950 kernels and the C-ABI (include/bsdc.h) of the step-5 duplex path.
//
// One launch does, per MI family, everything rules convert_Bstrain -> extend -> groupsort_convert
// -> callduplex do (main.snake.py:121-164) after the host has formed the families:
//   phase 1  B-strand conversion        tools/1.convert_AG_to_CT.py:84-183
//   phase 2  gap extension              tools/2.extend_gap.py:58-110 (4-record groups, :112-140)
//   phase 3  overlapping-bases consensus    fgbio, --consensus-call-overlapping-bases=true
//   phase 4  source reads                   fgbio toSourceRead (orientation, read-through, trailing N)
//   phase 5  most-common-alignment filter   fgbio filterToMostCommonAlignment
//   phase 6  single-strand likelihood vote  fgbio VanillaUmiConsensusCaller (pre 45 / post 30)
//   phase 7  duplex combine                 fgbio DuplexConsensusCaller.duplexConsensus
// The fgbio rows are restated from its public behaviour (parity unpinned).
//
// Layout: a family's records are staged once from HBM into an arena (LDS for the small-family
// kernel: one wavefront per family; LDS or global scratch for the large-family kernel: one
// 256-thread workgroup per family), every phase works in the arena, and only the consensus pair
// (packed nt16 + quals) goes back to HBM.  All integer / byte work; the vote's likelihood sums
// are exact fixed-point int64 so any summation order is bit-identical to the CPU restatement.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bsdc.h"

namespace {

constexpr int kWave = 64;
constexpr int kLargeThreads = 256;
constexpr int kSmallWaves = 4;  // wavefronts (families) per small-kernel workgroup
constexpr double kLrScale = 1099511627776.0;  // 2^40
constexpr double kLrInvScale = 9.094947017729282379150390625e-13;

// nt16 codes
constexpr uint8_t kA = 1, kC = 2, kG = 4, kT = 8, kN = 15;

struct RecMeta {  // 48 B, one per record of the family, in the arena
    int32_t pos;     // current leftmost position
    int32_t len;     // current length
    uint32_t slot;   // arena offset of the base slot (quals at slot + cap)
    int32_t cap;     // slot capacity (input length + 2)
    int32_t start;   // index of the first base inside the slot
    uint32_t link;
    uint32_t gidx;   // global record index
    int32_t tid;
    int32_t srclen;  // source-read length (phase 4)
    int32_t reflen;  // current reference length
    uint16_t flag;
    uint8_t rd;
    uint8_t set;     // 0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2, 0xFF none
    int32_t in_len;
};
static_assert(sizeof(RecMeta) == 48, "RecMeta layout");

struct Tables {
    long long lr[256];
    float thr[96];
};

__host__ __device__ inline int64_t round16(int64_t x) { return (x + 15) & ~int64_t(15); }

// Arena layout of one family (offsets from the arena base).
struct ArenaLayout {
    uint32_t meta, lists, ssb, ssq, simp, slots, total;
    int32_t ssw;
    __host__ __device__ ArenaLayout(int n, int64_t sum_len, int max_len, int64_t complex_ops) {
        ssw = (int32_t)round16(max_len + 2);
        int64_t o = 0;
        meta = (uint32_t)o;
        o += round16((int64_t)n * (int64_t)sizeof(RecMeta));
        lists = (uint32_t)o;
        o += round16((int64_t)n * 8);
        ssb = (uint32_t)o;
        o += 4 * (int64_t)ssw;
        ssq = (uint32_t)o;
        o += 4 * (int64_t)ssw;
        simp = (uint32_t)o;
        if (complex_ops > 0) o += round16(4 * (complex_ops + 4 * (int64_t)n));
        slots = (uint32_t)o;
        o += round16(2 * sum_len + 4 * (int64_t)n);
        total = (uint32_t)o;
    }
};

// ------------------------------------------------------------------------------------------
// group abstraction: a wavefront (G = 64) or a workgroup (G = 256)
// ------------------------------------------------------------------------------------------
template <int G>
struct Grp {
    int t;
    int *red;  // LDS scratch of G/64 ints (G > 64 only)
    __device__ __forceinline__ void sync() const {
        if constexpr (G == kWave) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
    }
    __device__ __forceinline__ int max(int v) const {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v = ::max(v, __shfl_xor(v, o, kWave));
        if constexpr (G == kWave) {
            return v;
        } else {
            sync();
            if ((t & 63) == 0) red[t >> 6] = v;
            sync();
            int r = red[0];
#pragma unroll
            for (int w = 1; w < G / kWave; w++) r = ::max(r, red[w]);
            sync();
            return r;
        }
    }
    __device__ __forceinline__ int any(int v) const { return max(v ? 1 : 0); }
};

// ------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint8_t nib(const uint8_t *p, int64_t k) {
    const uint8_t b = p[k >> 1];
    return (k & 1) ? (b & 0xF) : (b >> 4);
}
// htsjdk complement: A<->T, C<->G, everything else unchanged
__device__ __forceinline__ uint8_t comp_nt16(uint8_t b) {
    return b == kA ? kT : b == kT ? kA : b == kC ? kG : b == kG ? kC : b;
}
__device__ __forceinline__ int base_idx(uint8_t b) {
    return b == kA ? 0 : b == kC ? 1 : b == kG ? 2 : b == kT ? 3 : -1;
}
__device__ __forceinline__ float det_expf(float x) {
    // keep in step with oracle/bsdc_oracle.c orc_det_expf: same reduction, same fma chain
    const float t = x * 1.44269504088896341f;
    const float n = rintf(t);
    float r = fmaf(n, -6.93145751953125e-1f, x);
    r = fmaf(n, -1.428606765330187e-6f, r);
    float p = 1.38888889e-3f;
    p = fmaf(p, r, 8.33333333e-3f);
    p = fmaf(p, r, 4.16666667e-2f);
    p = fmaf(p, r, 1.66666667e-1f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return ldexpf(p, (int)n);
}

struct RefView {
    const uint8_t *seq;
    const int64_t *off;
    const int64_t *len;
    int32_t n;
};

// reference nibble at contig position p (N past the contig end or for an absent contig)
__device__ __forceinline__ uint8_t ref_at(const RefView &R, int32_t tid, int64_t p) {
    if (tid < 0 || tid >= R.n) return kN;
    const int64_t o = R.off[tid];
    if (o < 0 || p < 0 || p >= R.len[tid]) return kN;
    return nib(R.seq, o + p);
}

// tool 1 per-base rule (tools/1.convert_AG_to_CT.py:123-150), in its local form: the value at i
// depends on m[i], m[i+1], ref[i], ref[i+1] only (the skip at :140 writes what the A rule would)
__device__ __forceinline__ uint8_t convert_rule(uint8_t m0, uint8_t m1, bool has_next, uint8_t f0, uint8_t f1) {
    if (m0 == kA) return f0 == kG ? kG : kA;
    if (m0 == kC) {
        if (f0 == kC && f1 == kG) return (has_next && m1 == kA) ? kT : kC;
        return kT;
    }
    return m0;
}

// Cigar of the current record for complex records: [npre x M1] + input ops (the last one
// shortened by one when tool 1 trimmed a base: RD, tools/1.convert_AG_to_CT.py:161-167) +
// [nsuf x M1].  Op k of the view, k < npre + n + nsuf; a zero-length op is skipped by callers.
struct CigView {
    const uint32_t *ops;
    int n;
    int npre, nsuf;
    int rdtrim;
    __device__ __forceinline__ int count() const { return npre + n + nsuf; }
    __device__ __forceinline__ void at(int k, int &op, int32_t &l) const {
        if (k < npre || k >= npre + n) {
            op = 0;
            l = 1;
            if (rdtrim && n == 0 && k == npre - 1) l = 0;
            return;
        }
        const uint32_t c = ops[k - npre];
        op = (int)(c & 0xF);
        l = (int32_t)(c >> 4);
        if (rdtrim && k == npre + n - 1) l -= 1;
    }
};

// read offset aligned to reference position p, or -1
__device__ int read_at_ref(const CigView &c, int32_t pos, int32_t len, int64_t p) {
    int64_t rp = pos;
    int32_t qp = 0;
    const int nk = c.count();
    for (int k = 0; k < nk; k++) {
        int op;
        int32_t l;
        c.at(k, op, l);
        if (op == 0 || op == 7 || op == 8) {
            if (p >= rp && p < rp + l) {
                const int32_t q = qp + (int32_t)(p - rp);
                return q < len ? q : -1;
            }
            rp += l;
            qp += l;
        } else if (op == 1 || op == 4) {
            qp += l;
        } else if (op == 2 || op == 3) {
            if (p >= rp && p < rp + l) return -1;
            rp += l;
        }
    }
    return -1;
}

struct KParams {
    bsdc_family_batch B;
    bsdc_consensus O;
    RefView R;
    const Tables *tab;
    int32_t mode;
    int32_t overlap;
};

// ------------------------------------------------------------------------------------------
// one family, processed by group g in arena A
// ------------------------------------------------------------------------------------------
template <int G>
__device__ void process_family(const KParams &P, const Grp<G> &g, uint8_t *A, const long long *lr,
                               const float *thr, uint32_t fam) {
    const bsdc_family_batch &B = P.B;
    const uint32_t r0 = B.fam_off[fam];
    const int n = (int)(B.fam_off[fam + 1] - r0);
    const uint32_t off0 = n > 0 ? B.rec_off[r0] : 0u;
    const bool do_convert = P.mode & BSDC_MODE_CONVERT;
    const bool do_extend = P.mode & BSDC_MODE_EXTEND;
    const bool do_vote = P.mode & BSDC_MODE_VOTE;

    // complex-cigar op count of the family (sizes the arena's simplified-cigar region)
    int64_t cops = 0;
    int maxlen_f = 0;
    {
        int c = 0, ml = 0;
        for (int r = g.t; r < n; r += G) {
            const uint32_t lk = B.rec_link[r0 + r];
            if (lk & BSDC_LINK_COMPLEX) c += (int)(B.cig_info[r0 + r] & 0xFFFF);
            ml = ::max(ml, (int)(B.rec_lenflag[r0 + r] & 0xFFFF));
        }
        // sum via max-of-prefix is not available; complex families are rare: use a group sum by max trick
        // (sum over lanes with shuffles)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, kWave);
        if constexpr (G > kWave) {
            g.sync();
            if ((g.t & 63) == 0) g.red[g.t >> 6] = c;
            g.sync();
            int s = 0;
            for (int w = 0; w < G / kWave; w++) s += g.red[w];
            c = s;
            g.sync();
        }
        cops = c;
        maxlen_f = g.max(ml);
    }
    const ArenaLayout L(n, 0, maxlen_f, cops);  // slot region placed last; its size is not needed here
    RecMeta *M = reinterpret_cast<RecMeta *>(A + L.meta);
    uint16_t *lists = reinterpret_cast<uint16_t *>(A + L.lists);
    uint8_t *ssb = A + L.ssb;
    uint8_t *ssq = A + L.ssq;
    uint32_t *simp = reinterpret_cast<uint32_t *>(A + L.simp);
    uint8_t *slots = A + L.slots;
    const int ssw = L.ssw;

    // ---- phase 0: record metadata ----
    for (int r = g.t; r < n; r += G) {
        const uint32_t gi = r0 + r;
        const uint32_t lf = B.rec_lenflag[gi];
        RecMeta m;
        m.in_len = (int32_t)(lf & 0xFFFF);
        m.flag = (uint16_t)(lf >> 16);
        m.pos = B.rec_pos[gi];
        m.len = m.in_len;
        m.cap = m.in_len + 2;
        m.slot = 2u * (B.rec_off[gi] - off0) + 4u * (uint32_t)r;
        m.start = 1;
        m.link = B.rec_link[gi];
        m.gidx = gi;
        m.tid = B.rec_tid[gi];
        m.srclen = 0;
        m.reflen = (m.link & BSDC_LINK_COMPLEX) ? (int32_t)(B.cig_info[gi] >> 16) : m.in_len;
        m.rd = 0;
        m.set = 0xFF;
        M[r] = m;
    }
    g.sync();

    // ---- phase 1: stage bases + tool-1 conversion (tools/1.convert_AG_to_CT.py:84-183) ----
    for (int r = 0; r < n; r++) {
        const RecMeta m = M[r];
        const int32_t Lin = m.in_len;
        const int64_t ib = (int64_t)B.rec_off[m.gidx];
        uint8_t *sb = slots + m.slot;
        uint8_t *sq = sb + m.cap;
        if (do_convert && (m.link & BSDC_LINK_CONVERT)) {
            const int32_t Lm = Lin + 1;                       // 'N' + seq
            const int32_t np = m.pos - 1 > 0 ? m.pos - 1 : 0; // :92
            for (int j = g.t; j < Lm; j += G) {
                const uint8_t f0 = ref_at(P.R, m.tid, (int64_t)np + j);
                const uint8_t f1 = ref_at(P.R, m.tid, (int64_t)np + j + 1);
                const uint8_t m0 = j == 0 ? f0 : nib(B.seq, ib + j - 1);  // :121 seed
                const bool has_next = j + 1 < Lm;
                const uint8_t m1 = has_next ? nib(B.seq, ib + j) : kN;
                const uint8_t o = convert_rule(m0, m1, has_next, f0, f1);
                sb[j] = o;
                sq[j] = j == 0 ? (uint8_t)40 : B.qual[ib + j - 1];     // :174-177 'I' + quals
                if (j == Lm - 1) {
                    // :157-170 trailing C before a reference G is trimmed
                    const uint8_t f2 = ref_at(P.R, m.tid, (int64_t)np + Lm);
                    const uint8_t rd = (f2 == kG && o == kC) ? 1 : 0;
                    RecMeta &w = M[r];
                    w.rd = rd;
                    w.len = Lm - rd;
                    w.start = 0;
                    w.pos = np;
                    w.reflen = m.reflen + 1 - ((rd && m.reflen > 0) ? 1 : 0);
                }
            }
        } else {
            for (int j = g.t; j < Lin; j += G) {
                sb[1 + j] = nib(B.seq, ib + j);
                sq[1 + j] = B.qual[ib + j];
            }
        }
    }
    g.sync();

    // ---- phase 2: gap extension of 4-record groups (tools/2.extend_gap.py:58-110) ----
    if (do_extend) {
        for (int r = g.t; r < n; r += G) {
            const RecMeta m = M[r];
            const int p = (int)((m.link >> BSDC_LINK_PARTNER_SHIFT) & 3u);
            const RecMeta pm = M[p];
            const uint8_t *pb = slots + pm.slot;
            const uint8_t *pq = pb + pm.cap;
            if (m.link & BSDC_LINK_EXT_RIGHT) {
                // :70-80 the converted partner's first base / qual, POS-1, [(M,1)] + cigar
                // the partner is converted (start 0 when converted in this launch, else 1); its
                // first base is never touched by its own append (length >= 1)
                const int ps = (do_convert && (pm.link & BSDC_LINK_CONVERT)) ? 0 : 1;
                uint8_t *sb = slots + m.slot;
                sb[0] = pb[ps];
                sb[m.cap] = pq[ps];
                RecMeta &w = M[r];
                w.start = 0;
                w.len = m.len + 1;
                w.pos = m.pos - 1;
                w.reflen = m.reflen + 1;
            }
        }
        g.sync();
        for (int r = g.t; r < n; r += G) {
            const RecMeta m = M[r];
            const int p = (int)((m.link >> BSDC_LINK_PARTNER_SHIFT) & 3u);
            const bool rd = (do_convert && (m.link & BSDC_LINK_CONVERT)) ? (m.rd != 0) : ((m.link & BSDC_LINK_RD_IN) != 0);
            if ((m.link & BSDC_LINK_EXT_LEFT) && rd) {
                // :92-101 the partner's last base / qual (after its prepend), cigar + [(M,1)]
                const RecMeta pm = M[p];
                const uint8_t *pb = slots + pm.slot;
                uint8_t *sb = slots + m.slot;
                const int li = pm.start + pm.len - 1;
                sb[m.start + m.len] = pb[li];
                sb[m.cap + m.start + m.len] = pb[pm.cap + li];
                RecMeta &w = M[r];
                w.len = m.len + 1;
                w.reflen = m.reflen + 1;
            }
        }
        g.sync();
    }

    // ---- stage dump: the records as tool 2 writes them ----
    if (P.mode & BSDC_MODE_DUMP) {
        for (int r = 0; r < n; r++) {
            const RecMeta m = M[r];
            const int64_t d = (int64_t)B.rec_off[m.gidx] + 2 * (int64_t)m.gidx;
            const uint8_t *sb = slots + m.slot + m.start;
            for (int j = g.t; j < m.len; j += G) {
                P.O.dump_seq[d + j] = sb[j];
                P.O.dump_qual[d + j] = sb[m.cap + j];
            }
            if (g.t == 0) {
                P.O.dump_pos[m.gidx] = m.pos;
                P.O.dump_len[m.gidx] = (uint16_t)m.len;
                const bool conv = do_convert && (m.link & BSDC_LINK_CONVERT);
                const bool rd = conv ? (m.rd != 0) : ((m.link & BSDC_LINK_RD_IN) != 0);
                uint8_t tg = 0;
                if (rd) tg |= 1;
                if (conv) tg |= 2 | 4;
                if (do_extend && (m.link & BSDC_LINK_EXT_RIGHT)) tg |= 4;
                if (do_extend && (m.link & BSDC_LINK_EXT_LEFT) && rd) tg |= 8;
                P.O.dump_tags[m.gidx] = tg;
            }
        }
    }
    if (!do_vote) return;

    // complex-cigar view of record r in its current state
    auto cigview = [&](const RecMeta &m) {
        CigView c;
        c.ops = B.cigar + B.cig_off[m.gidx];
        c.n = (int)(B.cig_info[m.gidx] & 0xFFFF);
        const bool conv = do_convert && (m.link & BSDC_LINK_CONVERT);
        const bool rd = conv ? (m.rd != 0) : ((m.link & BSDC_LINK_RD_IN) != 0);
        c.npre = (conv || (do_extend && (m.link & BSDC_LINK_EXT_RIGHT))) ? 1 : 0;
        c.nsuf = (do_extend && (m.link & BSDC_LINK_EXT_LEFT) && rd) ? 1 : 0;
        c.rdtrim = (conv && rd) ? 1 : 0;
        return c;
    };

    // ---- phase 3: overlapping-bases consensus, per template ----
    if (P.overlap) {
        for (int r = 0; r < n; r++) {
            const RecMeta a = M[r];
            const uint32_t mate = a.link & BSDC_LINK_MATE_MASK;
            if (mate == BSDC_LINK_MATE_MASK || !(a.link & BSDC_LINK_USABLE)) continue;
            const RecMeta b = M[mate];
            if (!(b.link & BSDC_LINK_USABLE)) continue;
            if ((a.flag & 4) || (b.flag & 4) || a.tid != b.tid) continue;
            if (a.reflen <= 0 || b.reflen <= 0) continue;
            const int32_t s = ::max(a.pos, b.pos);
            const int32_t e = ::min(a.pos + a.reflen - 1, b.pos + b.reflen - 1);
            if (s > e) continue;
            const bool ca = a.link & BSDC_LINK_COMPLEX, cb = b.link & BSDC_LINK_COMPLEX;
            uint8_t *ab = slots + a.slot + a.start;
            uint8_t *aq = slots + a.slot + a.cap + a.start;
            uint8_t *bb = slots + b.slot + b.start;
            uint8_t *bq = slots + b.slot + b.cap + b.start;
            for (int32_t p = s + g.t; p <= e; p += G) {
                const int ia = ca ? read_at_ref(cigview(a), a.pos, a.len, p) : (p - a.pos < a.len ? p - a.pos : -1);
                const int ibb = cb ? read_at_ref(cigview(b), b.pos, b.len, p) : (p - b.pos < b.len ? p - b.pos : -1);
                if (ia < 0 || ibb < 0) continue;
                const uint8_t x = ab[ia], y = bb[ibb];
                if (x == kN || y == kN) continue;
                const int qa = aq[ia], qb = bq[ibb];
                if (x == y) {
                    const uint8_t q = (uint8_t)::min(qa + qb, 93);
                    aq[ia] = q;
                    bq[ibb] = q;
                } else if (qa > qb) {
                    bb[ibb] = x;
                    aq[ia] = bq[ibb] = (uint8_t)(qa - qb);
                } else if (qb > qa) {
                    ab[ia] = y;
                    aq[ia] = bq[ibb] = (uint8_t)(qb - qa);
                } else {
                    ab[ia] = bb[ibb] = kN;
                    aq[ia] = bq[ibb] = 2;
                }
            }
        }
        g.sync();
    }

    // ---- phase 4: source reads (orientation, read-through trim, trailing-N trim) ----
    for (int r = g.t; r < n; r += G) {
        RecMeta &m = M[r];
        if (!(m.link & BSDC_LINK_USABLE)) continue;
        const bool neg = m.flag & 16;
        int32_t keep = m.len;
        if (m.link & BSDC_LINK_RT) {
            const int32_t *rt = B.rt + 4 * (int64_t)m.gidx;
            const int32_t next_pos = rt[0], tlen = rt[1], mate_us = rt[2], mate_ue = rt[3];
            // fgbio isFrPair (htsjdk getPairOrientation == FR); RT is only set on records that are
            // paired, mapped, mate mapped, on the mate's contig and carry an MC tag
            const bool mneg = m.flag & 32;
            bool fr = false;
            if (neg != mneg) {
                const int64_t posfive = neg ? (int64_t)next_pos : (int64_t)m.pos;
                const int64_t negfive = neg ? (int64_t)m.pos + m.reflen - 1 : (int64_t)m.pos + tlen;
                fr = posfive < negfive;
            }
            if (fr) {
                const bool cx = m.link & BSDC_LINK_COMPLEX;
                if (!neg) {
                    const int64_t end = (int64_t)m.pos + m.reflen - 1;
                    if (end > mate_ue) {
                        int32_t kk;
                        if (!cx) {
                            kk = (int32_t)::min<int64_t>((int64_t)mate_ue - m.pos + 1, m.len);
                            if (kk < 0) kk = 0;
                        } else {
                            int last = -1;
                            const CigView c = cigview(m);
                            for (int64_t p = m.pos; p <= mate_ue && p < (int64_t)m.pos + m.reflen; p++) {
                                const int q = read_at_ref(c, m.pos, m.len, p);
                                if (q >= 0) last = q;
                            }
                            kk = last + 1;
                        }
                        keep = ::min(keep, kk);
                    }
                } else {
                    if ((int64_t)m.pos < mate_us) {
                        int32_t kk;
                        if (!cx) {
                            const int64_t first = (int64_t)mate_us - m.pos;
                            kk = first >= m.len ? 0 : (int32_t)(m.len - first);
                        } else {
                            int first = m.len;
                            const CigView c = cigview(m);
                            for (int64_t p = (int64_t)m.pos + m.reflen - 1; p >= mate_us && p >= m.pos; p--) {
                                const int q = read_at_ref(c, m.pos, m.len, p);
                                if (q >= 0) first = q;
                            }
                            kk = m.len - first;
                        }
                        keep = ::min(keep, kk);
                    }
                }
            }
        }
        const uint8_t *sb = slots + m.slot + m.start;
        while (keep > 0) {
            const uint8_t b = neg ? sb[m.len - keep] : sb[keep - 1];
            if (b != kN) break;
            keep--;
        }
        m.srclen = keep;
        if (keep > 0) {
            const bool r1 = m.flag & 0x40;
            const bool ab = m.link & BSDC_LINK_AB;
            m.set = ab ? (r1 ? 0 : 1) : (r1 ? 2 : 3);
        }
    }
    g.sync();

    // ---- phase 5: most-common-alignment filter (only families with a non-M-only cigar) ----
    int has_complex = 0;
    for (int r = g.t; r < n; r += G) has_complex |= (M[r].link & BSDC_LINK_COMPLEX) && M[r].set != 0xFF;
    if (g.any(has_complex)) {
        if (g.t == 0) {
            // simplified cigars (sequencing orientation, M/=/X -> M, merged, truncated)
            uint32_t *so = simp;                 // ops
            uint32_t *sofs = simp + cops + 2 * n; // per record: offset | count << 16 (n entries)
            uint32_t fill = 0;
            for (int r = 0; r < n; r++) {
                const RecMeta &m = M[r];
                sofs[r] = 0;
                if (m.set == 0xFF) continue;
                const uint32_t base = fill;
                int cnt = 0;
                if (!(m.link & BSDC_LINK_COMPLEX)) {
                    so[fill++] = ((uint32_t)m.srclen << 4) | 0u;
                    cnt = 1;
                } else {
                    const CigView c = cigview(m);
                    const bool neg = m.flag & 16;
                    const int tot = c.count();
                    int32_t q = 0;
                    for (int j = 0; j < tot && q < m.srclen; j++) {
                        const int k = neg ? tot - 1 - j : j;
                        int op;
                        int32_t l;
                        c.at(k, op, l);
                        if (l <= 0) continue;
                        if (op == 7 || op == 8) op = 0;
                        if (op == 4 || op == 5) continue;
                        if (op == 0 || op == 1) {
                            if (q + l > m.srclen) l = m.srclen - q;
                            q += l;
                        }
                        if (cnt > 0 && (int)(so[fill - 1] & 0xF) == op) {
                            so[fill - 1] = ((((so[fill - 1] >> 4) + (uint32_t)l)) << 4) | (uint32_t)op;
                        } else {
                            so[fill++] = ((uint32_t)l << 4) | (uint32_t)op;
                            cnt++;
                        }
                    }
                }
                sofs[r] = base | ((uint32_t)cnt << 16);
            }
            // X = {AB-R1, BA-R2} (sets 0, 3), Y = {AB-R2, BA-R1} (sets 1, 2); AB records first
            uint16_t *ord = lists;  // scratch: n entries
            uint8_t *member = ssb;  // scratch bitmap rows are too big in general: use group ids
            (void)member;
            for (int xy = 0; xy < 2; xy++) {
                const int sa = xy == 0 ? 0 : 1, sbb = xy == 0 ? 3 : 2;
                int cnt = 0;
                for (int r = 0; r < n; r++)
                    if (M[r].set == sa) ord[cnt++] = (uint16_t)r;
                for (int r = 0; r < n; r++)
                    if (M[r].set == sbb) ord[cnt++] = (uint16_t)r;
                if (cnt < 2) continue;
                // stable sort by srclen descending
                for (int i = 1; i < cnt; i++) {
                    const uint16_t x = ord[i];
                    int j = i - 1;
                    while (j >= 0 && M[ord[j]].srclen < M[x].srclen) {
                        ord[j + 1] = ord[j];
                        j--;
                    }
                    ord[j + 1] = x;
                }
                // groups: defining read + size; membership recomputed for the winner below
                int ng = 0;
                uint16_t gdef[64];
                int gsize[64];
                bool overflow = false;
                for (int i = 0; i < cnt; i++) {
                    const uint32_t ai = sofs[ord[i]];
                    const uint32_t *ac = so + (ai & 0xFFFF);
                    const int an = (int)(ai >> 16);
                    bool found = false;
                    for (int gi = 0; gi < ng; gi++) {
                        const uint32_t bi = sofs[gdef[gi]];
                        const uint32_t *bc = so + (bi & 0xFFFF);
                        const int bn = (int)(bi >> 16);
                        bool pre = an <= bn;
                        for (int k = 0; pre && k < an - 1; k++) pre = ac[k] == bc[k];
                        if (pre && an > 0) pre = (ac[an - 1] & 0xF) == (bc[an - 1] & 0xF) && (ac[an - 1] >> 4) <= (bc[an - 1] >> 4);
                        if (pre) {
                            gsize[gi]++;
                            found = true;
                        }
                    }
                    if (!found) {
                        if (ng < 64) {
                            gdef[ng] = ord[i];
                            gsize[ng] = 1;
                            ng++;
                        } else {
                            overflow = true;
                        }
                    }
                }
                (void)overflow;
                if (ng <= 1) continue;
                int best = 0;
                for (int gi = 1; gi < ng; gi++)
                    if (gsize[gi] > gsize[best]) best = gi;
                const uint32_t bi = sofs[gdef[best]];
                const uint32_t *bc = so + (bi & 0xFFFF);
                const int bn = (int)(bi >> 16);
                for (int i = 0; i < cnt; i++) {
                    const uint32_t ai = sofs[ord[i]];
                    const uint32_t *ac = so + (ai & 0xFFFF);
                    const int an = (int)(ai >> 16);
                    bool pre = an <= bn;
                    for (int k = 0; pre && k < an - 1; k++) pre = ac[k] == bc[k];
                    if (pre && an > 0) pre = (ac[an - 1] & 0xF) == (bc[an - 1] & 0xF) && (ac[an - 1] >> 4) <= (bc[an - 1] >> 4);
                    if (!pre) M[ord[i]].set = 0xFF;
                }
            }
        }
        g.sync();
    }

    // ---- phase 6a: per-set read lists (family order) and consensus lengths ----
    __shared__ int s_cnt[kLargeThreads / kWave > kSmallWaves ? kLargeThreads / kWave : kSmallWaves][4];
    __shared__ int s_lc[kLargeThreads / kWave > kSmallWaves ? kLargeThreads / kWave : kSmallWaves][4];
    const int wslot = G == kWave ? (int)(threadIdx.x >> 6) : 0;
    if (g.t == 0) {
        int cnt[4] = {0, 0, 0, 0}, lc[4] = {0, 0, 0, 0};
        for (int r = 0; r < n; r++) {
            const int s = M[r].set;
            if (s == 0xFF) continue;
            lists[s * n + cnt[s]++] = (uint16_t)r;
            lc[s] = ::max(lc[s], M[r].srclen);
        }
        for (int s = 0; s < 4; s++) {
            s_cnt[wslot][s] = cnt[s];
            s_lc[wslot][s] = lc[s];
        }
    }
    g.sync();
    int cnt[4], lc[4];
    for (int s = 0; s < 4; s++) {
        cnt[s] = s_cnt[wslot][s];
        lc[s] = s_lc[wslot][s];
    }
    g.sync();

    // ---- phase 6b: single-strand vote, lane = (set, column) ----
    const int tot = lc[0] + lc[1] + lc[2] + lc[3];
    for (int k = g.t; k < tot; k += G) {
        int s = 0, c = k;
        while (c >= lc[s]) {
            c -= lc[s];
            s++;
        }
        long long D0 = 0, D1 = 0, D2 = 0, D3 = 0;
        const uint16_t *lst = lists + s * n;
        for (int i = 0; i < cnt[s]; i++) {
            const RecMeta &m = M[lst[i]];
            if (c >= m.srclen) continue;
            const bool neg = m.flag & 16;
            const int j = neg ? m.len - 1 - c : c;
            uint8_t b = slots[m.slot + m.start + j];
            const uint8_t q = slots[m.slot + m.cap + m.start + j];
            if (neg) b = comp_nt16(b);
            const long long v = lr[q];
            D0 += b == kA ? v : 0;
            D1 += b == kC ? v : 0;
            D2 += b == kG ? v : 0;
            D3 += b == kT ? v : 0;
        }
        int best = 0;
        long long Db = D0;
        if (D1 > Db) { best = 1; Db = D1; }
        if (D2 > Db) { best = 2; Db = D2; }
        if (D3 > Db) { best = 3; Db = D3; }
        const long long Ds[4] = {D0, D1, D2, D3};
        float S = 0.0f;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            if (b == best) continue;
            const float x = (float)((double)(Ds[b] - Db) * kLrInvScale);
            if (x < -80.0f) continue;
            S += det_expf(x);
        }
        // Q = max k with S <= thr[k] (thr non-increasing), binary search over 1..93
        int lo = 0, hi = 93;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (S <= thr[mid])
                lo = mid;
            else
                hi = mid - 1;
        }
        const int Q = lo;
        ssb[s * ssw + c] = Q < 2 ? kN : (uint8_t)(1u << best);
        ssq[s * ssw + c] = Q < 2 ? (uint8_t)2 : (uint8_t)Q;
    }
    g.sync();

    // ---- phase 7: duplex combine and output (R1 = AB-R1 + BA-R2, R2 = AB-R2 + BA-R1) ----
    const bool has[4] = {cnt[0] > 0 && lc[0] > 0, cnt[1] > 0 && lc[1] > 0, cnt[2] > 0 && lc[2] > 0, cnt[3] > 0 && lc[3] > 0};
    int olen[2];
    int sa_[2] = {0, 1}, sb_[2] = {3, 2};
    bool ok[2];
    for (int e = 0; e < 2; e++) {
        const int sa = sa_[e], sb2 = sb_[e];
        ok[e] = has[sa] || has[sb2];
        olen[e] = (has[sa] && has[sb2]) ? ::min(lc[sa], lc[sb2]) : has[sa] ? lc[sa] : has[sb2] ? lc[sb2] : 0;
    }
    const bool emit = ok[0] && ok[1];
    const int32_t stride = P.O.stride;
    if (emit) {
        for (int e = 0; e < 2; e++) {
            const int sa = sa_[e], sb2 = sb_[e];
            const int64_t slot = (2 * (int64_t)fam + e) * stride;
            const int npair = (olen[e] + 1) >> 1;
            for (int k = g.t; k < npair; k += G) {
                uint8_t ob[2] = {0, 0}, oq[2] = {0, 0};
                for (int h = 0; h < 2; h++) {
                    const int c = 2 * k + h;
                    if (c >= olen[e]) break;
                    uint8_t b, q;
                    if (has[sa] && has[sb2]) {
                        const uint8_t xb = ssb[sa * ssw + c], yb = ssb[sb2 * ssw + c];
                        const int xq = ssq[sa * ssw + c], yq = ssq[sb2 * ssw + c];
                        int rq;
                        uint8_t rb;
                        if (xb == yb) {
                            rb = xb;
                            rq = xq + yq;
                        } else if (xq > yq) {
                            rb = xb;
                            rq = xq - yq;
                        } else if (yq > xq) {
                            rb = yb;
                            rq = yq - xq;
                        } else {
                            rb = xb;
                            rq = 2;
                        }
                        if (rq > 93) rq = 93;
                        if (xb == kN || yb == kN || rq == 2) {
                            rb = kN;
                            rq = 2;
                        }
                        b = rb;
                        q = (uint8_t)rq;
                    } else {
                        const int s1 = has[sa] ? sa : sb2;
                        b = ssb[s1 * ssw + c];
                        q = ssq[s1 * ssw + c];
                    }
                    ob[h] = b;
                    oq[h] = q;
                }
                P.O.seq[slot / 2 + k] = (uint8_t)((ob[0] << 4) | ob[1]);
                P.O.qual[slot + 2 * k] = oq[0];
                if (2 * k + 1 < olen[e]) P.O.qual[slot + 2 * k + 1] = oq[1];
            }
        }
    }
    if (g.t == 0) {
        uint8_t st = emit ? 1 : 0;
        if (has[0] || has[1]) st |= 2;
        if (has[2] || has[3]) st |= 4;
        P.O.status[fam] = st;
        P.O.len[2 * fam] = (uint16_t)(emit ? olen[0] : 0);
        P.O.len[2 * fam + 1] = (uint16_t)(emit ? olen[1] : 0);
    }
}

__device__ __forceinline__ void load_tables(const Tables *tab, long long *lr, float *thr) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lr[i] = tab->lr[i];
    for (int i = threadIdx.x; i < 96; i += blockDim.x) thr[i] = tab->thr[i];
    __syncthreads();
}

// small families: one wavefront per family, arena in LDS
__global__ __launch_bounds__(kWave *kSmallWaves) void k_small(KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    long long *lr = reinterpret_cast<long long *>(smem);
    float *thr = reinterpret_cast<float *>(smem + 2048);
    load_tables(P.tab, lr, thr);
    const int w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * kSmallWaves + w;
    if (i >= P.B.n_small) return;
    uint8_t *A = smem + 2048 + 384 + (size_t)w * (size_t)P.B.small_arena;
    Grp<kWave> g{(int)(threadIdx.x & 63), nullptr};
    process_family<kWave>(P, g, A, lr, thr, P.B.small_fams[i]);
}

// large families: one workgroup per family; arena in LDS (IN_LDS) or in global scratch
template <bool IN_LDS>
__global__ __launch_bounds__(kLargeThreads) void k_large(KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int red[kLargeThreads / kWave];
    long long *lr = reinterpret_cast<long long *>(smem);
    float *thr = reinterpret_cast<float *>(smem + 2048);
    load_tables(P.tab, lr, thr);
    const int64_t i = blockIdx.x;
    if (i >= P.B.n_large) return;
    uint8_t *A = IN_LDS ? smem + 2048 + 384 : P.O.scratch + (size_t)i * (size_t)P.B.large_arena;
    Grp<kLargeThreads> g{(int)threadIdx.x, red};
    process_family<kLargeThreads>(P, g, A, lr, thr, P.B.large_fams[i]);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
struct bsdc_ctx {
    int device;
    bsdc_params params;
    Tables host_tab;
    Tables *dev_tab = nullptr;
    uint8_t *ref_seq = nullptr;
    int64_t *ref_off = nullptr;
    int64_t *ref_len = nullptr;
    int32_t n_contig = 0;
    std::string err;
};

static void make_tables(const bsdc_params &p, Tables &t) {
    // keep in step with oracle/bsdc_oracle.c orc_tables
    const double e_post = pow(10.0, -p.error_rate_post_umi / 10.0);
    const double e_pre = pow(10.0, -p.error_rate_pre_umi / 10.0);
    for (int q = 0; q < 256; q++) {
        const double e = pow(10.0, -(double)q / 10.0);
        const double a = e_post + e - (4.0 / 3.0) * e_post * e;
        const double lnc = log1p(-a);
        const double lne = log(a / 3.0);
        t.lr[q] = llround((lnc - lne) * kLrScale);
    }
    t.thr[0] = INFINITY;
    for (int k = 1; k < 94; k++) {
        const double pk = pow(10.0, -((double)k - 0.001) / 10.0);
        const double tt = (pk - e_pre) / (1.0 - (4.0 / 3.0) * e_pre);
        t.thr[k] = tt < 0.0 ? -1.0f : (float)(tt / (1.0 - tt));
    }
    t.thr[94] = t.thr[95] = -1.0f;
}

#define HIP_OK(ctx, call)                                                                     \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            if (ctx) (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);          \
            return BSDC_EDEVICE;                                                              \
        }                                                                                     \
    } while (0)

extern "C" {

int32_t bsdc_abi_version(void) { return BSDC_ABI_VERSION; }

int64_t bsdc_family_arena_bytes(int32_t n_rec, int64_t sum_len, int32_t max_len, int64_t complex_ops) {
    ArenaLayout L(n_rec, sum_len, max_len, complex_ops);
    return (int64_t)L.total;
}

int32_t bsdc_ctx_create(int32_t device, const bsdc_params *params, bsdc_ctx **out) {
    if (!out || !params) return BSDC_EINVAL;
    *out = nullptr;
    if (params->min_reads != 0 || params->min_input_base_quality < 0) return BSDC_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return BSDC_EDEVICE;
    bsdc_ctx *c = new bsdc_ctx();
    c->device = device;
    c->params = *params;
    make_tables(*params, c->host_tab);
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&c->dev_tab, sizeof(Tables)) != hipSuccess ||
        hipMemcpy(c->dev_tab, &c->host_tab, sizeof(Tables), hipMemcpyHostToDevice) != hipSuccess) {
        delete c;
        return BSDC_EDEVICE;
    }
    *out = c;
    return 0;
}

void bsdc_ctx_destroy(bsdc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipFree(c->dev_tab);
    (void)hipFree(c->ref_seq);
    (void)hipFree(c->ref_off);
    (void)hipFree(c->ref_len);
    delete c;
}

const char *bsdc_last_error(const bsdc_ctx *c) { return c ? c->err.c_str() : "null context"; }

int32_t bsdc_get_tables(const bsdc_ctx *c, int64_t *lr256, float *thr94) {
    if (!c) return BSDC_EINVAL;
    for (int i = 0; i < 256; i++) lr256[i] = c->host_tab.lr[i];
    for (int i = 0; i < 94; i++) thr94[i] = c->host_tab.thr[i];
    return 0;
}

void bsdc_model_tables(double pre, double post, int64_t *lr256, float *thr94) {
    bsdc_params p{};
    p.error_rate_pre_umi = pre;
    p.error_rate_post_umi = post;
    Tables t;
    make_tables(p, t);
    for (int i = 0; i < 256; i++) lr256[i] = t.lr[i];
    for (int i = 0; i < 94; i++) thr94[i] = t.thr[i];
}

int32_t bsdc_load_reference(bsdc_ctx *c, const uint8_t *packed, int64_t n_nib, const int64_t *coff,
                            const int64_t *clen, int32_t n_contig) {
    if (!c || n_contig < 0 || (n_nib > 0 && !packed)) return BSDC_EINVAL;
    HIP_OK(c, hipSetDevice(c->device));
    (void)hipFree(c->ref_seq);
    (void)hipFree(c->ref_off);
    (void)hipFree(c->ref_len);
    c->ref_seq = nullptr;
    c->ref_off = c->ref_len = nullptr;
    const size_t nb = (size_t)((n_nib + 1) / 2) + 16;
    HIP_OK(c, hipMalloc(&c->ref_seq, nb));
    HIP_OK(c, hipMemset(c->ref_seq, 0xFF, nb));
    if (n_nib > 0) HIP_OK(c, hipMemcpy(c->ref_seq, packed, (size_t)((n_nib + 1) / 2), hipMemcpyHostToDevice));
    const size_t nc = sizeof(int64_t) * (size_t)(n_contig > 0 ? n_contig : 1);
    HIP_OK(c, hipMalloc(&c->ref_off, nc));
    HIP_OK(c, hipMalloc(&c->ref_len, nc));
    if (n_contig > 0) {
        HIP_OK(c, hipMemcpy(c->ref_off, coff, sizeof(int64_t) * n_contig, hipMemcpyHostToDevice));
        HIP_OK(c, hipMemcpy(c->ref_len, clen, sizeof(int64_t) * n_contig, hipMemcpyHostToDevice));
    }
    c->n_contig = n_contig;
    return 0;
}

int32_t bsdc_run(bsdc_ctx *c, const bsdc_family_batch *b, bsdc_consensus *o, int32_t mode, void *stream) {
    if (!c || !b || !o) return BSDC_EINVAL;
    if (b->small_arena % 16 || b->large_arena % 16 || o->stride % 16 || o->stride < b->max_len + 2) {
        c->err = "bad arena/stride sizes";
        return BSDC_EINVAL;
    }
    if ((mode & BSDC_MODE_CONVERT) && !c->ref_seq) {
        c->err = "reference not loaded";
        return BSDC_EINVAL;
    }
    if ((mode & BSDC_MODE_DUMP) && (!o->dump_pos || !o->dump_len || !o->dump_tags || !o->dump_seq || !o->dump_qual)) {
        c->err = "dump buffers missing";
        return BSDC_EINVAL;
    }
    HIP_OK(c, hipSetDevice(c->device));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    KParams P;
    P.B = *b;
    P.O = *o;
    P.R.seq = c->ref_seq;
    P.R.off = c->ref_off;
    P.R.len = c->ref_len;
    P.R.n = c->n_contig;
    P.tab = c->dev_tab;
    P.mode = mode;
    P.overlap = c->params.consensus_call_overlapping_bases;
    const size_t tab_lds = 2048 + 384;
    if (b->n_small > 0) {
        const size_t lds = tab_lds + (size_t)kSmallWaves * (size_t)b->small_arena;
        if (lds > 160 * 1024) {
            c->err = "small arena too large";
            return BSDC_EINVAL;
        }
        const int64_t blocks = (b->n_small + kSmallWaves - 1) / kSmallWaves;
        hipLaunchKernelGGL(k_small, dim3((unsigned)blocks), dim3(kWave * kSmallWaves), lds, s, P);
        HIP_OK(c, hipGetLastError());
    }
    if (b->n_large > 0) {
        const size_t lds = tab_lds + (size_t)b->large_arena;
        if (lds <= 64 * 1024) {
            hipLaunchKernelGGL(k_large<true>, dim3((unsigned)b->n_large), dim3(kLargeThreads), lds, s, P);
        } else {
            if (!o->scratch) {
                c->err = "large families need scratch";
                return BSDC_EINVAL;
            }
            hipLaunchKernelGGL(k_large<false>, dim3((unsigned)b->n_large), dim3(kLargeThreads), tab_lds, s, P);
        }
        HIP_OK(c, hipGetLastError());
    }
    return 0;
}

int32_t bsdc_convert(bsdc_ctx *c, const bsdc_family_batch *b, bsdc_consensus *o, void *stream) {
    return bsdc_run(c, b, o, BSDC_MODE_CONVERT | BSDC_MODE_DUMP, stream);
}
int32_t bsdc_extend(bsdc_ctx *c, const bsdc_family_batch *b, bsdc_consensus *o, void *stream) {
    return bsdc_run(c, b, o, BSDC_MODE_EXTEND | BSDC_MODE_DUMP, stream);
}
int32_t bsdc_duplex_call(bsdc_ctx *c, const bsdc_family_batch *b, bsdc_consensus *o, int32_t with_tools,
                         void *stream) {
    return bsdc_run(c, b, o, BSDC_MODE_VOTE | (with_tools ? (BSDC_MODE_CONVERT | BSDC_MODE_EXTEND) : 0), stream);
}

}  // extern "C"
