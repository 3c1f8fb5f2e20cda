// bsdc_kernels.hip -- gfx950 kernels and the C-ABI (include/bsdc.h) of the step-5 duplex path.
//
// One launch does, per MI family, everything rules convert_Bstrain -> extend -> groupsort_convert
// -> callduplex do (main.snake.py:121-164) after the host has formed the families:
//   B-strand conversion        tools/1.convert_AG_to_CT.py:84-183
//   gap extension              tools/2.extend_gap.py:58-110 (4-record groups, :112-140)
//   overlapping-bases consensus    fgbio, --consensus-call-overlapping-bases=true
//   source reads                   fgbio toSourceRead (orientation, read-through, trailing N)
//   most-common-alignment filter   fgbio filterToMostCommonAlignment
//   single-strand likelihood vote  fgbio VanillaUmiConsensusCaller (pre 45 / post 30)
//   duplex combine                 fgbio DuplexConsensusCaller.duplexConsensus
// The fgbio rows are restated from its public behaviour (parity unpinned).
//
// Two kernels:
//  * k_small -- one wavefront per family (families of <= 64 records whose arena fits the
//    bucket's LDS budget).  The family's slots are ONE contiguous, 32-aligned image in HBM
//    (include/bsdc.h); every 16-byte chunk of it (quals, packed bases) and of the converted
//    records' reference windows is requested up front (<= 4 loads in flight per lane), unpacked
//    into LDS, and everything after that is LDS + registers.  Per-record metadata lives in the
//    record's lane; loops over records are wave-uniform and read it with readlane.
//  * k_large -- one 256-thread workgroup per family, generic (arena in LDS or HBM scratch).
// All integer / byte work; the vote's likelihood sums are exact fixed-point integers (2^-20 nats),
// so any summation order is bit-identical to the CPU restatement (oracle/).  The one exception is
// the rare near-tie column, which takes fgbio's own pick: its double-precision sums, added in
// fgbio's read order (fp64_pick).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/bsdc.h"
#include "../../include/bsdc_layout.h"

namespace {

constexpr int kWave = 64;
#ifndef SMALL_WAVES
#define SMALL_WAVES 7  // k_small waves per SIMD the register budget is cut for (7: <= 64 VGPRs, <= 96 SGPRs)
#endif
#ifndef SMALL_SGPRS
#define SMALL_SGPRS (SMALL_WAVES >= 8 ? 80 : 96)  // SGPR budget: <= 80 -> 8, <= 96 -> 7 waves per SIMD (MI355X_MICROARCH.md)
#endif
#ifndef SMALL_STAGE_U
#define SMALL_STAGE_U 4  // k_small staging: image chunk loads in flight per lane
#endif
constexpr int kStageU = SMALL_STAGE_U;
// Wave priority (s_setprio) while a wavefront issues its first global loads: from the kernel's table
// loads until its family's reference-window loads are out, then back to 0 (profiles/r06/README.md,
// prio/: C2 2.99 -> 2.93 ms, tag leg 3.39 -> 3.29).  The loads leave before other waves' LDS and VALU
// work, so more of the HBM latency overlaps; holding the priority through the wait for the data
// gains nothing, nor does the output pack at the raised priority.  1: from the family's metadata loads
// on (about two thirds of the gain); 0: off.
#ifndef SMALL_PRIO
#define SMALL_PRIO 2
#endif
#ifndef SMALL_PRIO_LEVEL
#define SMALL_PRIO_LEVEL 3  // the raised priority (1..3: 1 measured the same)
#endif
#ifndef SMALL_PRIO_END
#define SMALL_PRIO_END 1  // where it drops back to 0: 0 after the image loads (less gain), 1 after the window loads, 2 after staging (no gain)
#endif
#ifndef LARGE_PRIO
#define LARGE_PRIO 1  // k_large's staging loads issue at wave priority 3 (C3 -0.3%, C4 -1%; its convert's reference loads too, or from the kernel's entry, and k_join's table loads: no more); 0: off
#endif
#ifndef SMALL_QDMA
#define SMALL_QDMA 1  // k_small stages the quals with LDS-DMA (global_load_lds_dwordx4); 0: through VGPRs
#endif
#ifndef LARGE_THREADS
#define LARGE_THREADS 256  // k_large workgroup size (a multiple of 64)
#endif
constexpr int kLargeThreads = LARGE_THREADS;
#ifndef LARGE_THREADS_BIG
#define LARGE_THREADS_BIG 512  // k_large workgroup size of the LDS-heavy buckets
#endif
constexpr int kLargeThreadsBig = LARGE_THREADS_BIG;  // 512 or 768
#ifndef JOIN_THREADS
#define JOIN_THREADS 512
#endif
#ifndef JOIN_U
#define JOIN_U 4
#endif
constexpr int kJoinThreads = JOIN_THREADS;  // k_join's workgroup (k_tie's too)
constexpr int kJoinU = JOIN_U;              // parts' loads in flight per (set, column) in k_join
#ifndef LARGE_BIG_BUCKET
#define LARGE_BIG_BUCKET 2
#endif
// large buckets q >= this (3, 2, 1 workgroups per CU, scratch) use kLargeThreadsBig: 512-thread
// workgroups from the 3-per-CU class on (24 waves per CU there; profiles/r05/README.md)
constexpr int kLargeBigBucket = LARGE_BIG_BUCKET;
#ifndef LARGE_VOTE_U
#define LARGE_VOTE_U 4  // k_large vote pass A: reads in flight per lane
#endif
constexpr int kVoteU = LARGE_VOTE_U;
#ifndef LARGE_OVL_CHUNKS
#define LARGE_OVL_CHUNKS 2  // k_large overlap: SWAR dwords (4 positions each) per task
#endif
constexpr int kOvlChunks = LARGE_OVL_CHUNKS;
#ifndef LARGE_OVL_U
#define LARGE_OVL_U 2  // k_large overlap: tasks per thread whose loads are in flight together
#endif
constexpr int kOvlU = LARGE_OVL_U;
#ifndef LARGE_OVL_BSTORE
#define LARGE_OVL_BSTORE 1  // k_large overlap, mate b's unaligned whole dwords: 0 bytes, 1 one unaligned dword, 2 16-bit halves
#endif
#ifndef SMALL_OVL_BSTORE
#define SMALL_OVL_BSTORE 1  // the same for k_small's overlap (overlap_dw): 0 bytes, 1 one unaligned dword
#endif
#ifndef LARGE_CONV_H
#define LARGE_CONV_H 2  // k_large convert: SWAR dwords (4 positions each) per task, 1 or 2
#endif
constexpr int kConvH = LARGE_CONV_H;
static_assert(kConvH == 1 || kConvH == 2, "16 reference nibbles cover at most 9 positions");
#ifndef LARGE_CONV_U
#define LARGE_CONV_U 4  // k_large convert: tasks per thread per round (their reference loads in flight together)
#endif
constexpr int kLConvU = LARGE_CONV_U;
#ifndef LARGE_STAGE_U
#define LARGE_STAGE_U 8  // k_large staging: 16-B image chunks per thread in flight
#endif
constexpr int kLStageU = LARGE_STAGE_U;
constexpr int kSmallMaxWaves = 8;              // wavefronts (families) per small-kernel workgroup, at most
constexpr int kSmallMinWaves = SMALL_WAVES >= 8 ? 8 : 6;  // occupancy target the register budget is cut for
constexpr int kSmallSimdWaves = SMALL_WAVES;   // waves per SIMD its registers allow
constexpr int kLdsBytes = 160 * 1024;           // LDS per CU
constexpr double kLrScale = 1048576.0;          // 2^20
constexpr int kSqBuckets = 136;                 // phred buckets of S: 4 per octave over [2^-32, 4)
constexpr int kSqBase = (127 - 32) << 2;         // (float bits >> 21) of 2^-32
constexpr int kTabBytesL = 1024 + 1024 + 384 + 144;  // the prefix k_large uses (zero, lr, thr, sq)
constexpr int kTabBytes = kTabBytesL + 2048 + 192;  // the Tables image in LDS
constexpr int kArenaGuard = 16;  // k_small: LDS bytes before the first and after the last arena
// k_small base bytes in LDS: nt16 code | 0x10 for A, C, G, T (set at staging, see unpack32)
constexpr uint32_t kLinkRdDev = 1u << 27;       // device-internal: tool 1 trimmed a base (RD=1)

// nt16 codes
constexpr uint32_t kA = 1, kC = 2, kG = 4, kT = 8, kN = 15;

struct Tables {
    int32_t zero[256];  // row 0 of the vote's [valid][q] table: a non-ACGT base adds nothing
    int32_t lr[256];    // round((ln(1-a) - ln(a/3)) * 2^20), a = P(error) of a Q base after the post-UMI step
    float thr[96];      // Q >= k  <=>  S <= thr[k]
    uint8_t sq[144];    // Q at the top of S bucket j (S bits >> 21 = kSqBase + j; bucket 0 also below)
    uint8_t qlo[2048];  // agreement case (S = 3 e^-D): Q at D = 2^16 k
    int32_t dthr[48];   // agreement case: smallest D with Q >= q (INT32_MAX: never)
};
// The device copy: the LDS image above plus fgbio's per-read terms in double precision, read from
// HBM on the rare near-tie path only: lnc[q] = ln P(correct), lne3[q] = ln P(error) / 3 of a Q base
// after the post-UMI step, computed the way fgbio's LogProbability computes them (make_fp64).
struct DevTables {
    Tables t;
    double lnc[256];
    double lne3[256];
};

using bsdc_layout::ArenaLayout;
using bsdc_layout::ref_chunks;
using bsdc_layout::round16;
using bsdc_layout::SmallLayout;

// ------------------------------------------------------------------------------------------
// shared device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t nib(const uint8_t *p, int64_t k) {
    const uint32_t b = p[k >> 1];
    return (k & 1) ? (b & 0xF) : (b >> 4);
}
// htsjdk complement (A<->T, C<->G); other codes only need to stay non-ACGT: nt16 4-bit reversal
__device__ __forceinline__ uint32_t comp_nt16(uint32_t b) { return __builtin_bitreverse32(b) >> 28; }
__device__ __forceinline__ bool is_acgt(uint32_t b) { return b != 0 && (b & (b - 1)) == 0 && b < 16; }
__device__ __forceinline__ int acgt_idx(uint32_t b) { return __builtin_ctz(b); }

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

// S = sum over the three other bases of e^(D_b - D_best), each term skipped below e^-80
__device__ __forceinline__ float term(long long d) {
    const float x = (float)((double)d * 9.5367431640625e-07);
    return x < -80.0f ? 0.0f : det_expf(x);
}
// the same for |d| < 2^31: scaling by 2^-20 is exact, so rounding d to float first gives the
// identical float (no i64 -> f64 -> f32 conversions)
__device__ __forceinline__ float term32(int32_t d) {
    const float x = (float)d * 9.5367431640625e-07f;
    return x < -80.0f ? 0.0f : det_expf(x);
}

// Q = max k with S <= thr[k] (thr is non-increasing, S >= 0).  Tables::sq[j] is Q at the top of
// S's bucket (4 buckets per octave, so at most one threshold inside for the usual parameters), a
// lower bound on Q(S); step up while the next threshold still holds -- exact for any thr.
// `thr` points into a Tables image: sq follows it.
__device__ __forceinline__ int phred_of(float S, const float *thr) {
    const uint8_t *sq = reinterpret_cast<const uint8_t *>(thr + 96);
    const int j = ::min(::max((int)(__float_as_uint(S) >> 21) - kSqBase, 0), kSqBuckets - 1);
    int q = sq[j];
    while (q < 93 && S <= thr[q + 1]) q++;
    return q;
}

// Per-column statistics of a single-strand consensus read (BSDC_MODE_TAGS), as fgbio
// VanillaUmiConsensusCaller keeps them for the consensus tags: the call itself (N / 2 below the
// caller's --min-consensus-base-quality, KParams::qmin, or without an A/C/G/T read), depth = reads
// with an A/C/G/T at the column, errors = depth - reads showing the RAW best base (before the
// mask).  Both counts saturate at 32767 (fgbio stores Shorts).  They are fused into the vote: an
// agreeing column's depth is its read count and its errors 0; a disagreeing one's come from the
// per-base counts of the general call (k_small's queue, k_large's pass B).
template <typename T>
__device__ __forceinline__ int first_max4(T d0, T d1, T d2, T d3) {
    int best = 0;
    T m = d0;
    if (d1 > m) { best = 1; m = d1; }
    if (d2 > m) { best = 2; m = d2; }
    if (d3 > m) { best = 3; }
    return best;
}
// Near tie: each read's 2^-20 term is rounded by up to half a unit, so a
// gap between the best and the second sum of at most one unit per read of the set (nset) can hide
// fgbio's order.  Those columns take fgbio's own pick (fp64_pick).
template <typename T>
__device__ __forceinline__ bool near_tie(T d0, T d1, T d2, T d3, int best, int nset) {
    const T m = best == 0 ? d0 : best == 1 ? d1 : best == 2 ? d2 : d3;
    T sec = best == 0 ? d1 : d0;
    if (best != 1 && d1 > sec) sec = d1;
    if (best != 2 && d2 > sec) sec = d2;
    if (best != 3 && d3 > sec) sec = d3;
    return (long long)m - (long long)sec <= (long long)nset;
}
// fgbio's pick on a near tie: ConsensusBaseBuilder.add's four double-precision log-likelihood sums
// (lnc for the read's base, lne3 for each other base), accumulated read by read in fgbio's read
// order, then the first maximum by strict >.  That order is filterToMostCommonAlignment's output:
// source length descending, ties in family record order, which is ascending image address here
// (a family's slots are laid out in record order).  It reproduces fgbio's rounding too, so an exact
// tie of quality multisets resolves as fgbio's summation order resolves it.  Rare, so the order
// is found by selection: each step takes the smallest (length desc, address) key above the last.
// Desc::get(i, addr, len, rev): the set's i-th read; its column col is image byte addr + col
// (forward) or addr - col (reverse); bases at bimg, quals at qimg, same offsets.
#ifndef FP64_PICK_ATTR
#define FP64_PICK_ATTR  // (out of line, noinline: C2 k_small 3.065 -> 3.101 ms, profiles/r03/ab/README.md)
#endif
template <class Desc>
__device__ FP64_PICK_ATTR int fp64_pick(const Desc &ds, int n, int col, const uint8_t *bimg, const uint8_t *qimg, const double *lnc,
                         const double *lne3) {
    double L0 = 0.0, L1 = 0.0, L2 = 0.0, L3 = 0.0;
    uint64_t lo = 0;
    for (;;) {
        uint64_t kb = ~0ull;
        uint32_t ab = 0;
        bool rb = false;
        for (int i = 0; i < n; i++) {
            uint32_t a;
            int len;
            bool rv;
            ds.get(i, a, len, rv);
            if (len <= col) continue;
            const uint64_t key = ((uint64_t)(0x7FFFFFFFu - (uint32_t)len) << 32) | a;  // (len < 2^31)
            if (key >= lo && key < kb) {
                kb = key;
                ab = a;
                rb = rv;
            }
        }
        if (kb == ~0ull) break;
        lo = kb + 1;
        const uint32_t x = rb ? ab - (uint32_t)col : ab + (uint32_t)col;
        const uint32_t code = rb ? comp_nt16(bimg[x]) : (bimg[x] & 0x0Fu);
        if (!is_acgt(code)) continue;  // fgbio adds no N
        const int q = qimg[x];
        const double c = lnc[q], e = lne3[q];
        L0 += code == kA ? c : e;
        L1 += code == kC ? c : e;
        L2 += code == kG ? c : e;
        L3 += code == kT ? c : e;
    }
    return first_max4(L0, L1, L2, L3);
}
struct SmallDesc {  // k_small: u32 {address, length << 16 (15 bits), reverse << 31}
    const uint32_t *d;
    __device__ __forceinline__ void get(int i, uint32_t &a, int &len, bool &rv) const {
        const uint32_t x = d[i];
        a = x & 0xFFFFu;
        len = (int)((x >> 16) & 0x7FFFu);
        rv = (x >> 31) != 0;
    }
};
struct LargeDesc {  // k_large: uint2 {address, length | reverse << 31}
    const uint2 *d;
    __device__ __forceinline__ void get(int i, uint32_t &a, int &len, bool &rv) const {
        const uint2 x = d[i];
        a = x.x;
        len = (int)(x.y & 0x7FFFFFFFu);
        rv = (x.y >> 31) != 0;
    }
};
// tool 1 per-base rule (tools/1.convert_AG_to_CT.py:123-150), in its local form: the value at i
// depends on m[i], m[i+1], ref[i], ref[i+1] only (the skip at :140 writes what the A rule would)
__device__ __forceinline__ uint32_t convert_rule(uint32_t m0, uint32_t m1, bool has_next, uint32_t f0, uint32_t f1) {
    if (m0 == kA) return f0 == kG ? kG : kA;
    if (m0 == kC) {
        if (f0 == kC && f1 == kG) return (has_next && m1 == kA) ? kT : kC;
        return kT;
    }
    return m0;
}

// ---- SWAR: four nt16 codes, one per byte ----
__device__ __forceinline__ uint32_t eq4(uint32_t x, uint32_t code) {
    // 0x0F in every byte equal to `code`, 0 elsewhere (bytes hold 0..15)
    const uint32_t t = x ^ (code * 0x01010101u);
    const uint32_t z = ((t + 0x0F0F0F0Fu) & 0x10101010u) ^ 0x10101010u;
    return z - (z >> 4);
}
__device__ __forceinline__ uint32_t sel4(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

// The same rule on k_small's base bytes: m, m1 hold code | 0x10 for A/C/G/T, f0, f1 plain codes;
// nxt80 = 0x80 where position j+k has a next base.  Equality tests are zero tests of the XOR
// (bytes <= 0x1F), and the two rewrites are XORs: A (0x01) -> G (0x04) is ^ 0x05, C -> T ^ 0x0A,
// which keep the 0x10 flag.
// (FLAG = false: m, m1 hold plain codes too -- k_large)
template <bool FLAG = true>
__device__ __forceinline__ uint32_t convert4f(uint32_t m, uint32_t m1, uint32_t f0, uint32_t f1, uint32_t nxt80) {
    auto is = [](uint32_t x, uint32_t code) {  // 0x80 in the bytes of x equal to code
        return ~((x ^ code) + 0x7F7F7F7Fu) & 0x80808080u;
    };
    constexpr uint32_t kA4 = FLAG ? 0x11111111u : 0x01010101u, kC4 = FLAG ? 0x12121212u : 0x02020202u;
    const uint32_t ag = is(m, kA4) & is(f0, 0x04040404u);
    const uint32_t keepc = is(f0, 0x02020202u) & is(f1, 0x04040404u) & ~(is(m1, kA4) & nxt80);
    const uint32_t ct = is(m, kC4) & ~keepc;
    return m ^ ((ag >> 7) | (ag >> 5)) ^ ((ct >> 6) | (ct >> 4));
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

__device__ __forceinline__ CigView make_cigview(const bsdc_family_batch &B, uint32_t gidx, uint32_t link, bool conv,
                                                bool rd, bool do_extend) {
    CigView c;
    c.ops = B.cigar + B.cig_off[gidx];
    c.n = (int)(B.cig_info[gidx] & 0xFFFF);
    c.npre = (conv || (do_extend && (link & BSDC_LINK_EXT_RIGHT))) ? 1 : 0;
    c.nsuf = (do_extend && (link & BSDC_LINK_EXT_LEFT) && rd) ? 1 : 0;
    c.rdtrim = (conv && rd) ? 1 : 0;
    return c;
}

// fgbio toSourceRead's read-through trim (isFrPair + the stale mate fields), on a record of
// current position `pos`, length `len`, reference length `reflen`
__device__ int32_t readthrough_keep(const bsdc_family_batch &B, uint32_t gidx, uint32_t flag, int32_t pos,
                                    int32_t len, int32_t reflen, bool complex_, const CigView *cv) {
    const int32_t *rt = B.rt + 4 * (int64_t)gidx;
    const int32_t next_pos = rt[0], tlen = rt[1], mate_us = rt[2], mate_ue = rt[3];
    const bool neg = flag & 16, mneg = flag & 32;
    if (neg == mneg) return len;
    const int64_t posfive = neg ? (int64_t)next_pos : (int64_t)pos;
    const int64_t negfive = neg ? (int64_t)pos + reflen - 1 : (int64_t)pos + tlen;
    if (!(posfive < negfive)) return len;
    int32_t keep = len;
    if (!neg) {
        const int64_t end = (int64_t)pos + reflen - 1;
        if (end > mate_ue) {
            int32_t kk;
            if (!complex_) {
                kk = (int32_t)::min<int64_t>((int64_t)mate_ue - pos + 1, len);
                if (kk < 0) kk = 0;
            } else {
                int last = -1;
                for (int64_t p = pos; p <= mate_ue && p < (int64_t)pos + reflen; p++) {
                    const int q = read_at_ref(*cv, pos, len, p);
                    if (q >= 0) last = q;
                }
                kk = last + 1;
            }
            keep = ::min(keep, kk);
        }
    } else if ((int64_t)pos < mate_us) {
        int32_t kk;
        if (!complex_) {
            const int64_t first = (int64_t)mate_us - pos;
            kk = first >= len ? 0 : (int32_t)(len - first);
        } else {
            int first = len;
            for (int64_t p = (int64_t)pos + reflen - 1; p >= mate_us && p >= pos; p--) {
                const int q = read_at_ref(*cv, pos, len, p);
                if (q >= 0) first = q;
            }
            kk = len - first;
        }
        keep = ::min(keep, kk);
    }
    return keep;
}

// Simplified cigar of a source read (sequencing orientation, M/=/X/S -> M, merged, truncated to
// srclen query bases) into `so`; returns the op count.
__device__ int simplified_cigar(const CigView *cv, bool complex_, bool neg, int32_t srclen, uint32_t *so) {
    if (!complex_) {
        so[0] = ((uint32_t)srclen << 4) | 0u;
        return 1;
    }
    int cnt = 0;
    const int tot = cv->count();
    int32_t q = 0;
    for (int j = 0; j < tot && q < srclen; j++) {
        const int k = neg ? tot - 1 - j : j;
        int op;
        int32_t l;
        cv->at(k, op, l);
        if (l <= 0) continue;
        if (op == 7 || op == 8 || op == 4) op = 0;  // fgbio simplifyCigar: S, =, X -> M
        if (op == 5) continue;
        if (op == 0 || op == 1) {
            if (q + l > srclen) l = srclen - q;
            q += l;
        }
        if (cnt > 0 && (int)(so[cnt - 1] & 0xF) == op)
            so[cnt - 1] = (((so[cnt - 1] >> 4) + (uint32_t)l) << 4) | (uint32_t)op;
        else
            so[cnt++] = ((uint32_t)l << 4) | (uint32_t)op;
    }
    return cnt;
}

__device__ __forceinline__ bool cigar_prefix(const uint32_t *ac, int an, const uint32_t *bc, int bn) {
    bool pre = an <= bn;
    for (int k = 0; pre && k < an - 1; k++) pre = ac[k] == bc[k];
    if (pre && an > 0) pre = (ac[an - 1] & 0xF) == (bc[an - 1] & 0xF) && (ac[an - 1] >> 4) <= (bc[an - 1] >> 4);
    return pre;
}

// fgbio filterToMostCommonAlignment on one of X / Y, single thread.  `ord` (scratch, n entries)
// holds the candidate records; srclen[] / sofs[] / so[] describe them; rejected ones get set 0xFF.
// gdef / gsize: 64 u16 each of LDS scratch (arrays on the stack would give the whole kernel a
// scratch allocation for this rare path)
__device__ void filter_group(uint16_t *ord, int cnt, const uint16_t *srclen, const uint32_t *sofs, const uint32_t *so,
                             uint8_t *set, uint16_t *gdef, uint16_t *gsize) {
    if (cnt < 2) return;
    for (int i = 1; i < cnt; i++) {  // stable sort by source length, descending
        const uint16_t x = ord[i];
        int j = i - 1;
        while (j >= 0 && srclen[ord[j]] < srclen[x]) {
            ord[j + 1] = ord[j];
            j--;
        }
        ord[j + 1] = x;
    }
    int ng = 0;
    for (int i = 0; i < cnt; i++) {
        const uint32_t ai = sofs[ord[i]];
        bool found = false;
        for (int gi = 0; gi < ng; gi++) {
            const uint32_t bi = sofs[gdef[gi]];
            if (cigar_prefix(so + (ai & 0xFFFF), (int)(ai >> 16), so + (bi & 0xFFFF), (int)(bi >> 16))) {
                gsize[gi]++;
                found = true;
            }
        }
        if (!found && ng < 64) {
            gdef[ng] = ord[i];
            gsize[ng] = 1;
            ng++;
        }
    }
    if (ng <= 1) return;
    int best = 0;
    for (int gi = 1; gi < ng; gi++)
        if (gsize[gi] > gsize[best]) best = gi;
    const uint32_t bi = sofs[gdef[best]];
    for (int i = 0; i < cnt; i++) {
        const uint32_t ai = sofs[ord[i]];
        if (!cigar_prefix(so + (ai & 0xFFFF), (int)(ai >> 16), so + (bi & 0xFFFF), (int)(bi >> 16))) set[ord[i]] = 0xFF;
    }
}

struct KParams {
    bsdc_family_batch B;
    bsdc_consensus O;
    const uint8_t *ref;  // packed nt16 genome
    const DevTables *tab;
    int32_t mode;
    int32_t overlap;
    int32_t ref_chunks;       // 16-B chunks per reference window (ref_chunks(max_len))
    uint32_t ref_chunks_inv;  // ceil(2^32 / ref_chunks)
    int32_t qmin;             // bsdc_params.min_consensus_base_quality: single-strand Q below it -> (N, 2)
};

// (TAGS) a single-strand column's depth and errors: bytes (saturated) for every family, and the
// exact u16 values in the family's wide row when it has one (include/bsdc.h ss_wide)
__device__ __forceinline__ void put_ss_stats(const KParams &P, int64_t fam, int s, int64_t col, uint32_t depth,
                                             uint32_t err) {
    const int64_t at = (4 * fam + s) * P.O.stride + col;
    P.O.ss_depth[at] = (uint8_t)::min(depth, 255u);
    P.O.ss_err[at] = (uint8_t)::min(err, 255u);
    const int32_t w = P.O.ss_wide ? P.O.ss_wide[fam] : -1;
    if (w >= 0) {
        const int64_t aw = (4 * (int64_t)w + s) * P.O.stride + col;
        P.O.ss_wdepth[aw] = (uint16_t)::min(depth, 32767u);
        P.O.ss_werr[aw] = (uint16_t)::min(err, 32767u);
    }
}

// the first `bytes` of the Tables image (k_small: all of it; k_large: the kTabBytesL prefix)
template <int BYTES>
__device__ __forceinline__ void load_tables(const Tables *tab, uint8_t *dst) {
    static_assert(sizeof(Tables) == kTabBytes, "Tables image");
    static_assert(offsetof(Tables, sq) == offsetof(Tables, thr) + sizeof(float) * 96, "sq follows thr");
    static_assert(offsetof(Tables, qlo) == kTabBytesL, "k_large's prefix");
    const uint4 *src = reinterpret_cast<const uint4 *>(tab);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (int i = threadIdx.x; i < BYTES / 16; i += blockDim.x) d[i] = src[i];
    __syncthreads();
}

// duplex combine of two SS columns (fgbio DuplexConsensusCaller.duplexConsensus)
__device__ __forceinline__ void duplex_col(uint32_t xb, uint32_t xq, uint32_t yb, uint32_t yq, uint32_t &ob, uint32_t &oq) {
    uint32_t rb;
    int rq;
    if (xb == yb) {
        rb = xb;
        rq = (int)(xq + yq);
    } else if (xq > yq) {
        rb = xb;
        rq = (int)(xq - yq);
    } else if (yq > xq) {
        rb = yb;
        rq = (int)(yq - xq);
    } else {
        rb = xb;
        rq = 2;
    }
    if (rq > 93) rq = 93;
    if (xb == kN || yb == kN || rq == 2) {
        rb = kN;
        rq = 2;
    }
    ob = rb;
    oq = (uint32_t)rq;
}

// ==========================================================================================
// k_small: one wavefront per family, everything in LDS
// ==========================================================================================
struct SMeta {  // 16 B, LDS copy of a record's registers (only for the rare serial path)
    uint32_t gidx;
    int32_t pos;
    uint32_t link;
    uint16_t len;
    uint16_t flag;
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int mbcnt(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
// value of a per-lane register held by `lane` (wave-uniform lane index)
__device__ __forceinline__ int32_t rl(int32_t v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ uint32_t rlu(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }
__device__ __forceinline__ uint32_t lds32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
__device__ __forceinline__ void st32(uint8_t *p, uint32_t v) { *reinterpret_cast<uint32_t *>(p) = v; }
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
// unaligned LDS dword (gfx950 LDS runs in unaligned mode: one ds_read_b32)
__device__ __forceinline__ uint32_t ldsu32(const uint8_t *p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ void stu32(uint8_t *p, uint32_t v) { __builtin_memcpy(p, &v, 4); }
// 16 B per lane from global memory straight into LDS at lds + 16 * lane (lds wave-uniform)
__device__ __forceinline__ void glds16(const uint8_t *g, uint8_t *lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}
__device__ __forceinline__ void st16(uint8_t *p, uint16_t v) { *reinterpret_cast<uint16_t *>(p) = v; }  // 2-aligned p
// The LDS dword at any byte offset p of `base` (16-aligned) from two aligned loads and a byte
// align: gfx950 LDS stalls an unaligned dword access (SQ_LDS_UNALIGNED_STALL)
__device__ __forceinline__ uint32_t lds_any32(const uint8_t *base, int32_t p) {
    const int32_t a = p & ~3;
    const uint32_t lo = *reinterpret_cast<const uint32_t *>(base + a);
    const uint32_t hi = *reinterpret_cast<const uint32_t *>(base + a + 4);
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)p & 3u);
}
// 0x80 in every byte of x that is 0 (bytes <= 0x80)
__device__ __forceinline__ uint32_t zero80(uint32_t x) { return ~(x + 0x7F7F7F7Fu) & 0x80808080u; }
__device__ __forceinline__ uint32_t expand80(uint32_t m80);
// Overlapping-bases consensus of 4 consecutive positions of one template: mate a's bytes at ia,
// mate b's at ib, rem (>= 1) positions of the overlap left.  Same rules as the per-position path
// (agree: both quals min(qa + qb, 93); disagree: the higher quality's base on both, quals
// |qa - qb|; equal quals: N / 2; an N on either side: untouched).  Base bytes carry the 0x10
// A/C/G/T flag (N = 0x0F has none); quals must be < 128 (the caller checks).
struct Ovl4 {
    uint32_t x, y, qa, qb;  // mate a's / b's 4 bases, 4 quals
};
__device__ __forceinline__ Ovl4 ovl4_load(const uint8_t *bimg, const uint8_t *qimg, uint32_t ia, uint32_t ib) {
    return Ovl4{lds_any32(bimg, (int32_t)ia), lds_any32(bimg, (int32_t)ib), lds_any32(qimg, (int32_t)ia),
                lds_any32(qimg, (int32_t)ib)};
}
// (`in`: 0xFF in the bytes inside the overlap)
__device__ __forceinline__ Ovl4 ovl4_compute_m(const Ovl4 &in4, uint32_t in) {
    const uint32_t X = in4.x, Y = in4.y, QA = in4.qa, QB = in4.qb;
    const uint32_t act = expand80(~(zero80(X ^ 0x0F0F0F0Fu) | zero80(Y ^ 0x0F0F0F0Fu)) & 0x80808080u) & in;
    const uint32_t eq = expand80(zero80(X ^ Y));
    const uint32_t ge = expand80(((QA | 0x80808080u) - QB) & 0x80808080u);  // qa >= qb
    const uint32_t qe = expand80(zero80(QA ^ QB));
    const uint32_t sum = QA + QB;                                           // <= 254
    const uint32_t over = expand80((sum | ((sum & 0x7F7F7F7Fu) + 0x22222222u)) & 0x80808080u);  // >= 94
    const uint32_t sum93 = (sum & ~over) | (0x5D5D5D5Du & over);
    const uint32_t ad = ((((QA | 0x80808080u) - QB) & ge) | (((QB | 0x80808080u) - QA) & ~ge)) & 0x7F7F7F7Fu;
    const uint32_t nq = (sum93 & eq) | (((ad & ~qe) | (0x02020202u & qe)) & ~eq);
    const uint32_t w = (X & ge) | (Y & ~ge);              // the higher quality's base
    const uint32_t v = (w & ~qe) | (0x0F0F0F0Fu & qe);    // equal quals: N
    const uint32_t nx = (X & eq) | (v & ~eq), ny = (Y & eq) | (v & ~eq);
    const uint32_t ox = (nx & act) | (X & ~act), oy = (ny & act) | (Y & ~act);
    const uint32_t oqa = (nq & act) | (QA & ~act), oqb = (nq & act) | (QB & ~act);
    return Ovl4{ox, oy, oqa, oqb};
}
__device__ __forceinline__ Ovl4 ovl4_compute(const Ovl4 &in4, int rem) {
    return ovl4_compute_m(in4, rem >= 4 ? 0xFFFFFFFFu : (1u << (8 * rem)) - 1u);
}
// One dword of a template's overlap, aligned to mate a: dword d of a's bytes from (xa & ~3)
// holds overlap positions 4d - (xa & 3) .. + 3 (the overlap is ovl positions from xa in a and xb
// in b).  a's bases and quals are loaded as aligned dwords (and stored so when the dword lies
// inside the overlap); b's come from two aligned loads each and go back byte by byte, only inside
// the overlap (a dword store when b is aligned too and the dword is whole): gfx950 stalls unaligned LDS accesses.
__device__ __forceinline__ void overlap_dw(uint8_t *bimg, uint8_t *qimg, uint32_t xa, uint32_t xb, int ovl, int d) {
    const int p0 = 4 * d - (int)(xa & 3u);
    const uint32_t A0 = (xa & ~3u) + 4u * (uint32_t)d;
    const int32_t B0 = (int32_t)xb + p0;
    const int lo = ::max(-p0, 0), hi = ::min(ovl - p0, 4);
    if (hi <= lo) return;
    const uint32_t inm = (0xFFFFFFFFu >> (32 - 8 * (hi - lo))) << (8 * lo);
    // b's bytes from its first overlap byte B0 + lo, moved up to byte lo with zeros below: B0 itself
    // may lie before the image, and a byte from there (>= 128: not a qual) would borrow into the
    // next byte in the SWAR qual compare
    const int32_t Bl = B0 + lo;
    const uint32_t sh = 8u * (uint32_t)lo;
    const Ovl4 o = ovl4_compute_m(
        Ovl4{lds32(bimg + A0), lds_any32(bimg, Bl) << sh, lds32(qimg + A0), lds_any32(qimg, Bl) << sh}, inm);
    // a's dword goes back whole even when the overlap covers part of it: slots are 4-aligned and
    // hold one record each (bsdc.h), so its other bytes are a's own, outside the overlap, and
    // ovl4_compute_m returns them as loaded; no other lane writes them in this phase
    const bool whole = inm == 0xFFFFFFFFu;
    st32(bimg + A0, o.x);
    st32(qimg + A0, o.qa);
    if (whole && (B0 & 3) == 0) {
        st32(bimg + B0, o.y);
        st32(qimg + B0, o.qb);
#if SMALL_OVL_BSTORE == 1
    } else if (whole) {  // b's unaligned dword: one unaligned ds_write_b32 each (fewer LDS ops than 4 bytes)
        stu32(bimg + B0, o.y);
        stu32(qimg + B0, o.qb);
#endif
    } else {  // b's partial dword: bytes (b's bytes just outside the overlap may precede b's slot)
        for (int k = lo; k < hi; k++) {
            bimg[B0 + k] = (uint8_t)(o.y >> (8 * k));
            qimg[B0 + k] = (uint8_t)(o.qb >> (8 * k));
        }
    }
}
// overlap_dw in two halves, so a thread can have several dwords' loads in flight before any of
// their stores (the dwords of different tasks share no byte): ovl_dw_load reads and masks,
// ovl_dw_store computes and writes
struct OvlDw {
    Ovl4 in;
    uint32_t A0, inm;
    int32_t B0;
    int lo, hi;
};
__device__ __forceinline__ OvlDw ovl_dw_load(const uint8_t *bimg, const uint8_t *qimg, uint32_t xa, uint32_t xb, int ovl,
                                            int d) {
    OvlDw t;
    const int p0 = 4 * d - (int)(xa & 3u);
    t.A0 = (xa & ~3u) + 4u * (uint32_t)d;
    t.B0 = (int32_t)xb + p0;
    t.lo = ::max(-p0, 0);
    t.hi = ::min(ovl - p0, 4);
    t.inm = t.hi > t.lo ? (0xFFFFFFFFu >> (32 - 8 * (t.hi - t.lo))) << (8 * t.lo) : 0u;
    if (t.hi > t.lo) {
        const int32_t Bl = t.B0 + t.lo;
        const uint32_t sh = 8u * (uint32_t)t.lo;
        t.in = Ovl4{lds32(bimg + t.A0), lds_any32(bimg, Bl) << sh, lds32(qimg + t.A0), lds_any32(qimg, Bl) << sh};
    }
    return t;
}
__device__ __forceinline__ void ovl_dw_store(uint8_t *bimg, uint8_t *qimg, const OvlDw &t) {
    if (t.hi <= t.lo) return;
    const Ovl4 o = ovl4_compute_m(t.in, t.inm);
    const bool whole = t.inm == 0xFFFFFFFFu;  // (as overlap_dw: a's dword goes back whole)
    st32(bimg + t.A0, o.x);
    st32(qimg + t.A0, o.qa);
    if (whole && (t.B0 & 3) == 0) {
        st32(bimg + t.B0, o.y);
        st32(qimg + t.B0, o.qb);
#if LARGE_OVL_BSTORE == 1
    } else if (whole) {  // b's unaligned dword: one unaligned ds_write_b32 each
        stu32(bimg + t.B0, o.y);
        stu32(qimg + t.B0, o.qb);
#elif LARGE_OVL_BSTORE == 2
    } else if (whole && (t.B0 & 1) == 0) {  // b's dword on a 2-byte boundary: two ds_write_b16 each
        st16(bimg + t.B0, (uint16_t)o.y);
        st16(bimg + t.B0 + 2, (uint16_t)(o.y >> 16));
        st16(qimg + t.B0, (uint16_t)o.qb);
        st16(qimg + t.B0 + 2, (uint16_t)(o.qb >> 16));
    } else if (whole) {  // odd: byte, 16-bit, byte
        bimg[t.B0] = (uint8_t)o.y;
        st16(bimg + t.B0 + 1, (uint16_t)(o.y >> 8));
        bimg[t.B0 + 3] = (uint8_t)(o.y >> 24);
        qimg[t.B0] = (uint8_t)o.qb;
        st16(qimg + t.B0 + 1, (uint16_t)(o.qb >> 8));
        qimg[t.B0 + 3] = (uint8_t)(o.qb >> 24);
#endif
    } else {
        for (int k = t.lo; k < t.hi; k++) {
            bimg[t.B0 + k] = (uint8_t)(o.y >> (8 * k));
            qimg[t.B0 + k] = (uint8_t)(o.qb >> (8 * k));
        }
    }
}
__device__ __forceinline__ void ovl4_store(uint8_t *bimg, uint8_t *qimg, uint32_t ia, uint32_t ib, int rem, const Ovl4 &o) {
    if (rem >= 4) {
        stu32(bimg + ia, o.x);
        stu32(bimg + ib, o.y);
        stu32(qimg + ia, o.qa);
        stu32(qimg + ib, o.qb);
    } else {  // the bytes past the overlap may belong to another template's read: byte stores
        for (int k = 0; k < rem; k++) {
            bimg[ia + k] = (uint8_t)(o.x >> (8 * k));
            bimg[ib + k] = (uint8_t)(o.y >> (8 * k));
            qimg[ia + k] = (uint8_t)(o.qa >> (8 * k));
            qimg[ib + k] = (uint8_t)(o.qb >> (8 * k));
        }
    }
}
__device__ __forceinline__ void overlap4(uint8_t *bimg, uint8_t *qimg, uint32_t ia, uint32_t ib, int rem) {
    ovl4_store(bimg, qimg, ia, ib, rem, ovl4_compute(ovl4_load(bimg, qimg, ia, ib), rem));
}
// D0..D3 += lr2[v_j][q_j] for the 4 bytes of b (base bytes, kValid flag = v) and q (quals).  The
// index (v << 8 | q) * 4 is built two columns at a time: v_perm interleaves [q_j, v_j] into 16-bit
// halves (<= 511, so one 32-bit shift scales both halves).
__device__ __forceinline__ void lookup4(const int32_t *lr2, uint32_t b, uint32_t q, int32_t &D0, int32_t &D1,
                                        int32_t &D2, int32_t &D3) {
    const uint32_t v = (b >> 4) & 0x01010101u;
    const uint32_t lo = __builtin_amdgcn_perm(v, q, 0x05010400u) << 2;
    const uint32_t hi = __builtin_amdgcn_perm(v, q, 0x07030602u) << 2;
    const uint8_t *base = reinterpret_cast<const uint8_t *>(lr2);
    D0 += *reinterpret_cast<const int32_t *>(base + (lo & 0xFFFFu));
    D1 += *reinterpret_cast<const int32_t *>(base + (lo >> 16));
    D2 += *reinterpret_cast<const int32_t *>(base + (hi & 0xFFFFu));
    D3 += *reinterpret_cast<const int32_t *>(base + (hi >> 16));
}
// The same with the valid flags given as 0 / 1 per byte (v)
__device__ __forceinline__ void lookup4v(const int32_t *lr2, uint32_t v, uint32_t q, int32_t &D0, int32_t &D1,
                                         int32_t &D2, int32_t &D3) {
    const uint32_t lo = __builtin_amdgcn_perm(v, q, 0x05010400u) << 2;
    const uint32_t hi = __builtin_amdgcn_perm(v, q, 0x07030602u) << 2;
    const uint8_t *base = reinterpret_cast<const uint8_t *>(lr2);
    D0 += *reinterpret_cast<const int32_t *>(base + (lo & 0xFFFFu));
    D1 += *reinterpret_cast<const int32_t *>(base + (lo >> 16));
    D2 += *reinterpret_cast<const int32_t *>(base + (hi & 0xFFFFu));
    D3 += *reinterpret_cast<const int32_t *>(base + (hi >> 16));
}
// 0x01 in every byte of x (plain nt16 codes, <= 15) that is one-hot (A, C, G or T), 0 elsewhere
__device__ __forceinline__ uint32_t onehot01(uint32_t x) {
    // one v_perm as a 16-entry byte table: selectors 0-7 pick the table bytes {0, 0x81, 1, 0, 1, 0,
    // 0, 0}; 8 (T) sign-extends table byte 1 (0x81: 0xFF); 9-11 sign-extend bytes 3, 5, 7 (0);
    // 12 gives 0 and 13-15 give 0xFF, cleared by the x >= 13 test (x + 3 reaches bit 4)
    const uint32_t r = __builtin_amdgcn_perm(0x00000001u, 0x00018100u, x);
    return r & ~((x + 0x03030303u) >> 4) & 0x01010101u;
}
// Mask of the bytes of a lane's dword that lie at or past a read's end, given k8 = 8 x (columns
// the read still covers from this lane's first column), for a forward read (bytes ascend) or a
// reverse one (bytes descend).  64-bit shifts give the k8 = 0 and k8 >= 32 ends for free.
__device__ __forceinline__ uint32_t bytes_past(int k8, bool reverse) {
    const uint32_t s = (uint32_t)::min(::max(k8, 0), 32);
    return reverse ? (uint32_t)(0xFFFFFFFFull >> s) : (uint32_t)(~0ull << s);
}
// byte-wise helpers; every byte they see is < 128
__device__ __forceinline__ uint32_t expand80(uint32_t m80) { return m80 | (m80 - (m80 >> 7)); }  // 0x80 -> 0xFF
__device__ __forceinline__ uint32_t bytes_nonzero(uint32_t x) {  // 0xFF where the byte (< 128) is not 0
    return expand80((x + 0x7F7F7F7Fu) & 0x80808080u);
}
// Single-strand results of 4 columns -> duplex (fgbio DuplexConsensusCaller.duplexConsensus), in
// bytes.  bmX: one-hot bases seen by side X (0 = none), QX: its phred from the likelihood sum.
// Q < qmin -> (N, 2); one side absent -> the other side; both -> agree: sum, else the higher
// quality's base with the difference, equal qualities -> 2; capped at 93; N or 2 -> (N, 2).
// qadd = (128 - qmin) x 0x01010101: a byte Q (<= 93) + (128 - qmin) reaches bit 7 iff Q >= qmin.
__device__ __forceinline__ void resolve4(bool ha, bool hb, uint32_t bmA, uint32_t QA, uint32_t bmB, uint32_t QB,
                                         uint32_t qadd, uint32_t &ob, uint32_t &oq, uint32_t *ss) {
    const uint32_t okA = expand80((QA + qadd) & 0x80808080u);  // Q >= qmin
    const uint32_t okB = expand80((QB + qadd) & 0x80808080u);
    const uint32_t bA = (bmA & okA) | (0x0F0F0F0Fu & ~okA), qA = (QA & okA) | (0x02020202u & ~okA);
    const uint32_t bB = (bmB & okB) | (0x0F0F0F0Fu & ~okB), qB = (QB & okB) | (0x02020202u & ~okB);
    ss[0] = bA;  // the single-strand results: side A bases, quals, side B bases, quals
    ss[1] = qA;
    ss[2] = bB;
    ss[3] = qB;
    if (!(ha && hb)) {
        ob = ha ? bA : bB;
        oq = ha ? qA : qB;
        return;
    }
    const uint32_t same = ~bytes_nonzero(bA ^ bB);
    const uint32_t dAB = (qA | 0x80808080u) - qB;                 // 128 + qA - qB per byte
    const uint32_t geA = expand80(dAB & 0x80808080u);              // qA >= qB
    const uint32_t dBA = (qB | 0x80808080u) - qA;
    const uint32_t ad = ((dAB & geA) | (dBA & ~geA)) & 0x7F7F7F7Fu;  // |qA - qB|
    const uint32_t sum = qA + qB;
    const uint32_t over = expand80((sum + 0x22222222u) & 0x80808080u);  // sum >= 94 (sums <= 186)
    const uint32_t sum93 = (sum & ~over) | (0x5D5D5D5Du & over);
    const uint32_t ad2 = ad | (0x02020202u & ~bytes_nonzero(ad));  // equal qualities -> 2
    uint32_t rb = (bA & (same | geA)) | (bB & ~(same | geA));
    uint32_t rq = (sum93 & same) | (ad2 & ~same);
    const uint32_t isN = ((bA + 0x01010101u) | (bB + 0x01010101u)) & 0x10101010u;  // a side is N (15)
    const uint32_t is2 = ~bytes_nonzero(rq ^ 0x02020202u);
    const uint32_t nm = expand80(isN << 3) | is2;
    ob = (rb & ~nm) | (0x0F0F0F0Fu & nm);
    oq = (rq & ~nm) | (0x02020202u & nm);
}
// htsjdk complement of one-hot codes in every byte (nibble bit reversal; 0 stays 0)
__device__ __forceinline__ uint32_t comp4(uint32_t x) {
    return (__builtin_bitreverse32(__builtin_bswap32(x)) >> 4) & 0x0F0F0F0Fu;
}
// 16 packed bytes (32 nibbles, high first) -> 32 base bytes.  With FLAG, each byte also gets
// 0x10 when its base is A, C, G or T (one bit of 4 set), computed on the packed nibbles:
// bits a..d of every nibble at once, one-hot = any & !two.
template <bool FLAG>
__device__ __forceinline__ void unpack32(uint4 v, uint8_t *dst) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t lo = w[k] & 0x0F0F0F0Fu;
        uint32_t hi = (w[k] >> 4) & 0x0F0F0F0Fu;
        if (FLAG) {
            const uint32_t a = w[k], b = w[k] >> 1, c = w[k] >> 2, d = w[k] >> 3;
            const uint32_t ab = a | b, cd = c | d;
            const uint32_t two = (a & b) | (c & d) | (ab & cd);
            const uint32_t vm = (ab | cd) & ~two & 0x11111111u;  // bit 4k: nibble k is one-hot
            lo |= (vm << 4) & 0x10101010u;
            hi |= vm & 0x10101010u;
        }
        o[2 * k] = __builtin_amdgcn_perm(lo, hi, 0x05010400u);
        o[2 * k + 1] = __builtin_amdgcn_perm(lo, hi, 0x07030602u);
    }
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = make_uint4(o[0], o[1], o[2], o[3]);
    d[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// TAGS: also the single-strand reads + column statistics (BSDC_MODE_TAGS; its own instance, so the
// hot instance carries none of that code)
// one family on one wavefront (k_small's body): A = the wave's LDS arena, T = the workgroup's
// LDS copy of the tables, fi = the family's index in this size class's list
template <bool TAGS>
__device__ __forceinline__ void small_family(const KParams &P, const Tables *T, uint8_t *A, const uint32_t *fams,
                                             int64_t fi, int t) {
    const int32_t *lr2 = T->zero;  // [2][256]: row (base byte >> 4) = 1 for A/C/G/T
    const float *thr = T->thr;
    const uint8_t *qlo = T->qlo;
    const int32_t *dthr = T->dthr;
    const bsdc_family_batch &B = P.B;
    const bool do_convert = P.mode & BSDC_MODE_CONVERT;
    const bool do_extend = P.mode & BSDC_MODE_EXTEND;
    const bool do_vote = P.mode & BSDC_MODE_VOTE;
    const int max_len = B.max_len;
    const int stop = (P.mode >> BSDC_MODE_STOP_SHIFT) & 15;  // profiling ablation (0 = full kernel)

    // list entry: family id, first record, record count | image size / 32 << 8, image base (the
    // index made wave-uniform: one scalar load, s_load_dwordx4, instead of a vector load and five
    // readfirstlanes)
    const uint4 ent = reinterpret_cast<const uint4 *>(fams)[__builtin_amdgcn_readfirstlane((int)fi)];
    const uint32_t fam = __builtin_amdgcn_readfirstlane(ent.x);
    const uint32_t r0 = __builtin_amdgcn_readfirstlane(ent.y);
    const int n = (int)(__builtin_amdgcn_readfirstlane(ent.z) & 0xFF);
    const uint32_t img = (__builtin_amdgcn_readfirstlane(ent.z) >> 8) * 32u;
    const uint32_t base_g = __builtin_amdgcn_readfirstlane(ent.w);

    // ---- staging: record metadata, every 16-byte chunk of the image and the converted records'
    // reference windows.  Metadata loads go first so the window loads (whose addresses they hold)
    // are issued while the image chunks are still in flight; up to 4 chunk loads per lane per
    // round ----
    if (SMALL_PRIO == 1) __builtin_amdgcn_s_setprio(SMALL_PRIO_LEVEL);
    const bool has = t < n;
    uint4 rc = make_uint4(0, 0, 0, 0);
    uint2 win = make_uint2(0, 0);
    uint32_t cinfo = 0;
    if (has) {
        rc = reinterpret_cast<const uint4 *>(B.rec)[r0 + t];
        win = reinterpret_cast<const uint2 *>(B.rec_win)[r0 + t];
        cinfo = B.cig_info[r0 + t];
    }
    const int nqc = (int)(img >> 4), nch = nqc + (int)(img >> 5);  // qual chunks, + packed-base chunks
    uint8_t *bimg = A;          // SmallLayout: bimg = 0, qimg = img
    uint8_t *qimg = A + img;
    auto load_img = [&](int k) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < nqc)
            v = *reinterpret_cast<const uint4 *>(B.qual + base_g + 16 * (uint32_t)k);
        else if (k < nch)
            v = *reinterpret_cast<const uint4 *>(B.seq + (base_g >> 1) + 16 * (uint32_t)(k - nqc));
        return v;
    };
    uint32_t qor = 0;  // OR of every qual byte this lane stages (0x80 set: a qual >= 128)
#if SMALL_QDMA
    // quals straight into LDS: one 1 KiB wave-instruction per 64 chunks, no VGPR round trip (the
    // image is as contiguous in LDS as in HBM); the qual >= 128 test then reads them back
    for (int u = 0; u < ((nqc + 63) >> 6); u++) {
        const int k = t + 64 * u;
        if (k < nqc) glds16(B.qual + base_g + 16u * (uint32_t)k, qimg + 1024 * u);
    }
#endif
    auto store_img = [&](int k, uint4 v) {
        if (k < nqc && !SMALL_QDMA) {
            *reinterpret_cast<uint4 *>(qimg + 16 * k) = v;
            qor |= v.x | v.y | v.z | v.w;
        } else if (k >= nqc && k < nch) {
            unpack32<true>(v, bimg + 32 * (k - nqc));
        }
    };
    // lanes take qual chunks and packed-base chunks in separate rounds (the unpack runs once per
    // round of base chunks instead of in every round where some lane has one): chunk k of round u
    // is qual chunk t + 64 u for u < uq, packed-base chunk t + 64 (u - uq) after
    const int uq = SMALL_QDMA ? 0 : (nqc + 63) >> 6;
    auto kmap = [&](int u) {
        if (u < uq) return t + 64 * u < nqc ? t + 64 * u : nch;
        const int kb = t + 64 * (u - uq);
        return kb < nch - nqc ? nqc + kb : nch;
    };
    uint4 v[kStageU];
#pragma unroll
    for (int u = 0; u < kStageU; u++) v[u] = load_img(kmap(u));
    if (SMALL_PRIO && SMALL_PRIO_END == 0) __builtin_amdgcn_s_setprio(0);

    const uint32_t gslot = rc.x;
    int32_t pos = (int32_t)rc.y;
    const int32_t L = (int32_t)(rc.z & 0xFFFF);
    const uint32_t flag = rc.z >> 16;
    uint32_t link = rc.w;
    const bool conv = has && do_convert && (link & BSDC_LINK_CONVERT);
    const bool cplx = has && (link & BSDC_LINK_COMPLEX);
    if (!cplx) cinfo = 0;
    const uint64_t conv_mask = ballot(conv);
    const int nconv = __builtin_popcountll(conv_mask);
    const int ci = mbcnt(conv_mask);
    int cops = (int)(cinfo & 0xFFFF);
    if (ballot(cops != 0)) {  // (most families: no complex cigar, no six-step reduction)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) cops += __shfl_xor(cops, o, kWave);
    }
    const SmallLayout Lo(n, img, nconv, cops, max_len);
    uint8_t *refw = A + Lo.ref;
    const int ws = Lo.ws;
    uint32_t *lc = reinterpret_cast<uint32_t *>(A + Lo.misc);
    uint8_t *convlane = A + Lo.misc + 16;                              // converted record -> its lane
    uint32_t *convwin = reinterpret_cast<uint32_t *>(A + Lo.lists);  // until the descriptors exist
    const uint32_t slot = gslot - base_g;                              // record slot in the image
    if (conv) {
        convwin[ci] = win.x;
        convlane[ci] = (uint8_t)t;
    }
    if (t < 4) lc[t] = 0;
    wave_sync();
    // window chunk k -> (converted record k / rcn, part k % rcn); rcn and its 2^32 reciprocal are
    // launch constants (floor(k * rinv / 2^32) is exact for k, rcn < 2^16)
    const uint32_t rcn = (uint32_t)P.ref_chunks, rinv = P.ref_chunks_inv;
    const int wtot = nconv * (int)rcn;
    auto load_win = [&](int k) {
        uint4 x = make_uint4(0, 0, 0, 0);
        if (k < wtot) {
            const uint32_t cr = __umulhi((uint32_t)k, rinv), part = (uint32_t)k - cr * rcn;
            x = *reinterpret_cast<const uint4 *>(P.ref + ((convwin[cr] >> 1) & ~15u) + 16 * part);
        }
        return x;
    };
    auto store_win = [&](int k, uint4 x) {
        if (k < wtot) {
            const uint32_t cr = __umulhi((uint32_t)k, rinv), part = (uint32_t)k - cr * rcn;
            unpack32<false>(x, refw + cr * ws + 32 * part);
        }
    };
    uint4 wv[2];
#pragma unroll
    for (int u = 0; u < 2; u++) wv[u] = load_win(t + 64 * u);
    if (SMALL_PRIO && SMALL_PRIO_END == 1) __builtin_amdgcn_s_setprio(0);  // (every first-round load is issued)
#pragma unroll
    for (int u = 0; u < kStageU; u++) store_img(kmap(u), v[u]);
    const int ub = (nch - nqc + 63) >> 6;  // rounds of base chunks
    for (int u0 = kStageU; u0 < uq + ub; u0 += kStageU) {  // families with more image chunks
#pragma unroll
        for (int u = 0; u < kStageU; u++) v[u] = load_img(kmap(u0 + u));
#pragma unroll
        for (int u = 0; u < kStageU; u++) store_img(kmap(u0 + u), v[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; u++) store_win(t + 64 * u, wv[u]);
    for (int k0 = 128; k0 < wtot; k0 += 128) {
#pragma unroll
        for (int u = 0; u < 2; u++) wv[u] = load_win(k0 + t + 64 * u);
#pragma unroll
        for (int u = 0; u < 2; u++) store_win(k0 + t + 64 * u, wv[u]);
    }
#if SMALL_QDMA
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA'd quals have landed
    wave_sync();
    for (int k = t; k < nqc; k += 64) {
        const uint4 q = *reinterpret_cast<const uint4 *>(qimg + 16 * k);
        qor |= q.x | q.y | q.z | q.w;
    }
#endif
    wave_sync();
    if (SMALL_PRIO && SMALL_PRIO_END == 2) __builtin_amdgcn_s_setprio(0);
    if (stop == 1) return;

    // ---- tool 1: every converted record at once -- 16 lanes per record, 4 positions per lane per
    // step (tools/1.convert_AG_to_CT.py:84-183) ----
    int32_t start = 1, len = L;
    bool rd = false;
    for (int cr0 = 0; cr0 < nconv; cr0 += 4) {
        const int cr = cr0 + (t >> 4);
        const bool act = cr < nconv;
        const int src = act ? convlane[cr] : 0;
        const uint32_t s_slot = (uint32_t)__shfl((int)slot, src, kWave);
        const int32_t s_L = __shfl(L, src, kWave);
        const uint32_t s_win = (uint32_t)__shfl((int)win.x, src, kWave);
        const int32_t s_avail = __shfl((int)win.y, src, kWave);
        bool my_rd = false;
        if (act) {
            const int32_t Lm = s_L + 1;
            const uint32_t wbase = (uint32_t)(cr * ws) + (s_win & 31u);
            for (int j4 = 4 * (t & 15); j4 < Lm; j4 += 64) {
                uint32_t m = lds32(bimg + s_slot + j4);
                const uint32_t mn = lds32(bimg + s_slot + j4 + 4);
                const uint32_t a = wbase + (uint32_t)j4;
                const uint32_t d0 = lds32(refw + (a & ~3u)), d1 = lds32(refw + (a & ~3u) + 4);
                const uint32_t sh = a & 3u;
                uint32_t f0 = alignbyte(d1, d0, sh);
                uint32_t f1 = sh == 3 ? d1 : alignbyte(d1, d0, sh + 1);
                if (j4 + 5 > s_avail) {  // past the contig end / absent contig: N
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (j4 + k >= s_avail) f0 = (f0 & ~(0xFFu << (8 * k))) | (kN << (8 * k));
                        if (j4 + k + 1 >= s_avail) f1 = (f1 & ~(0xFFu << (8 * k))) | (kN << (8 * k));
                    }
                }
                if (j4 == 0) {  // :121 seed, m[0] = ref[0] (flagged when A/C/G/T)
                    const uint32_t r0b = f0 & 0xFFu;
                    m = (m & ~0xFFu) | r0b | ((r0b != 0 && (r0b & (r0b - 1)) == 0) ? 0x10u : 0u);
                }
                const uint32_t m1 = alignbyte(mn, m, 1);
                uint32_t nxt = 0x80808080u;
                const int last = Lm - 1 - j4;  // the record's last position has no next base
                if (last >= 0 && last < 4) nxt &= ~(0xFFu << (8 * last));
                const uint32_t out = convert4f(m, m1, f0, f1, nxt);
                st32(bimg + s_slot + j4, out);
                if (last >= 0 && last < 4)  // :157-170 a final C before a reference G is trimmed
                    my_rd = ((out >> (8 * last)) & 0x0F) == kC && ((f1 >> (8 * last)) & 0x0F) == kG;
            }
            if ((t & 15) == 0) qimg[s_slot] = 40;  // :174-177 'I' + quals
        }
        const uint64_t bal = ballot(my_rd);
        if (conv && (ci >> 2) == (cr0 >> 2) && ((bal >> (16 * (ci & 3))) & 0xFFFFu)) rd = true;
    }
    if (conv) {
        start = 0;
        len = L + 1 - (rd ? 1 : 0);
        pos = pos - 1 > 0 ? pos - 1 : 0;
    }
    if (!do_convert && has && (link & BSDC_LINK_RD_IN)) rd = true;
    if (rd) link |= kLinkRdDev;
    wave_sync();
    if (stop == 2) return;

    // ---- tool 2: gap extension of 4-record groups (tools/2.extend_gap.py:58-110) ----
    if (do_extend) {
        const int p = (int)((link >> BSDC_LINK_PARTNER_SHIFT) & 3u);
        const uint32_t p_slot = (uint32_t)__shfl((int)slot, p, kWave);
        const int32_t p_start = __shfl(start, p, kWave);
        const int32_t p_len = __shfl(len, p, kWave);
        const bool er = has && (link & BSDC_LINK_EXT_RIGHT);
        const bool el = has && (link & BSDC_LINK_EXT_LEFT) && rd;
        uint32_t b0 = 0, q0 = 0, bl = 0, ql = 0;
        if (er) {  // :70-80 the converted partner's first base / qual
            b0 = bimg[p_slot + p_start];
            q0 = qimg[p_slot + p_start];
        }
        if (el) {  // :92-101 the partner's last base / qual, after its own prepend
            if (p_len > 0) {
                bl = bimg[p_slot + p_start + p_len - 1];
                ql = qimg[p_slot + p_start + p_len - 1];
            } else {
                bl = bimg[slot + start];
                ql = qimg[slot + start];
            }
        }
        if (er) {
            bimg[slot + start - 1] = (uint8_t)b0;
            qimg[slot + start - 1] = (uint8_t)q0;
            start -= 1;
            len += 1;
            pos -= 1;
        }
        if (el) {
            bimg[slot + start + len] = (uint8_t)bl;
            qimg[slot + start + len] = (uint8_t)ql;
            len += 1;
        }
        wave_sync();
    }

    // current reference length
    int32_t reflen = len;
    if (cplx) {
        reflen = (int32_t)(cinfo >> 16) + (conv ? 1 : 0) - ((conv && rd) ? 1 : 0) +
                 ((do_extend && (link & BSDC_LINK_EXT_RIGHT)) ? 1 : 0) +
                 ((do_extend && (link & BSDC_LINK_EXT_LEFT) && rd) ? 1 : 0);
    }

    // ---- stage dump ----
    if (P.mode & BSDC_MODE_DUMP) {
        for (int r = 0; r < n; r++) {
            const uint32_t s_slot = rlu(slot, r), s_g = rlu(gslot, r);
            const int32_t s_start = rl(start, r), s_len = rl(len, r);
            for (int j = t; j < s_len; j += 64) {
                P.O.dump_seq[s_g + j] = bimg[s_slot + s_start + j] & 0x0F;
                P.O.dump_qual[s_g + j] = qimg[s_slot + s_start + j];
            }
        }
        if (has) {
            const uint32_t gi = r0 + t;
            P.O.dump_pos[gi] = pos;
            P.O.dump_len[gi] = (uint16_t)len;
            uint8_t tg = 0;
            if (rd) tg |= 1;
            if (conv) tg |= 2 | 4;
            if (do_extend && (link & BSDC_LINK_EXT_RIGHT)) tg |= 4;
            if (do_extend && (link & BSDC_LINK_EXT_LEFT) && rd) tg |= 8;
            P.O.dump_tags[gi] = tg;
        }
    }
    if (!do_vote || stop == 3) return;

    // ---- overlapping-bases consensus ----
    // Every R1 lane gets its mate's state by lane shuffles and computes the template's overlap.
    // Templates with simple cigars then run 4 at a time, 16 lanes each, 4 positions per lane
    // (overlap4); a complex cigar, or a family with a quality byte >= 128, takes the
    // per-position path one template at a time.
    const uint32_t mate = link & BSDC_LINK_MATE_MASK;
    const bool usable = has && (link & BSDC_LINK_USABLE);
    if (P.overlap) {
        const bool mate_ok = usable && mate != BSDC_LINK_MATE_MASK && !(flag & 4);
        const int ml = mate_ok ? (int)mate : t;
        const uint32_t b_link = (uint32_t)__shfl((int)link, ml, kWave), b_flag = (uint32_t)__shfl((int)flag, ml, kWave);
        const int32_t b_pos = __shfl(pos, ml, kWave), b_reflen = __shfl(reflen, ml, kWave);
        const uint32_t b_base = (uint32_t)__shfl((int)(slot + (uint32_t)start), ml, kWave);
        const int32_t s0 = ::max(pos, b_pos), e0 = ::min(pos + reflen - 1, b_pos + b_reflen - 1);
        const bool ok = mate_ok && (b_link & BSDC_LINK_USABLE) && !(b_flag & 4) && reflen > 0 && b_reflen > 0 &&
                        s0 <= e0;
        const bool wild = ballot((qor & 0x80808080u) != 0) != 0;
        const bool fast = ok && !((link | b_link) & BSDC_LINK_COMPLEX) && !wild;
        uint64_t tm = ballot(ok && !fast);
        while (tm) {
            const int a = __builtin_ctzll(tm);
            tm &= tm - 1;
            const int b = (int)rlu(mate, a);
            const uint32_t la_ = rlu(link, a), lb_ = rlu(link, b);
            const int32_t pa = rl(pos, a), pb = rl(pos, b), la = rl(len, a), lb = rl(len, b);
            const int32_t ps0 = rl(s0, a), pe0 = rl(e0, a);
            const uint32_t sa = rlu(slot, a) + (uint32_t)rl(start, a), sb = rlu(slot, b) + (uint32_t)rl(start, b);
            const bool ca = la_ & BSDC_LINK_COMPLEX, cb = lb_ & BSDC_LINK_COMPLEX;
            CigView va, vb;
            if (ca) va = make_cigview(B, r0 + a, la_, do_convert && (la_ & BSDC_LINK_CONVERT), (la_ & kLinkRdDev) != 0, do_extend);
            if (cb) vb = make_cigview(B, r0 + b, lb_, do_convert && (lb_ & BSDC_LINK_CONVERT), (lb_ & kLinkRdDev) != 0, do_extend);
            for (int32_t p = ps0 + t; p <= pe0; p += 64) {
                const int ia = ca ? read_at_ref(va, pa, la, p) : (p - pa < la ? p - pa : -1);
                const int ib = cb ? read_at_ref(vb, pb, lb, p) : (p - pb < lb ? p - pb : -1);
                if (ia < 0 || ib < 0) continue;
                const uint32_t x = bimg[sa + ia], y = bimg[sb + ib];
                if (x == kN || y == kN) continue;
                const int qa = qimg[sa + ia], qb = qimg[sb + ib];
                if (x == y) {
                    const uint8_t q = (uint8_t)::min(qa + qb, 93);
                    qimg[sa + ia] = q;
                    qimg[sb + ib] = q;
                } else if (qa > qb) {
                    bimg[sb + ib] = (uint8_t)x;
                    qimg[sa + ia] = qimg[sb + ib] = (uint8_t)(qa - qb);
                } else if (qb > qa) {
                    bimg[sa + ia] = (uint8_t)y;
                    qimg[sa + ia] = qimg[sb + ib] = (uint8_t)(qb - qa);
                } else {
                    bimg[sa + ia] = bimg[sb + ib] = (uint8_t)kN;
                    qimg[sa + ia] = qimg[sb + ib] = 2;
                }
            }
        }
        const uint64_t fm = ballot(fast);
        const int nt = __builtin_popcountll(fm);
        if (nt > 0) {
            uint32_t *tinfo = reinterpret_cast<uint32_t *>(A + Lo.ref);  // R: the windows are dead
            if (fast) {
                const int i = mbcnt(fm);
                tinfo[3 * i] = slot + (uint32_t)start + (uint32_t)(s0 - pos);
                tinfo[3 * i + 1] = b_base + (uint32_t)(s0 - b_pos);
                tinfo[3 * i + 2] = (uint32_t)(e0 - s0 + 1);
            }
            wave_sync();
            for (int g0 = 0; g0 < nt; g0 += 4) {
                const int g = g0 + (t >> 4);
                if (g < nt) {
                    const uint32_t xa = tinfo[3 * g], xb = tinfo[3 * g + 1];
                    const int ovl = (int)tinfo[3 * g + 2];
                    const int nd = ((int)(xa & 3u) + ovl + 3) >> 2;
                    for (int d = t & 15; d < nd; d += 16) overlap_dw(bimg, qimg, xa, xb, ovl, d);
                }
            }
        }
        wave_sync();
    }

    if (stop == 4) return;
    // ---- source reads: read-through trim, trailing-N trim, strand/end set ----
    const bool neg = flag & 16;
    int32_t srclen = 0;
    uint32_t set = 0xFF;
    if (usable) {
        int32_t keep = len;
        CigView cv;
        if (cplx) cv = make_cigview(B, r0 + t, link, conv, rd, do_extend);
        if (link & BSDC_LINK_RT) keep = readthrough_keep(B, r0 + t, flag, pos, len, reflen, cplx, &cv);
        const uint8_t *sbp = bimg + slot + start;
        while (keep > 0) {
            const uint32_t bb = neg ? sbp[len - keep] : sbp[keep - 1];
            if (bb != kN) break;
            keep--;
        }
        srclen = keep;
        if (keep > 0) {
            const bool r1 = flag & 0x40;
            set = (link & BSDC_LINK_AB) ? (r1 ? 0u : 1u) : (r1 ? 2u : 3u);
        }
    }

    // ---- most-common-alignment filter (only families with a non-M-only cigar; serial) ----
    if (ballot(cplx && set != 0xFF)) {
        SMeta *meta = reinterpret_cast<SMeta *>(A + Lo.meta);
        uint8_t *setv = A + Lo.setv;
        uint16_t *ordv = reinterpret_cast<uint16_t *>(A + Lo.ordv);
        uint16_t *srcl = reinterpret_cast<uint16_t *>(A + Lo.srcl);
        if (has) {
            meta[t].gidx = r0 + t;
            meta[t].pos = pos;
            meta[t].link = link;
            meta[t].len = (uint16_t)len;
            meta[t].flag = (uint16_t)flag;
            srcl[t] = (uint16_t)srclen;
            setv[t] = (uint8_t)set;
        }
        wave_sync();
        if (t == 0) {
            uint32_t *so = reinterpret_cast<uint32_t *>(A + Lo.simp);
            uint16_t *grp = reinterpret_cast<uint16_t *>(A + Lo.grp);
            uint32_t *sofs = so + cops + 2 * n;
            uint32_t fill = 0;
            for (int r = 0; r < n; r++) {
                sofs[r] = 0;
                if (setv[r] == 0xFF) continue;
                const SMeta m = meta[r];
                const bool mc = m.link & BSDC_LINK_COMPLEX;
                const bool mconv = do_convert && (m.link & BSDC_LINK_CONVERT);
                CigView v;
                if (mc) v = make_cigview(B, m.gidx, m.link, mconv, (m.link & kLinkRdDev) != 0, do_extend);
                const int c = simplified_cigar(&v, mc, m.flag & 16, srcl[r], so + fill);
                sofs[r] = fill | ((uint32_t)c << 16);
                fill += (uint32_t)c;
            }
            for (int xy = 0; xy < 2; xy++) {
                const int s1 = xy == 0 ? 0 : 1, s2 = xy == 0 ? 3 : 2;
                int cnt = 0;
                for (int r = 0; r < n; r++)
                    if (setv[r] == s1) ordv[cnt++] = (uint16_t)r;
                for (int r = 0; r < n; r++)
                    if (setv[r] == s2) ordv[cnt++] = (uint16_t)r;
                filter_group(ordv, cnt, srcl, sofs, so, setv, grp, grp + 64);
            }
        }
        wave_sync();
        if (has) set = setv[t];
        wave_sync();
    }

    // ---- read descriptors by set (forward reads first) and consensus lengths ----
    // R1 = AB-R1 + BA-R2, R2 = AB-R2 + BA-R1.  Descriptor of a source read: its column c is image
    // byte sbase + c (forward) or sbase - c (reverse); srclen < 2^15.
    const uint32_t sbase = slot + start + (neg ? (uint32_t)(len - 1) : 0u);
    const uint32_t desc = sbase | ((uint32_t)srclen << 16) | (neg ? 0x80000000u : 0u);
    uint32_t *dlist = reinterpret_cast<uint32_t *>(A + Lo.lists);  // <= 64 descriptors, set by set
    int cnt[4], nfw[4], off[4];
    {
        int o = 0;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint64_t mf = ballot(set == (uint32_t)s && !neg), mr = ballot(set == (uint32_t)s && neg);
            nfw[s] = __builtin_popcountll(mf);
            cnt[s] = nfw[s] + __builtin_popcountll(mr);
            off[s] = o;
            if (set == (uint32_t)s) dlist[o + (neg ? nfw[s] + mbcnt(mr) : mbcnt(mf))] = desc;
            o += cnt[s];
        }
    }
    if (set != 0xFF) atomicMax(&lc[set], (uint32_t)srclen);
    wave_sync();
    // lane j holds descriptor j: the vote reads them with v_readlane (no LDS round trip per read)
    const uint32_t dreg = t < off[3] + cnt[3] ? dlist[t] : 0u;
    int lcs[4];
#pragma unroll
    for (int s = 0; s < 4; s++) lcs[s] = (int)__builtin_amdgcn_readfirstlane(lc[s]);
    if (stop == 5) return;

    // ---- single-strand vote + duplex combine, per end ----
    // A lane owns 4 consecutive columns of one end.  Per read it loads their 4 bases and 4 quals as
    // one (unaligned) LDS dword each -- the dword ending at sbase - c for a reverse read, whose
    // bytes run backwards --, clears the bases of columns past the read's end, ORs the one-hot
    // bases, and adds Tables::lr2[base][qual] for each column: rows of non-ACGT codes (and the
    // cleared 0) are zero, so no per-base test is needed.  A column where each side's reads agree
    // (OR has <= 1 bit set) is resolved from its sum alone (Tables::qlo / dthr); the rest (any
    // disagreement, any N, a negative sum) are queued for the general four-likelihood path.
    bool hs[4];
#pragma unroll
    for (int s = 0; s < 4; s++) hs[s] = cnt[s] > 0;
    const bool emit = (hs[0] || hs[3]) && (hs[1] || hs[2]);
    const int32_t stride = P.O.stride;
    int olen[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int sa = e == 0 ? 0 : 1, sb = e == 0 ? 3 : 2;
        olen[e] = (hs[sa] && hs[sb]) ? ::min(lcs[sa], lcs[sb]) : hs[sa] ? lcs[sa] : hs[sb] ? lcs[sb] : 0;
    }
    if (emit && stop != 6) {
        const int ow = Lo.ow;
        const uint32_t qadd = (uint32_t)(128 - P.qmin) * 0x01010101u;
        uint8_t *outb = A + Lo.outb;  // [2][ow] duplex bases
        uint8_t *outq = A + Lo.outq;  // [2][ow] duplex quals
        uint16_t *sq = reinterpret_cast<uint16_t *>(A + Lo.squeue);
        int nq = 0;
        for (int e = 0; e < 2; e++) {
            const int ol = olen[e];
            const int sa = e == 0 ? 0 : 1, sb = e == 0 ? 3 : 2;
            // the two sets' figures as wave-uniform selects, not indexed by sa / sb: e is a loop
            // variable, and a dynamically indexed array goes to scratch (the TAGS instance's did)
            const int cA = e == 0 ? cnt[0] : cnt[1], cB = e == 0 ? cnt[3] : cnt[2];
            const int fA = e == 0 ? nfw[0] : nfw[1], fB = e == 0 ? nfw[3] : nfw[2];
            const int oA = e == 0 ? off[0] : off[1], oB = e == 0 ? off[3] : off[2];
            const bool hA = cA > 0, hB = cB > 0;
            // TAGS: the single-strand reads run to their own lengths, which can pass the duplex's
            // (min of the two); columns past a side's own length are not that side's
            const int la = hA ? (e == 0 ? lcs[0] : lcs[1]) : 0, lb = hB ? (e == 0 ? lcs[3] : lcs[2]) : 0;
            const int lv = TAGS ? ::max(la, lb) : ol;
            for (int c0 = 0; c0 < lv; c0 += 256) {
                const int c = c0 + 4 * t, c8 = 8 * c;
                int32_t D[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
                uint32_t mf[2] = {0, 0}, mr[2] = {0, 0};  // one-hot ORs of forward / reverse reads
                uint32_t nf[2] = {0, 0}, nr[2] = {0, 0};  // TAGS: reads with an A/C/G/T, per column byte
                if (c < lv) {
#pragma unroll
                    for (int side = 0; side < 2; side++) {
                        const int o = side == 0 ? oA : oB;
                        // one read: its 4 columns from c (descriptor d is wave-uniform; d = 0 is a
                        // read of length 0 and adds nothing, which pads the pairs below)
                        auto fwd = [&](uint32_t d) {
                            // bytes at or past the read's end: (-1 << 8 * covered) as 64 bits
                            const uint32_t x = bytes_past(8 * (int)((d >> 16) & 0x7FFF) - c8, false);
                            const int32_t a = (int32_t)(d & 0xFFFFu) + c;
                            const uint32_t b = lds_any32(bimg, a) & ~x, q = lds_any32(qimg, a);
                            mf[side] |= b;
                            const uint32_t v = (b >> 4) & 0x01010101u;
                            lookup4v(lr2, v, q, D[side][0], D[side][1], D[side][2], D[side][3]);
                            if (TAGS) nf[side] += v;
                        };
                        auto rev = [&](uint32_t d) {  // bytes run backwards: byte 3 - j is column c + j
                            const uint32_t x = bytes_past(8 * (int)((d >> 16) & 0x7FFF) - c8, true);
                            const int32_t a = (int32_t)(d & 0xFFFFu) - c - 3;
                            const uint32_t b = lds_any32(bimg, a) & ~x, q = lds_any32(qimg, a);
                            mr[side] |= b;
                            const uint32_t v = (b >> 4) & 0x01010101u;
                            lookup4v(lr2, v, q, D[side][3], D[side][2], D[side][1], D[side][0]);
                            if (TAGS) nr[side] += v;
                        };
                        // reads two at a time (both reads' loads in flight together), then an odd one
                        const int nf = side == 0 ? fA : fB, na = side == 0 ? cA : cB;
                        int i = 0;
                        for (; i + 1 < nf; i += 2) {
                            const uint32_t d0 = rlu(dreg, o + i), d1 = rlu(dreg, o + i + 1);
                            fwd(d0);
                            fwd(d1);
                        }
                        if (i < nf) fwd(rlu(dreg, o + i));
                        for (i = nf; i + 1 < na; i += 2) {
                            const uint32_t d0 = rlu(dreg, o + i), d1 = rlu(dreg, o + i + 1);
                            rev(d0);
                            rev(d1);
                        }
                        if (i < na) rev(rlu(dreg, o + i));
                    }
                }
                uint32_t bm[2], multi[2];
#pragma unroll
                for (int side = 0; side < 2; side++) {
                    bm[side] = (mf[side] & 0x0F0F0F0Fu) | comp4(__builtin_bswap32(mr[side] & 0x0F0F0F0Fu));
                    const uint32_t x = bm[side];
                    multi[side] = x & ((x | 0x10101010u) - 0x01010101u);  // per byte: more than one base seen
                }
                // per side and column: Q from the sum alone (valid when the column is not slow)
                // (a sum of at most one unit per read of the set is a potential near tie with the
                // unseen bases' 0: it takes the general path too)
                uint32_t Qp[2] = {0, 0}, negm[2] = {0, 0};
#pragma unroll
                for (int side = 0; side < 2; side++) {
                    const int32_t nset = side == 0 ? cA : cB;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int32_t dsum = D[side][j];
                        negm[side] |= dsum <= nset ? 0xFFu << (8 * j) : 0u;
                        const int32_t d = ::min(::max(dsum, 0), (int32_t)((1 << 27) - 1));
                        const uint32_t q0 = qlo[d >> 16];
                        Qp[side] |= (q0 + (d >= dthr[q0 + 1] ? 1u : 0u)) << (8 * j);
                    }
                }
                uint32_t ob4, oq4, ss[4];
                resolve4(hA, hB, bm[0], Qp[0], bm[1], Qp[1], qadd, ob4, oq4, ss);
                // (TAGS) the bytes of columns inside each side's own length; without TAGS every
                // column below ol is inside both present sides
                const uint32_t inA = TAGS ? ~bytes_past(8 * (la - c), false) : ~0u;
                const uint32_t inB = TAGS ? ~bytes_past(8 * (lb - c), false) : ~0u;
                // slow columns: a side saw more than one base, or a negative sum.  The queued
                // path recomputes only the slow side(s): the other side's single-strand result
                // rides in the column's output bytes (base | 0x10 if it is side B; qual 0 = none).
                const uint32_t slowA = hA ? (bytes_nonzero(multi[0] & 0x7F7F7F7Fu) | negm[0]) & inA : 0u;
                const uint32_t slowB = hB ? (bytes_nonzero(multi[1] & 0x7F7F7F7Fu) | negm[1]) & inB : 0u;
                const uint32_t slow4 = slowA | slowB;
                if (slow4) {
                    const uint32_t useA = hA ? ~slowA : 0u, useB = (hB ? ~slowB : 0u) & ~useA;
                    const uint32_t fb = (ss[0] & useA) | ((ss[2] | 0x10101010u) & useB);
                    const uint32_t fq = (ss[1] & useA) | (ss[3] & useB);
                    ob4 = (ob4 & ~slow4) | (fb & slow4);
                    oq4 = (oq4 & ~slow4) | (fq & slow4);
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const bool qd = ((slow4 >> (8 * j)) & 0xFFu) != 0 && c + j < lv;
                    const uint64_t ms = ballot(qd);
                    if (qd) sq[nq + mbcnt(ms)] = (uint16_t)((e << 15) | (c + j));
                    nq += __builtin_popcountll(ms);
                }
                if (c < lv) {
                    st32(outb + e * ow + c, ob4);
                    st32(outq + e * ow + c, oq4);
                }
                // TAGS: the single-strand reads and their column statistics, fused into the vote
                // (fgbio's per-read / per-base consensus tags).  A column whose side agrees (not
                // slow) is that side's one base at its Q (or N / 2 below the mask), depth = its
                // A/C/G/T reads, errors 0.  Whole dwords: a slow column's bytes are rewritten by
                // the queue below (the same wavefront's later store to the same address: no
                // ordering is needed between the lanes of one wavefront), and the bytes past the
                // set's own length (c + 3 < stride) are never read (ss_len).  Writing only the
                // agreeing columns' bytes cost the tag leg 0.4 ms on C2 (profiles/r06/README.md).
                if (TAGS && c < lv) {
#pragma unroll
                    for (int side = 0; side < 2; side++) {
                        const int s = side == 0 ? sa : sb;
                        if (!(side == 0 ? hA : hB)) continue;
                        const uint32_t n4 = nf[side] + __builtin_bswap32(nr[side]);  // (<= 64 reads: bytes)
                        const int64_t at = (4 * (int64_t)fam + s) * stride + c;
                        *reinterpret_cast<uint32_t *>(P.O.ss_base + at) = ss[2 * side];
                        *reinterpret_cast<uint32_t *>(P.O.ss_qual + at) = ss[2 * side + 1];
                        *reinterpret_cast<uint32_t *>(P.O.ss_depth + at) = n4;
                        *reinterpret_cast<uint32_t *>(P.O.ss_err + at) = 0u;
                    }
                }
            }
        }
        // queued columns: the general path (all four likelihoods, up to three exp terms).  Two lanes
        // per queued (end, column): lane 2k the end's side A, lane 2k+1 its side B, each walking its
        // own side's reads; the side-A lane then combines the pair (partner value by lane shuffle).
        wave_sync();
        if (stop == 7) nq = 0;
        const uint32_t hsm = (hs[0] ? 1u : 0u) | (hs[1] ? 2u : 0u) | (hs[2] ? 4u : 0u) | (hs[3] ? 8u : 0u);
        const int side = t & 1;
        for (int k0 = 0; k0 < 2 * nq && stop != 9; k0 += 64) {
            const int k = (k0 + t) >> 1;
            const bool act = k < nq;
            const uint32_t ent = act ? sq[k] : 0u;
            const int e = (int)(ent >> 15), c = (int)(ent & 0x7FFF);
            // this lane's set: side A of end 0 / 1 is set 0 / 1, side B is set 3 / 2
            const int s = side == 0 ? e : 3 - e;
            const int ns = s == 0 ? cnt[0] : s == 1 ? cnt[1] : s == 2 ? cnt[2] : cnt[3];
            const int os = s == 0 ? off[0] : s == 1 ? off[1] : s == 2 ? off[2] : off[3];
            const bool have = act && ((hsm >> s) & 1u);
            const uint32_t kb = act ? outb[e * ow + c] : 0u, kq = act ? outq[e * ow + c] : 0u;  // kept side
            uint32_t vb = 0, vq = 0;
            if (have && kq != 0 && (int)((kb >> 4) & 1) == side) {
                vb = kb & 0x0F;
                vq = kq;
            } else if (have) {
                int32_t D0 = 0, D1 = 0, D2 = 0, D3 = 0;
                uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;  // TAGS: reads per base
                uint32_t seen = 0;  // bit 4 of a base byte: A/C/G/T
                for (int i = 0; i < ns; i++) {
                    const uint32_t d = dlist[os + i];
                    if (c >= (int)((d >> 16) & 0x7FFF)) continue;
                    const uint32_t idx = (d & 0x80000000u) ? (d & 0xFFFF) - c : (d & 0xFFFF) + c;
                    const uint32_t braw = bimg[idx];
                    seen |= braw;
                    const int32_t v = lr2[(braw >> 4) * 256u + qimg[idx]];
                    const uint32_t bb = (d & 0x80000000u) ? comp_nt16(braw) : (braw & 0x0F);
                    D0 += bb == kA ? v : 0;
                    D1 += bb == kC ? v : 0;
                    D2 += bb == kG ? v : 0;
                    D3 += bb == kT ? v : 0;
                    if (TAGS) {
                        n0 += bb == kA ? 1u : 0u;
                        n1 += bb == kC ? 1u : 0u;
                        n2 += bb == kG ? 1u : 0u;
                        n3 += bb == kT ? 1u : 0u;
                    }
                }
                int best = first_max4(D0, D1, D2, D3);
                if (near_tie(D0, D1, D2, D3, best, ns))  // rare: fgbio's fp64 read-order pick
                    best = fp64_pick(SmallDesc{dlist + os}, ns, c, bimg, qimg, P.tab->lnc, P.tab->lne3);
                const int32_t Db = best == 0 ? D0 : best == 1 ? D1 : best == 2 ? D2 : D3;
                float S = 0.0f;  // |D| < 2^30 here (<= 64 reads)
                if (best != 0) S += term32(D0 - Db);
                if (best != 1) S += term32(D1 - Db);
                if (best != 2) S += term32(D2 - Db);
                if (best != 3) S += term32(D3 - Db);
                const int Q = phred_of(S, thr);
                const bool nocall = !(seen & 0x10u) || Q < P.qmin;  // no A/C/G/T read, or below the mask
                vb = nocall ? kN : (1u << best);
                vq = nocall ? 2u : (uint32_t)Q;
                if (TAGS) {  // this side's single-strand column (the fused tag statistics)
                    const uint32_t depth = n0 + n1 + n2 + n3;
                    const uint32_t nb = best == 0 ? n0 : best == 1 ? n1 : best == 2 ? n2 : n3;
                    const int64_t at = (4 * (int64_t)fam + s) * stride + c;
                    P.O.ss_base[at] = (uint8_t)vb;
                    P.O.ss_qual[at] = (uint8_t)vq;
                    P.O.ss_depth[at] = (uint8_t)depth;  // (<= 64 reads)
                    P.O.ss_err[at] = (uint8_t)(depth - nb);
                }
            }
            const uint32_t pb = (uint32_t)__shfl_xor((int)vb, 1, kWave), pq = (uint32_t)__shfl_xor((int)vq, 1, kWave);
            if (act && side == 0) {
                const bool ha = (hsm >> e) & 1u, hb = (hsm >> (3 - e)) & 1u;
                uint32_t ob, oq;
                if (ha && hb) {
                    duplex_col(vb, vq, pb, pq, ob, oq);
                } else {
                    ob = ha ? vb : pb;
                    oq = ha ? vq : pq;
                }
                outb[e * ow + c] = (uint8_t)ob;
                outq[e * ow + c] = (uint8_t)oq;
            }
        }
        wave_sync();
        // pack and store: lanes 0-31 end 0, lanes 32-63 end 1, 8 columns per lane
        if (stop != 7 && stop != 8) {
            const int e = t >> 5;
            const int ol = e ? olen[1] : olen[0];
            for (int c0 = 8 * (t & 31); c0 < ol; c0 += 256) {
                uint2 bv = *reinterpret_cast<const uint2 *>(outb + e * ow + c0);
                uint2 qv = *reinterpret_cast<const uint2 *>(outq + e * ow + c0);
                const int k8 = 8 * (ol - c0);  // columns of the 8 inside the consensus, x 8
                const uint32_t keep0 = ~bytes_past(k8, false), keep1 = ~bytes_past(k8 - 32, false);
                bv.x &= keep0;
                bv.y &= keep1;
                const uint32_t qlo2 = qv.x & keep0, qhi2 = qv.y & keep1;
                // bytes b0..b7 -> nibbles b0 b1 | b2 b3 | ... (BAM order, high nibble first)
                const uint32_t t0 = (bv.x << 4) | (bv.x >> 8), t1 = (bv.y << 4) | (bv.y >> 8);
                const uint32_t pk = __builtin_amdgcn_perm(t1, t0, 0x06040200u);
                const int64_t so = (2 * (int64_t)fam + e) * stride;
                *reinterpret_cast<uint32_t *>(P.O.seq + so / 2 + c0 / 2) = pk;
                *reinterpret_cast<uint2 *>(P.O.qual + so + c0) = make_uint2(qlo2, qhi2);
            }
        }
    }
    // single-strand lengths of the consensus tags (their columns: the vote above, emitted families)
    if (TAGS && t < 4) P.O.ss_len[4 * fam + t] = (uint16_t)(t == 0 ? (hs[0] ? lcs[0] : 0) : t == 1 ? (hs[1] ? lcs[1] : 0)
                                                             : t == 2 ? (hs[2] ? lcs[2] : 0) : (hs[3] ? lcs[3] : 0));
    if (t == 0) {
        uint8_t st = emit ? 1 : 0;
        if (hs[0] || hs[1]) st |= 2;
        if (hs[2] || hs[3]) st |= 4;
        P.O.status[fam] = st;
        P.O.len[2 * fam] = (uint16_t)(emit ? olen[0] : 0);
        P.O.len[2 * fam + 1] = (uint16_t)(emit ? olen[1] : 0);
    }
}

// One wavefront per family, the grid covering the size class's list (persistent waves taking
// families from a counter measured 4.4x slower: the loop costs registers).
template <bool TAGS>
__global__ __launch_bounds__(kWave *kSmallMaxWaves, kSmallMinWaves) __attribute__((amdgpu_num_sgpr(SMALL_SGPRS))) void k_small(
    KParams P, const uint32_t *fams, int64_t nfams, int32_t arena) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];  // the wavefronts' arenas
    __shared__ __attribute__((aligned(16))) Tables s_tab;           // static: its address folds into offsets
    if (((P.mode >> BSDC_MODE_STOP_SHIFT) & 15) == 15) return;  // profiling: launch cost alone
    if (SMALL_PRIO == 2) __builtin_amdgcn_s_setprio(SMALL_PRIO_LEVEL);  // (from the table loads on)
    // (the tables by LDS-DMA with the barrier at the end of staging measured the same, 2.937 against
    // 2.940 ms: profiles/r06/prio/)
    load_tables<kTabBytes>(&P.tab->t, reinterpret_cast<uint8_t *>(&s_tab));
    if (((P.mode >> BSDC_MODE_STOP_SHIFT) & 15) == 14) return;  // profiling: + the table copy
    const int w = threadIdx.x >> 6;
    const int t = threadIdx.x & 63;
    const int64_t fi = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
    // (the arenas start kArenaGuard bytes into smem: a dword load that straddles the start of a
    // family image -- its bytes before the image masked -- stays inside the allocation)
    uint8_t *A = smem + kArenaGuard + (size_t)w * (size_t)arena;
    if (fi < nfams) small_family<TAGS>(P, &s_tab, A, fams, fi, t);
}

// ==========================================================================================
// k_large: one 256-thread workgroup per family (arena in LDS or in HBM scratch)
// ==========================================================================================
struct RecMeta {  // 48 B, one per record of the family, in the arena
    int32_t pos;     // current leftmost position
    int32_t len;     // current length
    uint32_t slot;   // arena offset of the base slot (quals at slot + cap)
    int32_t avail;   // converted: valid reference nibbles of its window (rec_win[1])
    int32_t start;   // index of the first base inside the slot
    uint32_t link;
    uint32_t gidx;   // global record index
    uint32_t win;    // converted: reference window start nibble
    int32_t srclen;  // source-read length
    int32_t reflen;  // current reference length
    uint16_t flag;
    uint8_t rd;
    uint8_t set;     // 0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2, 0xFF none
    int32_t in_len;
};
static_assert(sizeof(RecMeta) == bsdc_layout::kRecMetaBytes, "RecMeta layout");


template <int G>
__device__ __forceinline__ int block_sum(int v, int *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    int s = 0;
    for (int w = 0; w < G / kWave; w++) s += red[w];
    __syncthreads();
    return s;
}
template <int G>
__device__ __forceinline__ int block_max(int v, int *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = ::max(v, __shfl_xor(v, o, kWave));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    int s = red[0];
    for (int w = 1; w < G / kWave; w++) s = ::max(s, red[w]);
    __syncthreads();
    return s;
}

// the sum of a and the max of b over the workgroup, one barrier (red: 2 G / 64 ints)
template <int G>
__device__ __forceinline__ void block_sum_max(int a, int b, int *red, int &sum, int &mx) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o, kWave);
        b = ::max(b, __shfl_xor(b, o, kWave));
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = a;
        red[G / kWave + (threadIdx.x >> 6)] = b;
    }
    __syncthreads();
    sum = 0;
    mx = red[G / kWave];
    for (int w = 0; w < G / kWave; w++) {
        sum += red[w];
        mx = ::max(mx, red[G / kWave + w]);
    }
}

// Duplex combine and output of one family from its single-strand rows (LDS, [4][ssw] bases
// ssb / quals ssq, lengths lcv, reads cnt): R1 = AB-R1 (+) BA-R2, R2 = AB-R2 (+) BA-R1, a strand
// present on one side passing through; with TAGS the single-strand rows and lengths of the
// consensus tags (their depth / errors went out with the calls); status and lengths.
template <int G, bool TAGS>
__device__ void large_emit(const KParams &P, uint32_t fam, const int *cnt, const int *lcv, const uint8_t *ssb,
                           const uint8_t *ssq, int ssw, bool tag_rows) {
    const int tt = threadIdx.x;
    bool hs[4];
    for (int s = 0; s < 4; s++) hs[s] = cnt[s] > 0 && lcv[s] > 0;
    const bool emit = (hs[0] || hs[3]) && (hs[1] || hs[2]);
    const int32_t stride = P.O.stride;
    int olen[2];
    for (int e = 0; e < 2; e++) {
        const int sa = e == 0 ? 0 : 1, sb2 = e == 0 ? 3 : 2;
        olen[e] = (hs[sa] && hs[sb2]) ? ::min(lcv[sa], lcv[sb2]) : hs[sa] ? lcv[sa] : hs[sb2] ? lcv[sb2] : 0;
    }
    if (emit) {
        for (int e = 0; e < 2; e++) {
            const int sa = e == 0 ? 0 : 1, sb2 = e == 0 ? 3 : 2;
            const int64_t so = (2 * (int64_t)fam + e) * stride;
            const int npair = (olen[e] + 1) >> 1;
            for (int k = tt; k < npair; k += G) {
                uint32_t ob[2] = {0, 0}, oq[2] = {0, 0};
                for (int h = 0; h < 2; h++) {
                    const int col = 2 * k + h;
                    if (col >= olen[e]) break;
                    if (hs[sa] && hs[sb2]) {
                        duplex_col(ssb[sa * ssw + col], ssq[sa * ssw + col], ssb[sb2 * ssw + col], ssq[sb2 * ssw + col],
                                   ob[h], oq[h]);
                    } else {
                        const int s1 = hs[sa] ? sa : sb2;
                        ob[h] = ssb[s1 * ssw + col];
                        oq[h] = ssq[s1 * ssw + col];
                    }
                }
                P.O.seq[so / 2 + k] = (uint8_t)((ob[0] << 4) | ob[1]);
                P.O.qual[so + 2 * k] = (uint8_t)oq[0];
                if (2 * k + 1 < olen[e]) P.O.qual[so + 2 * k + 1] = (uint8_t)oq[1];
            }
        }
    }
    if (TAGS && tag_rows) {
        for (int s = 0; s < 4; s++) {
            const int ls = hs[s] ? lcv[s] : 0;
            const int64_t row = (4 * (int64_t)fam + s) * stride;
            for (int c = tt; c < ls; c += G) {
                P.O.ss_base[row + c] = ssb[s * ssw + c];
                P.O.ss_qual[row + c] = ssq[s * ssw + c];
            }
        }
        if (tt < 4) P.O.ss_len[4 * fam + tt] = (uint16_t)(hs[tt] ? lcv[tt] : 0);
    }
    if (tt == 0) {
        uint8_t st = emit ? 1 : 0;
        if (hs[0] || hs[1]) st |= 2;
        if (hs[2] || hs[3]) st |= 4;
        P.O.status[fam] = st;
        P.O.len[2 * fam] = (uint16_t)(emit ? olen[0] : 0);
        P.O.len[2 * fam + 1] = (uint16_t)(emit ? olen[1] : 0);
    }
}

// The parts' sums in scratch (include/bsdc.h split_partial_off): header [part][8] int32 (set
// reads, set lengths), then per (part, set) rows of the output stride's pitch: int32x4 likelihood
// sums (slot k: the set's k-th multi-base column), u8x4 A/C/G/T read counts and int32 one-base sums
// (or slot numbers) by column.

// a[s] for a lane-varying or loop-variable s, as selects: a dynamically indexed local array goes to
// scratch (k_large's PART instances had 32-48 B of it)
// Only the PART instances take the selects: in the whole-family instances the arrays stay in
// registers anyway, and the selects cost C3's large set 1.4% (profiles/r05/README.md)
template <bool SEL>
__device__ __forceinline__ int pick4(const int (&a)[4], int s) {
    if constexpr (SEL)
        return s == 0 ? a[0] : s == 1 ? a[1] : s == 2 ? a[2] : a[3];
    else
        return a[s];
}
// more than one of the four per-base read counts (u8 each) is nonzero
__device__ __forceinline__ bool multi_base(uint32_t m) {
    return ((m & 0xFFu) != 0) + ((m & 0xFF00u) != 0) + ((m & 0xFF0000u) != 0) + ((m & 0xFF000000u) != 0) > 1;
}
// A part's column: its read counts per base (u8 x4; without TAGS only the OR of its A/C/G/T codes,
// u8), and the likelihood sum of its one base when only one has reads (`one`, 4 B: most columns),
// else the slot of its four sums (`one` = k, `sum` row slot k, 16 B; k_join reads them only then).
struct PartSums {
    int32_t *head;
    uint4 *sum;
    uint32_t *cnt;
    int32_t pitch;
    __device__ __forceinline__ PartSums(const KParams &P) {
        uint8_t *b = P.O.scratch + P.B.split_partial_off;
        const int64_t np = P.B.n_split_parts;
        pitch = P.O.stride;
        head = reinterpret_cast<int32_t *>(b);
        sum = reinterpret_cast<uint4 *>(b + round16(32 * np));
        cnt = reinterpret_cast<uint32_t *>(b + round16(32 * np) + 16 * 4 * np * (int64_t)pitch);
        one = reinterpret_cast<int32_t *>(b + round16(32 * np) + 20 * 4 * np * (int64_t)pitch);
    }
    int32_t *one;   // the sum of a column whose reads show one base (its count byte the only one set)
    // Without TAGS the parts keep no read counts: a column's OR of the A/C/G/T codes its reads show
    // (u8, one-hot bits) is all the join needs.  The OR rows lie back to back at the count region's
    // start (a part's four 150-B rows in five lines: spaced like the counts, each row took two)
    __device__ __forceinline__ uint8_t *orb(int64_t at) const { return reinterpret_cast<uint8_t *>(cnt) + at; }
    __device__ __forceinline__ int64_t at(int64_t part, int s, int col) const { return (4 * part + s) * (int64_t)pitch + col; }
};

// PART: the entry is one part of a split family (include/bsdc.h split_parts): everything up to
// the vote as for a family, then the part's per-column sums and counts go to scratch (PartSums)
// instead of the calls; k_join adds the parts up.
template <int G, bool TAGS, bool PART = false>
__device__ void process_large(const KParams &P, uint8_t *A, uint8_t *s_tab, const int32_t *lr, const float *thr, uint4 ent,
                              int *red, int *s_cnt, int *s_lc, int *s_cur) {
    const int tt = threadIdx.x;
    const bsdc_family_batch &B = P.B;
    // list entry: family, first record (a part: its first part record), n, image bytes
    const uint32_t fam = ent.x, r0 = ent.y, img = ent.w;
    const int n = PART ? (int)(ent.z & 0xFFu) : (int)ent.z;  // (a part: | its split family << 8)
    const bool do_convert = P.mode & BSDC_MODE_CONVERT;
    const bool do_extend = P.mode & BSDC_MODE_EXTEND;
    const bool do_vote = P.mode & BSDC_MODE_VOTE;
    const uint4 *REC = reinterpret_cast<const uint4 *>(B.rec);
    const uint4 *PR = reinterpret_cast<const uint4 *>(B.split_part_recs);  // (PART) batch record, slot, mate, batch slot
    // the image's first entry in the batch: the family's first slot, or a part's staged chunks'
    // first entry (its first record's batch slot less its slot in the staged image)
    const uint32_t off0 = n > 0 ? (PART ? PR[r0].w - PR[r0].y : REC[r0].x) : 0u;
    const int stop = (P.mode >> BSDC_MODE_STOP_SHIFT) & 15;  // profiling ablation (0 = full kernel)

    // ---- one round of global loads for everything the family needs first: the tables (s_cnt[0]
    // cleared by the caller), up to kLStageU 16-byte image chunks per thread (quals, packed bases)
    // and the record metadata.  The image and the metadata sit at offsets the list entry alone
    // gives (ArenaLayout), so nothing waits for the family's max length / cigar size ----
    // the family image as in HBM: bases (one byte each) at slots + slot, quals at slots + img + slot
    // (a base at slots + x has its qual at slots + img + x)
    const ArenaLayout L0(n, 2 * (int64_t)img, 0, 0);  // meta / clist / slots only
    uint8_t *slots = A + L0.slots;
    uint8_t *qimg = slots + img;
    RecMeta *M = reinterpret_cast<RecMeta *>(A + L0.meta);
    uint16_t *clist = reinterpret_cast<uint16_t *>(A + L0.clist);  // the converted records
    uint32_t qor = 0;  // OR of the family's quals: a byte >= 128 keeps the overlap off the SWAR path
    // 16-B chunks: quals, then packed bases (a part's records lie back to back: its chunks too)
    const int nqc = (int)(img >> 4), nch = nqc + (int)(img >> 5);
    auto load_chunk = [&](int k) {
        const uint8_t *src = k < nqc ? B.qual + off0 + 16 * (uint32_t)k : B.seq + (off0 >> 1) + 16 * (uint32_t)(k - nqc);
        return *reinterpret_cast<const uint4 *>(src);
    };
    auto store_chunk = [&](int k, uint4 v) {
        if (k < nqc) {
            *reinterpret_cast<uint4 *>(qimg + 16 * k) = v;
            qor |= v.x | v.y | v.z | v.w;
        } else {
            unpack32<false>(v, slots + 32 * (k - nqc));
        }
    };
    // (quals by LDS-DMA here measured slower: profiles/r05/README.md)
    auto chunk_of = [&](int i) { return i; };
    const int nreg = nch;
    uint4 v[kLStageU];
    if (LARGE_PRIO) __builtin_amdgcn_s_setprio(3);
#pragma unroll
    for (int u = 0; u < kLStageU; u++)
        if (tt + u * G < nreg) v[u] = load_chunk(chunk_of(tt + u * G));
    uint4 tv = make_uint4(0, 0, 0, 0);
    if (tt < kTabBytesL / 16) tv = reinterpret_cast<const uint4 *>(&P.tab->t)[tt];
    int c = 0, ml = 0;
    for (int r = tt; r < n; r += G) {
        const uint4 pr = PART ? PR[r0 + r] : make_uint4(0, 0, 0, 0);
        const uint32_t gi = PART ? pr.x : r0 + r;
        const uint4 rc = REC[gi];
        const uint32_t ci = B.cig_info[gi];
        const uint2 wn = reinterpret_cast<const uint2 *>(B.rec_win)[gi];
        RecMeta m;
        m.in_len = (int32_t)(rc.z & 0xFFFF);
        m.flag = (uint16_t)(rc.z >> 16);
        m.pos = (int32_t)rc.y;
        m.len = m.in_len;

        m.slot = PART ? pr.y : rc.x - off0;
        m.start = 1;
        m.link = PART ? (rc.w & ~(uint32_t)BSDC_LINK_MATE_MASK) | (pr.z & 0xFFFFu) : rc.w;  // (a part: its local mate)
        m.gidx = gi;
        const bool conv = do_convert && (m.link & BSDC_LINK_CONVERT);
        m.win = conv ? wn.x : 0u;
        m.avail = conv ? (int32_t)wn.y : 0;
        m.srclen = 0;
        const bool cx = m.link & BSDC_LINK_COMPLEX;
        m.reflen = cx ? (int32_t)(ci >> 16) : m.in_len;
        m.rd = 0;
        m.set = 0xFF;
        M[r] = m;
        if (cx) c += (int)(ci & 0xFFFF);
        ml = ::max(ml, m.in_len);
        if (conv) clist[atomicAdd(&s_cnt[0], 1)] = (uint16_t)r;
    }
#pragma unroll
    for (int u = 0; u < kLStageU; u++)
        if (tt + u * G < nreg) store_chunk(chunk_of(tt + u * G), v[u]);
    if (tt < kTabBytesL / 16) reinterpret_cast<uint4 *>(s_tab)[tt] = tv;
    for (int k0 = tt + kLStageU * G; k0 < nreg; k0 += kLStageU * G) {  // families of more chunks
#pragma unroll
        for (int u = 0; u < kLStageU; u++)
            if (k0 + u * G < nreg) v[u] = load_chunk(chunk_of(k0 + u * G));
#pragma unroll
        for (int u = 0; u < kLStageU; u++)
            if (k0 + u * G < nreg) store_chunk(chunk_of(k0 + u * G), v[u]);
    }
    int cops, maxlen_f;
    block_sum_max<G>(c, ml, red, cops, maxlen_f);  // (its barrier publishes the arena and the tables)
    if (LARGE_PRIO) __builtin_amdgcn_s_setprio(0);  // (dropping it before the record metadata loop: C3 8.59 against 8.54 ms)
    const ArenaLayout Lo(n, 2 * (int64_t)img, maxlen_f, cops);
    uint16_t *lists = reinterpret_cast<uint16_t *>(A + Lo.lists);
    uint8_t *ssb = A + Lo.ssb;
    uint8_t *ssq = A + Lo.ssq;
    uint32_t *simp = reinterpret_cast<uint32_t *>(A + Lo.simp);
    uint16_t *grp = reinterpret_cast<uint16_t *>(A + Lo.grp);  // filter_group scratch, X then Y (complex families)
    const int ssw = Lo.ssw;
    if (stop == 1) return;

    // ---- tool 1 (tools/1.convert_AG_to_CT.py:84-183): every converted record at once, 4 positions
    // per thread, flattened over (converted record, dword).  Each chunk of G dwords reads first and
    // writes after a barrier: a dword's rule also reads the next dword's original bases ----
    if (do_convert) {
        const int nc = s_cnt[0];
        // a task is kConvH dwords (4 positions each) of one converted record; the 16 reference
        // nibbles at the task's aligned 8 bytes cover 4 * kConvH + 1 positions for kConvH <= 2
        constexpr int H = kConvH, TP = 4 * kConvH;
        const int SD = (maxlen_f + 1 + TP - 1) / TP;  // tasks per converted record, at most
        const int total = nc * SD;
        constexpr int kConvU = kLConvU;  // tasks per thread per round: their global loads go out together
        for (int base = 0; base < total; base += kConvU * G) {
            int rr[kConvU], jj[kConvU], av[kConvU];
            uint32_t w0[kConvU], w1[kConvU];
#pragma unroll
            for (int u = 0; u < kConvU; u++) {
                const int k = base + u * G + tt;
                rr[u] = -1;
                jj[u] = 0;
                if (k < total) {
                    const int ci = k / SD, j4 = TP * (k - ci * SD);
                    const int r = clist[ci];
                    if (j4 < M[r].in_len + 1) {
                        rr[u] = r;
                        jj[u] = j4;
                        // nibbles win + j4 .. + TP (high nibble first) lie in the 8 aligned bytes at a4
                        const uint64_t x0 = (uint64_t)M[r].win + (uint64_t)j4;
                        const uint32_t *rw = reinterpret_cast<const uint32_t *>(P.ref + ((x0 >> 1) & ~3ull));
                        w0[u] = rw[0];
                        w1[u] = rw[1];
                        av[u] = M[r].avail;
                    }
                }
            }
            uint32_t out[kConvU][H], wa[kConvU][H];
            bool ok[kConvU][H];
#pragma unroll
            for (int u = 0; u < kConvU; u++) {
#pragma unroll
                for (int h = 0; h < H; h++) ok[u][h] = false;
                if (rr[u] < 0) continue;
                const int r = rr[u];
                const RecMeta m = M[r];
                const int32_t Lm = m.in_len + 1;
                const uint64_t x00 = (uint64_t)m.win + (uint64_t)jj[u];
                const uint64_t W = (uint64_t)w0[u] | ((uint64_t)w1[u] << 32);
                const int u00 = (int)(x00 - 2 * ((x00 >> 1) & ~3ull));
#pragma unroll
                for (int h = 0; h < H; h++) {
                    const int j4 = jj[u] + 4 * h;
                    if (j4 >= Lm) continue;
                    ok[u][h] = true;
                    uint32_t m4 = lds32(slots + m.slot + j4);
                    const uint32_t mn = lds32(slots + m.slot + j4 + 4);
                    const int u0 = u00 + 4 * h;
                    uint32_t f0 = 0, f1 = 0;
#pragma unroll
                    for (int q = 0; q < 5; q++) {
                        const int x = u0 + q;
                        const uint32_t nb = (uint32_t)(W >> (8 * (x >> 1) + ((x & 1) ? 0 : 4))) & 0xFu;
                        const uint32_t fb = j4 + q < av[u] ? nb : kN;
                        if (q < 4) f0 |= fb << (8 * q);
                        if (q > 0) f1 |= fb << (8 * (q - 1));
                    }
                    if (j4 == 0) m4 = (m4 & ~0xFFu) | (f0 & 0xFFu);  // :121 seed, m[0] = ref[0]
                    const uint32_t m1 = alignbyte(mn, m4, 1);
                    uint32_t nxt = 0x80808080u;
                    const int last = Lm - 1 - j4;  // the record's last position has no next base
                    if (last < 4) nxt &= ~(0xFFu << (8 * last));
                    out[u][h] = convert4f<false>(m4, m1, f0, f1, nxt);
                    wa[u][h] = m.slot + (uint32_t)j4;
                    if (j4 == 0) qimg[m.slot] = 40;  // :174-177 'I' + quals
                    if (last < 4) {  // :157-170 a final C before a reference G is trimmed
                        const uint8_t rdv = (((out[u][h] >> (8 * last)) & 0xFF) == kC && ((f1 >> (8 * last)) & 0xFF) == kG) ? 1 : 0;
                        RecMeta &w = M[r];
                        w.rd = rdv;
                        w.len = Lm - rdv;
                        w.start = 0;
                        w.pos = m.pos - 1 > 0 ? m.pos - 1 : 0;
                        w.reflen = m.reflen + 1 - ((rdv && m.reflen > 0) ? 1 : 0);
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kConvU; u++)
#pragma unroll
                for (int h = 0; h < H; h++)
                    if (ok[u][h]) st32(slots + wa[u][h], out[u][h]);
            __syncthreads();
        }
    }
    if (!do_convert) {
        for (int r = tt; r < n; r += G)
            if (M[r].link & BSDC_LINK_RD_IN) M[r].rd = 1;
        __syncthreads();
    }
    if (stop == 2) return;

    // ---- gap extension ----
    if (do_extend) {
        for (int r = tt; r < n; r += G) {
            const RecMeta m = M[r];
            if (!(m.link & BSDC_LINK_EXT_RIGHT)) continue;
            const int p = (int)((m.link >> BSDC_LINK_PARTNER_SHIFT) & 3u);
            const RecMeta pm = M[p];
            uint8_t *sb = slots + m.slot;
            sb[0] = slots[pm.slot + pm.start];
            sb[img] = slots[pm.slot + img + pm.start];
            RecMeta &w = M[r];
            w.start = 0;
            w.len = m.len + 1;
            w.pos = m.pos - 1;
            w.reflen = m.reflen + 1;
        }
        __syncthreads();
        for (int r = tt; r < n; r += G) {
            const RecMeta m = M[r];
            if (!((m.link & BSDC_LINK_EXT_LEFT) && m.rd)) continue;
            const int p = (int)((m.link >> BSDC_LINK_PARTNER_SHIFT) & 3u);
            const RecMeta pm = M[p];
            uint8_t *sb = slots + m.slot;
            const int li = pm.start + pm.len - 1;
            sb[m.start + m.len] = slots[pm.slot + li];
            sb[img + m.start + m.len] = slots[pm.slot + img + li];
            RecMeta &w = M[r];
            w.len = m.len + 1;
            w.reflen = m.reflen + 1;
        }
        __syncthreads();
    }

    if (P.mode & BSDC_MODE_DUMP) {
        for (int r = 0; r < n; r++) {
            const RecMeta m = M[r];
            const int64_t d = (int64_t)B.rec[4 * (size_t)m.gidx];
            const uint8_t *sb = slots + m.slot + m.start;
            for (int j = tt; j < m.len; j += G) {
                P.O.dump_seq[d + j] = sb[j];
                P.O.dump_qual[d + j] = sb[img + j];
            }
            if (tt == 0) {
                P.O.dump_pos[m.gidx] = m.pos;
                P.O.dump_len[m.gidx] = (uint16_t)m.len;
                const bool conv = do_convert && (m.link & BSDC_LINK_CONVERT);
                uint8_t tg = 0;
                if (m.rd) tg |= 1;
                if (conv) tg |= 2 | 4;
                if (do_extend && (m.link & BSDC_LINK_EXT_RIGHT)) tg |= 4;
                if (do_extend && (m.link & BSDC_LINK_EXT_LEFT) && m.rd) tg |= 8;
                P.O.dump_tags[m.gidx] = tg;
            }
        }
    }
    if (!do_vote || stop == 3) return;

    auto cigv = [&](const RecMeta &m) {
        return make_cigview(B, m.gidx, m.link, do_convert && (m.link & BSDC_LINK_CONVERT), m.rd != 0, do_extend);
    };

    // ---- overlapping-bases consensus ----
    // A thread per R1 record finds its template's overlap.  Templates with simple cigars (and a
    // family without quals >= 128) run flattened over (template, 4 positions) through overlap4;
    // the rest take the per-position path, one wave per template.  Templates share no bytes.
    const bool wild = block_max<G>((qor & 0x80808080u) != 0 ? 1 : 0, red) != 0;
    if (stop == 11) return;
    if (P.overlap) {
        uint32_t *tl = reinterpret_cast<uint32_t *>(lists);  // fast: 3 words each from the front; slow: 1 from the back
        if (tt == 0) {
            s_cnt[0] = 0;
            s_cnt[1] = 0;
        }
        __syncthreads();
        for (int r = tt; r < n; r += G) {
            const RecMeta a = M[r];
            const uint32_t mate = a.link & BSDC_LINK_MATE_MASK;
            if (mate == BSDC_LINK_MATE_MASK || !(a.link & BSDC_LINK_USABLE)) continue;
            const RecMeta b = M[mate];
            if (!(b.link & BSDC_LINK_USABLE) || (a.flag & 4) || (b.flag & 4)) continue;
            if (a.reflen <= 0 || b.reflen <= 0) continue;
            const int32_t s0 = ::max(a.pos, b.pos);
            const int32_t e0 = ::min(a.pos + a.reflen - 1, b.pos + b.reflen - 1);
            if (s0 > e0) continue;
            if (!wild && !((a.link | b.link) & BSDC_LINK_COMPLEX)) {
                const int i = atomicAdd(&s_cnt[0], 1);
                tl[3 * i] = a.slot + (uint32_t)a.start + (uint32_t)(s0 - a.pos);
                tl[3 * i + 1] = b.slot + (uint32_t)b.start + (uint32_t)(s0 - b.pos);
                tl[3 * i + 2] = (uint32_t)(e0 - s0 + 1);
            } else {
                tl[2 * n - 1 - atomicAdd(&s_cnt[1], 1)] = (uint32_t)r;
            }
        }
        __syncthreads();
        if (stop == 12) return;
        const int nfast = s_cnt[0], nslow = s_cnt[1];
        // a task is 4 * kOvlChunks positions of one template (kOvlChunks SWAR dwords): the task ->
        // template map, the entry loads and the address math are paid once per task
        // aligned on mate a: the longest overlap spans (maxlen + 2 + 3) / 4 + 1 dwords of a
        const int SDo = ((maxlen_f + 2 + 3) / 4 + 1 + kOvlChunks - 1) / kOvlChunks;  // tasks of the longest overlap
        // kOvlU tasks per thread per round: all their loads, then all their stores (no byte of
        // the image belongs to two tasks)
        for (int k0 = tt; k0 < nfast * SDo; k0 += kOvlU * G) {
            OvlDw t[kOvlU][kOvlChunks];
#pragma unroll
            for (int u = 0; u < kOvlU; u++) {
                const int k = k0 + u * G;
                const bool act = k < nfast * SDo;
                const int g = act ? k / SDo : 0, d0 = kOvlChunks * (k - g * SDo);
                const uint32_t xa = tl[3 * g], xb = tl[3 * g + 1];
                const int ovl = act ? (int)tl[3 * g + 2] : 0;
#pragma unroll
                for (int c = 0; c < kOvlChunks; c++) t[u][c] = ovl_dw_load(slots, qimg, xa, xb, ovl, d0 + c);
            }
#pragma unroll
            for (int u = 0; u < kOvlU; u++)
#pragma unroll
                for (int c = 0; c < kOvlChunks; c++) ovl_dw_store(slots, qimg, t[u][c]);
        }
        for (int i = tt >> 6; i < nslow; i += G / kWave) {
            const int r = (int)tl[2 * n - 1 - i];
            const RecMeta a = M[r];
            const RecMeta b = M[a.link & BSDC_LINK_MATE_MASK];
            const int32_t s0 = ::max(a.pos, b.pos);
            const int32_t e0 = ::min(a.pos + a.reflen - 1, b.pos + b.reflen - 1);
            const bool ca = a.link & BSDC_LINK_COMPLEX, cb = b.link & BSDC_LINK_COMPLEX;
            CigView va, vb;
            if (ca) va = cigv(a);
            if (cb) vb = cigv(b);
            uint8_t *ab = slots + a.slot + a.start;
            uint8_t *aq = qimg + a.slot + a.start;
            uint8_t *bb = slots + b.slot + b.start;
            uint8_t *bq = qimg + b.slot + b.start;
            for (int32_t p = s0 + (tt & (kWave - 1)); p <= e0; p += kWave) {
                const int ia = ca ? read_at_ref(va, a.pos, a.len, p) : (p - a.pos < a.len ? p - a.pos : -1);
                const int ibb = cb ? read_at_ref(vb, b.pos, b.len, p) : (p - b.pos < b.len ? p - b.pos : -1);
                if (ia < 0 || ibb < 0) continue;
                const uint32_t x = ab[ia], y = bb[ibb];
                if (x == kN || y == kN) continue;
                const int qa = aq[ia], qb = bq[ibb];
                if (x == y) {
                    const uint8_t q = (uint8_t)::min(qa + qb, 93);
                    aq[ia] = q;
                    bq[ibb] = q;
                } else if (qa > qb) {
                    bb[ibb] = (uint8_t)x;
                    aq[ia] = bq[ibb] = (uint8_t)(qa - qb);
                } else if (qb > qa) {
                    ab[ia] = (uint8_t)y;
                    aq[ia] = bq[ibb] = (uint8_t)(qb - qa);
                } else {
                    ab[ia] = bb[ibb] = (uint8_t)kN;
                    aq[ia] = bq[ibb] = 2;
                }
            }
        }
        __syncthreads();
    }
    if (stop == 4) return;

    // ---- source reads ----
    for (int r = tt; r < n; r += G) {
        RecMeta &m = M[r];
        if (!(m.link & BSDC_LINK_USABLE)) continue;
        const bool negr = m.flag & 16;
        int32_t keep = m.len;
        const bool cx = m.link & BSDC_LINK_COMPLEX;
        CigView cv;
        if (cx) cv = cigv(m);
        if (m.link & BSDC_LINK_RT) keep = readthrough_keep(B, m.gidx, m.flag, m.pos, m.len, m.reflen, cx, &cv);
        const uint8_t *sb = slots + m.slot + m.start;
        while (keep > 0) {
            const uint32_t b = negr ? sb[m.len - keep] : sb[keep - 1];
            if (b != kN) break;
            keep--;
        }
        m.srclen = keep;
        if (keep > 0) {
            const bool r1 = m.flag & 0x40;
            const bool abs_ = m.link & BSDC_LINK_AB;
            m.set = abs_ ? (r1 ? 0 : 1) : (r1 ? 2 : 3);
        }
    }
    __syncthreads();
    if (stop == 10) return;

    // ---- most-common-alignment filter ----
    // Simplified cigars in parallel (each record's ops at an offset from a block scan of its op
    // bound), then the two groups (X = AB-R1 + BA-R2, Y = AB-R2 + BA-R1) by one thread each.
    int hc = 0;
    for (int r = tt; r < n; r += G) hc |= (M[r].link & BSDC_LINK_COMPLEX) && M[r].set != 0xFF;
    if (block_max<G>(hc, red)) {
        uint32_t *so = simp;
        uint32_t *sofs = simp + cops + 2 * n;
        uint16_t *srcl = reinterpret_cast<uint16_t *>(simp + cops + 3 * n);  // n u16 in the last n words
        uint8_t *setv = reinterpret_cast<uint8_t *>(srcl + n);               // ... and n bytes after them
        uint32_t run = 0;
        for (int base = 0; base < n; base += G) {
            const int r = base + tt;
            uint32_t v = 0;
            if (r < n) v = (M[r].link & BSDC_LINK_COMPLEX) ? (B.cig_info[M[r].gidx] & 0xFFFF) + 2u : 1u;  // ops bound
            uint32_t incl = v;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, o, kWave);
                if ((tt & (kWave - 1)) >= o) incl += y;
            }
            if ((tt & (kWave - 1)) == kWave - 1) red[tt >> 6] = (int)incl;
            __syncthreads();
            uint32_t woff = 0, ctot = 0;
            for (int w = 0; w < G / kWave; w++) {
                woff += w < (tt >> 6) ? (uint32_t)red[w] : 0u;
                ctot += (uint32_t)red[w];
            }
            if (r < n) {
                const RecMeta m = M[r];
                const uint32_t off = run + woff + incl - v;
                sofs[r] = 0;
                srcl[r] = (uint16_t)m.srclen;
                setv[r] = m.set;
                if (m.set != 0xFF) {
                    const bool mc = m.link & BSDC_LINK_COMPLEX;
                    CigView cv;
                    if (mc) cv = cigv(m);
                    const int c2 = simplified_cigar(&cv, mc, m.flag & 16, m.srclen, so + off);
                    sofs[r] = off | ((uint32_t)c2 << 16);
                }
            }
            run += ctot;
            __syncthreads();
        }
        if ((tt & (kWave - 1)) == 0 && (tt >> 6) < 2) {
            const int xy = tt >> 6;
            const int s1 = xy == 0 ? 0 : 1, s2 = xy == 0 ? 3 : 2;
            uint16_t *ord = lists + xy * n;
            int c = 0;
            for (int r = 0; r < n; r++)
                if (setv[r] == s1) ord[c++] = (uint16_t)r;
            for (int r = 0; r < n; r++)
                if (setv[r] == s2) ord[c++] = (uint16_t)r;
            filter_group(ord, c, srcl, sofs, so, setv, grp + 128 * xy, grp + 128 * xy + 64);
        }
        __syncthreads();
        for (int r = tt; r < n; r += G) M[r].set = setv[r];
        __syncthreads();
    }

    // ---- read descriptors by set, consensus lengths ----
    // desc[soff[s] + i] = {address of column 0, srclen | reverse << 31}; a reverse read's columns
    // run backwards from its last base.  Order within a set is free: the vote sums are integers.
    uint2 *desc = reinterpret_cast<uint2 *>(lists);
    if (tt < 4) {
        s_cnt[tt] = 0;
        s_lc[tt] = 0;
        s_cur[tt] = 0;
        s_cur[4 + tt] = 0;
    }
    __syncthreads();
    for (int r = tt; r < n; r += G) {
        const RecMeta &m = M[r];
        if (m.set == 0xFF) continue;
        atomicAdd(&s_cnt[m.set], 1);
        atomicMax(&s_lc[m.set], m.srclen);
    }
    __syncthreads();
    int cnt[4], lcv[4], soff[4];
    for (int s = 0, o = 0; s < 4; s++) {
        cnt[s] = s_cnt[s];
        lcv[s] = s_lc[s];
        soff[s] = o;
        o += cnt[s];
    }
    for (int r = tt; r < n; r += G) {  // forward reads from the front of the set, reverse from the back
        const RecMeta &m = M[r];
        if (m.set == 0xFF) continue;
        const bool negr = m.flag & 16;
        const int i = negr ? pick4<PART>(cnt, m.set) - 1 - atomicAdd(&s_cur[4 + m.set], 1) : atomicAdd(&s_cur[m.set], 1);
        desc[pick4<PART>(soff, m.set) + i] = make_uint2(m.slot + (uint32_t)m.start + (negr ? (uint32_t)(m.len - 1) : 0u),
                                           (uint32_t)m.srclen | (negr ? 0x80000000u : 0u));
    }
    __syncthreads();
    int nfw[4];
    for (int s = 0; s < 4; s++) nfw[s] = s_cur[s];
    if (stop == 5) return;

    // ---- single-strand vote ----
    // A thread owns consecutive columns of one set and walks its reads: one dword of bases and
    // one of quals per read (a reverse read's dword byte-swapped and complemented), columns past
    // the read's end cleared, lr[q] added to the base's sum.  Sets of <= 128 reads: 4 columns per
    // thread, int32 sums (exact: |lr| < 2^24).  Deeper sets: 2 columns per thread, int32 sums
    // flushed to int64 every 128 reads.
    auto resolve = [&](int s, int col, long long D0, long long D1, long long D2, long long D3, uint32_t n01, uint32_t n23) {
        int best = first_max4(D0, D1, D2, D3);
        if (near_tie(D0, D1, D2, D3, best, pick4<PART>(cnt, s)))  // rare: fgbio's fp64 read-order pick
            best = fp64_pick(LargeDesc{desc + pick4<PART>(soff, s)}, pick4<PART>(cnt, s), col, slots, qimg, P.tab->lnc, P.tab->lne3);
        const long long Db = best == 0 ? D0 : best == 1 ? D1 : best == 2 ? D2 : D3;
        float S = 0.0f;
        if (best != 0) S += term(D0 - Db);
        if (best != 1) S += term(D1 - Db);
        if (best != 2) S += term(D2 - Db);
        if (best != 3) S += term(D3 - Db);
        const int Q = phred_of(S, thr);
        // pass A left the OR of the column's A/C/G/T codes in ssb: 0 = no A/C/G/T read
        const bool nocall = ssb[s * ssw + col] == 0 || Q < P.qmin;
        ssb[s * ssw + col] = nocall ? (uint8_t)kN : (uint8_t)(1u << best);
        ssq[s * ssw + col] = nocall ? (uint8_t)2 : (uint8_t)Q;
        if (TAGS) {  // the column's depth / errors (the raw best base's reads) for the consensus tags
            const uint32_t depth = (n01 & 0xFFFFu) + (n01 >> 16) + (n23 & 0xFFFFu) + (n23 >> 16);
            const uint32_t nb = ((best < 2 ? n01 : n23) >> (16 * (best & 1))) & 0xFFFFu;
            put_ss_stats(P, fam, s, col, depth, depth - nb);
        }
    };
    // PART: a multi-base column's per-base sums (int32: a part holds < 255 reads a set) and counts
    // (PART) pass B's marked columns are the multi-base ones; the k-th of set s leaves its four
    // sums in slot k of the set's row (its `one`, written in pass A, holds k)
    auto part_write = [&](int s, int col, int k, long long D0, long long D1, long long D2, long long D3, uint32_t n01,
                          uint32_t n23) {
        const PartSums ps(P);
        if (TAGS) {
            ps.cnt[ps.at(blockIdx.x, s, col)] =
                (n01 & 0xFFu) | ((n01 >> 8) & 0xFF00u) | ((n23 & 0xFFu) << 16) | ((n23 >> 16) << 24);
        }
        ps.sum[ps.at(blockIdx.x, s, k)] =
            make_uint4((uint32_t)(int32_t)D0, (uint32_t)(int32_t)D1, (uint32_t)(int32_t)D2, (uint32_t)(int32_t)D3);
    };
    // Wavefronts by set: wave w works on set w % 4; with 8 waves (512 threads) the two waves of a
    // set split its reads (PARTS = 2).
    // Pass A: a lane owns 4 columns and walks the wave's reads, forward ones then reverse ones,
    // 4 in flight; descriptors are read 64 at a time, one per lane, and broadcast with v_readlane.
    // Per column: one likelihood sum over the reads showing an A/C/G/T there (Tables zero / lr
    // rows: a non-ACGT code adds 0) and the OR of those A/C/G/T codes.  A column whose OR is one
    // code, with a sum above one unit per read (no near tie with the unseen bases' 0), is resolved
    // from the sum alone: S = 3 e^-T, as the four-sum path computes it (an N or IUPAC code there
    // adds nothing to any of the four sums).  Every other column (a disagreement, no A/C/G/T at
    // all, a small or negative sum) is marked (ssq = 0).
    // Pass B: the marked columns, 8 lanes each: the lanes split the reads, sum per base, reduce
    // by lane shuffles, and the first lane makes the general call (resolve).
    constexpr int NW = G / kWave, PARTS = NW / 4;
    static_assert(NW == 4 * PARTS && PARTS >= 1 && PARTS <= 3, "k_large: 4, 8 or 12 wavefronts");
    const int32_t *lr2 = lr - 256;  // TablesL: zero[256] then lr[256]
    const int lane = tt & (kWave - 1), wv = tt >> 6, ws = wv & 3, wpart = wv >> 2;
    int64_t *psum = reinterpret_cast<int64_t *>(A + Lo.meta);        // [4][ssw] part-1 sums (RecMeta is dead)
    uint8_t *por = reinterpret_cast<uint8_t *>(psum + 4 * ssw);     // [4][ssw] part-1 ORs
    uint16_t *pcn = reinterpret_cast<uint16_t *>(por + 4 * ssw);     // [4][ssw] part-1 A/C/G/T read counts (TAGS)
    {
        const int na = pick4<PART>(cnt, ws), lc = pick4<PART>(lcv, ws), nf = pick4<PART>(nfw, ws);
        const uint2 *dl = desc + pick4<PART>(soff, ws);
        const int rb = wpart * na / PARTS, re = (wpart + 1) * na / PARTS;  // this wave's share of the set's reads
        const int lmax = ::max(::max(lcv[0], lcv[1]), ::max(lcv[2], lcv[3]));
        int nmk = 0;  // (PART) the set's marked columns before this block
        for (int cb = 0; cb < lmax; cb += 4 * kWave) {  // the same trip count in every wave (barriers inside)
            const int c = cb + 4 * lane, c8 = 8 * c;
            long long T0 = 0, T1 = 0, T2 = 0, T3 = 0;
            uint32_t orm = 0;
            uint32_t cn01 = 0, cn23 = 0;  // TAGS: A/C/G/T reads per column, u16 pairs
            if (cb < lc) {
                int32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
                uint32_t c4 = 0;  // (bytes, <= 64 reads between flushes)
                auto fwd = [&](uint32_t ex, uint32_t ey) {
                    const int sl = (int)ey;
                    const uint32_t keep = ~bytes_past(8 * sl - c8, false);
                    const int32_t a = (int32_t)ex + (sl > c ? c : 0);
                    const uint32_t b = lds_any32(slots, a) & keep, q = lds_any32(qimg, a);
                    const uint32_t v = onehot01(b);
                    orm |= b & (v * 0xFFu);
                    lookup4v(lr2, v, q, t0, t1, t2, t3);
                    if (TAGS) c4 += v;
                };
                auto rev = [&](uint32_t ex, uint32_t ey) {  // bytes run backwards from the read's last base
                    const int sl = (int)(ey & 0x7FFFFFFFu);
                    const uint32_t keep = ~bytes_past(8 * sl - c8, true);
                    const int32_t a = (int32_t)ex - (sl > c ? c : 0) - 3;
                    const uint32_t b = comp4(__builtin_bswap32(lds_any32(slots, a) & keep));
                    const uint32_t q = __builtin_bswap32(lds_any32(qimg, a));
                    const uint32_t v = onehot01(b);
                    orm |= b & (v * 0xFFu);
                    lookup4v(lr2, v, q, t0, t1, t2, t3);
                    if (TAGS) c4 += v;
                };
                auto flush = [&]() {  // int32 partials over <= 64 reads: exact
                    T0 += t0;
                    T1 += t1;
                    T2 += t2;
                    T3 += t3;
                    t0 = t1 = t2 = t3 = 0;
                    if (TAGS) {
                        cn01 += __builtin_amdgcn_perm(0u, c4, 0x0c010c00u);
                        cn23 += __builtin_amdgcn_perm(0u, c4, 0x0c030c02u);
                        c4 = 0;
                    }
                };
                const int fe = ::min(re, nf);
                for (int r0 = rb; r0 < fe; r0 += kWave) {
                    const uint2 dr = r0 + lane < fe ? dl[r0 + lane] : make_uint2(0u, 0u);
                    const int nr = ::min(kWave, fe - r0);
                    int i = 0;
                    for (; i + kVoteU - 1 < nr; i += kVoteU) {  // kVoteU reads' loads in flight
#pragma unroll
                        for (int u = 0; u < kVoteU; u++) fwd(rlu(dr.x, i + u), rlu(dr.y, i + u));
                    }
                    for (; i < nr; i++) fwd(rlu(dr.x, i), rlu(dr.y, i));
                    flush();
                }
                for (int r0 = ::max(rb, nf); r0 < re; r0 += kWave) {
                    const uint2 dr = r0 + lane < re ? dl[r0 + lane] : make_uint2(0u, 0u);
                    const int nr = ::min(kWave, re - r0);
                    int i = 0;
                    for (; i + kVoteU - 1 < nr; i += kVoteU) {  // kVoteU reads' loads in flight
#pragma unroll
                        for (int u = 0; u < kVoteU; u++) rev(rlu(dr.x, i + u), rlu(dr.y, i + u));
                    }
                    for (; i < nr; i++) rev(rlu(dr.x, i), rlu(dr.y, i));
                    flush();
                }
            }
            // the other parts' partials meet in one region, the last part first, each later one
            // adding its own, then part 0 reads them (one barrier per part)
#pragma unroll
            for (int pp = PARTS - 1; pp >= 1; pp--) {
                if (wpart == pp && cb < lc) {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (c + j < lc) {
                            const long long tj = j == 0 ? T0 : j == 1 ? T1 : j == 2 ? T2 : T3;
                            const uint8_t oj = (uint8_t)(orm >> (8 * j));
                            const uint16_t nj = (uint16_t)((j < 2 ? cn01 : cn23) >> (16 * (j & 1)));
                            if (pp == PARTS - 1) {
                                psum[ws * ssw + c + j] = tj;
                                por[ws * ssw + c + j] = oj;
                                if (TAGS) pcn[ws * ssw + c + j] = nj;
                            } else {
                                psum[ws * ssw + c + j] += tj;
                                por[ws * ssw + c + j] |= oj;
                                if (TAGS) pcn[ws * ssw + c + j] += nj;
                            }
                        }
                }
                __syncthreads();
            }
            if (wpart == 0 && cb < lc) {
                // PART: the lane's 4 columns' records -- ORs (one dword) or, with TAGS, counts (one
                // 16-B vector; a multi-base column's are pass B's) -- and one-base sums (one vector),
                // stored after the loop: per-column 4-B stores at a 16-B lane stride wrote each line
                // several times (C4 part dispatch: 1034 -> 263 MB written, profiles/r05/README.md)
                uint32_t or4 = 0, cnt4[4] = {0u, 0u, 0u, 0u};
                int32_t one4[4] = {0, 0, 0, 0};
                // PART: a multi-base column's four sums go to the slot of its rank among the set's
                // marked columns (pass B's mlist order), and its `one` holds that rank: the join's
                // lanes then read neighbouring columns' sums from neighbouring slots (by column, a
                // sparse 16-B read per line cost k_join 2.2x the bytes the parts wrote)
                uint32_t mrank = 0;
                if (PART) {
                    uint32_t mk4 = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        uint32_t ob = (orm >> (8 * j)) & 0xFFu;
                        if (PARTS >= 2 && c + j < lc) ob |= por[ws * ssw + c + j];
                        if (c + j < lc && (ob & (ob - 1)) != 0) mk4 |= 1u << j;
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) mrank += mbcnt(ballot((mk4 >> j) & 1u));
                    mrank += (uint32_t)nmk;
#pragma unroll
                    for (int j = 0; j < 4; j++) nmk += __builtin_popcountll(ballot((mk4 >> j) & 1u));
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int col = c + j;
                    if (col >= lc) break;
                    uint32_t ob = (orm >> (8 * j)) & 0xFFu;
                    long long Tj = j == 0 ? T0 : j == 1 ? T1 : j == 2 ? T2 : T3;
                    uint32_t nj = TAGS ? ((j < 2 ? cn01 : cn23) >> (16 * (j & 1))) & 0xFFFFu : 0u;
                    if (PARTS >= 2) {
                        Tj += psum[ws * ssw + col];
                        ob |= por[ws * ssw + col];
                        if (TAGS) nj += pcn[ws * ssw + col];
                    }
                    if (PART) {  // one base (or none) seen: the part's sums are that base's; else pass B
                        if ((ob & (ob - 1)) == 0) {
                            const int bi = ob ? __builtin_ctz(ob) : 0;
                            one4[j] = ob ? (int32_t)Tj : 0;
                            cnt4[j] = ob ? nj << (8 * bi) : 0u;
                            ssq[ws * ssw + col] = 1;
                        } else {
                            one4[j] = (int32_t)mrank++;
                            ssq[ws * ssw + col] = 0;
                        }
                        or4 |= ob << (8 * j);
                    } else if (ob != 0 && (ob & (ob - 1)) == 0 && Tj > na) {
                        const float e = term(-Tj);
                        const float S = ((0.0f + e) + e) + e;
                        const int Q = phred_of(S, thr);
                        ssb[ws * ssw + col] = Q < P.qmin ? (uint8_t)kN : (uint8_t)ob;
                        ssq[ws * ssw + col] = Q < P.qmin ? (uint8_t)2 : (uint8_t)Q;
                        if (TAGS) {  // one base seen: depth = its reads, errors 0
                            put_ss_stats(P, fam, ws, col, nj, 0u);
                        }
                    } else {
                        ssb[ws * ssw + col] = (uint8_t)ob;  // (the OR: pass B's no-call test)
                        ssq[ws * ssw + col] = 0;
                    }
                }
                // (only lanes with columns: a lane past lc would write into the next row; c < lc
                // gives c + 3 < stride, c being a multiple of 4 and stride of 16)
                if (PART && c < lc) {
                    const PartSums ps(P);
                    const int64_t at = ps.at(blockIdx.x, ws, c);
                    if (TAGS)
                        *reinterpret_cast<uint4 *>(ps.cnt + at) = make_uint4(cnt4[0], cnt4[1], cnt4[2], cnt4[3]);
                    else
                        *reinterpret_cast<uint32_t *>(ps.orb(at)) = or4;
                    *reinterpret_cast<int4 *>(ps.one + at) = make_int4(one4[0], one4[1], one4[2], one4[3]);
                }
            }
            if (PARTS >= 2) __syncthreads();
        }
    }
    __syncthreads();
    if (stop == 6) return;
    // Pass B.  The marked columns of each set are listed (ballot compaction; the list lives in the
    // part-sum region, dead now), then lane j of a wave owns the set's j-th marked column (the two
    // waves of a set take alternate blocks of 64) and walks all the set's reads, 4 in flight, with
    // the descriptors broadcast as in pass A: four per-base sums, then the general call (resolve).
    uint16_t *mlist = reinterpret_cast<uint16_t *>(psum);  // [4][ssw]
    if (wpart == 0) {
        const int lc = pick4<PART>(lcv, ws);
        int nm = 0;
        for (int cb = 0; cb < lc; cb += kWave) {
            const int col = cb + lane;
            const bool mk = col < lc && ssq[ws * ssw + col] == 0;
            const uint64_t bal = ballot(mk);
            if (mk) mlist[ws * ssw + nm + mbcnt(bal)] = (uint16_t)col;
            nm += __builtin_popcountll(bal);
        }
        if (lane == 0) s_lc[ws] = nm;
    }
    __syncthreads();
    {
        const int s = ws, na = pick4<PART>(cnt, s), nm = s_lc[s];
        const uint2 *dl = desc + pick4<PART>(soff, s);
        // With two waves per set (PARTS = 2) both take the same 64 marked columns and split the
        // set's reads; part 1's four sums meet part 0's through LDS (int32: exact for <= 127
        // reads a part, |lr| < 2^24), after mlist in the part-sum region.  Workgroup-uniform:
        // every set must fit, and every wave runs the same number of blocks (barriers inside).
        const int64_t region = ::max((int64_t)round16((int64_t)n * (int64_t)bsdc_layout::kRecMetaBytes) + round16(2 * (int64_t)n),
                                     (int64_t)bsdc_layout::kVoteRegionPerCol * ssw);
        const int64_t pbo = round16(8 * (int64_t)ssw);
        const bool split = PARTS >= 2 && pbo + (PARTS - 1) * 4 * kWave * 24 <= region &&
                           ::max(::max(cnt[0], cnt[1]), ::max(cnt[2], cnt[3])) <= 127 * PARTS;
        int32_t *pb = reinterpret_cast<int32_t *>(reinterpret_cast<uint8_t *>(psum) + pbo);  // [4][64][6]
        const int nmax = ::max(::max(s_lc[0], s_lc[1]), ::max(s_lc[2], s_lc[3]));
        const int rb = split ? wpart * na / PARTS : 0, re = split ? (wpart + 1) * na / PARTS : na;
        const int kstart = split ? 0 : kWave * wpart, kstep = split ? kWave : kWave * PARTS;
        const int kend = split ? nmax : nm;
        // One wave on a set with <= 32 marked columns: its two halves take the same columns and
        // half the reads each (the lower half reads [0, h), the upper [h, na)), then add up.
        const bool half = !split && nm <= 32 && na >= 16;
        const int h = (na + 1) >> 1, hl = lane & 31;
        for (int k0 = kstart; k0 < kend; k0 += kstep) {
            const int cl = half ? hl : lane;
            const bool act = k0 + cl < nm && (!half || lane < 32);
            const int col = k0 + cl < nm ? mlist[s * ssw + k0 + cl] : 0;
            long long D0 = 0, D1 = 0, D2 = 0, D3 = 0;
            int32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
            uint32_t n01 = 0, n23 = 0;  // TAGS: reads per base, u16 pairs (A | C << 16, G | T << 16)
            auto one = [&](uint32_t ex, uint32_t ey) {
                const int sl = (int)(ey & 0x7FFFFFFFu);
                const bool rv = ey >> 31, in = col < sl;
                const int32_t a = !in ? (int32_t)ex : rv ? (int32_t)ex - col : (int32_t)ex + col;
                const uint32_t braw = slots[a] & 0x0Fu, bb = rv ? comp_nt16(braw) : braw;
                const int32_t v = in ? lr[qimg[a]] : 0;
                d0 += bb == kA ? v : 0;
                d1 += bb == kC ? v : 0;
                d2 += bb == kG ? v : 0;
                d3 += bb == kT ? v : 0;
                if (TAGS && in) {
                    n01 += bb == kA ? 1u : bb == kC ? 0x10000u : 0u;
                    n23 += bb == kG ? 1u : bb == kT ? 0x10000u : 0u;
                }
            };
            if (half) {
                for (int r0 = 0; r0 < h; r0 += 32) {
                    // lane j < 32: read r0 + j; lane 32 + j: read h + r0 + j (0 descriptors add nothing)
                    const int rj = (lane < 32 ? 0 : h) + r0 + hl;
                    const bool okj = r0 + hl < h && rj < na;
                    const uint2 dr = okj ? dl[rj] : make_uint2(0u, 0u);
                    const int nr = ::min(32, h - r0);
                    auto pick = [&](uint32_t v, int i) { return lane < 32 ? rlu(v, i) : rlu(v, 32 + i); };
                    int i = 0;
                    for (; i + 7 < nr; i += 8) {  // 8 reads' loads in flight
#pragma unroll
                        for (int u = 0; u < 8; u++) one(pick(dr.x, i + u), pick(dr.y, i + u));
                    }
                    for (; i < nr; i++) one(pick(dr.x, i), pick(dr.y, i));
                    D0 += d0;  // int32 partials over <= 32 reads: exact
                    D1 += d1;
                    D2 += d2;
                    D3 += d3;
                    d0 = d1 = d2 = d3 = 0;
                }
                auto add_up = [&](long long &x) {  // + the upper half's partial (lane + 32)
                    const int lo = __shfl_xor((int)(uint32_t)x, 32, kWave), hi = __shfl_xor((int)(x >> 32), 32, kWave);
                    x += (long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
                };
                add_up(D0);
                add_up(D1);
                add_up(D2);
                add_up(D3);
                if (TAGS) {
                    n01 += (uint32_t)__shfl_xor((int)n01, 32, kWave);
                    n23 += (uint32_t)__shfl_xor((int)n23, 32, kWave);
                }
            }
            for (int r0 = rb; r0 < re && k0 < nm && !half; r0 += kWave) {
                const uint2 dr = r0 + lane < re ? dl[r0 + lane] : make_uint2(0u, 0u);
                const int nr = ::min(kWave, re - r0);
                int i = 0;
                for (; i + 7 < nr; i += 8) {  // 8 reads' loads in flight
#pragma unroll
                    for (int u = 0; u < 8; u++) one(rlu(dr.x, i + u), rlu(dr.y, i + u));
                }
                for (; i < nr; i++) one(rlu(dr.x, i), rlu(dr.y, i));
                D0 += d0;  // int32 partials over <= 64 reads: exact
                D1 += d1;
                D2 += d2;
                D3 += d3;
                d0 = d1 = d2 = d3 = 0;
            }
            if (split) {  // parts 1.. leave their sums in their own slots; part 0 adds them up
                if (wpart >= 1 && act) {
                    int32_t *pw = pb + 6 * (((wpart - 1) * 4 + s) * kWave + lane);
                    pw[0] = (int32_t)D0;
                    pw[1] = (int32_t)D1;
                    pw[2] = (int32_t)D2;
                    pw[3] = (int32_t)D3;
                    if (TAGS) {
                        pw[4] = (int32_t)n01;
                        pw[5] = (int32_t)n23;
                    }
                }
                __syncthreads();
                if (wpart == 0 && act) {
#pragma unroll
                    for (int pp = 1; pp < PARTS; pp++) {
                        const int32_t *pw = pb + 6 * (((pp - 1) * 4 + s) * kWave + lane);
                        D0 += pw[0];
                        D1 += pw[1];
                        D2 += pw[2];
                        D3 += pw[3];
                        if (TAGS) {
                            n01 += (uint32_t)pw[4];
                            n23 += (uint32_t)pw[5];
                        }
                    }
                    if (PART)
                        part_write(s, col, k0 + cl, D0, D1, D2, D3, n01, n23);
                    else
                        resolve(s, col, D0, D1, D2, D3, TAGS ? n01 : 0u, TAGS ? n23 : 0u);
                }
                __syncthreads();
            } else if (act) {
                if (PART)
                    part_write(s, col, k0 + cl, D0, D1, D2, D3, n01, n23);
                else
                    resolve(s, col, D0, D1, D2, D3, n01, n23);
            }
        }
    }
    __syncthreads();
    if (stop == 7) return;
    if (PART) {  // the part's set sizes and lengths; k_join does the rest
        if (tt < 8) PartSums(P).head[8 * (int64_t)blockIdx.x + tt] = tt < 4 ? pick4<PART>(cnt, tt) : pick4<PART>(lcv, tt - 4);
        return;
    }

    // ---- duplex combine and output ----
    large_emit<G, TAGS>(P, fam, cnt, lcv, ssb, ssq, ssw, stop == 0);
}

static_assert(BSDC_LARGE_LDS_MAX + kTabBytesL + 256 <= kLdsBytes, "large-family LDS budget");
struct TablesL {  // k_large's LDS copy: the prefix of Tables it reads
    int32_t zero[256];
    int32_t lr[256];
    float thr[96];
    uint8_t sq[144];
};
static_assert(sizeof(TablesL) == kTabBytesL, "TablesL image");
// G = 256 threads for the buckets that fit 3 or more workgroups per CU, 512 for the LDS-heavy ones
// (2 or 1 per CU, HBM scratch): twice the wavefronts in flight for the same LDS.
template <bool IN_LDS, int G, bool TAGS, bool PART = false>
__global__ __launch_bounds__(G, G == 256 ? 5 : 2) void k_large(KParams P, const uint4 *fams, int64_t nfams, int32_t arena,
                                                                int64_t scratch_off) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];  // the family's arena (IN_LDS)
    __shared__ __attribute__((aligned(16))) TablesL s_tab;  // loaded by process_large with the image
    __shared__ int red[2 * G / kWave];
    __shared__ int s_cnt[4], s_lc[4], s_cur[8];
    const TablesL *T = &s_tab;
    if (((P.mode >> BSDC_MODE_STOP_SHIFT) & 15) == 15) return;  // profiling: launch cost alone
    if (((P.mode >> BSDC_MODE_STOP_SHIFT) & 15) == 14) {        // profiling: + the table copy
        load_tables<kTabBytesL>(&P.tab->t, reinterpret_cast<uint8_t *>(&s_tab));
        return;
    }
    const int32_t *lr = T->lr;
    const float *thr = T->thr;
    const int64_t i = blockIdx.x;
    if (i >= nfams) return;
    if (threadIdx.x == 0) s_cnt[0] = 0;  // the converted-record count (process_large's first phase)
    __syncthreads();
    uint8_t *A = IN_LDS ? smem : P.O.scratch + scratch_off + (size_t)i * (size_t)arena;
    process_large<G, TAGS, PART>(P, A, reinterpret_cast<uint8_t *>(&s_tab), lr, thr, fams[i], red, s_cnt, s_lc, s_cur);
}

// A split family's join on one workgroup of G threads (k_join): rows = 8 x stride bytes of LDS for
// its single-strand rows + kJoinParts x 8 bytes for the parts' set lengths, tab = the TablesL copy.
constexpr int kJoinParts = 256;
template <int G, bool TAGS>
__device__ void join_family(const KParams &P, uint4 e0, uint4 e1, uint8_t *rows, uint8_t *tab, int *red, int *s_cnt,
                            int *s_lc, int *s_cur, int *s_tie) {
    const int tt = threadIdx.x;
    const TablesL &T = *reinterpret_cast<const TablesL *>(tab);
    const PartSums ps(P);
    const int64_t p0 = e1.x;
    const int np = (int)e1.y;
    // the parts' set lengths, [set][part] in LDS after the rows (kJoinParts at most; more read them
    // from HBM): a column's loop over the parts then issues only its sum and count loads
    uint16_t *hl = reinterpret_cast<uint16_t *>(rows + 8 * P.O.stride);
    const bool hl_lds = np <= kJoinParts;
    __syncthreads();  // (s_cnt / s_lc / s_tie are the caller's too)
    if (hl_lds)
        for (int k = tt; k < 4 * np; k += G) hl[(k & 3) * kJoinParts + (k >> 2)] = (uint16_t)ps.head[8 * (p0 + (k >> 2)) + 4 + (k & 3)];
    if (tt < 4) {
        int c = 0, l = 0;
        for (int p = 0; p < np; p++) {
            c += ps.head[8 * (p0 + p) + tt];
            l = ::max(l, ps.head[8 * (p0 + p) + 4 + tt]);
        }
        s_cnt[tt] = c;
        s_lc[tt] = c > 0 ? l : 0;
    }
    if (tt == 0) *s_tie = 0;
    __syncthreads();
    int cnt[4], lcv[4];
    for (int s = 0; s < 4; s++) {
        cnt[s] = s_cnt[s];
        lcv[s] = s_lc[s];
    }
    const int pitch = P.O.stride;
    uint8_t *ssb = rows, *ssq = rows + 4 * pitch;
    const int ntot = lcv[0] + lcv[1] + lcv[2] + lcv[3];
    for (int k = tt; k < ntot; k += G) {
        int s = 0, c = k;
        while (c >= lcv[s]) {
            c -= lcv[s];
            s++;
        }
        long long D0 = 0, D1 = 0, D2 = 0, D3 = 0;
        uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;  // (without TAGS: n0 = the OR of the parts' ORs)
        auto add = [&](uint4 d, uint32_t m) {
            D0 += (int32_t)d.x;
            D1 += (int32_t)d.y;
            D2 += (int32_t)d.z;
            D3 += (int32_t)d.w;
            if (TAGS) {
                n0 += m & 0xFFu;
                n1 += (m >> 8) & 0xFFu;
                n2 += (m >> 16) & 0xFFu;
                n3 += m >> 24;
            } else {
                n0 |= m;
            }
        };
        // a part's column record -- counts (TAGS) or OR (one-hot bits) -- shows more than one base
        auto multi = [&](uint32_t x) { return TAGS ? multi_base(x) : (x & (x - 1)) != 0; };
        // one part's column as four sums: its one base's sum, or the four sums (multi-base)
        auto four = [&](uint32_t x, int32_t o, uint4 sm) {
            if (multi(x)) return sm;
            const uint32_t b = TAGS ? (x & 0xFFu ? 0u : x & 0xFF00u ? 1u : x & 0xFF0000u ? 2u : 3u)
                                    : (x & 1u ? 0u : x & 2u ? 1u : x & 4u ? 2u : 3u);
            return make_uint4(b == 0 ? (uint32_t)o : 0u, b == 1 ? (uint32_t)o : 0u, b == 2 ? (uint32_t)o : 0u,
                              b == 3 ? (uint32_t)o : 0u);
        };
        auto rec = [&](int64_t at) { return TAGS ? ps.cnt[at] : (uint32_t)*ps.orb(at); };
        if (hl_lds) {
            // kJoinU parts' loads in flight, every load unconditional (a part past the set's end,
            // or past the family's parts, reads an in-range slot and is masked after; a one-base
            // column's sums load reads one shared line): no branch around a load, so no wait per part
            for (int pb = 0; pb < np; pb += kJoinU) {
                uint32_t m[kJoinU];
                int32_t o[kJoinU];
                bool in[kJoinU];
#pragma unroll
                for (int u = 0; u < kJoinU; u++) {
                    const int pc = ::min(pb + u, np - 1);
                    in[u] = pb + u < np && c < (int)hl[s * kJoinParts + pc];
                    // a lane past the part's set length reads the row's first column instead of
                    // bytes the part never wrote (a line each: 70 MB of C4's join reads)
                    const int cc = in[u] ? c : 0;
                    m[u] = rec(ps.at(p0 + pc, s, cc));
                    o[u] = ps.one[ps.at(p0 + pc, s, cc)];
                }
                uint4 sm[kJoinU];
#pragma unroll
                for (int u = 0; u < kJoinU; u++) {
                    m[u] = in[u] ? m[u] : 0u;
                    o[u] = in[u] ? o[u] : 0;
                    const int pc = ::min(pb + u, np - 1);
                    sm[u] = ps.sum[multi(m[u]) ? ps.at(p0 + pc, s, o[u]) : 0];  // (a multi-base column's `one`: its slot)
                }
#pragma unroll
                for (int u = 0; u < kJoinU; u++) add(four(m[u], o[u], sm[u]), m[u]);
            }
        } else {  // (more than kJoinParts parts: their set lengths from HBM, part by part)
            for (int p = 0; p < np; p++) {
                if (c >= ps.head[8 * (p0 + p) + 4 + s]) continue;  // (a part whose set ends before c wrote nothing there)
                const uint32_t x = rec(ps.at(p0 + p, s, c));
                const int32_t o = ps.one[ps.at(p0 + p, s, c)];
                add(four(x, o, multi(x) ? ps.sum[ps.at(p0 + p, s, o)] : make_uint4(0u, 0u, 0u, 0u)), x);
            }
        }
        const int best = first_max4(D0, D1, D2, D3);
        if (near_tie(D0, D1, D2, D3, best, cnt[s])) {
            *s_tie = 1;
            continue;
        }
        const long long Db = best == 0 ? D0 : best == 1 ? D1 : best == 2 ? D2 : D3;
        float S = 0.0f;
        if (best != 0) S += term(D0 - Db);
        if (best != 1) S += term(D1 - Db);
        if (best != 2) S += term(D2 - Db);
        if (best != 3) S += term(D3 - Db);
        const int Q = phred_of(S, T.thr);
        const uint32_t depth = n0 + n1 + n2 + n3;  // (without TAGS: nonzero iff a read shows an A/C/G/T)
        const bool nocall = depth == 0 || Q < P.qmin;
        ssb[s * pitch + c] = nocall ? (uint8_t)kN : (uint8_t)(1u << best);
        ssq[s * pitch + c] = nocall ? (uint8_t)2 : (uint8_t)Q;
        if (TAGS) {
            const uint32_t nb = best == 0 ? n0 : best == 1 ? n1 : best == 2 ? n2 : n3;
            put_ss_stats(P, e0.x, s, c, depth, depth - nb);
        }
    }
    __syncthreads();
    if (*s_tie) {  // (rare) the whole family in its HBM arena, fgbio's pick on the near ties
        if (tt == 0) s_cnt[0] = 0;
        __syncthreads();
        process_large<G, TAGS, false>(P, P.O.scratch + 16 * (int64_t)e1.z, tab, T.lr, T.thr, e0, red, s_cnt, s_lc, s_cur);
        return;
    }
    large_emit<G, TAGS>(P, e0.x, cnt, lcv, ssb, ssq, pitch, true);
}

// One workgroup per split family (include/bsdc.h): the parts' sums and counts added up per
// (set, column) -- exact integers, so the parts' order does not matter --, the single-strand call
// of each column (as k_large's resolve), then duplex combine and output (large_emit).  A near-tie
// column needs fgbio's read-order double sums over all the set's reads, which the parts did not
// keep: then the family runs whole in its HBM fallback arena (process_large), as the HBM bucket does.
template <bool TAGS>
__global__ __launch_bounds__(kJoinThreads, 1024 / kJoinThreads) void k_join(KParams P, const uint4 *sfams, int64_t nsf) {
    constexpr int G = kJoinThreads;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];  // single-strand rows: bases, quals [4][stride]
    __shared__ __attribute__((aligned(16))) TablesL s_tab;
    __shared__ int red[2 * G / kWave];
    __shared__ int s_cnt[4], s_lc[4], s_cur[8];
    __shared__ int s_tie;
    const int64_t i = blockIdx.x;
    if (i >= nsf) return;
    load_tables<kTabBytesL>(&P.tab->t, reinterpret_cast<uint8_t *>(&s_tab));
    join_family<G, TAGS>(P, sfams[2 * i], sfams[2 * i + 1], smem, reinterpret_cast<uint8_t *>(&s_tab), red, s_cnt,
                         s_lc, s_cur, &s_tie);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------
#ifndef BSDC_FORK
#define BSDC_FORK 1
#endif
#ifndef BSDC_FORK_STREAMS
#define BSDC_FORK_STREAMS 4
#endif
constexpr int kForkStreams = BSDC_FORK_STREAMS;

struct bsdc_ctx {
    int device;
    bsdc_params params;
    DevTables host_tab;
    DevTables *dev_tab = nullptr;
    uint8_t *ref_seq = nullptr;
    int64_t ref_nibbles = 0;
    std::string err;
    // (BSDC_FORK) side streams the bucket dispatches of one call fan out to, joined back to the
    // caller's stream by events, so one dispatch's tail overlaps the next
    hipStream_t side[kForkStreams] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kForkStreams] = {};
};

static float det_expf_host(float x) {
    const float tq = x * 1.44269504088896341f;
    const float n = rintf(tq);
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

static int phred_agree(int64_t D, const float *thr) {
    const float x = (float)((double)(-D) * 9.5367431640625e-07);
    const float e = x < -80.0f ? 0.0f : det_expf_host(x);
    const float S = ((0.0f + e) + e) + e;
    int Q = 0;
    for (int k = 1; k < 94; k++) {
        if (S <= thr[k])
            Q = k;
        else
            break;
    }
    return Q;
}

static void make_tables(double pre, double post, Tables &t) {
    // keep in step with oracle/bsdc_oracle.c orc_tables
    const double e_post = pow(10.0, -post / 10.0);
    const double e_pre = pow(10.0, -pre / 10.0);
    for (int q = 0; q < 256; q++) {
        const double e = pow(10.0, -(double)q / 10.0);
        const double a = e_post + e - (4.0 / 3.0) * e_post * e;
        const double lnc = log1p(-a);
        const double lne = log(a / 3.0);
        t.lr[q] = (int32_t)llround((lnc - lne) * kLrScale);
    }
    for (int q = 0; q < 256; q++) t.zero[q] = 0;
    t.thr[0] = INFINITY;
    for (int k = 1; k < 94; k++) {
        const double pk = pow(10.0, -((double)k - 0.001) / 10.0);
        const double tt = (pk - e_pre) / (1.0 - (4.0 / 3.0) * e_pre);
        t.thr[k] = tt < 0.0 ? -1.0f : (float)(tt / (1.0 - tt));
    }
    t.thr[94] = t.thr[95] = -1.0f;
    // sq[j] = Q at the largest S of bucket j (bits (kSqBase + j + 1) << 21, minus one ulp): Q is
    // non-increasing in S, so it is a lower bound on Q over the bucket (and below it, for j = 0)
    for (int j = 0; j < 144; j++) {
        const int jj = j < kSqBuckets ? j : kSqBuckets - 1;
        const uint32_t bits = ((uint32_t)(kSqBase + jj + 1) << 21) - 1u;
        float S;
        memcpy(&S, &bits, 4);
        int q = 0;
        for (int k = 1; k < 94; k++)
            if (S <= t.thr[k]) q = k;
        t.sq[j] = (uint8_t)q;
    }
    // agreement case: every other base has D = 0, S = ((0 + e) + e) + e with e = term(-D); Q(D)
    // is the oracle's arithmetic on the host (same float ops), tabulated exactly:
    // Q(D) = qlo[D >> 16] + (D >= dthr[qlo[D >> 16] + 1]).  tests/test_abi.py checks every D.
    auto qof = [&](int64_t D) { return phred_agree(D, t.thr); };
    for (int k = 0; k < 2048; k++) t.qlo[k] = (uint8_t)qof((int64_t)k << 16);
    for (int q = 0; q < 48; q++) {
        if (q == 0) {
            t.dthr[q] = 0;
            continue;
        }
        int64_t lo = 0, hi = (int64_t)1 << 27;  // smallest D in [0, 2^27) with Q(D) >= q, else 2^31-1
        if (qof(hi - 1) < q) {
            t.dthr[q] = 0x7FFFFFFF;
            continue;
        }
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (qof(mid) >= q)
                hi = mid;
            else
                lo = mid + 1;
        }
        t.dthr[q] = (int32_t)lo;
    }
}

// fgbio's per-read terms in double precision, its LogProbability arithmetic restated (PARITY
// UNPINNED): pErr = probabilityOfErrorTwoTrials(ln e_post, ln e(q)); lnc = not(pErr), lne3 = pErr -
// ln 3.  The near-tie pick adds these, so the operation order is kept in step with oracle/
// bsdc_oracle.c orc_tables_fp64 and tests/fgbio_vote.py qual_tables (tests/test_fgbio_vote.py
// compares the three bit for bit).
static double lp_or(double a, double b) {
    const double m = a > b ? a : b, n = a > b ? b : a;
    return m == -INFINITY ? m : m + log1p(exp(n - m));
}
static double lp_not(double x) { return x > -log(2.0) ? log(-expm1(x)) : log1p(-exp(x)); }
static double lp_a_or_not_b(double a, double b) { return b == -INFINITY ? a : a + log1p(-exp(b - a)); }
static void make_fp64(double post, double *lnc, double *lne3) {
    const double ln10 = log(10.0), ln3 = log(3.0), ln43 = log(4.0 / 3.0);
    const double x = -post * ln10 / 10.0;
    for (int q = 0; q < 256; q++) {
        const double y = -(double)q * ln10 / 10.0;
        const double pe = lp_a_or_not_b(lp_or(x, y), ln43 + x + y);
        lnc[q] = lp_not(pe);
        lne3[q] = pe - ln3;
    }
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

int32_t bsdc_host_register(int32_t device, void *ptr, int64_t nbytes) {
    if (!ptr || nbytes <= 0) return BSDC_EINVAL;
    if (hipSetDevice(device) != hipSuccess || hipHostRegister(ptr, (size_t)nbytes, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();  // (not sticky: the next launch check must not see it)
        return BSDC_EDEVICE;
    }
    return 0;
}

int32_t bsdc_host_unregister(int32_t device, void *ptr) {
    if (!ptr) return BSDC_EINVAL;
    if (hipSetDevice(device) != hipSuccess || hipHostUnregister(ptr) != hipSuccess) {
        (void)hipGetLastError();
        return BSDC_EDEVICE;
    }
    return 0;
}

static bool params_ok(const bsdc_params *p) {
    return p->min_reads == 0 && p->min_input_base_quality >= 0 && p->min_consensus_base_quality >= 0 &&
           p->min_consensus_base_quality <= 94;
}

int32_t bsdc_ctx_set_params(bsdc_ctx *c, const bsdc_params *params) {
    if (!c || !params) return BSDC_EINVAL;
    if (!params_ok(params)) {
        c->err = "bad params";
        return BSDC_EINVAL;
    }
    if (params->error_rate_pre_umi != c->params.error_rate_pre_umi ||
        params->error_rate_post_umi != c->params.error_rate_post_umi) {
        // new tables: no launch of this context may still read the old ones
        HIP_OK(c, hipSetDevice(c->device));
        HIP_OK(c, hipDeviceSynchronize());
        make_tables(params->error_rate_pre_umi, params->error_rate_post_umi, c->host_tab.t);
        make_fp64(params->error_rate_post_umi, c->host_tab.lnc, c->host_tab.lne3);
        HIP_OK(c, hipMemcpy(c->dev_tab, &c->host_tab, sizeof(DevTables), hipMemcpyHostToDevice));
    }
    c->params = *params;  // the rest is read at launch time (bsdc_run)
    return 0;
}
void bsdc_ctx_destroy(bsdc_ctx *c);

int64_t bsdc_family_arena_bytes(int32_t n_rec, int64_t slot_bytes, int32_t max_len, int64_t complex_ops) {
    ArenaLayout L(n_rec, slot_bytes, max_len, complex_ops);
    return (int64_t)L.total;
}

int64_t bsdc_small_arena_bytes(int32_t n_rec, int64_t img, int32_t n_conv, int64_t complex_ops, int32_t max_len) {
    SmallLayout L(n_rec, img, n_conv, complex_ops, max_len);
    return (int64_t)L.total;
}

void bsdc_model_tables(double pre, double post, int64_t *lr256, float *thr94) {
    Tables t;
    make_tables(pre, post, t);
    for (int i = 0; i < 256; i++) lr256[i] = t.lr[i];
    for (int i = 0; i < 94; i++) thr94[i] = t.thr[i];
}

void bsdc_agree_tables(double pre, double post, uint8_t *qlo2048, int32_t *dthr48) {
    Tables t;
    make_tables(pre, post, t);
    memcpy(qlo2048, t.qlo, sizeof t.qlo);
    memcpy(dthr48, t.dthr, sizeof t.dthr);
}

void bsdc_model_tables_fp64(double pre, double post, double *lnc256, double *lne3_256) {
    (void)pre;
    make_fp64(post, lnc256, lne3_256);
}

void bsdc_phred_buckets(double pre, double post, uint8_t *sq144) {
    Tables t;
    make_tables(pre, post, t);
    memcpy(sq144, t.sq, sizeof t.sq);
}

int32_t bsdc_ctx_create(int32_t device, const bsdc_params *params, bsdc_ctx **out) {
    if (!out || !params) return BSDC_EINVAL;
    *out = nullptr;
    if (!params_ok(params)) return BSDC_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return BSDC_EDEVICE;
    bsdc_ctx *c = new bsdc_ctx();
    c->device = device;
    c->params = *params;
    make_tables(params->error_rate_pre_umi, params->error_rate_post_umi, c->host_tab.t);
    make_fp64(params->error_rate_post_umi, c->host_tab.lnc, c->host_tab.lne3);
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&c->dev_tab, sizeof(DevTables)) != hipSuccess ||
        hipMemcpy(c->dev_tab, &c->host_tab, sizeof(DevTables), hipMemcpyHostToDevice) != hipSuccess) {
        bsdc_ctx_destroy(c);
        return BSDC_EDEVICE;
    }
    if (BSDC_FORK) {  // the side streams and their events: all of them, or the context fails
        bool ok = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; ok && i < kForkStreams; i++)
            ok = hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&c->ev_join[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            bsdc_ctx_destroy(c);
            return BSDC_EDEVICE;
        }
    }
    *out = c;
    return 0;
}

void bsdc_ctx_destroy(bsdc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipFree(c->dev_tab);
    (void)hipFree(c->ref_seq);
    for (int i = 0; i < kForkStreams; i++) {
        if (c->side[i]) (void)hipStreamDestroy(c->side[i]);
        if (c->ev_join[i]) (void)hipEventDestroy(c->ev_join[i]);
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    delete c;
}

const char *bsdc_last_error(const bsdc_ctx *c) { return c ? c->err.c_str() : "null context"; }

int32_t bsdc_get_tables(const bsdc_ctx *c, int64_t *lr256, float *thr94) {
    if (!c) return BSDC_EINVAL;
    for (int i = 0; i < 256; i++) lr256[i] = c->host_tab.t.lr[i];
    for (int i = 0; i < 94; i++) thr94[i] = c->host_tab.t.thr[i];
    return 0;
}

int32_t bsdc_load_reference(bsdc_ctx *c, const uint8_t *packed, int64_t n_nib, const int64_t *coff,
                            const int64_t *clen, int32_t n_contig) {
    (void)coff;
    (void)clen;
    if (!c || n_contig < 0 || n_nib < 0 || (n_nib > 0 && !packed)) return BSDC_EINVAL;
    HIP_OK(c, hipSetDevice(c->device));
    (void)hipFree(c->ref_seq);
    c->ref_seq = nullptr;
    // +512 B: window chunks may read past the genome end (their nibbles are masked as N)
    const size_t nb = (size_t)((n_nib + 1) / 2) + 512;
    HIP_OK(c, hipMalloc(&c->ref_seq, nb));
    HIP_OK(c, hipMemset(c->ref_seq, 0xFF, nb));
    if (n_nib > 0) HIP_OK(c, hipMemcpy(c->ref_seq, packed, (size_t)((n_nib + 1) / 2), hipMemcpyHostToDevice));
    c->ref_nibbles = n_nib;
    return 0;
}

int32_t bsdc_run(bsdc_ctx *c, const bsdc_family_batch *b, bsdc_consensus *o, int32_t mode, void *stream) {
    if (!c || !b || !o) return BSDC_EINVAL;
    if (o->stride % 16 || o->stride < b->max_len + 2 || b->max_len > 0xFFFF - 8) {
        c->err = "bad stride";
        return BSDC_EINVAL;
    }
    if (b->n_split_parts > 0 && (b->split_part_arena % 16 || b->split_part_arena <= 0 ||
                                 b->split_part_arena > BSDC_LARGE_LDS_MAX || !o->scratch || !b->split_parts || !b->split_fams)) {
        c->err = "bad split families";
        return BSDC_EINVAL;
    }
    for (int q = 0; q < BSDC_LARGE_BUCKETS; q++) {
        if (b->n_large[q] > 0 && (b->large_arena[q] % 16 || b->large_arena[q] <= 0)) {
            c->err = "bad large arena size";
            return BSDC_EINVAL;
        }
        if (b->n_large[q] > 0 && b->large_arena[q] > BSDC_LARGE_LDS_MAX && !o->scratch) {
            c->err = "large families need scratch";
            return BSDC_EINVAL;
        }
    }
    for (int q = 0; q < BSDC_SMALL_BUCKETS; q++) {
        if (b->n_small[q] > 0 &&
            (b->small_arena[q] % 16 || b->small_arena[q] <= 0 ||
             (size_t)kTabBytes + 2 * (size_t)kArenaGuard + 4 * (size_t)b->small_arena[q] > kLdsBytes)) {
            c->err = "bad small arena size";
            return BSDC_EINVAL;
        }
    }
    if ((mode & BSDC_MODE_CONVERT) && !c->ref_seq) {
        c->err = "reference not loaded";
        return BSDC_EINVAL;
    }
    if ((mode & BSDC_MODE_TAGS) && (!(mode & BSDC_MODE_VOTE) || !o->ss_len || !o->ss_base || !o->ss_qual ||
                                    !o->ss_depth || !o->ss_err)) {
        c->err = "BSDC_MODE_TAGS needs BSDC_MODE_VOTE and the ss_* outputs";
        return BSDC_EINVAL;
    }
    if ((mode & BSDC_MODE_TAGS) && o->ss_wide && (!o->ss_wdepth || !o->ss_werr)) {
        c->err = "ss_wide needs ss_wdepth and ss_werr";
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
    P.ref = c->ref_seq;
    P.tab = c->dev_tab;
    P.mode = mode;
    P.overlap = c->params.consensus_call_overlapping_bases;
    P.ref_chunks = ref_chunks(b->max_len);
    P.ref_chunks_inv = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)P.ref_chunks - 1) / (uint64_t)P.ref_chunks);
    P.qmin = c->params.min_consensus_base_quality;
    // the dispatches: on `s`, or (BSDC_FORK) spread over the side streams (created with the
    // context) after an event on `s`
    int nd = 0, used = 0;
    int32_t rc = 0;
    auto fail = [&](hipError_t e, const char *what) {
        c->err = std::string(what) + ": " + hipGetErrorString(e);
        rc = BSDC_EDEVICE;
    };
    auto next_stream = [&]() -> hipStream_t {
        if (!BSDC_FORK) return s;
        hipError_t e;
        if (nd == 0 && (e = hipEventRecord(c->ev_fork, s)) != hipSuccess) {
            fail(e, "hipEventRecord(fork)");
            return nullptr;
        }
        const int i = nd++ % kForkStreams;
        if (!(used & (1 << i))) {
            if ((e = hipStreamWaitEvent(c->side[i], c->ev_fork, 0)) != hipSuccess) {
                fail(e, "hipStreamWaitEvent(side)");
                return nullptr;
            }
            used |= 1 << i;
        }
        return c->side[i];
    };
    // split families: their parts (k_large part mode, LDS arenas, 256 threads), then one join
    // workgroup per family, in order on one stream
    auto launch_split = [&]() {
        if (rc != 0 || b->n_split_parts <= 0 || b->n_split_fams <= 0) return;
        const int32_t a = b->split_part_arena;
        const bool tg = (mode & BSDC_MODE_TAGS) != 0;
        const hipStream_t ls = next_stream();
        if (rc != 0) return;
        const uint4 *pf = reinterpret_cast<const uint4 *>(b->split_parts);
        const uint4 *sf = reinterpret_cast<const uint4 *>(b->split_fams);
        const size_t jl = 8 * (size_t)o->stride + 8 * kJoinParts;
        // k_join reads the sums header the parts write at the end of their vote: without
        // BSDC_MODE_VOTE (the tools-only launches dump tool-2 records and stop before it) or with a
        // profiling stop knob (the parts return early) that scratch is never written, so no join
        const bool join = (mode & BSDC_MODE_VOTE) && ((mode >> BSDC_MODE_STOP_SHIFT) & 15) == 0;
        if (tg) {
            hipLaunchKernelGGL((k_large<true, kLargeThreads, true, true>), dim3((unsigned)b->n_split_parts), dim3(kLargeThreads),
                               (size_t)a, ls, P, pf, b->n_split_parts, a, (int64_t)0);
            if (join)
                hipLaunchKernelGGL((k_join<true>), dim3((unsigned)b->n_split_fams), dim3(kJoinThreads), jl, ls, P, sf,
                                   b->n_split_fams);
        } else {
            hipLaunchKernelGGL((k_large<true, kLargeThreads, false, true>), dim3((unsigned)b->n_split_parts),
                               dim3(kLargeThreads), (size_t)a, ls, P, pf, b->n_split_parts, a, (int64_t)0);
            if (join)
                hipLaunchKernelGGL((k_join<false>), dim3((unsigned)b->n_split_fams), dim3(kJoinThreads), jl, ls, P, sf,
                                   b->n_split_fams);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) fail(e, "split launch");
    };
    auto launch_small_all = [&]() {
    if (!(mode & BSDC_MODE_SKIP_SMALL) && rc == 0) {
        const uint32_t *f = b->small_fams;
        for (int q = 0; q < BSDC_SMALL_BUCKETS && rc == 0; q++) {
            const int64_t nf = b->n_small[q];
            if (nf > 0) {
                // wavefronts per workgroup (they share one copy of the tables): 4 or 8, whichever
                // keeps more wavefronts resident per CU; the smaller on a tie
                // (a workgroup's wavefronts spread over the 4 SIMDs: at most kSmallSimdWaves each)
                const int64_t a = b->small_arena[q];
                const int64_t g2 = 2 * kArenaGuard;
                const int64_t w4 = 4 * std::min<int64_t>(kSmallSimdWaves, kLdsBytes / (kTabBytes + g2 + 4 * a));
                const int64_t w8 = 8 * std::min<int64_t>(kSmallSimdWaves / 2, kLdsBytes / (kTabBytes + g2 + 8 * a));
                const int nw = w8 > w4 ? 8 : 4;
                const size_t lds = (size_t)nw * (size_t)a + (size_t)g2;  // + the static tables
                const int64_t blocks = (nf + nw - 1) / nw;
                const hipStream_t ls = next_stream();
                if (rc) break;
                if (mode & BSDC_MODE_TAGS)
                    hipLaunchKernelGGL(k_small<true>, dim3((unsigned)blocks), dim3(kWave * nw), lds, ls, P, f, nf, b->small_arena[q]);
                else
                    hipLaunchKernelGGL(k_small<false>, dim3((unsigned)blocks), dim3(kWave * nw), lds, ls, P, f, nf, b->small_arena[q]);
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) fail(e, "k_small launch");
            }
            f += 4 * nf;
        }
    }
    };
    auto launch_large_all = [&]() {
    if (!(mode & BSDC_MODE_SKIP_LARGE) && rc == 0) {
        // one dispatch per non-empty bucket: its LDS arena size sets how many workgroups share a CU
        const uint4 *f = reinterpret_cast<const uint4 *>(b->large_fams);
        // every bucket beyond the LDS budget has its own region of `scratch` (the dispatches may
        // run at once on the side streams)
        int64_t soff = 0;
        for (int q = 0; q < BSDC_LARGE_BUCKETS && rc == 0; q++) {
            const int64_t nf = b->n_large[q];
            const int32_t a = b->large_arena[q];
            if (nf > 0) {
                const bool big = q >= kLargeBigBucket;  // 3, 2 or 1 workgroups per CU, or HBM scratch
                const hipStream_t ls = next_stream();
                if (rc) break;
                const bool tg = (mode & BSDC_MODE_TAGS) != 0;
                if (a <= BSDC_LARGE_LDS_MAX && !big) {
                    if (tg)
                        hipLaunchKernelGGL((k_large<true, kLargeThreads, true>), dim3((unsigned)nf), dim3(kLargeThreads), (size_t)a, ls, P, f,
                                           nf, a, (int64_t)0);
                    else
                        hipLaunchKernelGGL((k_large<true, kLargeThreads, false>), dim3((unsigned)nf), dim3(kLargeThreads), (size_t)a, ls, P,
                                           f, nf, a, (int64_t)0);
                } else if (a <= BSDC_LARGE_LDS_MAX) {
                    if (tg)
                        hipLaunchKernelGGL((k_large<true, kLargeThreadsBig, true>), dim3((unsigned)nf), dim3(kLargeThreadsBig), (size_t)a, ls,
                                           P, f, nf, a, (int64_t)0);
                    else
                        hipLaunchKernelGGL((k_large<true, kLargeThreadsBig, false>), dim3((unsigned)nf), dim3(kLargeThreadsBig), (size_t)a,
                                           ls, P, f, nf, a, (int64_t)0);
                } else {
                    if (tg)
                        hipLaunchKernelGGL((k_large<false, kLargeThreadsBig, true>), dim3((unsigned)nf), dim3(kLargeThreadsBig), 0, ls, P, f,
                                           nf, a, soff);
                    else
                        hipLaunchKernelGGL((k_large<false, kLargeThreadsBig, false>), dim3((unsigned)nf), dim3(kLargeThreadsBig), 0, ls, P,
                                           f, nf, a, soff);
                    soff += nf * (int64_t)a;
                }
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) fail(e, "k_large launch");
            }
            f += nf;
        }
        launch_split();  // (first instead: not faster, profiles/r05/README.md)
    }
    };
    // small families first (the large families' dispatches first: not faster, profiles/r05/README.md)
    launch_small_all();
    launch_large_all();
    // join: `s` waits for every side stream used -- also after a failed launch, so that no work
    // already queued on a side stream outlives the caller's view of the batch's buffers
    for (int i = 0; i < kForkStreams; i++)
        if (used & (1 << i)) {
            hipError_t e = hipEventRecord(c->ev_join[i], c->side[i]);
            if (e == hipSuccess) e = hipStreamWaitEvent(s, c->ev_join[i], 0);
            if (e != hipSuccess) {  // cannot order it on `s`: wait for the side stream itself
                (void)hipStreamSynchronize(c->side[i]);
                if (rc == 0) fail(e, "join");
            }
        }
    return rc;
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
