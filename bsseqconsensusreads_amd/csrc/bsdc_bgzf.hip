// BGZF block compression on the GPU (gfx950): one 256-thread workgroup per 65280-byte block of
// an uncompressed BAM stream -> a gzip member with one dynamic-Huffman DEFLATE block (RFC 1951),
// the BGZF header with BSIZE (SAM/BAM spec 4.1).  The host adds CRC32 + ISIZE when it writes the
// blocks out (it holds the uncompressed bytes), and stores a block whose deflate would not fit.
//
// The algorithm is oracle/bgzf_ref.c's, step for step, so the bytes are identical (tests):
//  A. match candidates in rounds of 256 consecutive positions: a position's candidate is the last
//     earlier position of its round with the same 4 bytes (each thread scans the round's values in
//     LDS back from its own), else what the LDS hash table holds; then the round inserts its
//     positions (atomicMax: the largest wins a slot).  The candidates, as distances in HBM
//     scratch, link every position to an earlier one: a hash chain;
//  B. thread t parses its 255-byte segment: at each position the longest match (>= 3, not past the
//     segment, first on a tie) of distances 1, 2, 4 and the first 8 positions down the chain (from
//     A2: each position's chain distances precomputed in parallel), the search ending at a match
//     of 64;
//     lazy: a match shorter than 32 yields a literal when the next position has a longer one;
//     tokens to HBM scratch, symbol frequencies by LDS atomics;
//  C. thread 0 builds the length-limited Huffman codes (the restatement's two-queue build), the
//     run-length coded code lengths and their own code, and writes the block header bits;
//  D. each thread's bit count, a block scan -> bit offsets;
//  E. each thread writes its bits: whole 32-bit words as plain stores, its first and last
//     (shared) words by atomicOr into the zeroed slot.
// Bytes per block: 65280 in, ~9.3 KB out for the tagged step-5 output (ratio 7.0 against libdeflate
// level 5's 7.26, profiles/deflate_levels.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bsdc.h"

namespace {

constexpr int kT = 256;          // threads per block = positions per candidate round
constexpr int kSeg = 255;        // bytes per thread segment (kT * kSeg = 65280 = BGZF block)
constexpr int kBlock = kT * kSeg;
constexpr int kHashBits = 11;  // 2048 slots: the block, the table and the rest fit 80 KB of LDS (2 workgroups per CU)
constexpr int kMaxDist = 32768;
constexpr int kChain = 8;        // chain positions tried per match search
constexpr int kLazy = 32;        // matches shorter than this look one position ahead
constexpr int kNice = 64;        // a match this long ends the search
constexpr int kOutCap = 65536 - 26;  // deflate bytes that still fit a BGZF block

__constant__ uint8_t cClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// the RFC 1951 length / distance code tables as arithmetic (a divergent index into a __constant__
// table is a vector memory load; these are on every token of phases B, D and E)
__device__ __forceinline__ int len_code(int l) {  // 3 <= l <= 258
    if (l < 11) return l - 3;
    if (l == 258) return 28;
    const int n = l - 3, e = 31 - __builtin_clz((unsigned)n);
    return 4 * (e - 1) + ((n >> (e - 2)) & 3);
}
__device__ __forceinline__ int len_base(int c) { return c < 8 ? c + 3 : c == 28 ? 258 : ((4 + (c & 3)) << ((c >> 2) - 1)) + 3; }
__device__ __forceinline__ int len_extra(int c) { return c < 8 || c == 28 ? 0 : (c >> 2) - 1; }
__device__ __forceinline__ int dist_code(int d) {  // 1 <= d <= 32768
    if (d <= 4) return d - 1;
    const int n = d - 1, e = 31 - __builtin_clz((unsigned)n);
    return 2 * e + ((n >> (e - 1)) & 1);
}
__device__ __forceinline__ int dist_base(int e) { return e < 4 ? e + 1 : ((2 + (e & 1)) << ((e >> 1) - 1)) + 1; }
__device__ __forceinline__ int dist_extra(int e) { return e < 4 ? 0 : (e >> 1) - 1; }

// Huffman code lengths (bgzf_ref.c bgzf_huffman_lengths) by the whole workgroup: the leaves'
// order by (frequency, symbol) as a parallel rank count (every thread ranks its symbols against
// all), then thread 0 builds the two-queue tree and the depths; the frequency halving retry is
// workgroup-uniform.  Same lengths as the restatement's insertion sort + build.
struct HuffScratch {
    uint32_t f[288];
    int16_t leaf[288];
    uint32_t w[576];
    int16_t parent[576];
    int32_t nl, maxd;
};
__device__ void huffman_lengths(const uint32_t *freq_in, int n, int limit, uint8_t *len, HuffScratch &s) {
    const int t = threadIdx.x;
    for (int i = t; i < n; i += blockDim.x) s.f[i] = freq_in[i];
    __syncthreads();
    for (;;) {
        for (int i = t; i < n; i += blockDim.x) {
            len[i] = 0;
            const uint32_t fi = s.f[i];
            if (!fi) continue;
            int r = 0;
            for (int j = 0; j < n; j++) {
                const uint32_t fj = s.f[j];
                r += fj != 0 && (fj < fi || (fj == fi && j < i));
            }
            s.leaf[r] = (int16_t)i;
        }
        if (t == 0) {
            int nl = 0;
            for (int i = 0; i < n; i++) nl += s.f[i] != 0;
            s.nl = nl;
        }
        __syncthreads();
        if (t == 0) {
            const int nl = s.nl;
            int maxd = 0;
            if (nl == 1) {
                len[s.leaf[0]] = 1;
            } else if (nl > 1) {
                for (int i = 0; i < nl; i++) {
                    s.w[i] = s.f[s.leaf[i]];
                    s.parent[i] = -1;
                }
                int qa = 0, qi = nl, ni = nl;
                for (int k = 0; k < nl - 1; k++) {
                    int pick[2];
                    for (int q = 0; q < 2; q++) {
                        if (qa < nl && (qi >= ni || s.w[qa] <= s.w[qi])) pick[q] = qa++;
                        else pick[q] = qi++;
                    }
                    s.w[ni] = s.w[pick[0]] + s.w[pick[1]];
                    s.parent[ni] = -1;
                    s.parent[pick[0]] = s.parent[pick[1]] = (int16_t)ni;
                    ni++;
                }
                // depths root-down: parents come after their children (the root is ni - 1); w reused
                s.w[ni - 1] = 0;
                for (int i = ni - 2; i >= 0; i--) {
                    s.w[i] = s.w[s.parent[i]] + 1;
                    if (i < nl) {
                        len[s.leaf[i]] = (uint8_t)s.w[i];
                        maxd = ::max(maxd, (int)s.w[i]);
                    }
                }
            }
            s.maxd = maxd;
        }
        __syncthreads();
        if (s.maxd <= limit) return;
        for (int i = t; i < n; i += blockDim.x)
            if (s.f[i]) s.f[i] = (s.f[i] >> 1) | 1u;
        __syncthreads();
    }
}
__device__ void canonical_codes(const uint8_t *len, int n, uint16_t *code) {
    int bl_count[16];
    for (int b = 0; b < 16; b++) bl_count[b] = 0;
    for (int i = 0; i < n; i++) bl_count[len[i]]++;
    bl_count[0] = 0;
    int next[16], c = 0;
    next[0] = 0;
    for (int b = 1; b < 16; b++) {
        c = (c + bl_count[b - 1]) << 1;
        next[b] = c;
    }
    for (int i = 0; i < n; i++) {
        code[i] = 0;
        if (!len[i]) continue;
        const uint32_t v = (uint32_t)next[len[i]]++;
        code[i] = (uint16_t)(__builtin_bitreverse32(v) >> (32 - len[i]));
    }
}

// bit writer of one thread over its own bit range of the slot's words: the first and the last
// word may be shared with a neighbour (atomicOr), the words in between are its own (stores)
struct BitOut {
    uint32_t *words;
    int64_t bit;       // next bit position
    int64_t first_w;   // the range's first word (shared)
    uint64_t acc;      // pending bits, LSB first, of word (bit >> 5) onwards
    int nacc;          // bits in acc
    int64_t accw;      // word index of acc's bit 0
    __device__ void init(uint32_t *w, int64_t b) {
        words = w;
        bit = b;
        first_w = b >> 5;
        accw = b >> 5;
        acc = 0;
        nacc = (int)(b & 31);  // bits of the first word below our range: zeros
    }
    __device__ void flush_word(bool last) {
        const uint32_t v = (uint32_t)acc;
        if (accw == first_w || last) atomicOr(words + accw, v);
        else words[accw] = v;
        acc >>= 32;
        nacc -= 32;
        accw++;
    }
    __device__ void put(uint32_t v, int n) {  // n <= 16
        if (n == 0) return;
        acc |= (uint64_t)(v & ((1u << n) - 1u)) << nacc;
        nacc += n;
        bit += n;
        if (nacc >= 32) flush_word(false);
    }
    __device__ void finish() {
        if (nacc > 0) flush_word(true);
    }
};

struct Late {  // phases C-D: in the hash table's place (dead after phase A)
    HuffScratch hs;
    uint8_t sym[320], ext[320];
    uint32_t bits[kT];
};
struct __attribute__((aligned(16))) Smem {
    uint8_t in[kBlock + 16];  // (+16: the match compare reads whole dwords; bytes past n are never counted)
    union {
        uint32_t table[1 << kHashBits];
        Late late;
    } u;
    alignas(16) uint32_t rv[kT];  // phase A: the round's 4-byte values
    uint32_t lf[286], df[30], cf[19];
    uint8_t ll[286], dl[30], cl[19];
    uint16_t lc[286], dc[30], cc[19];
    int32_t hdr_bits, ns, hlit, hdist, hclen;
};
static_assert(sizeof(Late) <= sizeof(uint32_t) << kHashBits, "phase C-D scratch fits the table");
static_assert(sizeof(Smem) <= 80 * 1024, "two workgroups per CU");
static_assert(kChain == 8, "a position's chain is one 16-byte word");

// phase timing for profiles/bgzf_phases.sh (a build with -DBSDC_BGZF_PHASES; none in the product):
// thread 0's wall clock (100 MHz) at the phase ends, per block of the last launch
#ifdef BSDC_BGZF_PHASES
__device__ uint64_t g_bgzf_phase[8192 * 8];
#define BGZF_PHASE(k) \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_bgzf_phase[blockIdx.x * 8 + (k)] = wall_clock64()
#else
#define BGZF_PHASE(k) (void)0
#endif

// the code-length sequence run-length coded (bgzf_ref.c bgzf_rle_lengths)
__device__ int rle_lengths(const uint8_t *ll, int hlit, const uint8_t *dl, int hdist, uint8_t *sym, uint8_t *ext) {
    auto L = [&](int i) { return i < hlit ? ll[i] : dl[i - hlit]; };
    const int n = hlit + hdist;
    int k = 0;
    for (int i = 0; i < n;) {
        const int v = L(i);
        int run = 1;
        while (i + run < n && L(i + run) == v) run++;
        if (v == 0) {
            int r = run;
            while (r >= 11) {
                const int t = r > 138 ? 138 : r;
                sym[k] = 18;
                ext[k++] = (uint8_t)(t - 11);
                r -= t;
            }
            if (r >= 3) {
                sym[k] = 17;
                ext[k++] = (uint8_t)(r - 3);
                r = 0;
            }
            while (r-- > 0) {
                sym[k] = 0;
                ext[k++] = 0;
            }
        } else {
            sym[k] = (uint8_t)v;
            ext[k++] = 0;
            int r = run - 1;
            while (r >= 3) {
                const int t = r > 6 ? 6 : r;
                sym[k] = 16;
                ext[k++] = (uint8_t)(t - 3);
                r -= t;
            }
            while (r-- > 0) {
                sym[k] = (uint8_t)v;
                ext[k++] = 0;
            }
        }
        i += run;
    }
    return k;
}

// blocks blk0 .. blk0 + gridDim.x - 1 of in[0, n_total); slot b of `slots` (65536 bytes) receives
// block blk0 + b's header and deflate bytes, sizes[blk0 + b] its BGZF size (0: does not fit)
__global__ __launch_bounds__(kT, 2) void k_bgzf(const uint8_t *__restrict__ in_all, int64_t n_total, int64_t blk0,
                                                 uint8_t *__restrict__ slots, int32_t *__restrict__ sizes,
                                                 uint16_t *__restrict__ dist_scr, uint32_t *__restrict__ tok_scr,
                                                 uint16_t *__restrict__ chain_scr) {
    __shared__ Smem S;
    const int t = threadIdx.x;
    BGZF_PHASE(0);
    const int64_t blk = blk0 + blockIdx.x;
    const int64_t base = blk * kBlock;
    if (base >= n_total) return;
    const int n = (int)::min<int64_t>(kBlock, n_total - base);
    uint8_t *slot = slots + (size_t)blockIdx.x * 65536;
    uint32_t *words = reinterpret_cast<uint32_t *>(slot + 16);  // the deflate data starts at byte 18 = bit 16 of word 0
    uint16_t *dist = dist_scr + (size_t)blockIdx.x * 65536;
    uint32_t *tok = tok_scr + (size_t)blockIdx.x * kBlock;
    uint16_t *chain = chain_scr + (size_t)blockIdx.x * kBlock * kChain;

    // ---- load the block (dwords, then the tail), clear the table, the frequencies, the slot ----
    const uint8_t *src = in_all + base;
    for (int i = t; i < n; i += kT) S.in[i] = src[i];  // (nothing reads past n)
    for (int i = t; i < (1 << kHashBits); i += kT) S.u.table[i] = 0;
    for (int i = t; i < 286; i += kT) S.lf[i] = 0;
    if (t < 30) S.df[t] = 0;
    for (int i = t; i < 65536 / 4; i += kT) reinterpret_cast<uint32_t *>(slot)[i] = 0;
    __syncthreads();
    BGZF_PHASE(1);

    // ---- A. candidates.  The round barriers only order the LDS table (s_waitcnt lgkmcnt(0) +
    // s_barrier): a __syncthreads() would also wait for every round's HBM stores of `dist`, which
    // only phase B reads, after the full barrier below ----
    for (int r0 = 0; r0 < n; r0 += kT) {
        const int p = r0 + t;
        const bool has4 = p + 3 < n;
        uint32_t h = 0, v = 0;
        int32_t c = -1;
        if (has4) {
            v = (uint32_t)S.in[p] | (uint32_t)S.in[p + 1] << 8 | (uint32_t)S.in[p + 2] << 16 |
                (uint32_t)S.in[p + 3] << 24;
            h = (v * 2654435761u) >> (32 - kHashBits);
            c = (int32_t)S.u.table[h] - 1;
        }
        S.rv[t] = v;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (has4) {
            // the last j < t with the same value (every earlier position of the round has 4
            // bytes): a branch-free scan of the round's values up to this wave's end, 16-byte
            // broadcast reads
            const int w0 = t & ~63;  // the earlier waves' positions: all before t
            int q = -1;
#pragma unroll 4
            for (int j = 0; j < w0; j += 4) {
                const uint4 r = *reinterpret_cast<const uint4 *>(&S.rv[j]);
                q = ::max(q, r.x == v ? j : -1);
                q = ::max(q, r.y == v ? j + 1 : -1);
                q = ::max(q, r.z == v ? j + 2 : -1);
                q = ::max(q, r.w == v ? j + 3 : -1);
            }
            uint64_t m = 0;  // this wave's positions: a match mask, then the highest below t
#pragma unroll
            for (int j = 0; j < 64; j += 4) {
                const uint4 r = *reinterpret_cast<const uint4 *>(&S.rv[w0 + j]);
                m |= (uint64_t)(r.x == v) << j | (uint64_t)(r.y == v) << (j + 1) | (uint64_t)(r.z == v) << (j + 2) |
                     (uint64_t)(r.w == v) << (j + 3);
            }
            m &= (1ull << (t & 63)) - 1;
            if (m) q = w0 + 63 - __clzll((long long)m);
            if (q >= 0) c = r0 + q;
            atomicMax(&S.u.table[h], (uint32_t)p + 1);
        }
        if (p < n) dist[p] = (uint16_t)(c >= 0 ? p - c : 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    __syncthreads();  // (the dist stores)
    BGZF_PHASE(2);

    // ---- A2. every position's chain: the distances of its first kChain chain positions within
    // kMaxDist (0 ends the list), 16 bytes a position.  Pointer chasing through `dist`, 16
    // positions at a time per thread so their loads overlap ----
    {
        constexpr int kG = 16;
        for (int p0 = t; p0 < n; p0 += kT * kG) {
            int D[kG];
            uint32_t w[kG][kChain / 2];
#pragma unroll
            for (int u = 0; u < kG; u++) {
                const int p = p0 + u * kT;
                D[u] = p < n ? dist[p] : 0;
#pragma unroll
                for (int k = 0; k < kChain / 2; k++) w[u][k] = 0;
            }
#pragma unroll
            for (int k = 0; k < kChain; k++) {
#pragma unroll
                for (int u = 0; u < kG; u++) {
                    if (D[u] > kMaxDist) D[u] = 0;
                    w[u][k >> 1] |= (uint32_t)D[u] << (16 * (k & 1));
                }
                if (k + 1 < kChain) {
#pragma unroll
                    for (int u = 0; u < kG; u++)
                        if (D[u]) {
                            const int dc = dist[p0 + u * kT - D[u]];
                            D[u] = dc ? D[u] + dc : 0;
                        }
                }
            }
#pragma unroll
            for (int u = 0; u < kG; u++) {
                const int p = p0 + u * kT;
                if (p < n)
                    *reinterpret_cast<uint4 *>(chain + (size_t)p * kChain) = make_uint4(w[u][0], w[u][1], w[u][2], w[u][3]);
            }
        }
    }
    __syncthreads();  // (the chain stores, for phase B)
    BGZF_PHASE(3);

    // ---- B. parse of this thread's segment ----
    const int s0 = t * kSeg, s1 = ::min(n, s0 + kSeg);
    int nt = 0;
    uint32_t *mytok = tok + s0;
    // the longest match at i: distances 1, 2, 4, then down the chain (a candidate that does not
    // match at the current best length cannot be longer, so it is not walked)
    auto best_match = [&](int i, int &bl, int &bd) {
        const int maxl = ::min(s1 - i, 258);
        bl = 0;
        bd = 0;
        auto tryd = [&](int d) {
            if (d > i || bl >= ::min(maxl, kNice) || S.in[i + bl] != S.in[i - d + bl]) return;
            // 4 bytes a compare (two aligned dwords per side, funnel-shifted; each dword read
            // once), clamped to maxl
            const uint32_t *w = reinterpret_cast<const uint32_t *>(S.in);
            const int a = i, b = i - d;
            const uint32_t sa = (uint32_t)(a & 3), sb = (uint32_t)(b & 3);
            int wa = a >> 2, wb = b >> 2;
            uint32_t alo = w[wa], blo = w[wb];
            int l = 0;
            for (;;) {
                const uint32_t ahi = w[wa + 1], bhi = w[wb + 1];
                const uint32_t x = __builtin_amdgcn_alignbyte(ahi, alo, sa) ^ __builtin_amdgcn_alignbyte(bhi, blo, sb);
                if (x) {
                    l += __builtin_ctz(x) >> 3;
                    break;
                }
                l += 4;
                if (l >= maxl) break;
                alo = ahi;
                blo = bhi;
                wa++;
                wb++;
            }
            l = ::min(l, maxl);
            if (l > bl) {
                bl = l;
                bd = d;
            }
        };
        const uint4 cw = *reinterpret_cast<const uint4 *>(chain + (size_t)i * kChain);
        tryd(1);
        tryd(2);
        tryd(4);
        const uint32_t cws[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
        for (int k = 0; k < kChain; k++) {
            const int d = (int)((cws[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
            if (!d) break;
            tryd(d);
        }
    };
    bool have_next = false;
    int next_l = 0, next_d = 0;
    for (int i = s0; i < s1;) {
        int bestl, bestd;
        if (have_next) {
            bestl = next_l;
            bestd = next_d;
            have_next = false;
        } else {
            best_match(i, bestl, bestd);
        }
        if (bestl >= 3 && bestl < kLazy && i + 1 < s1) {
            best_match(i + 1, next_l, next_d);
            if (next_l > bestl) {  // a literal here, the longer match next
                bestl = 0;
                have_next = true;
            }
        }
        if (bestl >= 3) {
            mytok[nt++] = 0x80000000u | (uint32_t)bestl << 16 | (uint32_t)bestd;
            atomicAdd(&S.lf[257 + len_code(bestl)], 1u);
            atomicAdd(&S.df[dist_code(bestd)], 1u);
            i += bestl;
        } else {
            mytok[nt++] = S.in[i];
            atomicAdd(&S.lf[S.in[i]], 1u);
            i++;
        }
    }
    __syncthreads();
    BGZF_PHASE(4);

    // ---- C. codes (the Huffman builds by the workgroup) and the header (thread 0) ----
    if (t == 0) S.lf[256]++;
    __syncthreads();
    huffman_lengths(S.lf, 286, 15, S.ll, S.u.late.hs);
    huffman_lengths(S.df, 30, 15, S.dl, S.u.late.hs);
    if (t == 0) {
        int used_d = 0;
        for (int i = 0; i < 30; i++) used_d |= S.dl[i] != 0;
        if (!used_d) S.dl[0] = 1;
        int hlit = 286;
        while (hlit > 257 && S.ll[hlit - 1] == 0) hlit--;
        int hdist = 30;
        while (hdist > 1 && S.dl[hdist - 1] == 0) hdist--;
        const int ns = rle_lengths(S.ll, hlit, S.dl, hdist, S.u.late.sym, S.u.late.ext);
        for (int i = 0; i < 19; i++) S.cf[i] = 0;
        for (int i = 0; i < ns; i++) S.cf[S.u.late.sym[i]]++;
        S.ns = ns;
        S.hlit = hlit;
        S.hdist = hdist;
    }
    __syncthreads();
    huffman_lengths(S.cf, 19, 7, S.cl, S.u.late.hs);
    if (t == 0) {
        const int ns = S.ns;
        int hclen = 19;
        while (hclen > 4 && S.cl[cClOrder[hclen - 1]] == 0) hclen--;
        canonical_codes(S.ll, 286, S.lc);
        canonical_codes(S.dl, 30, S.dc);
        canonical_codes(S.cl, 19, S.cc);
        int hb = 3 + 5 + 5 + 4 + 3 * hclen;
        for (int i = 0; i < ns; i++) {
            const int s = S.u.late.sym[i];
            hb += S.cl[s] + (s == 16 ? 2 : s == 17 ? 3 : s == 18 ? 7 : 0);
        }
        S.hdr_bits = hb;
        S.hclen = hclen;
    }
    __syncthreads();
    BGZF_PHASE(5);

    // ---- D. bits per thread, offsets ----
    uint32_t mb = 0;
    for (int k = 0; k < nt; k++) {
        const uint32_t x = mytok[k];
        if (!(x >> 31)) {
            mb += S.ll[x];
        } else {
            const int l = (int)((x >> 16) & 0x1FF), d = (int)(x & 0xFFFF);
            const int c = len_code(l), e = dist_code(d);
            mb += S.ll[257 + c] + len_extra(c) + S.dl[e] + dist_extra(e);
        }
    }
    if (t == kT - 1) mb += S.ll[256];  // end of block
    S.u.late.bits[t] = mb;
    __syncthreads();
    BGZF_PHASE(6);
    // exclusive scan over the 256 counts (one wave per 64, then the wave totals)
    int64_t off = S.hdr_bits;
    for (int j = 0; j < t; j++) off += S.u.late.bits[j];
    int64_t total = S.hdr_bits;
    for (int j = 0; j < kT; j++) total += S.u.late.bits[j];
    const int64_t clen = (total + 7) >> 3;
    if (clen > kOutCap) {  // does not fit: the host stores this block
        if (t == 0) sizes[blk] = 0;
        return;
    }

    // ---- E. the bits: header (thread 0, from bit 0), then every thread's tokens ----
    // the slot's words start 16 bytes in, so deflate bit b is bit 16 + b of the word stream
    BitOut o;
    if (t == 0) {
        o.init(words, 16);
        o.put(1, 1);
        o.put(2, 2);
        o.put((uint32_t)(S.hlit - 257), 5);
        o.put((uint32_t)(S.hdist - 1), 5);
        o.put((uint32_t)(S.hclen - 4), 4);
        for (int i = 0; i < S.hclen; i++) o.put(S.cl[cClOrder[i]], 3);
        for (int i = 0; i < S.ns; i++) {
            const int s = S.u.late.sym[i];
            o.put(S.cc[s], S.cl[s]);
            if (s == 16) o.put(S.u.late.ext[i], 2);
            if (s == 17) o.put(S.u.late.ext[i], 3);
            if (s == 18) o.put(S.u.late.ext[i], 7);
        }
    } else {
        o.init(words, 16 + off);
    }
    for (int k = 0; k < nt; k++) {
        const uint32_t x = mytok[k];
        if (!(x >> 31)) {
            o.put(S.lc[x], S.ll[x]);
            continue;
        }
        const int l = (int)((x >> 16) & 0x1FF), d = (int)(x & 0xFFFF);
        const int c = len_code(l), e = dist_code(d);
        o.put(S.lc[257 + c], S.ll[257 + c]);
        o.put((uint32_t)(l - len_base(c)), len_extra(c));
        o.put(S.dc[e], S.dl[e]);
        o.put((uint32_t)(d - dist_base(e)), dist_extra(e));
    }
    if (t == kT - 1) o.put(S.lc[256], S.ll[256]);
    o.finish();
    __syncthreads();
    BGZF_PHASE(7);
    if (t == 0) {  // the gzip header with the BC extra field (bytes 16-17 = BSIZE - 1)
        const int bsize = (int)(18 + clen + 8);
        const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0};
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        for (int i = 0; i < 4; i++) {
            w0 |= (uint32_t)hdr[i] << (8 * i);
            w1 |= (uint32_t)hdr[4 + i] << (8 * i);
            w2 |= (uint32_t)hdr[8 + i] << (8 * i);
            w3 |= (uint32_t)hdr[12 + i] << (8 * i);
        }
        uint32_t *sw = reinterpret_cast<uint32_t *>(slot);
        sw[0] = w0;
        sw[1] = w1;
        sw[2] = w2;
        sw[3] = w3;
        // word 4 holds BSIZE - 1 in its low 16 bits and the first deflate bits above: OR it in
        atomicOr(sw + 4, (uint32_t)(bsize - 1) & 0xFFFFu);
        sizes[blk] = bsize;
    }
}

// the blocks' bytes back to back: block b's first sizes[b] bytes to out + the sum of the sizes
// before it (this launch's and the earlier launches' blocks of the same stream: at most a few
// thousand, summed by the workgroup, so the host need not wait for the sizes between launches)
__global__ void k_bgzf_pack(const uint8_t *__restrict__ slots, const int32_t *__restrict__ sizes,
                            uint8_t *__restrict__ out, int64_t blk0) {
    __shared__ int64_t part[256 / 64];
    const int64_t b = blockIdx.x;
    const int64_t upto = blk0 + b;
    int64_t acc = 0;
    for (int64_t j = threadIdx.x; j < upto; j += blockDim.x) acc += max(sizes[j], 0);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    const int64_t off = part[0] + part[1] + part[2] + part[3];
    const int n = sizes[upto];
    const uint8_t *s = slots + (size_t)b * 65536;
    uint8_t *d = out + off;
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace

extern "C" {

// BGZF compression of a device byte stream (include/bsdc.h): blocks of 65280 bytes, max_blocks
// at a time.  bsdc_bgzf_deflate compresses blocks blk0 .. blk0 + nblk - 1 into the scratch's
// slots and writes their sizes (BGZF block size with the 8 trailer bytes counted but not written;
// 0 = the block does not fit and is stored by the host); bsdc_bgzf_pack then copies each slot's
// bytes to out + (the sum of sizes[0 .. b)), the blocks of every launch back to back.
int64_t bsdc_bgzf_scratch_bytes(int64_t max_blocks) {
    return max_blocks * (65536 + 65536 * 2 + (int64_t)kBlock * 4 + (int64_t)kBlock * 2 * kChain);
}

int32_t bsdc_bgzf_deflate(const uint8_t *d_in, int64_t n, int64_t blk0, int64_t nblk, uint8_t *d_scratch,
                          int32_t *d_sizes, void *stream) {
    if (nblk <= 0) return 0;
    if (blk0 * kBlock >= n) return -22;
    uint8_t *slots = d_scratch;
    uint16_t *dist = reinterpret_cast<uint16_t *>(d_scratch + nblk * 65536);
    uint32_t *tok = reinterpret_cast<uint32_t *>(d_scratch + nblk * (65536 + 65536 * 2));
    uint16_t *chain = reinterpret_cast<uint16_t *>(d_scratch + nblk * (65536 + 65536 * 2 + (int64_t)kBlock * 4));
    hipLaunchKernelGGL(k_bgzf, dim3((unsigned)nblk), dim3(kT), 0, (hipStream_t)stream, d_in, n, blk0, slots, d_sizes,
                       dist, tok, chain);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int32_t bsdc_bgzf_pack(const uint8_t *d_scratch, const int32_t *d_sizes, int64_t blk0, int64_t nblk, uint8_t *d_out,
                       void *stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(k_bgzf_pack, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, d_scratch, d_sizes, d_out,
                       blk0);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

#ifdef BSDC_BGZF_PHASES
int32_t bsdc_bgzf_phases(uint64_t *host, int64_t n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bgzf_phase), (size_t)n * sizeof(uint64_t)) == hipSuccess ? 0 : -5;
}
#endif

}  // extern "C"
