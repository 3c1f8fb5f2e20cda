/* Sequential restatement of the GPU BGZF block encoder (csrc/bsdc_bgzf.hip) -- TEST
 * INFRASTRUCTURE ONLY: tests/test_bgzf.py checks that zlib inflates its blocks back to the input,
 * and tests/test_gpu_bgzf.py that the kernel's blocks equal these byte for byte.
 *
 * Not a reference-tool algorithm: the reference writes BAM through htsjdk / pysam (zlib deflate).
 * This is this repository's own DEFLATE (RFC 1951) encoder, shaped for one 256-thread workgroup
 * per BGZF block (SAM/BAM spec section 4.1):
 *  1. match candidates, in rounds of kThreads consecutive positions: a position's candidate is
 *     the last earlier position of its own round with the same 4 bytes, else what the 4-byte hash
 *     table holds; then the round's positions are inserted (the largest position wins a slot), so
 *     the table gives the most recent position with the same hash before the round.  The
 *     candidates link every position to an earlier one: a hash chain;
 *  2. parse of kSeg-byte segments (one per thread): at each position the longest match (at least
 *     3, never past the segment end, first one on a tie) of the distances 1, 2, 4 and the first
 *     kChain positions down the chain within kMaxDist, the search ending at a kNice match; lazy: a match shorter than kLazy yields a
 *     literal when the next position has a longer one;
 *  3. one dynamic-Huffman block (BFINAL=1, BTYPE=2): length-limited Huffman codes (frequencies
 *     halved until the longest code fits), canonical codes, code lengths run-length coded with
 *     16/17/18;
 *  4. the BGZF wrapper: gzip header with the BC extra field, CRC32, ISIZE.
 * Every step is deterministic, so kernel and restatement produce the same bytes. */
#include <stdint.h>
#include <string.h>

#include "bgzf_ref.h"

enum { kThreads = 256, kSeg = 255, kHashBits = 11, kMaxDist = 32768, kChain = 8, kLazy = 32, kNice = 64 };

static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                       513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static uint32_t hash4(const uint8_t *p) {
    const uint32_t v = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    return (v * 2654435761u) >> (32 - kHashBits);
}
static int len_code(int l) {
    int c = 0;
    while (c < 28 && kLenBase[c + 1] <= l) c++;
    return c;
}
static int dist_code(int d) {
    int c = 0;
    while (c < 29 && kDistBase[c + 1] <= d) c++;
    return c;
}

/* Huffman code lengths of n symbols (freq 0: length 0), longest <= limit.  Two queues over the
 * leaves sorted by (frequency, symbol); on equal weight the leaf queue goes first.  Too deep:
 * every nonzero frequency becomes (f >> 1) | 1 and the code is built again.  One used symbol gets
 * length 1. */
void bgzf_huffman_lengths(const uint32_t *freq_in, int n, int limit, uint8_t *len) {
    uint32_t f[288];
    for (int i = 0; i < n; i++) f[i] = freq_in[i];
    for (;;) {
        int leaf[288], nl = 0;
        for (int i = 0; i < n; i++) {
            len[i] = 0;
            if (f[i]) leaf[nl++] = i;
        }
        if (nl == 0) return;
        if (nl == 1) {
            len[leaf[0]] = 1;
            return;
        }
        for (int i = 1; i < nl; i++) {  // insertion sort by (freq, symbol)
            const int x = leaf[i];
            int j = i - 1;
            while (j >= 0 && (f[leaf[j]] > f[x] || (f[leaf[j]] == f[x] && leaf[j] > x))) {
                leaf[j + 1] = leaf[j];
                j--;
            }
            leaf[j + 1] = x;
        }
        /* nodes 0..nl-1 leaves (in sorted order), nl.. internal */
        uint64_t w[576];
        int parent[576];
        for (int i = 0; i < nl; i++) {
            w[i] = f[leaf[i]];
            parent[i] = -1;
        }
        int qa = 0, qi = nl, ni = nl;  /* leaf queue head, internal queue head, next internal */
        for (int k = 0; k < nl - 1; k++) {
            int pick[2];
            for (int s = 0; s < 2; s++) {
                if (qa < nl && (qi >= ni || w[qa] <= w[qi])) pick[s] = qa++;
                else pick[s] = qi++;
            }
            w[ni] = w[pick[0]] + w[pick[1]];
            parent[ni] = -1;
            parent[pick[0]] = parent[pick[1]] = ni;
            ni++;
        }
        int depth[576];
        depth[ni - 1] = 0;
        int maxd = 0;
        for (int i = ni - 2; i >= 0; i--) {  /* parents come after their children */
            depth[i] = depth[parent[i]] + 1;
            if (i < nl) {
                len[leaf[i]] = (uint8_t)depth[i];
                if (depth[i] > maxd) maxd = depth[i];
            }
        }
        if (maxd <= limit) return;
        for (int i = 0; i < n; i++)
            if (f[i]) f[i] = (f[i] >> 1) | 1u;
    }
}

/* canonical codes (RFC 1951 3.2.2), bit-reversed for the LSB-first stream */
void bgzf_canonical_codes(const uint8_t *len, int n, uint16_t *code) {
    int bl_count[16] = {0};
    for (int i = 0; i < n; i++) bl_count[len[i]]++;
    bl_count[0] = 0;
    int next[16], c = 0;
    for (int b = 1; b < 16; b++) {
        c = (c + bl_count[b - 1]) << 1;
        next[b] = c;
    }
    for (int i = 0; i < n; i++) {
        code[i] = 0;
        if (!len[i]) continue;
        const int v = next[len[i]]++;
        int r = 0;
        for (int b = 0; b < len[i]; b++) r |= ((v >> b) & 1) << (len[i] - 1 - b);
        code[i] = (uint16_t)r;
    }
}

typedef struct {
    uint8_t *out;
    int64_t cap, bit;  /* bytes available; bits written */
    int over;
} Bits;
static void put(Bits *b, uint32_t v, int nbits) {
    for (int i = 0; i < nbits; i++) {
        const int64_t byte = b->bit >> 3;
        if (byte >= b->cap) {
            b->over = 1;
            return;
        }
        if ((b->bit & 7) == 0) b->out[byte] = 0;
        b->out[byte] |= (uint8_t)(((v >> i) & 1u) << (b->bit & 7));
        b->bit++;
    }
}

/* the code-length sequence run-length coded: symbols (0-18) and their extra values */
int bgzf_rle_lengths(const uint8_t *lens, int n, uint8_t *sym, uint8_t *ext) {
    int k = 0;
    for (int i = 0; i < n;) {
        const int v = lens[i];
        int run = 1;
        while (i + run < n && lens[i + run] == v) run++;
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

static uint32_t crc_table[256];
static int crc_ready;
static uint32_t crc32_bytes(const uint8_t *p, int64_t n) {
    if (!crc_ready) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            crc_table[i] = c;
        }
        crc_ready = 1;
    }
    uint32_t c = 0xFFFFFFFFu;
    for (int64_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

/* the longest match at i (0 if none of length >= 1): distances 1, 2, 4, then down the chain,
 * until one is kNice long */
static void best_match(const uint8_t *in, const int32_t *cand, int i, int s1, int *pl, int *pd) {
    const int maxl = s1 - i < 258 ? s1 - i : 258;
    int cd[3 + kChain] = {1, 2, 4};
    int nc = 3;
    for (int c = cand[i]; c >= 0 && nc < 3 + kChain && i - c <= kMaxDist; c = cand[c]) cd[nc++] = i - c;
    int bestl = 0, bestd = 0;
    for (int k = 0; k < nc; k++) {
        const int d = cd[k];
        if (d > i) continue;
        int l = 0;
        while (l < maxl && in[i + l] == in[i - d + l]) l++;
        if (l > bestl) {
            bestl = l;
            bestd = d;
        }
        if (bestl >= kNice) break;
    }
    *pl = bestl;
    *pd = bestd;
}

/* One BGZF block of in[0, n) (1 <= n <= 65280) into out (65536 bytes): its size, or 0 when the
 * dynamic block does not fit (the caller then stores the block). */
int bgzf_ref_block(const uint8_t *in, int n, uint8_t *out) {
    static uint32_t table[1 << kHashBits];
    static int32_t cand[65536];
    memset(table, 0, sizeof table);
    for (int r0 = 0; r0 < n; r0 += kThreads) {
        const int r1 = r0 + kThreads < n ? r0 + kThreads : n;
        for (int p = r0; p < r1; p++) {
            cand[p] = -1;
            if (p + 3 >= n) continue;
            cand[p] = (int32_t)table[hash4(in + p)] - 1;
            for (int q = p - 1; q >= r0; q--)
                if (memcmp(in + q, in + p, 4) == 0) {
                    cand[p] = q;
                    break;
                }
        }
        for (int p = r0; p < r1; p++)
            if (p + 3 < n) {
                const uint32_t h = hash4(in + p);
                if (table[h] < (uint32_t)p + 1) table[h] = (uint32_t)p + 1;
            }
    }
    /* tokens: literal b -> b; match -> 0x80000000 | len << 16 | dist */
    static uint32_t tok[65536];
    int nt = 0;
    uint32_t lf[286] = {0}, df[30] = {0};
    for (int s0 = 0; s0 < n; s0 += kSeg) {
        const int s1 = s0 + kSeg < n ? s0 + kSeg : n;
        for (int i = s0; i < s1;) {
            int bestl, bestd;
            best_match(in, cand, i, s1, &bestl, &bestd);
            if (bestl >= 3 && bestl < kLazy && i + 1 < s1) {
                int l2, d2;
                best_match(in, cand, i + 1, s1, &l2, &d2);
                if (l2 > bestl) bestl = 0;  /* a literal here, the longer match next */
            }
            if (bestl >= 3) {
                tok[nt++] = 0x80000000u | (uint32_t)bestl << 16 | (uint32_t)bestd;
                lf[257 + len_code(bestl)]++;
                df[dist_code(bestd)]++;
                i += bestl;
            } else {
                tok[nt++] = in[i];
                lf[in[i]]++;
                i++;
            }
        }
    }
    lf[256]++;
    uint8_t ll[286], dl[30];
    bgzf_huffman_lengths(lf, 286, 15, ll);
    bgzf_huffman_lengths(df, 30, 15, dl);
    int used_d = 0;
    for (int i = 0; i < 30; i++) used_d |= dl[i] != 0;
    if (!used_d) dl[0] = 1;  /* no match: one distance code of length 1 (RFC 1951 3.2.7) */
    int hlit = 286;
    while (hlit > 257 && ll[hlit - 1] == 0) hlit--;
    int hdist = 30;
    while (hdist > 1 && dl[hdist - 1] == 0) hdist--;
    uint8_t lens[316], sym[320], ext[320];
    memcpy(lens, ll, (size_t)hlit);
    memcpy(lens + hlit, dl, (size_t)hdist);
    const int ns = bgzf_rle_lengths(lens, hlit + hdist, sym, ext);
    uint32_t cf[19] = {0};
    for (int i = 0; i < ns; i++) cf[sym[i]]++;
    uint8_t cl[19];
    bgzf_huffman_lengths(cf, 19, 7, cl);
    int hclen = 19;
    while (hclen > 4 && cl[kClOrder[hclen - 1]] == 0) hclen--;
    uint16_t lc[286], dc[30], cc[19];
    bgzf_canonical_codes(ll, 286, lc);
    bgzf_canonical_codes(dl, 30, dc);
    bgzf_canonical_codes(cl, 19, cc);

    Bits b = {out + 18, 65536 - 26, 0, 0};
    put(&b, 1, 1);  /* BFINAL */
    put(&b, 2, 2);  /* BTYPE = dynamic */
    put(&b, (uint32_t)(hlit - 257), 5);
    put(&b, (uint32_t)(hdist - 1), 5);
    put(&b, (uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; i++) put(&b, cl[kClOrder[i]], 3);
    for (int i = 0; i < ns; i++) {
        put(&b, cc[sym[i]], cl[sym[i]]);
        if (sym[i] == 16) put(&b, ext[i], 2);
        if (sym[i] == 17) put(&b, ext[i], 3);
        if (sym[i] == 18) put(&b, ext[i], 7);
    }
    for (int k = 0; k < nt; k++) {
        const uint32_t t = tok[k];
        if (!(t >> 31)) {
            put(&b, lc[t], ll[t]);
            continue;
        }
        const int l = (int)((t >> 16) & 0x1FF), d = (int)(t & 0xFFFF);
        const int c = len_code(l), e = dist_code(d);
        put(&b, lc[257 + c], ll[257 + c]);
        put(&b, (uint32_t)(l - kLenBase[c]), kLenExtra[c]);
        put(&b, dc[e], dl[e]);
        put(&b, (uint32_t)(d - kDistBase[e]), kDistExtra[e]);
    }
    put(&b, lc[256], ll[256]);
    if (b.over) return 0;
    const int clen = (int)((b.bit + 7) >> 3);
    const int bsize = 18 + clen + 8;
    static const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0};
    memcpy(out, hdr, 16);
    out[16] = (uint8_t)((bsize - 1) & 0xFF);
    out[17] = (uint8_t)((bsize - 1) >> 8);
    const uint32_t crc = crc32_bytes(in, n);
    for (int i = 0; i < 4; i++) out[18 + clen + i] = (uint8_t)(crc >> (8 * i));
    for (int i = 0; i < 4; i++) out[22 + clen + i] = (uint8_t)((uint32_t)n >> (8 * i));
    return bsize;
}
