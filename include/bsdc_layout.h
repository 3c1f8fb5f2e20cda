/* bsdc_layout.h -- LDS arena layouts of the two family kernels, shared by the HIP kernels
 * (csrc/bsdc_kernels.hip) and the host batch builder (csrc/bsdc_host.cpp), so that the arena a
 * bucket reserves and the arena a kernel carves are one formula.  Not part of the C-ABI. */
#ifndef BSDC_LAYOUT_H
#define BSDC_LAYOUT_H
#include <stdint.h>

#if defined(__HIPCC__)
#define BSDC_HD __host__ __device__
#else
#define BSDC_HD
#endif

namespace bsdc_layout {

BSDC_HD inline int64_t round16(int64_t x) { return (x + 15) & ~int64_t(15); }
// 16-B chunks that cover one converted record's packed reference window
BSDC_HD inline int ref_chunks(int max_len) { return (15 + (max_len + 4) / 2 + 15) / 16; }
constexpr int kRecMetaBytes = 48;  // k_large's per-record metadata (RecMeta)
// k_large's vote scratch per output column, in the region RecMeta leaves dead: the second wave
// part's int64 sums (32), ORs (4) and A/C/G/T read counts (8, the tags)
constexpr int kVoteRegionPerCol = 44;

// Arena of one small family (k_small: one per wavefront).  Regions live only as long as their
// phase and share space:
//   bimg, qimg  the family image, bases / quals (whole kernel)
//   lists       reference-window starts (staging) -> read descriptors (vote), 4 B per record
//   misc        consensus lengths lc[4] (u32), then converted record -> lane (u8)
//   R           reference windows (staging, convert) | alignment-filter scratch (source reads) |
//               duplex rows + queued columns (vote)
struct SmallLayout {
    uint32_t bimg, qimg, lists, misc, ref, meta, setv, ordv, srcl, simp, grp, outb, outq, squeue, total;
    int32_t ws, ow;
    BSDC_HD SmallLayout(int n, int64_t img, int nconv, int64_t cops, int max_len) {
        ws = 32 * ref_chunks(max_len);
        ow = (int32_t)round16(max_len + 2);
        int64_t o = 0;
        bimg = (uint32_t)o;
        o += img;
        qimg = (uint32_t)o;
        o += img;
        lists = (uint32_t)o;
        o += round16(4 * (int64_t)n);
        misc = (uint32_t)o;  // lc[4] u32, then a byte per record
        o += 16 + round16(n);
        const int64_t R = o;
        ref = (uint32_t)R;
        const int64_t e_ref = R + (int64_t)nconv * ws;
        meta = (uint32_t)R;  // SMeta per record
        setv = meta + (uint32_t)round16(16 * (int64_t)n);
        ordv = setv + (uint32_t)round16(n);
        srcl = ordv + (uint32_t)round16(2 * (int64_t)n);
        simp = srcl + (uint32_t)round16(2 * (int64_t)n);
        grp = (uint32_t)((int64_t)simp + (cops > 0 ? round16(4 * (cops + 4 * (int64_t)n)) : 0));
        const int64_t e_f = (int64_t)grp + (cops > 0 ? 256 : 0);  // filter_group's 2 x 64 u16
        outb = (uint32_t)R;  // duplex bases, 2 ends
        outq = (uint32_t)(R + 2 * (int64_t)ow);
        squeue = (uint32_t)(R + 4 * (int64_t)ow);  // queued (end, column), u16: at most 2 ow of them
        const int64_t e_v = R + 8 * (int64_t)ow;
        int64_t e = e_ref > e_f ? e_ref : e_f;
        total = (uint32_t)(e > e_v ? e : e_v);
    }
};

// Arena layout of one large family (offsets from the arena base).  The family image comes first
// and the record metadata right after it: both offsets are known from the list entry alone, so
// the kernel stages the image and writes the metadata before it knows the family's longest read
// and cigar size (which place the regions after them).
struct ArenaLayout {
    uint32_t meta, clist, lists, ssb, ssq, simp, grp, slots, total;
    int32_t ssw;
    BSDC_HD ArenaLayout(int n, int64_t slot_bytes, int max_len, int64_t complex_ops) {
        ssw = (int32_t)round16(max_len + 2);
        int64_t o = 0;
        slots = (uint32_t)o;
        o += round16(slot_bytes);
        // RecMeta per record + the converted-record list (u16); in the vote (both dead) the second
        // wave part's sums
        meta = (uint32_t)o;
        clist = (uint32_t)(o + round16((int64_t)n * (int64_t)kRecMetaBytes));
        const int64_t mb = round16((int64_t)n * (int64_t)kRecMetaBytes) + round16(2 * (int64_t)n),
                      vb = kVoteRegionPerCol * (int64_t)ssw;
        o += mb > vb ? mb : vb;
        lists = (uint32_t)o;
        o += round16((int64_t)n * 8);
        ssb = (uint32_t)o;
        o += 4 * (int64_t)ssw;
        ssq = (uint32_t)o;
        o += 4 * (int64_t)ssw;
        simp = (uint32_t)o;
        if (complex_ops > 0) o += round16(4 * (complex_ops + 4 * (int64_t)n));
        grp = (uint32_t)o;  // filter_group's 2 x 64 u16, for X and for Y (complex families)
        if (complex_ops > 0) o += 512;
        total = (uint32_t)o;
    }
};

}  // namespace bsdc_layout
#endif
