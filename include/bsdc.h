/* bsdc.h -- C-ABI of libbsdc, the MI355X (gfx950) step-5 duplex path.
 *
 * The reference has no plugin API: its boundary is the file contract of the four Snakemake rules
 * convert_Bstrain -> extend -> groupsort_convert -> callduplex (main.snake.py:121-164).  Each entry
 * point below replaces one piece of that contract; INTEGRATION.md shows the ctypes binding the
 * Python host (bsseqconsensusreads_amd/_lib.py) uses, which is also what a maintainer of the
 * reference would add in place of the `python3 tools/...` / `fgbio ...` shell lines.
 *
 *   bsdc_convert      replaces tools/1.convert_AG_to_CT.py:69-186 (per-record B-strand conversion)
 *   bsdc_extend       replaces tools/2.extend_gap.py:112-140       (4-record gap extension)
 *   bsdc_duplex_call  replaces main.snake.py:155-164 fgbio CallDuplexConsensusReads (and, with
 *                     BSDC_MODE_CONVERT|BSDC_MODE_EXTEND in `mode`, the two tools in front of it)
 *
 * Conventions: every function returns 0 on success and a negative errno-style code on failure
 * (message via bsdc_last_error).  Batch and output pointers are DEVICE pointers owned by the
 * caller; work is enqueued on `stream` (a hipStream_t, NULL = the null stream) and is
 * asynchronous: the bucket dispatches fan out over four context-owned side streams after an
 * event on `stream`, and `stream` waits for all of them before any later work on it runs.  The
 * reference genome is copied into library-owned device memory.  One context per GPU per host
 * thread; no global mutable state.  Output order == input family order.
 */
#ifndef BSDC_H
#define BSDC_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define BSDC_ABI_VERSION 15
#define BSDC_SMALL_BUCKETS 8
#define BSDC_LARGE_BUCKETS 6
#define BSDC_LARGE_LDS_MAX 158912 /* LDS arena bytes one large-family workgroup may use */ /* LDS arena size classes of the wavefront-per-family kernel */

#define BSDC_EINVAL (-22)
#define BSDC_ENOMEM (-12)
#define BSDC_EDEVICE (-5)

/* fgbio CallDuplexConsensusReads flags as the pipeline passes them (main.snake.py:163) */
typedef struct {
    double error_rate_pre_umi;                /* --error-rate-pre-umi=45 */
    double error_rate_post_umi;               /* --error-rate-post-umi=30 */
    int32_t min_input_base_quality;           /* --min-input-base-quality=0 */
    int32_t consensus_call_overlapping_bases; /* --consensus-call-overlapping-bases=true */
    int32_t min_reads;                        /* --min-reads=0 (only 0 is supported) */
    int32_t min_consensus_base_quality;       /* single-strand calls with Q below it -> (N, 2), 0..94:
                                                 2 for step 5 (fgbio DuplexConsensusCaller's single-strand
                                                 caller masks at PhredScore.MinValue; main.snake.py:163
                                                 passes no such flag), 0 for step 1
                                                 (--min-consensus-base-quality=0, main.snake.py:54) */
} bsdc_params;

/* Per-record `link` word (host-built) */
#define BSDC_LINK_MATE_MASK 0xFFFFu   /* template mate (R2 of this R1) index within family; 0xFFFF = none */
#define BSDC_LINK_AB (1u << 16)       /* MI ends in /A */
#define BSDC_LINK_BA (1u << 17)       /* MI ends in /B */
#define BSDC_LINK_COMPLEX (1u << 18)  /* cigar is not a single M-like run: read cig_* */
#define BSDC_LINK_RT (1u << 19)       /* read-through trim candidate: read rt[] */
#define BSDC_LINK_CONVERT (1u << 20)  /* tool 1 converts this record (flag 1/83/163) */
#define BSDC_LINK_EXT_RIGHT (1u << 21) /* tool 2: gets the partner's first base prepended */
#define BSDC_LINK_EXT_LEFT (1u << 22) /* tool 2: gets the partner's last base appended if RD=1 */
#define BSDC_LINK_PARTNER_SHIFT 23    /* 2 bits: tool-2 partner index within the family */
#define BSDC_LINK_RD_IN (1u << 25)    /* RD tag of an already-converted input (extend-only mode) */
#define BSDC_LINK_USABLE (1u << 26)   /* paired primary record with an /A or /B MI */

/* A batch of MI families in HBM, structure-of-arrays.  Record r of family f is
 * fam_off[f] <= r < fam_off[f+1].  Records live in "slots": slot r starts at nibble/byte index
 * S = rec[4r] of `seq` (nt16 codes "=ACMGRSVTWYHKDBN", two per byte, high nibble first, as in
 * BAM) and of `qual`, is round4(len+2) long, and holds the record's bases/quals at S+1 .. S+len
 * (S+0 and S+len+1 are the prepend / append room of tools 1 and 2).  A family's slots are
 * contiguous and its first slot starts at a multiple of 32.  Soft clips are already stripped by
 * the host (tools 1 and 2 both strip them before anything else). */
typedef struct {
    int64_t n_rec;
    int64_t n_fam;
    const uint32_t *fam_off;     /* [n_fam+1] */
    const uint32_t *rec;         /* [4*n_rec] slot start, pos (int32, 0-based), len | flag << 16, link */
    const uint32_t *rec_win;     /* [2*n_rec] converted records: reference window start nibble
                                    (= contig start + max(pos-1,0)), valid nibbles (<= len+2) */
    const uint32_t *cig_off;     /* [n_rec]   complex records only: first op in `cigar` */
    const uint32_t *cig_info;    /* [n_rec]   complex only: n_ops | reflen << 16 */
    const uint32_t *cigar;       /*           BAM-encoded ops (soft/hard clips removed) */
    const int32_t *rt;           /* [4*n_rec] RT records only: next_pos, tlen, mate unclipped start, end */
    const uint8_t *seq;
    const uint8_t *qual;
    const uint32_t *small_fams;  /* families processed one wavefront each, BSDC_SMALL_BUCKETS consecutive buckets;
                                    4 words per family: family, first record,
                                    n_rec | (image bytes / 32) << 8, image base (first slot) */
    int64_t n_small[BSDC_SMALL_BUCKETS];      /* families per bucket */
    int32_t small_arena[BSDC_SMALL_BUCKETS];  /* LDS bytes per wavefront of each bucket (multiple of 16) */
    const uint32_t *large_fams;  /* families processed one workgroup each, BSDC_LARGE_BUCKETS consecutive
                                    buckets; 4 words per family: family, first record, n_rec,
                                    image bytes (from the first slot) */
    int64_t n_large[BSDC_LARGE_BUCKETS];      /* families per bucket */
    int32_t large_arena[BSDC_LARGE_BUCKETS];  /* bytes per workgroup of each bucket (multiple of 16); a
                                                 bucket beyond BSDC_LARGE_LDS_MAX keeps its arenas in `scratch` */
    int32_t max_len;             /* max record length */
    int32_t split_part_arena;    /* LDS bytes per part workgroup (256 threads) */
    /* Part mode (k_large): a family beyond the LDS buckets whose records hold no complex cigar and
     * no tool-2 role is cut into parts of whole templates that each fit split_part_arena; a part
     * runs everything up to the vote in LDS and leaves its per-column likelihood sums and read
     * counts in `scratch`; one workgroup per family then adds the parts up, calls, combines and
     * writes (a near-tie column -- rare -- makes that family run whole in its HBM arena instead). */
    const uint32_t *split_parts; /* 4 words per part: family, first part record, n_rec (< 256) | its row in
                                    split_fams << 8, image bytes */
    int64_t n_split_parts;
    const uint32_t *split_part_recs; /* 4 words per part record: batch record, slot in the part's image,
                                        part-local index of its mate (0xFFFF: none) | record length << 16,
                                        slot in the batch image */
    const uint32_t *split_fams;  /* 8 words per family: family, first record, n_rec, image bytes, first part,
                                    parts, fallback arena offset in scratch / 16, fallback arena bytes */
    int64_t n_split_fams;
    int64_t split_partial_off;   /* scratch offset of the parts' sums: [part][8] int32 (set reads, set
                                    lengths), then [part][4][stride] int32x4 sums (slot k: the set's
                                    k-th multi-base column), [part][4][stride] u8x4 counts (without
                                    BSDC_MODE_TAGS: the region's first [part][4][stride] bytes hold
                                    the columns' ORs of one-hot A/C/G/T codes instead), [part][4][stride]
                                    int32 one-base sums (a multi-base column: its sums' slot k) */
} bsdc_family_batch;

/* Outputs (device pointers).  Consensus slot (f, end) holds `stride` bases. */
typedef struct {
    int32_t stride;              /* >= max_len + 2, multiple of 16 */
    int32_t reserved;
    uint8_t *status;             /* [n_fam] bit0 pair emitted, bit1 AB strand used, bit2 BA strand used */
    uint16_t *len;               /* [2*n_fam] R1, R2 lengths */
    uint8_t *seq;                /* [2*n_fam*stride/2] packed nt16 */
    uint8_t *qual;               /* [2*n_fam*stride] */
    /* optional stage dump (NULL = off): the records after tool 1 + tool 2 */
    int32_t *dump_pos;           /* [n_rec] */
    uint16_t *dump_len;          /* [n_rec] */
    uint8_t *dump_tags;          /* [n_rec] bit0 RD=1, bit1 LA present, bit2 prepended M, bit3 appended M */
    uint8_t *dump_seq;           /* [slot start + j] one nt16 code per byte */
    uint8_t *dump_qual;
    uint8_t *scratch;            /* arenas of the large buckets beyond BSDC_LARGE_LDS_MAX, one region per
                                    bucket (their dispatches may run concurrently): the sum of
                                    n_large[q] * large_arena[q] over those buckets; then the split
                                    families' fallback arenas and the parts' sums (bsdc_family_batch);
                                    + 256 bytes */
    /* optional single-strand consensus reads and their per-column statistics (BSDC_MODE_TAGS),
     * the inputs of fgbio's per-read / per-base consensus tags (aD/aM/aE, ad/ae/ac/aq, ...;
     * cD/cM/cE, cd/ce for the molecular caller).  Row (f, s), s = 0 AB-R1, 1 AB-R2, 2 BA-R1,
     * 3 BA-R2, holds `stride` columns of family f's set s (sequencing orientation). */
    uint16_t *ss_len;            /* [4*n_fam] single-strand consensus length (0 = set empty) */
    uint8_t *ss_base;            /* [4*n_fam*stride] nt16 code per byte (N when Q < 2) */
    uint8_t *ss_qual;            /* [4*n_fam*stride] */
    uint8_t *ss_depth;           /* [4*n_fam*stride] reads with an A/C/G/T at the column (ABI 14: u8,
                                    saturated at 255; exact in ss_wdepth for a family with a wide row) */
    uint8_t *ss_err;             /* [4*n_fam*stride] depth - reads showing the raw (pre-mask) best base (u8,
                                    saturated; exact in ss_werr) */
    /* (ABI 14) families of more than 255 records, whose depths may not fit a byte: ss_wide[f] = the
     * family's wide row w (-1: none; the host numbers them), and rows (w, s) of ss_wdepth / ss_werr
     * hold its exact depths / errors, u16 saturated at 32767 as fgbio's tags.  NULL with no such
     * family.  (A family routed to the small kernels has at most 64 records.) */
    const int32_t *ss_wide;      /* [n_fam] */
    uint16_t *ss_wdepth;         /* [4*n_wide*stride] */
    uint16_t *ss_werr;           /* [4*n_wide*stride] */
} bsdc_consensus;

#define BSDC_MODE_CONVERT 1
#define BSDC_MODE_EXTEND 2
#define BSDC_MODE_VOTE 4
#define BSDC_MODE_DUMP 8
#define BSDC_MODE_TAGS 64       /* also write the ss_* outputs (with BSDC_MODE_VOTE) */
#define BSDC_MODE_SKIP_SMALL 16 /* profiling: do not launch the small-family kernel */
#define BSDC_MODE_SKIP_LARGE 32 /* profiling: do not launch the large-family kernel */
#define BSDC_MODE_STOP_SHIFT 8  /* profiling: (mode >> 8) & 15 = k > 0 stops the small kernel after phase k */

typedef struct bsdc_ctx bsdc_ctx;

int32_t bsdc_abi_version(void);
int32_t bsdc_ctx_create(int32_t device, const bsdc_params *params, bsdc_ctx **out);
/* Replace a context's flags (e.g. one GPU context serving both callers: step 1's flags at
 * main.snake.py:54, step 5's at :163).  New error rates rebuild the tables after a device sync. */
int32_t bsdc_ctx_set_params(bsdc_ctx *ctx, const bsdc_params *params);
void bsdc_ctx_destroy(bsdc_ctx *ctx);
const char *bsdc_last_error(const bsdc_ctx *ctx);

/* Reference genome, host pointers: nt16 codes of the upper-cased FASTA, packed two per byte;
 * contig_off[tid] = first nibble of contig tid (-1 = contig absent from the FASTA).  Batches
 * address it through rec_win, which the host derives from the same contig table. */
int32_t bsdc_load_reference(bsdc_ctx *ctx, const uint8_t *packed_nt16, int64_t n_nibbles,
                            const int64_t *contig_off, const int64_t *contig_len, int32_t n_contig);

/* The one launcher.  mode = OR of BSDC_MODE_*. */
int32_t bsdc_run(bsdc_ctx *ctx, const bsdc_family_batch *batch, bsdc_consensus *out, int32_t mode,
                 void *stream);

/* Named entry points of the three reference stages (== bsdc_run with a fixed mode). */
int32_t bsdc_convert(bsdc_ctx *ctx, const bsdc_family_batch *batch, bsdc_consensus *out, void *stream);
int32_t bsdc_extend(bsdc_ctx *ctx, const bsdc_family_batch *batch, bsdc_consensus *out, void *stream);
int32_t bsdc_duplex_call(bsdc_ctx *ctx, const bsdc_family_batch *batch, bsdc_consensus *out,
                         int32_t with_tools, void *stream);

/* Arena bytes one family needs (host-side helpers shared with the batch builder):
 * workgroup kernel (slot_bytes = 2 x the family's image bytes) and wavefront kernel (img = slot
 * span rounded to 32, n_conv = converted records, max_len = the batch's max record length). */
int64_t bsdc_family_arena_bytes(int32_t n_rec, int64_t slot_bytes, int32_t max_len, int64_t complex_ops);
int64_t bsdc_small_arena_bytes(int32_t n_rec, int64_t img, int32_t n_conv, int64_t complex_ops, int32_t max_len);

/* The likelihood tables the vote kernel uses (host copies), for cross-checks. */
int32_t bsdc_get_tables(const bsdc_ctx *ctx, int64_t *lr256, float *thresh94);
/* Same tables for given error rates, without a context (no GPU needed). */
void bsdc_model_tables(double error_rate_pre_umi, double error_rate_post_umi, int64_t *lr256, float *thresh94);
/* The near-tie tables: fgbio's per-read log-space terms in double precision,
   ln P(correct) and ln P(error) / 3 per phred, which a near-tie column sums in fgbio's read order. */
void bsdc_model_tables_fp64(double error_rate_pre_umi, double error_rate_post_umi, double *lnc256, double *lne3_256);
/* The vote's agreement-case tables: Q(D) = qlo[D >> 16] + (D >= dthr[qlo[D >> 16] + 1]). */
void bsdc_agree_tables(double error_rate_pre_umi, double error_rate_post_umi, uint8_t *qlo2048, int32_t *dthr48);
/* The general case's phred buckets: Q(S) = the largest k >= sq[j] with S <= thresh[k], j = the
   bucket of S ((float bits >> 21) - ((127 - 32) << 2), clamped to [0, 135]). */
void bsdc_phred_buckets(double error_rate_pre_umi, double error_rate_post_umi, uint8_t *sq144);

/* BGZF compression of the output BAM on the GPU (replaces the deflate of fgbio's / htsjdk's BAM
   writer behind CallDuplexConsensusReads --output, main.snake.py:159-163; csrc/bsdc_bgzf.hip):
   device bytes in[0, n) as blocks of 65280 bytes, one dynamic-Huffman DEFLATE block each.
   bsdc_bgzf_deflate compresses blocks blk0 .. blk0 + nblk - 1 into the scratch
   (bsdc_bgzf_scratch_bytes(nblk) bytes) and writes sizes[blk0 + b]: the BGZF block size, its
   CRC32 / ISIZE trailer counted but left to the host (libbsdc_io bsdc_bam_writer_put), or
   0 when the block does not fit (the host deflates it).  bsdc_bgzf_pack then copies block b's
   bytes from the scratch to out + (sizes[0] + .. + sizes[blk0 + b - 1]), so successive launches
   over one stream's blocks pack them back to back with no host round trip.  Device pointers;
   stream = hipStream_t. */
int64_t bsdc_bgzf_scratch_bytes(int64_t max_blocks);

/* Page-lock a caller's host range for DMA (hipHostRegister) / release it: a multi-GPU worker's
 * mappings of the shared segments its batches and outputs travel in (fleet.py), so uploads and
 * fetches run by DMA from / into them.  0, or BSDC_EDEVICE with the runtime's error cleared (a
 * range that stays pageable still works, at the pageable copy rate).  No reference counterpart:
 * the reference runs step 5 as one process per rule (main.snake.py:121-164, fgbio --threads). */
int32_t bsdc_host_register(int32_t device, void *ptr, int64_t nbytes);
int32_t bsdc_host_unregister(int32_t device, void *ptr);
int32_t bsdc_bgzf_deflate(const uint8_t *in, int64_t n, int64_t blk0, int64_t nblk, uint8_t *scratch,
                          int32_t *sizes, void *stream);
int32_t bsdc_bgzf_pack(const uint8_t *scratch, const int32_t *sizes, int64_t blk0, int64_t nblk, uint8_t *out,
                       void *stream);

#ifdef __cplusplus
}
#endif
#endif
