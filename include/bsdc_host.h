/* bsdc_host.h -- host-side family formation of the step-5 path (csrc/bsdc_host.cpp, built into
 * libbsdc_io.so): decoded records -> the family plan -> the device batch of include/bsdc.h for any
 * contiguous range of families.
 *
 * This is the C++ statement of batch.plan_families / batch.materialize (whose numpy statement the
 * tests keep as the restatement it is checked against, tests/test_host_plan.py).  It replaces the
 * per-record bookkeeping the reference does in Python dicts and lists:
 *   tool 1 dispatch               tools/1.convert_AG_to_CT.py:70-80
 *   tool 2 grouping, 4-groups     tools/2.extend_gap.py:155-186, :112-140
 *   TemplateCoordinate families   fgbio SortBam -s TemplateCoordinate (main.snake.py:152) and the
 *                                 duplex caller's runs of one MI (parity unpinned)
 * Plain C ABI: pointers and sizes only.  Errors: a negative BSDC_E* code and
 * bsdc_host_last_error() (thread-local message). */
#ifndef BSDC_HOST_H
#define BSDC_HOST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSDC_PLAN_FULL 0 /* raw step-5 input: tool 1 + tool 2 roles, then the vote */
#define BSDC_PLAN_VOTE 1 /* tool-2 output: the vote alone */
#define BSDC_PLAN_EMISSING_MI (-61) /* a kept record has no MI tag (tools/2.extend_gap.py:179-180) */

/* Decoded records, structure of arrays (records.RawRecords).  seq holds one nt16 code per byte. */
typedef struct bsdc_host_records {
    int64_t n;
    const uint16_t *flag;
    const int32_t *tid, *pos, *l_seq;
    const int64_t *seq_off; /* into seq and qual */
    const uint8_t *seq, *qual;
    const int64_t *cig_off;
    const int32_t *n_cig;
    const uint32_t *cigar;
    const int32_t *next_tid, *next_pos, *tlen;
    const int32_t *name_id, *mi_id; /* mi_id -1: no MI tag */
    const int8_t *mi_strand;        /* 0 /A, 1 /B, -1 neither */
    const int64_t *mc_off;          /* -1: no MC tag */
    const int32_t *mc_n;
    const uint32_t *mc_cigar;
    const int64_t *mi_rank, *name_rank; /* byte-order sort keys of the MI bases / names (NULL: the ids) */
} bsdc_host_records;

typedef struct bsdc_host_reference {
    int64_t n_contig;
    const int64_t *contig_off, *contig_len; /* nibble offset (-1: not in the FASTA), length */
    const uint8_t *packed;                  /* nt16 nibbles, high first */
} bsdc_host_reference;

typedef struct bsdc_plan bsdc_plan;

/* Plan the families of all records (mode BSDC_PLAN_*; tc_order 1: TemplateCoordinate runs of one
 * MI, 0: tool 2's MI groups).  n_threads <= 0: the OpenMP default.  *out is freed with
 * bsdc_plan_free. */
int32_t bsdc_plan_families(const bsdc_host_records *R, const bsdc_host_reference *ref, int32_t mode,
                           int32_t tc_order, int32_t n_threads, bsdc_plan **out);
void bsdc_plan_sizes(const bsdc_plan *h, int64_t *n_rec, int64_t *n_fam);

/* Plan arrays (batch.FamilyPlan): per plan record [n_rec], per family [n_fam (+1)], per input
 * record [n].  NULL members are skipped. */
typedef struct bsdc_plan_arrays {
    int64_t *order;      /* [n_rec] input record of each plan record, family order */
    int64_t *fam_off;    /* [n_fam + 1] */
    int32_t *fam_mi;     /* [n_fam] */
    int64_t *t2_rank;    /* [n_rec] tool-2 output position */
    uint8_t *fam_split;  /* [n_fam] a tool-2 extension partner lies outside the family */
    uint8_t *conv, *ext_right, *ext_left, *rd_in; /* [n] */
    int64_t *partner_raw, *sL, *L, *kfirst, *kn;  /* [n] */
} bsdc_plan_arrays;
void bsdc_plan_copy(const bsdc_plan *h, const bsdc_plan_arrays *a);
void bsdc_plan_free(bsdc_plan *h);

/* A plan as arrays (bsdc_plan_copy's output, or the numpy plan). */
typedef struct bsdc_host_plan_view {
    int64_t n_fam;
    const int64_t *order, *fam_off;
    const uint8_t *conv, *ext_right, *ext_left, *rd_in;
    const int64_t *partner_raw, *sL, *L, *kfirst, *kn;
} bsdc_host_plan_view;

typedef struct bsdc_batch bsdc_batch;
typedef struct bsdc_batch_sizes {
    int64_t n_rec, n_fam, n_slots, n_bases, n_cigar_max;
    int32_t max_len;
} bsdc_batch_sizes;

/* Device-batch arrays of families [f0, f1) (batch.FamilyBatch); seq [n_slots / 2] and qual
 * [n_slots] must be zeroed by the caller. */
typedef struct bsdc_batch_arrays {
    uint8_t *seq, *qual;          /* packed nt16 image / quals, slot layout */
    uint32_t *rec;                /* [4 n_rec] slot, pos, len | flag << 16, link */
    uint32_t *rec_win;            /* [2 n_rec] */
    int32_t *rt;                  /* [4 n_rec] */
    uint32_t *cig_off, *cig_info; /* [n_rec] */
    uint32_t *cigar;              /* [n_cigar_max] */
    int64_t *src;                 /* [n_rec] input record */
    uint32_t *fam_off;            /* [n_fam + 1] */
    uint32_t *fam_entry;          /* [4 n_fam] small-kernel list entry */
    int64_t *need_l, *img;        /* [n_fam] large arena bytes, image bytes */
    int8_t *cls;                  /* [n_fam] small bucket q, or BSDC_SMALL_BUCKETS + large bucket */
    const int64_t *large_caps;    /* [BSDC_LARGE_BUCKETS - 1] LDS arena caps of the large buckets */
} bsdc_batch_arrays;

/* Sizes the batch of plan families [f0, f1) (mode_full: tool 1 + 2 run in the launch). */
int32_t bsdc_materialize_prepare(const bsdc_host_records *R, const bsdc_host_reference *ref,
                                 const bsdc_host_plan_view *pv, int64_t f0, int64_t f1, int32_t mode_full,
                                 int32_t small_cap, int32_t n_threads, bsdc_batch **out, bsdc_batch_sizes *s);
/* Fills the arrays; *n_cigar_out = the cigar words written. */
int32_t bsdc_materialize_fill(bsdc_batch *b, const bsdc_batch_arrays *o, int64_t *n_cigar_out);
void bsdc_batch_free(bsdc_batch *b);

/* k_large's part mode (include/bsdc.h split_parts): cuts families of a batch's HBM-scratch bucket
 * into parts of whole templates (an R1 and the R2 its mate link names, or an unpaired record),
 * dealt in record order, each part's ArenaLayout within part_cap and at most max_part_rec records.
 * A family is cut only if none of its records has a complex cigar (the alignment filter needs the
 * whole set) or a tool-2 role, it has < 65536 records, and it yields at least two parts.
 * rec: the batch's [4 * n_rec] record words; ents: [n_ent][4] bucket entries (family, first
 * record, n_rec, image bytes).  bsdc_split_count writes each entry's part count (0 = not cut) and
 * record count in its parts, and returns the total parts; bsdc_split_fill writes the part entries
 * (family, first part record, n_rec, staged image entries) and part records (batch record, slot
 * in the part's staged image, part-local mate index or 0xFFFF | length << 16, new batch slot),
 * entry e's from first_part[e] / first_rec[e].  The new slots lay each cut family's image out part
 * after part, each part's records back to back from its first record's slot (the family's first
 * record first: the whole-family fallback reads the image from its slot); a part stages the
 * 32-entry chunks that cover its records, from its first slot rounded down to 32 (the staged image
 * entries).  bsdc_split_move then moves the bytes of seq (packed nt16) and qual and rewrites the
 * batch records' slots (rec_off [n_rec]); split_fams: [n_sf][8] (include/bsdc.h). */
int64_t bsdc_split_count(const uint32_t *rec, const uint32_t *ents, int64_t n_ent, int64_t part_cap, int32_t max_part_rec,
                         int32_t *nparts, int64_t *nrecs, int32_t n_threads);
void bsdc_split_fill(const uint32_t *rec, const uint32_t *ents, int64_t n_ent, int64_t part_cap, int32_t max_part_rec,
                     const int64_t *first_part, const int64_t *first_rec, uint32_t *parts, uint32_t *part_recs,
                     int32_t n_threads);
void bsdc_split_move(uint8_t *seq, uint8_t *qual, uint32_t *rec_off, const uint32_t *split_fams, int64_t n_sf,
                     const uint32_t *parts, const uint32_t *part_recs, int32_t n_threads);

const char *bsdc_host_last_error(void);
/* the input record of the last BSDC_PLAN_EMISSING_MI */
int64_t bsdc_host_error_record(void);

#ifdef __cplusplus
}
#endif
#endif
