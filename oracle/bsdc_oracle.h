/* bsdc_oracle.h -- CPU restatement of the step-5 duplex path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.  It is the
 * checker, never the product: the product path is libbsdc (HIP) and fails loudly without it.
 *
 * Stages restated (citations are /root/reference paths):
 *   tool 1  tools/1.convert_AG_to_CT.py:69-186     pinned by tests/golden/tool1_fuzz.json.gz
 *   tool 2  tools/2.extend_gap.py:112-190           pinned by tests/golden/tool12_families.json.gz
 *   vote    fgbio CallDuplexConsensusReads as invoked at main.snake.py:163
 *           (--error-rate-pre-umi=45 --error-rate-post-umi=30 --min-input-base-quality=0
 *            --min-reads=0 --consensus-call-overlapping-bases=true).  fgbio is not vendored,
 *           not installed and has no pinned version (README.md:15 "v1.5+"), so this part is
 *           PARITY UNPINNED: it restates the rules written down in DESIGN.md section 3.
 *
 * Input is one decoded record stream ("raw records", input order) plus the reference.
 * Bases are ASCII letters as a BAM decoder prints them ("=ACMGRSVTWYHKDBN").
 */
#ifndef BSDC_ORACLE_H
#define BSDC_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int64_t n;
    const uint16_t *flag;
    const int32_t *tid;
    const int32_t *pos;       /* 0-based leftmost aligned position */
    const int32_t *l_seq;
    const int64_t *seq_off;   /* into seq / qual */
    const uint8_t *seq;       /* ASCII */
    const uint8_t *qual;      /* raw phred */
    const int64_t *cig_off;
    const int32_t *n_cig;
    const uint32_t *cigar;    /* BAM encoding: len << 4 | op */
    const int32_t *mi_id;     /* MI tag with the /A,/B suffix removed, as an id; -1 = no MI tag */
    const int8_t *mi_strand;  /* 0 = ".../A", 1 = ".../B", -1 = neither */
    const int32_t *name_id;   /* QNAME as an id */
    const int32_t *next_tid;
    const int32_t *next_pos;
    const int32_t *tlen;
    const int64_t *mc_off;    /* MC tag cigar, -1 = no MC tag */
    const int32_t *mc_n;
    const uint32_t *mc_cigar;
    /* TemplateCoordinate order (family_order = 1): byte-order rank of each MI base string (per mi
     * id) and of each QNAME (per name id); library id per record (NULL = one library) */
    const int32_t *mi_lex;
    const int32_t *name_lex;
    const int32_t *lib_id;
} orc_records;

typedef struct {
    int32_t n_contig;          /* header contigs (tid space) */
    const int64_t *off;        /* into seq; -1 = contig absent from the FASTA */
    const int64_t *len;
    const uint8_t *seq;        /* FASTA letters, any case */
} orc_reference;

typedef struct {
    double error_rate_pre_umi;   /* phred, 45 */
    double error_rate_post_umi;  /* phred, 30 */
    int32_t min_input_base_quality; /* 0 */
    int32_t consensus_call_overlapping_bases; /* 1 */
    int32_t run_tools;           /* 1: raw input -> tool1 -> tool2 -> vote; 0: input is already tool-2 output */
    int32_t n_threads;           /* OpenMP threads, <= 0 = default */
    int32_t family_order;        /* 1: families = runs of one MI base in fgbio TemplateCoordinate order of the
                                    tool-2 records (SortBam at main.snake.py:152); 0: tool-2 MI groups */
    int32_t keep_sources;        /* 1: keep every family's source reads per set (orc_get_sources) */
    int32_t min_consensus_base_quality; /* single-strand calls below this phred -> (N, 2): 2 for the duplex
                                           caller's single-strand caller, 0 for main.snake.py:54 */
} orc_params;

typedef struct orc_result orc_result;

/* Runs the path. Returns NULL on an error (message in orc_last_error()). */
orc_result *orc_run(const orc_records *in, const orc_reference *ref, const orc_params *p);
const char *orc_last_error(void);
void orc_free(orc_result *r);

/* Stage dumps.  which = 1 (tool-1 output, input order) or 2 (tool-2 output, tool-2 order). */
int64_t orc_n_records(const orc_result *r, int which);
int64_t orc_total_bases(const orc_result *r, int which);
int64_t orc_total_cigar(const orc_result *r, int which);
/* Copies out record k's fields into flat arrays (offsets are running sums over k). */
void orc_get_records(const orc_result *r, int which, int64_t *src, int32_t *pos, int32_t *l_seq,
                     uint8_t *seq, uint8_t *qual, int32_t *n_cig, uint32_t *cigar, int32_t *rd,
                     int32_t *la);

/* Consensus per family, in family order (TemplateCoordinate runs, or tool-2 MI groups). */
int64_t orc_n_families(const orc_result *r);
/* Family membership: rec_off[nfam + 1], src[rec_off[nfam]] = input record index per family record. */
void orc_get_families(const orc_result *r, int64_t *rec_off, int64_t *src);
int32_t orc_max_cons_len(const orc_result *r);
/* stride = bases per (family, end) slot; bases ASCII (A,C,G,T,N); status 1 = pair emitted. */
void orc_get_consensus(const orc_result *r, int32_t stride, int32_t *mi_id, int32_t *status,
                       int32_t *len, uint8_t *bases, uint8_t *quals, int32_t *n_reads);

/* The four single-strand consensus reads per family (sets 0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2, row
 * 4*f + s, `stride` columns, len 0 = empty set) with the per-column depth and errors of fgbio's
 * consensus tags (PARITY UNPINNED). */
void orc_get_ss(const orc_result *r, int32_t stride, int32_t *len, uint8_t *bases, uint8_t *quals, int32_t *depth,
                int32_t *err);

/* The source reads the vote saw (keep_sources = 1): per family and set (row 4*f + s) the count of
 * reads, then every read in set order -- its length, its bases (ASCII, sequencing orientation, after
 * the overlapping-bases consensus, read-through and trailing-N trims) and quals.  For restating the
 * vote independently (tests/fgbio_vote.py). */
void orc_sources_size(const orc_result *r, int64_t *n_reads, int64_t *n_bases);
void orc_get_sources(const orc_result *r, int32_t *set_count, int32_t *len, uint8_t *bases, uint8_t *quals);

/* Tables of the likelihood model, for a cross-check against libbsdc's own. */
void orc_tables(double pre, double post, int64_t *lr_fixed256, float *phred_thresh94);
/* fgbio's per-read log-space terms in double precision: ln P(correct) and ln P(error) / 3 per phred */
void orc_tables_fp64(double pre, double post, double *lnc256, double *lne3_256);
float orc_det_expf(float x);
int64_t orc_check_agree(const uint8_t *qlo, const int32_t *dthr, const float *thr, int64_t dmax);

#ifdef __cplusplus
}
#endif
#endif
