/* bsdc_oracle.c -- sequential CPU restatement of the step-5 duplex path.
 * TEST INFRASTRUCTURE ONLY (see bsdc_oracle.h).  Written for clarity, character by character,
 * in the shape of the reference's own Python; the per-family vote loop is OpenMP-parallel only so
 * that it can double as the CPU baseline ("port") in bench.py.
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -ffp-contract=off; the flag keeps the vote's float
 * arithmetic in the exact order written, which the HIP kernel reproduces).
 */
#include "bsdc_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };

static __thread char g_err[512];
const char *orc_last_error(void) { return g_err; }
static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

/* ------------------------------------------------------------------------------------------ */
/* one record as the tools see it (a pysam AlignedSegment, reduced to the fields they touch)   */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int64_t src;      /* input record index */
    uint16_t flag;
    int32_t tid, pos;
    int32_t len;
    char *seq;        /* ASCII */
    uint8_t *qual;
    int32_t ncig;
    uint32_t *cig;
    int32_t rd, la;   /* -1 = tag absent */
} orec;

static int cig_op(uint32_t c) { return (int)(c & 0xF); }
static int32_t cig_len(uint32_t c) { return (int32_t)(c >> 4); }
static uint32_t mk_cig(int op, int32_t len) { return ((uint32_t)len << 4) | (uint32_t)op; }

static void orec_free(orec *r) {
    free(r->seq);
    free(r->qual);
    free(r->cig);
    r->seq = NULL;
    r->qual = NULL;
    r->cig = NULL;
}

static orec orec_from_input(const orc_records *in, int64_t k, int extra) {
    orec r;
    memset(&r, 0, sizeof r);
    r.src = k;
    r.flag = in->flag[k];
    r.tid = in->tid[k];
    r.pos = in->pos[k];
    r.len = in->l_seq[k];
    r.seq = (char *)malloc((size_t)r.len + extra + 1);
    r.qual = (uint8_t *)malloc((size_t)r.len + extra + 1);
    memcpy(r.seq, in->seq + in->seq_off[k], (size_t)r.len);
    memcpy(r.qual, in->qual + in->seq_off[k], (size_t)r.len);
    r.ncig = in->n_cig[k];
    r.cig = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)r.ncig + extra + 1));
    memcpy(r.cig, in->cigar + in->cig_off[k], sizeof(uint32_t) * (size_t)r.ncig);
    r.rd = -1;
    r.la = -1;
    return r;
}

static orec orec_clone(const orec *a, int extra) {
    orec r = *a;
    r.seq = (char *)malloc((size_t)a->len + extra + 1);
    r.qual = (uint8_t *)malloc((size_t)a->len + extra + 1);
    memcpy(r.seq, a->seq, (size_t)a->len);
    memcpy(r.qual, a->qual, (size_t)a->len);
    r.cig = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)a->ncig + extra + 1));
    memcpy(r.cig, a->cig, sizeof(uint32_t) * (size_t)a->ncig);
    return r;
}

/* remove_softclips: tools/1.convert_AG_to_CT.py:37-62 == tools/2.extend_gap.py:30-52 */
static void remove_softclips(orec *r) {
    if (r->ncig == 0) return;
    if (cig_op(r->cig[0]) == OP_S) {
        int32_t sc = cig_len(r->cig[0]);
        if (sc > r->len) sc = r->len;
        memmove(r->seq, r->seq + sc, (size_t)(r->len - sc));
        memmove(r->qual, r->qual + sc, (size_t)(r->len - sc));
        r->len -= sc;
        memmove(r->cig, r->cig + 1, sizeof(uint32_t) * (size_t)(r->ncig - 1));
        r->ncig -= 1;
    }
    if (r->ncig > 0 && cig_op(r->cig[r->ncig - 1]) == OP_S) {
        int32_t sc = cig_len(r->cig[r->ncig - 1]);
        /* python seq[:-sc] */
        r->len = sc >= r->len ? 0 : r->len - sc;
        r->ncig -= 1;
    }
}

static int has_op(const orec *r, int op) {
    for (int i = 0; i < r->ncig; i++)
        if (cig_op(r->cig[i]) == op) return 1;
    return 0;
}

static char upper(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }

/* ------------------------------------------------------------------------------------------ */
/* tool 1: tools/1.convert_AG_to_CT.py:69-186                                                 */
/* returns 0 = dropped, 1 = passed through (:70-72), 2 = converted (:73-186)                 */
/* ------------------------------------------------------------------------------------------ */
static int tool1_record(const orec *in, const orc_reference *ref, orec *out) {
    uint16_t f = in->flag;
    if (f == 0 || f == 99 || f == 147) { /* :70-72 */
        *out = orec_clone(in, 0);
        return 1;
    }
    if (!(f == 1 || f == 83 || f == 163)) return 0; /* every other flag is silently dropped */
    /* :79-80 reads with I, D or H are removed */
    if (has_op(in, OP_I) || has_op(in, OP_D) || has_op(in, OP_H)) return 0;
    orec r = orec_clone(in, 2);
    remove_softclips(&r); /* :81-83 */
    const int32_t L = r.len;          /* readseqlen_ori */
    const int32_t Lm = L + 1;         /* modified_length: 'N' + seq (:87-89) */
    const int32_t new_pos = in->pos - 1 > 0 ? in->pos - 1 : 0; /* :92 */
    /* :95-100 new cigar = [(M,1)] + trimmed (or [(M,1),(M,Lm-1)] when trimmed is empty) */
    uint32_t *nc = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)r.ncig + 2));
    int32_t nn = 0;
    nc[nn++] = mk_cig(OP_M, 1);
    if (r.ncig > 0) {
        for (int i = 0; i < r.ncig; i++) nc[nn++] = r.cig[i];
    } else {
        nc[nn++] = mk_cig(OP_M, Lm - 1);
    }
    /* :103-117 reference window [new_pos, new_pos + Lm + 1), upper-cased, N-padded; any fetch
     * failure (contig not in the FASTA) gives all N */
    char *rs = (char *)malloc((size_t)Lm + 2);
    int32_t need = Lm + 1;
    int have = 0;
    if (in->tid >= 0 && in->tid < ref->n_contig && ref->off[in->tid] >= 0) {
        int64_t clen = ref->len[in->tid];
        const uint8_t *cs = ref->seq + ref->off[in->tid];
        for (int32_t k = 0; k < need; k++) {
            int64_t p = (int64_t)new_pos + k;
            if (p < clen) {
                rs[k] = upper((char)cs[p]);
                have++;
            } else
                break;
        }
    }
    for (int32_t k = have; k < need; k++) rs[k] = 'N';
    /* :120-150 the per-base loop, literally */
    char *m = (char *)malloc((size_t)Lm + 1);
    m[0] = 'N';
    memcpy(m + 1, r.seq, (size_t)L);
    m[0] = rs[0]; /* :121 */
    int32_t i = 0;
    const int32_t rslen = need;
    while (i < Lm) {
        char rb = m[i];
        char fb = i < rslen ? rs[i] : 'N';
        if (rb == 'A') {
            if (fb == 'A')
                m[i] = 'A';
            else if (fb == 'G')
                m[i] = 'G';
        } else if (rb == 'C') {
            if (i < rslen - 1 && rs[i] == 'C' && rs[i + 1] == 'G') {
                if (i + 1 < Lm) {
                    if (m[i + 1] == 'A') {
                        m[i] = 'T';
                        m[i + 1] = 'G';
                        i += 1;
                    }
                }
            } else {
                m[i] = 'T';
            }
        }
        i += 1;
    }
    /* :157-170 right trim of a final C before a reference G */
    int32_t outlen = Lm;
    int32_t rd = 0;
    char extra = Lm < rslen ? rs[Lm] : 'N';
    uint8_t *tq = r.qual; /* trimmed_qual */
    int32_t tql = L;
    if (extra == 'G' && outlen > 0 && m[outlen - 1] == 'C') {
        outlen -= 1;
        rd = 1;
        int32_t ll = cig_len(nc[nn - 1]);
        if (ll > 1)
            nc[nn - 1] = mk_cig(cig_op(nc[nn - 1]), ll - 1);
        else
            nn -= 1;
        if (tql > 0) tql -= 1;
    }
    /* :173-183 */
    orec o;
    memset(&o, 0, sizeof o);
    o.src = in->src;
    o.flag = in->flag;
    o.tid = in->tid;
    o.pos = new_pos;
    o.len = outlen;
    o.seq = (char *)malloc((size_t)outlen + 3);
    memcpy(o.seq, m, (size_t)outlen);
    o.qual = (uint8_t *)malloc((size_t)outlen + 3);
    o.qual[0] = 'I' - 33; /* Q40 */
    memcpy(o.qual + 1, tq, (size_t)tql);
    o.ncig = nn;
    o.cig = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)nn + 3));
    memcpy(o.cig, nc, sizeof(uint32_t) * (size_t)nn);
    o.rd = rd;
    o.la = 1;
    *out = o;
    free(nc);
    free(rs);
    free(m);
    orec_free(&r);
    return 2;
}

/* ------------------------------------------------------------------------------------------ */
/* tool 2: tools/2.extend_gap.py                                                             */
/* ------------------------------------------------------------------------------------------ */
/* process_read_pair :58-110.  Returns via *left_out / *right_out which record plays each role. */
static void process_read_pair(orec *read1, orec *read2, orec **left_out, orec **right_out) {
    orec *left, *right;
    if (read1->flag == 83 || read1->flag == 163) {
        left = read1;
        right = read2;
    } else {
        left = read2;
        right = read1;
    }
    /* :70-80 LA==1: the partner gets the converted read's first base / qual and POS-1 */
    if (left->la == 1 && left->len > 0) {
        char fb = left->seq[0];
        uint8_t fq = left->qual[0];
        memmove(right->seq + 1, right->seq, (size_t)right->len);
        memmove(right->qual + 1, right->qual, (size_t)right->len);
        right->seq[0] = fb;
        right->qual[0] = fq;
        right->len += 1;
        right->pos -= 1;
        memmove(right->cig + 1, right->cig, sizeof(uint32_t) * (size_t)right->ncig);
        right->cig[0] = mk_cig(OP_M, 1);
        right->ncig += 1;
    }
    /* :92-101 RD==1: the converted read gets the partner's last base / qual */
    if (left->rd == 1 && right->len > 0) {
        left->seq[left->len] = right->seq[right->len - 1];
        left->qual[left->len] = right->qual[right->len - 1];
        left->len += 1;
        left->cig[left->ncig] = mk_cig(OP_M, 1);
        left->ncig += 1;
    }
    *left_out = left;
    *right_out = right;
}

typedef struct {
    orec *v;
    int64_t n, cap;
} orec_vec;
static void ovec_push(orec_vec *v, orec r) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->v = (orec *)realloc(v->v, sizeof(orec) * (size_t)v->cap);
    }
    v->v[v->n++] = r;
}

/* ------------------------------------------------------------------------------------------ */
/* the likelihood model (fgbio ConsensusCaller, restated)          */
/* ------------------------------------------------------------------------------------------ */
#define LR_SCALE 1048576.0 /* 2^20: likelihoods in exact fixed point, 2^-20 nats */
#define LR_INV_SCALE 9.5367431640625e-07

void orc_tables(double pre, double post, int64_t *lr, float *thr) {
    const double e_post = pow(10.0, -post / 10.0);
    const double e_pre = pow(10.0, -pre / 10.0);
    for (int q = 0; q < 256; q++) {
        const double e = pow(10.0, -(double)q / 10.0);
        /* probability of error over two trials: p1 + p2 - 4/3 p1 p2 */
        const double a = e_post + e - (4.0 / 3.0) * e_post * e;
        const double lnc = log1p(-a);
        const double lne = log(a / 3.0);
        lr[q] = llround((lnc - lne) * LR_SCALE);
    }
    /* Phred Q = floor(-10 log10 p' + 0.001): Q >= k  <=>  S <= thr[k], S = sum_{b!=b*} e^(L_b - L_b*) */
    thr[0] = INFINITY;
    for (int k = 1; k < 94; k++) {
        const double pk = pow(10.0, -((double)k - 0.001) / 10.0);
        const double t = (pk - e_pre) / (1.0 - (4.0 / 3.0) * e_pre);
        thr[k] = t < 0.0 ? -1.0f : (float)(t / (1.0 - t));
    }
}

/* fgbio's per-read terms in double-precision log space, as fgbio computes them (LogProbability
 * arithmetic, restated; PARITY UNPINNED): pErr = probabilityOfErrorTwoTrials(ln e_post, ln e(q)),
 * lnc[q] = not(pErr) (the read's base), lne3[q] = pErr - ln 3 (each other base).  The near-tie
 * decision of ss_consensus sums these in fgbio's read order.  Keep the operation order in step
 * with libbsdc (csrc/bsdc_kernels.hip make_fp64) and tests/fgbio_vote.py qual_tables. */
static double lp_or(double a, double b) {
    const double m = a > b ? a : b, n = a > b ? b : a;
    return m == -INFINITY ? m : m + log1p(exp(n - m));
}
static double lp_not(double x) { return x > -log(2.0) ? log(-expm1(x)) : log1p(-exp(x)); }
static double lp_a_or_not_b(double a, double b) { return b == -INFINITY ? a : a + log1p(-exp(b - a)); }
static double lp_two_trials(double x, double y) { return lp_a_or_not_b(lp_or(x, y), log(4.0 / 3.0) + x + y); }

void orc_tables_fp64(double pre, double post, double *lnc, double *lne3) {
    (void)pre;
    const double ln10 = log(10.0), ln3 = log(3.0);
    const double x = -post * ln10 / 10.0;
    for (int q = 0; q < 256; q++) {
        const double pe = lp_two_trials(x, -(double)q * ln10 / 10.0);
        lnc[q] = lp_not(pe);
        lne3[q] = pe - ln3;
    }
}

float orc_det_expf(float x) {
    /* exp for x in [-80, 0]: Cody-Waite reduction, degree-6 Taylor, explicit fma everywhere */
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

static int base_index(char b) {
    switch (b) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
    }
}

/* complement as htsjdk SequenceUtil.complement: A/C/G/T swapped, anything else unchanged */
static char complement(char b) {
    switch (b) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    default: return b;
    }
}

static int32_t ref_len_ops(const uint32_t *c, int32_t n) {
    int32_t s = 0;
    for (int i = 0; i < n; i++) {
        int op = cig_op(c[i]);
        if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) s += cig_len(c[i]);
    }
    return s;
}

/* read offset aligned to each reference position of the record: out[p - pos] (-1 = none) */
static void ref_to_read(const orec *r, int32_t *out, int32_t reflen) {
    for (int32_t k = 0; k < reflen; k++) out[k] = -1;
    int32_t rp = 0, qp = 0;
    for (int i = 0; i < r->ncig; i++) {
        int op = cig_op(r->cig[i]);
        int32_t l = cig_len(r->cig[i]);
        if (op == OP_M || op == OP_EQ || op == OP_X) {
            for (int32_t j = 0; j < l; j++) {
                if (rp + j < reflen && qp + j < r->len) out[rp + j] = qp + j;
            }
            rp += l;
            qp += l;
        } else if (op == OP_I || op == OP_S) {
            qp += l;
        } else if (op == OP_D || op == OP_N) {
            rp += l;
        }
    }
}

typedef struct {
    int32_t rec;     /* index into the family's record array */
    int32_t len;     /* source length */
    char *b;         /* sequencing-orientation bases */
    uint8_t *q;
    int32_t ncig;    /* simplified cigar, sequencing orientation, truncated */
    uint32_t *cig;
    int strand;      /* 0 AB, 1 BA */
    int r1;          /* first of pair */
} srcread;

/* overlapping-bases consensus of one template (r1, r2 both mapped, same contig) */
static void overlap_consensus(orec *a, orec *b) {
    if ((a->flag & 4) || (b->flag & 4) || a->tid != b->tid) return;
    int32_t la = ref_len_ops(a->cig, a->ncig), lb = ref_len_ops(b->cig, b->ncig);
    if (la <= 0 || lb <= 0) return;
    int32_t s = a->pos > b->pos ? a->pos : b->pos;
    int32_t ea = a->pos + la - 1, eb = b->pos + lb - 1;
    int32_t e = ea < eb ? ea : eb;
    if (s > e) return;
    int32_t *ma = (int32_t *)malloc(sizeof(int32_t) * (size_t)la);
    int32_t *mb = (int32_t *)malloc(sizeof(int32_t) * (size_t)lb);
    ref_to_read(a, ma, la);
    ref_to_read(b, mb, lb);
    for (int32_t p = s; p <= e; p++) {
        int32_t ia = ma[p - a->pos], ib = mb[p - b->pos];
        if (ia < 0 || ib < 0) continue;
        char ba = a->seq[ia], bb = b->seq[ib];
        if (ba == 'N' || bb == 'N') continue;
        int qa = a->qual[ia], qb = b->qual[ib];
        if (ba == bb) {
            int q = qa + qb;
            if (q > 93) q = 93;
            a->qual[ia] = (uint8_t)q;
            b->qual[ib] = (uint8_t)q;
        } else if (qa > qb) {
            b->seq[ib] = ba;
            a->qual[ia] = b->qual[ib] = (uint8_t)(qa - qb);
        } else if (qb > qa) {
            a->seq[ia] = bb;
            a->qual[ia] = b->qual[ib] = (uint8_t)(qb - qa);
        } else {
            a->seq[ia] = b->seq[ib] = 'N';
            a->qual[ia] = b->qual[ib] = 2;
        }
    }
    free(ma);
    free(mb);
}

/* htsjdk SamPairUtil.getPairOrientation(...) == FR, with fgbio's isFrPair preconditions */
static int is_fr_pair(const orec *r, const orc_records *in) {
    int64_t k = r->src;
    if (!(r->flag & 1) || (r->flag & 4) || (r->flag & 8)) return 0;
    if (in->next_tid[k] != r->tid) return 0;
    int neg = (r->flag & 16) != 0, mneg = (r->flag & 32) != 0;
    if (neg == mneg) return 0;
    int64_t posfive, negfive;
    if (neg) {
        posfive = in->next_pos[k];
        negfive = (int64_t)r->pos + ref_len_ops(r->cig, r->ncig) - 1;
    } else {
        posfive = r->pos;
        negfive = (int64_t)r->pos + in->tlen[k];
    }
    return posfive < negfive;
}

/* fgbio toSourceRead, restated: orientation, read-through trim against the (stale) mate fields,
 * trailing-N trim.  Returns 0 when nothing is left. */
static int to_source_read(const orec *r, const orc_records *in, srcread *s) {
    const int neg = (r->flag & 16) != 0;
    int32_t L = r->len;
    s->b = (char *)malloc((size_t)L + 1);
    s->q = (uint8_t *)malloc((size_t)L + 1);
    for (int32_t i = 0; i < L; i++) {
        if (neg) {
            s->b[i] = complement(r->seq[L - 1 - i]);
            s->q[i] = r->qual[L - 1 - i];
        } else {
            s->b[i] = r->seq[i];
            s->q[i] = r->qual[i];
        }
    }
    int32_t keep = L;
    int64_t k = r->src;
    if (in->mc_off[k] >= 0 && is_fr_pair(r, in)) {
        const uint32_t *mc = in->mc_cigar + in->mc_off[k];
        int32_t mn = in->mc_n[k];
        int32_t reflen = ref_len_ops(r->cig, r->ncig);
        int32_t *m = (int32_t *)malloc(sizeof(int32_t) * (size_t)(reflen > 0 ? reflen : 1));
        ref_to_read(r, m, reflen);
        if (!neg) {
            int32_t trail = 0;
            for (int i = mn - 1; i >= 0 && (cig_op(mc[i]) == OP_S || cig_op(mc[i]) == OP_H); i--) trail += cig_len(mc[i]);
            int64_t mate_end = (int64_t)in->next_pos[k] + ref_len_ops(mc, mn) - 1 + trail;
            int64_t end = (int64_t)r->pos + reflen - 1;
            if (end > mate_end) {
                int32_t last = -1;
                for (int32_t p = 0; p < reflen && (int64_t)r->pos + p <= mate_end; p++)
                    if (m[p] >= 0) last = m[p];
                int32_t kk = last + 1;
                if (kk < keep) keep = kk;
            }
        } else {
            int32_t lead = 0;
            for (int i = 0; i < mn && (cig_op(mc[i]) == OP_S || cig_op(mc[i]) == OP_H); i++) lead += cig_len(mc[i]);
            int64_t mate_start = (int64_t)in->next_pos[k] - lead;
            if ((int64_t)r->pos < mate_start) {
                int32_t first = L;
                for (int32_t p = reflen - 1; p >= 0 && (int64_t)r->pos + p >= mate_start; p--)
                    if (m[p] >= 0) first = m[p];
                int32_t kk = L - first;
                if (kk < keep) keep = kk;
            }
        }
        free(m);
    }
    while (keep > 0 && s->b[keep - 1] == 'N') keep--;
    s->len = keep;
    /* simplified cigar: sequencing orientation, M/=/X/S -> M, merged, truncated to `keep` query bases */
    s->cig = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)r->ncig + 1));
    s->ncig = 0;
    int32_t q = 0;
    for (int j = 0; j < r->ncig && q < keep; j++) {
        uint32_t c = neg ? r->cig[r->ncig - 1 - j] : r->cig[j];
        int op = cig_op(c);
        int32_t l = cig_len(c);
        if (op == OP_EQ || op == OP_X || op == OP_S) op = OP_M; /* soft-clipped bases stay in the source read */
        if (op == OP_H) continue;
        if (op == OP_M || op == OP_I) {
            if (q + l > keep) l = keep - q;
            q += l;
        }
        if (s->ncig > 0 && cig_op(s->cig[s->ncig - 1]) == op)
            s->cig[s->ncig - 1] = mk_cig(op, cig_len(s->cig[s->ncig - 1]) + l);
        else
            s->cig[s->ncig++] = mk_cig(op, l);
    }
    return keep > 0;
}

static int cigar_is_prefix(const srcread *a, const uint32_t *bc, int32_t bn) {
    if (a->ncig > bn) return 0;
    for (int i = 0; i < a->ncig - 1; i++)
        if (a->cig[i] != bc[i]) return 0;
    int i = a->ncig - 1;
    if (i < 0) return 1;
    return cig_op(a->cig[i]) == cig_op(bc[i]) && cig_len(a->cig[i]) <= cig_len(bc[i]);
}

/* fgbio filterToMostCommonAlignment, restated: sets keep[i] and order[] -- fgbio returns its
 * keepers in its sorted order (source length descending, ties in input order), which is the order
 * the consensus caller then adds the reads in */
static void filter_most_common(srcread **v, int n, int *keep, int *order) {
    for (int i = 0; i < n; i++) {
        keep[i] = 1;
        order[i] = i;
    }
    if (n < 2) return;
    /* stable sort by length, descending (insertion sort keeps ties in input order) */
    for (int i = 1; i < n; i++) {
        int x = order[i], j = i - 1;
        while (j >= 0 && v[order[j]]->len < v[x]->len) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = x;
    }
    int *gid_of_cig = (int *)malloc(sizeof(int) * (size_t)n); /* group -> defining read */
    int *gsize = (int *)calloc((size_t)n, sizeof(int));
    unsigned char *member = (unsigned char *)calloc((size_t)n * (size_t)n, 1); /* [g][read] */
    int ng = 0;
    for (int oi = 0; oi < n; oi++) {
        int i = order[oi];
        int found = 0;
        for (int g = 0; g < ng; g++) {
            const srcread *d = v[gid_of_cig[g]];
            if (cigar_is_prefix(v[i], d->cig, d->ncig)) {
                member[(size_t)g * n + i] = 1;
                gsize[g]++;
                found = 1;
            }
        }
        if (!found) {
            gid_of_cig[ng] = i;
            member[(size_t)ng * n + i] = 1;
            gsize[ng] = 1;
            ng++;
        }
    }
    if (ng > 1) {
        int best = 0;
        for (int g = 1; g < ng; g++)
            if (gsize[g] > gsize[best]) best = g;
        for (int i = 0; i < n; i++) keep[i] = member[(size_t)best * n + i];
    }
    free(gid_of_cig);
    free(gsize);
    free(member);
}

typedef struct {
    int32_t len;
    char *b;
    uint8_t *q;
    int32_t *depth; /* reads with an A/C/G/T at the column */
    int32_t *err;   /* depth - reads showing the raw (pre-mask) best base */
} ssread;

/* single-strand consensus (fgbio VanillaUmiConsensusCaller, min-reads 1), restated; with the
 * per-column depth and errors fgbio keeps for its consensus tags:
 *   errors = if (rawBase == NoCall) depth else depth - builder.observations(rawBase)
 * where rawBase is the likelihood call before the minimum-quality mask (PARITY UNPINNED). */
typedef struct {
    double lnc[256], lne3[256];
} fp64tab;

static int ss_consensus(srcread **v, int n, const int64_t *lr, const fp64tab *f64, const float *thr, int min_cbq,
                        ssread *out) {
    int32_t lc = 0;
    for (int i = 0; i < n; i++)
        if (v[i]->len > lc) lc = v[i]->len;
    if (n == 0 || lc == 0) return 0;
    out->len = lc;
    out->b = (char *)malloc((size_t)lc);
    out->q = (uint8_t *)malloc((size_t)lc);
    out->depth = (int32_t *)malloc(sizeof(int32_t) * (size_t)lc);
    out->err = (int32_t *)malloc(sizeof(int32_t) * (size_t)lc);
    for (int32_t c = 0; c < lc; c++) {
        int64_t D[4] = {0, 0, 0, 0};
        int32_t obs[4] = {0, 0, 0, 0};
        for (int i = 0; i < n; i++) {
            if (v[i]->len <= c) continue;
            int bi = base_index(v[i]->b[c]);
            if (bi < 0) continue;
            D[bi] += lr[v[i]->q[c]];
            obs[bi]++;
        }
        int best = 0;
        for (int b = 1; b < 4; b++)
            if (D[b] > D[best]) best = b;
        /* near tie: the 2^-20 sums carry up to half a unit of rounding per read, so a gap of at most
         * one unit per read of the set can hide fgbio's order.  There fgbio's own pick is taken:
         * ConsensusBaseBuilder.add's four double-precision sums, read by read in the set's order
         * (v[] is in fgbio's order, see family_call), first maximum by strict >.  That also
         * reproduces its rounding on exact ties (equal quality multisets on two bases). */
        int64_t second = INT64_MIN;
        for (int b = 0; b < 4; b++)
            if (b != best && D[b] > second) second = D[b];
        if (D[best] - second <= n) {
            double L[4] = {0.0, 0.0, 0.0, 0.0};
            for (int i = 0; i < n; i++) {
                if (v[i]->len <= c) continue;
                int bi = base_index(v[i]->b[c]);
                if (bi < 0) continue;
                const int q = v[i]->q[c];
                for (int b = 0; b < 4; b++) L[b] += b == bi ? f64->lnc[q] : f64->lne3[q];
            }
            best = 0;
            for (int b = 1; b < 4; b++)
                if (L[b] > L[best]) best = b;
        }
        float S = 0.0f;
        for (int b = 0; b < 4; b++) {
            if (b == best) continue;
            const float x = (float)((double)(D[b] - D[best]) * LR_INV_SCALE);
            if (x < -80.0f) continue;
            S += orc_det_expf(x);
        }
        int Q = 0;
        for (int k = 1; k < 94; k++) {
            if (S <= thr[k])
                Q = k;
            else
                break;
        }
        const int32_t depth = obs[0] + obs[1] + obs[2] + obs[3];
        /* no A/C/G/T read (fgbio: fewer contributions than min-reads 1) or below
         * --min-consensus-base-quality: (NoCall, NoCallQual = 2) */
        if (depth == 0 || Q < min_cbq) {
            out->b[c] = 'N';
            out->q[c] = 2;
        } else {
            out->b[c] = "ACGT"[best];
            out->q[c] = (uint8_t)Q;
        }
        out->depth[c] = depth > 32767 ? 32767 : depth;
        out->err[c] = depth - obs[best] > 32767 ? 32767 : depth - obs[best];
    }
    return 1;
}

/* duplex combine (fgbio DuplexConsensusCaller.duplexConsensus), restated */
static int duplex(const ssread *a, int has_a, const ssread *b, int has_b, char *ob, uint8_t *oq, int32_t *olen) {
    if (!has_a && !has_b) return 0;
    if (has_a != has_b) {
        const ssread *x = has_a ? a : b;
        memcpy(ob, x->b, (size_t)x->len);
        memcpy(oq, x->q, (size_t)x->len);
        *olen = x->len;
        return 1;
    }
    int32_t len = a->len < b->len ? a->len : b->len;
    for (int32_t i = 0; i < len; i++) {
        char ab = a->b[i], bb = b->b[i];
        int aq = a->q[i], bq = b->q[i];
        char rb;
        int rq;
        if (ab == bb) {
            rb = ab;
            rq = aq + bq;
        } else if (aq > bq) {
            rb = ab;
            rq = aq - bq;
        } else if (bq > aq) {
            rb = bb;
            rq = bq - aq;
        } else {
            rb = ab;
            rq = 2;
        }
        if (rq > 93) rq = 93;
        if (ab == 'N' || bb == 'N' || rq == 2) {
            rb = 'N';
            rq = 2;
        }
        ob[i] = rb;
        oq[i] = (uint8_t)rq;
    }
    *olen = len;
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
struct orc_result {
    orec_vec t1, t2;
    int64_t nfam;
    int32_t maxlen;
    int32_t *fam_mi;
    int32_t *fam_status;
    int32_t *fam_len;   /* [2*f + end] */
    int32_t *fam_nreads;
    char **fam_b;       /* [2*f + end] */
    uint8_t **fam_q;
    ssread *fam_ss;       /* [4*f + set] single-strand reads (len 0 = set empty) */
    int64_t *fam_rec_off; /* [nfam + 1] into fam_src */
    int64_t *fam_src;     /* input record index of each family record, family order */
    /* keep_sources: per family the vote's source reads, set by set */
    int32_t *src_count;   /* [4*f + set] */
    int32_t **src_len;    /* [f] -> lengths of the family's source reads */
    char **src_b;         /* [f] -> their bases, concatenated */
    uint8_t **src_q;
};

static void family_call(orec *recs, int n, const orc_records *in, const orc_params *p, const int64_t *lr,
                        const fp64tab *f64, const float *thr, struct orc_result *res, int64_t f) {
    res->fam_status[f] = 0;
    res->fam_len[2 * f] = res->fam_len[2 * f + 1] = 0;
    res->fam_b[2 * f] = res->fam_b[2 * f + 1] = NULL;
    res->fam_q[2 * f] = res->fam_q[2 * f + 1] = NULL;
    /* work on copies: the overlap consensus edits bases in place */
    orec *w = (orec *)malloc(sizeof(orec) * (size_t)(n > 0 ? n : 1));
    int *usable = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        w[i] = orec_clone(&recs[i], 0);
        /* paired primary records only; MI must carry /A or /B */
        usable[i] = (w[i].flag & 1) && !(w[i].flag & 0x900) && in->mi_strand[w[i].src] >= 0;
    }
    if (p->consensus_call_overlapping_bases) {
        for (int i = 0; i < n; i++) {
            if (!usable[i] || !(w[i].flag & 0x40)) continue;
            int first_r1 = 1;
            for (int j = 0; j < i; j++)
                if (usable[j] && (w[j].flag & 0x40) && in->name_id[w[j].src] == in->name_id[w[i].src]) first_r1 = 0;
            if (!first_r1) continue;
            for (int j = 0; j < n; j++) {
                if (usable[j] && (w[j].flag & 0x80) && in->name_id[w[j].src] == in->name_id[w[i].src]) {
                    overlap_consensus(&w[i], &w[j]);
                    break;
                }
            }
        }
    }
    srcread *src = (srcread *)calloc((size_t)(n > 0 ? n : 1), sizeof(srcread));
    int *ok = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    for (int i = 0; i < n; i++) {
        if (!usable[i]) continue;
        src[i].rec = i;
        src[i].strand = in->mi_strand[w[i].src];
        src[i].r1 = (w[i].flag & 0x40) != 0;
        ok[i] = to_source_read(&w[i], in, &src[i]);
    }
    /* X = AB-R1 ++ BA-R2, Y = AB-R2 ++ BA-R1 */
    srcread **X = (srcread **)malloc(sizeof(srcread *) * (size_t)(n + 1));
    srcread **Y = (srcread **)malloc(sizeof(srcread *) * (size_t)(n + 1));
    int nx = 0, ny = 0;
    for (int pass = 0; pass < 2; pass++) {
        for (int i = 0; i < n; i++) {
            if (!usable[i] || !ok[i]) continue;
            int ab = src[i].strand == 0;
            if (pass == 0 && ab && src[i].r1) X[nx++] = &src[i];
            if (pass == 1 && !ab && !src[i].r1) X[nx++] = &src[i];
            if (pass == 0 && ab && !src[i].r1) Y[ny++] = &src[i];
            if (pass == 1 && !ab && src[i].r1) Y[ny++] = &src[i];
        }
    }
    int *kx = (int *)malloc(sizeof(int) * (size_t)(nx + 1));
    int *ky = (int *)malloc(sizeof(int) * (size_t)(ny + 1));
    int *ox = (int *)malloc(sizeof(int) * (size_t)(nx + 1));
    int *oy = (int *)malloc(sizeof(int) * (size_t)(ny + 1));
    filter_most_common(X, nx, kx, ox);
    filter_most_common(Y, ny, ky, oy);
    srcread **sets[4];
    int ns[4] = {0, 0, 0, 0};
    for (int s = 0; s < 4; s++) sets[s] = (srcread **)malloc(sizeof(srcread *) * (size_t)(n + 1));
    /* sets: 0 AB-R1, 1 AB-R2, 2 BA-R1, 3 BA-R2, each in the filter's output order (fgbio splits
     * its keepers by strand, keeping their order) */
    for (int k = 0; k < nx; k++) {
        const int i = ox[k];
        if (kx[i]) {
            int s = X[i]->strand == 0 ? 0 : 3;
            sets[s][ns[s]++] = X[i];
        }
    }
    for (int k = 0; k < ny; k++) {
        const int i = oy[k];
        if (ky[i]) {
            int s = Y[i]->strand == 0 ? 1 : 2;
            sets[s][ns[s]++] = Y[i];
        }
    }
    free(ox);
    free(oy);
    if (p->keep_sources) {
        int64_t nr = 0, nb = 0;
        for (int s = 0; s < 4; s++) {
            res->src_count[4 * f + s] = ns[s];
            nr += ns[s];
            for (int i = 0; i < ns[s]; i++) nb += sets[s][i]->len;
        }
        res->src_len[f] = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nr + 1));
        res->src_b[f] = (char *)malloc((size_t)nb + 1);
        res->src_q[f] = (uint8_t *)malloc((size_t)nb + 1);
        int64_t ri = 0, bi = 0;
        for (int s = 0; s < 4; s++)
            for (int i = 0; i < ns[s]; i++) {
                const srcread *x = sets[s][i];
                res->src_len[f][ri++] = x->len;
                memcpy(res->src_b[f] + bi, x->b, (size_t)x->len);
                memcpy(res->src_q[f] + bi, x->q, (size_t)x->len);
                bi += x->len;
            }
    }
    ssread ss[4];
    int has[4];
    for (int s = 0; s < 4; s++) has[s] = ss_consensus(sets[s], ns[s], lr, f64, thr, p->min_consensus_base_quality, &ss[s]);
    int32_t nreads = 0;
    for (int s = 0; s < 4; s++) nreads += ns[s];
    res->fam_nreads[f] = nreads;
    char *b1 = (char *)malloc((size_t)res->maxlen + 8), *b2 = (char *)malloc((size_t)res->maxlen + 8);
    uint8_t *q1 = (uint8_t *)malloc((size_t)res->maxlen + 8), *q2 = (uint8_t *)malloc((size_t)res->maxlen + 8);
    int32_t l1 = 0, l2 = 0;
    int d1 = duplex(&ss[0], has[0], &ss[3], has[3], b1, q1, &l1);
    int d2 = duplex(&ss[1], has[1], &ss[2], has[2], b2, q2, &l2);
    if (d1 && d2) {
        res->fam_status[f] = 1;
        res->fam_len[2 * f] = l1;
        res->fam_len[2 * f + 1] = l2;
        res->fam_b[2 * f] = b1;
        res->fam_q[2 * f] = q1;
        res->fam_b[2 * f + 1] = b2;
        res->fam_q[2 * f + 1] = q2;
    } else {
        free(b1);
        free(b2);
        free(q1);
        free(q2);
    }
    for (int s = 0; s < 4; s++) {
        if (has[s])
            res->fam_ss[4 * f + s] = ss[s];  /* owned by the result */
        else
            memset(&res->fam_ss[4 * f + s], 0, sizeof(ssread));
        free(sets[s]);
    }
    for (int i = 0; i < n; i++) {
        free(src[i].b);
        free(src[i].q);
        free(src[i].cig);
        orec_free(&w[i]);
    }
    free(w);
    free(usable);
    free(src);
    free(ok);
    free(X);
    free(Y);
    free(kx);
    free(ky);
}

/* ------------------------------------------------------------------------------------------ */
/* family formation: fgbio SortBam -s TemplateCoordinate (main.snake.py:152) + the duplex       */
/* caller's grouping of consecutive records with one MI base (fgbio is not  */
/* vendored: PARITY UNPINNED).  Key: (tid, mate tid, unclipped 5' pos, mate unclipped 5' pos,    */
/* strands, library, MI base, name, upper-of-pair), the lower end of the template first; the     */
/* mate fields are the stale ones the tools leave (PNEXT, MC).                                    */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int32_t tid1, tid2, pos1, pos2;
    int32_t neg1, neg2, lib, mi, name, upper;
    int64_t ord; /* tool-2 output position: ties keep it (a stable sort) */
} tc_key;

static void unclipped_ends(const uint32_t *c, int32_t n, int32_t pos, int32_t *us, int32_t *ue) {
    int32_t lead = 0, trail = 0, i = 0, j = n - 1;
    for (; i < n && (cig_op(c[i]) == OP_S || cig_op(c[i]) == OP_H); i++) lead += cig_len(c[i]);
    for (; j >= i && (cig_op(c[j]) == OP_S || cig_op(c[j]) == OP_H); j--) trail += cig_len(c[j]);
    *us = pos - lead;
    *ue = pos + ref_len_ops(c, n) - 1 + trail;
}

static tc_key tc_key_of(const orec *r, const orc_records *in, int64_t ord) {
    tc_key k;
    int32_t us, ue, mus, mue;
    unclipped_ends(r->cig, r->ncig, r->pos, &us, &ue);
    const int32_t neg = (r->flag & 16) != 0;
    const int32_t t1 = r->tid, p1 = neg ? ue : us;
    int32_t t2 = INT32_MAX, p2 = INT32_MAX, n2 = 0;
    if ((r->flag & 1) && !(r->flag & 8)) {
        const int64_t s = r->src;
        t2 = in->next_tid[s];
        n2 = (r->flag & 32) != 0;
        if (in->mc_off[s] >= 0) {
            unclipped_ends(in->mc_cigar + in->mc_off[s], in->mc_n[s], in->next_pos[s], &mus, &mue);
        } else {
            mus = mue = in->next_pos[s];
        }
        p2 = n2 ? mue : mus;
    }
    const int lower = t1 < t2 || (t1 == t2 && (p1 < p2 || (p1 == p2 && neg <= n2)));
    k.tid1 = lower ? t1 : t2;
    k.pos1 = lower ? p1 : p2;
    k.neg1 = lower ? neg : n2;
    k.tid2 = lower ? t2 : t1;
    k.pos2 = lower ? p2 : p1;
    k.neg2 = lower ? n2 : neg;
    k.upper = !lower;
    k.lib = in->lib_id ? in->lib_id[r->src] : 0;
    k.mi = in->mi_lex[in->mi_id[r->src]];
    k.name = in->name_lex[in->name_id[r->src]];
    k.ord = ord;
    return k;
}

static int tc_cmp(const void *pa, const void *pb) {
    const tc_key *a = (const tc_key *)pa, *b = (const tc_key *)pb;
#define TC_CMP(f) if (a->f != b->f) return a->f < b->f ? -1 : 1
    TC_CMP(tid1);
    TC_CMP(tid2);
    TC_CMP(pos1);
    TC_CMP(pos2);
    TC_CMP(neg1);
    TC_CMP(neg2);
    TC_CMP(lib);
    TC_CMP(mi);
    TC_CMP(name);
    TC_CMP(upper);
    TC_CMP(ord);
#undef TC_CMP
    return 0;
}

orc_result *orc_run(const orc_records *in, const orc_reference *ref, const orc_params *p) {
    g_err[0] = 0;
#ifdef _OPENMP
    if (p->n_threads > 0) omp_set_num_threads(p->n_threads);
#endif
    orc_result *res = (orc_result *)calloc(1, sizeof(orc_result));
    const int64_t n = in->n;
    /* ---- tool 1 (per record) ---- */
    orec *t1 = (orec *)calloc((size_t)(n > 0 ? n : 1), sizeof(orec));
    int *t1k = (int *)calloc((size_t)(n > 0 ? n : 1), sizeof(int));
    if (p->run_tools) {
#pragma omp parallel for schedule(dynamic, 256)
        for (int64_t k = 0; k < n; k++) {
            orec r = orec_from_input(in, k, 0);
            t1k[k] = tool1_record(&r, ref, &t1[k]);
            orec_free(&r);
        }
    } else {
        for (int64_t k = 0; k < n; k++) {
            t1[k] = orec_from_input(in, k, 0);
            t1k[k] = 1;
        }
    }
    for (int64_t k = 0; k < n; k++)
        if (t1k[k]) ovec_push(&res->t1, t1[k]);
    free(t1);
    free(t1k);
    /* ---- tool 2: group by MI (first-seen order), :158-186 ---- */
    int32_t max_mi = -1;
    for (int64_t k = 0; k < in->n; k++)
        if (in->mi_id[k] > max_mi) max_mi = in->mi_id[k];
    int64_t *gfirst = (int64_t *)malloc(sizeof(int64_t) * (size_t)(max_mi + 2));
    for (int32_t i = 0; i <= max_mi; i++) gfirst[i] = -1;
    int64_t ng = 0;
    int32_t *gorder_mi = (int32_t *)malloc(sizeof(int32_t) * (size_t)(res->t1.n + 1));
    int64_t *gcount = (int64_t *)calloc((size_t)(res->t1.n + 1), sizeof(int64_t));
    int64_t *rec_group = (int64_t *)malloc(sizeof(int64_t) * (size_t)(res->t1.n + 1));
    for (int64_t k = 0; k < res->t1.n; k++) {
        orec *r = &res->t1.v[k];
        rec_group[k] = -1;
        if (p->run_tools && has_op(r, OP_H)) continue; /* :160-161 */
        int32_t mi = in->mi_id[r->src];
        if (mi < 0) { /* :179-180 */
            set_err("record %lld does not have MI tag.", (long long)r->src);
            free(gfirst);
            free(gorder_mi);
            free(gcount);
            free(rec_group);
            orc_free(res);
            return NULL;
        }
        if (gfirst[mi] < 0) {
            gfirst[mi] = ng;
            gorder_mi[ng] = mi;
            ng++;
        }
        rec_group[k] = gfirst[mi];
        gcount[gfirst[mi]]++;
    }
    /* bucket records by group, keeping order */
    int64_t *goff = (int64_t *)calloc((size_t)(ng + 1), sizeof(int64_t));
    for (int64_t g = 0; g < ng; g++) goff[g + 1] = goff[g] + gcount[g];
    int64_t *gfill = (int64_t *)calloc((size_t)(ng + 1), sizeof(int64_t));
    orec *grouped = (orec *)malloc(sizeof(orec) * (size_t)(goff[ng] + 1));
    for (int64_t k = 0; k < res->t1.n; k++) {
        int64_t g = rec_group[k];
        if (g < 0) continue;
        orec c = orec_clone(&res->t1.v[k], 2);
        if (p->run_tools && has_op(&c, OP_S)) remove_softclips(&c); /* :168-176 */
        grouped[goff[g] + gfill[g]++] = c;
    }
    int64_t *fam_off = (int64_t *)calloc((size_t)(ng + 1), sizeof(int64_t));
    for (int64_t g = 0; g < ng; g++) {
        orec *v = grouped + goff[g];
        int64_t cnt = goff[g + 1] - goff[g];
        fam_off[g] = res->t2.n;
        if (!p->run_tools || cnt != 4) { /* :114-115 */
            for (int64_t i = 0; i < cnt; i++) ovec_push(&res->t2, v[i]);
            continue;
        }
        /* :118-138 */
        int idx[4][4], nidx[4] = {0, 0, 0, 0}; /* flag slots 99,163,83,147 */
        const uint16_t fl[4] = {99, 163, 83, 147};
        for (int i = 0; i < 4; i++)
            for (int s = 0; s < 4; s++)
                if (v[i].flag == fl[s]) idx[s][nidx[s]++] = i;
        int slot[4][4];
        for (int s = 0; s < 4; s++)
            for (int j = 0; j < nidx[s]; j++) slot[s][j] = idx[s][j];
        if (nidx[0] && nidx[1]) {
            orec *l, *r;
            process_read_pair(&v[slot[0][0]], &v[slot[1][0]], &l, &r);
            int li = (int)(l - v), ri = (int)(r - v);
            slot[0][0] = li; /* flag_groups[99][0] = left (the 163 read) */
            slot[1][0] = ri;
        }
        if (nidx[2] && nidx[3]) {
            orec *l, *r;
            process_read_pair(&v[slot[2][0]], &v[slot[3][0]], &l, &r);
            slot[2][0] = (int)(l - v);
            slot[3][0] = (int)(r - v);
        }
        int used[4] = {0, 0, 0, 0};
        for (int s = 0; s < 4; s++)
            for (int j = 0; j < nidx[s]; j++) {
                ovec_push(&res->t2, v[slot[s][j]]);
                used[slot[s][j]] = 1;
            }
        for (int i = 0; i < 4; i++)
            if (!used[i]) orec_free(&v[i]);
    }
    fam_off[ng] = res->t2.n;
    /* family records: the tool-2 groups as they are, or runs of one MI in TemplateCoordinate order */
    orec *frecs = (orec *)malloc(sizeof(orec) * (size_t)(res->t2.n + 1)); /* shallow copies */
    if (p->family_order == 1) {
        tc_key *keys = (tc_key *)malloc(sizeof(tc_key) * (size_t)(res->t2.n + 1));
        for (int64_t k = 0; k < res->t2.n; k++) keys[k] = tc_key_of(&res->t2.v[k], in, k);
        qsort(keys, (size_t)res->t2.n, sizeof(tc_key), tc_cmp);
        fam_off = (int64_t *)realloc(fam_off, sizeof(int64_t) * (size_t)(res->t2.n + 2)); /* runs >= groups */
        int64_t nf = 0;
        for (int64_t k = 0; k < res->t2.n; k++) {
            frecs[k] = res->t2.v[keys[k].ord];
            const int32_t mi = in->mi_id[frecs[k].src];
            if (k == 0 || mi != in->mi_id[frecs[k - 1].src]) {
                fam_off[nf] = k;
                gorder_mi[nf] = mi;
                nf++;
            }
        }
        fam_off[nf] = res->t2.n;
        ng = nf;
        free(keys);
    } else {
        for (int64_t k = 0; k < res->t2.n; k++) frecs[k] = res->t2.v[k];
    }
    free(grouped);
    free(goff);
    free(gfill);
    free(gcount);
    free(rec_group);
    free(gfirst);
    /* ---- vote, per family ---- */
    int64_t lr[256];
    float thr[94];
    fp64tab f64;
    orc_tables(p->error_rate_pre_umi, p->error_rate_post_umi, lr, thr);
    orc_tables_fp64(p->error_rate_pre_umi, p->error_rate_post_umi, f64.lnc, f64.lne3);
    res->nfam = ng;
    res->fam_rec_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(ng + 1));
    res->fam_src = (int64_t *)malloc(sizeof(int64_t) * (size_t)(res->t2.n + 1));
    for (int64_t g = 0; g <= ng; g++) res->fam_rec_off[g] = fam_off[g];
    for (int64_t k = 0; k < res->t2.n; k++) res->fam_src[k] = frecs[k].src;
    int32_t maxlen = 0;
    for (int64_t k = 0; k < res->t2.n; k++)
        if (res->t2.v[k].len > maxlen) maxlen = res->t2.v[k].len;
    res->maxlen = maxlen;
    res->fam_mi = (int32_t *)malloc(sizeof(int32_t) * (size_t)(ng + 1));
    res->fam_status = (int32_t *)calloc((size_t)(ng + 1), sizeof(int32_t));
    res->fam_nreads = (int32_t *)calloc((size_t)(ng + 1), sizeof(int32_t));
    res->fam_len = (int32_t *)calloc((size_t)(2 * ng + 2), sizeof(int32_t));
    res->fam_b = (char **)calloc((size_t)(2 * ng + 2), sizeof(char *));
    res->fam_q = (uint8_t **)calloc((size_t)(2 * ng + 2), sizeof(uint8_t *));
    res->fam_ss = (ssread *)calloc((size_t)(4 * ng + 4), sizeof(ssread));
    for (int64_t g = 0; g < ng; g++) res->fam_mi[g] = gorder_mi[g];
    if (p->keep_sources) {
        res->src_count = (int32_t *)calloc((size_t)(4 * ng + 4), sizeof(int32_t));
        res->src_len = (int32_t **)calloc((size_t)(ng + 1), sizeof(int32_t *));
        res->src_b = (char **)calloc((size_t)(ng + 1), sizeof(char *));
        res->src_q = (uint8_t **)calloc((size_t)(ng + 1), sizeof(uint8_t *));
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t g = 0; g < ng; g++)
        family_call(frecs + fam_off[g], (int)(fam_off[g + 1] - fam_off[g]), in, p, lr, &f64, thr, res, g);
    free(frecs);
    free(gorder_mi);
    free(fam_off);
    return res;
}

void orc_free(orc_result *r) {
    if (!r) return;
    for (int64_t k = 0; k < r->t1.n; k++) orec_free(&r->t1.v[k]);
    for (int64_t k = 0; k < r->t2.n; k++) orec_free(&r->t2.v[k]);
    free(r->fam_rec_off);
    free(r->fam_src);
    free(r->t1.v);
    free(r->t2.v);
    for (int64_t i = 0; i < 2 * r->nfam; i++) {
        if (r->fam_b) free(r->fam_b[i]);
        if (r->fam_q) free(r->fam_q[i]);
    }
    for (int64_t i = 0; r->fam_ss && i < 4 * r->nfam; i++) {
        free(r->fam_ss[i].b);
        free(r->fam_ss[i].q);
        free(r->fam_ss[i].depth);
        free(r->fam_ss[i].err);
    }
    free(r->fam_ss);
    for (int64_t i = 0; r->src_len && i < r->nfam; i++) {
        free(r->src_len[i]);
        free(r->src_b[i]);
        free(r->src_q[i]);
    }
    free(r->src_count);
    free(r->src_len);
    free(r->src_b);
    free(r->src_q);
    free(r->fam_b);
    free(r->fam_q);
    free(r->fam_mi);
    free(r->fam_status);
    free(r->fam_len);
    free(r->fam_nreads);
    free(r);
}

static const orec_vec *pick(const orc_result *r, int which) { return which == 1 ? &r->t1 : &r->t2; }

int64_t orc_n_records(const orc_result *r, int which) { return pick(r, which)->n; }
int64_t orc_total_bases(const orc_result *r, int which) {
    const orec_vec *v = pick(r, which);
    int64_t s = 0;
    for (int64_t k = 0; k < v->n; k++) s += v->v[k].len;
    return s;
}
int64_t orc_total_cigar(const orc_result *r, int which) {
    const orec_vec *v = pick(r, which);
    int64_t s = 0;
    for (int64_t k = 0; k < v->n; k++) s += v->v[k].ncig;
    return s;
}
void orc_get_records(const orc_result *r, int which, int64_t *src, int32_t *pos, int32_t *l_seq, uint8_t *seq,
                     uint8_t *qual, int32_t *n_cig, uint32_t *cigar, int32_t *rd, int32_t *la) {
    const orec_vec *v = pick(r, which);
    int64_t so = 0, co = 0;
    for (int64_t k = 0; k < v->n; k++) {
        const orec *x = &v->v[k];
        src[k] = x->src;
        pos[k] = x->pos;
        l_seq[k] = x->len;
        memcpy(seq + so, x->seq, (size_t)x->len);
        memcpy(qual + so, x->qual, (size_t)x->len);
        so += x->len;
        n_cig[k] = x->ncig;
        memcpy(cigar + co, x->cig, sizeof(uint32_t) * (size_t)x->ncig);
        co += x->ncig;
        rd[k] = x->rd;
        la[k] = x->la;
    }
}

int64_t orc_n_families(const orc_result *r) { return r->nfam; }
void orc_get_families(const orc_result *r, int64_t *rec_off, int64_t *src) {
    for (int64_t g = 0; g <= r->nfam; g++) rec_off[g] = r->fam_rec_off[g];
    for (int64_t k = 0; k < r->fam_rec_off[r->nfam]; k++) src[k] = r->fam_src[k];
}
int32_t orc_max_cons_len(const orc_result *r) { return r->maxlen; }
void orc_get_consensus(const orc_result *r, int32_t stride, int32_t *mi_id, int32_t *status, int32_t *len,
                       uint8_t *bases, uint8_t *quals, int32_t *n_reads) {
    for (int64_t f = 0; f < r->nfam; f++) {
        mi_id[f] = r->fam_mi[f];
        status[f] = r->fam_status[f];
        n_reads[f] = r->fam_nreads[f];
        for (int e = 0; e < 2; e++) {
            int32_t l = r->fam_len[2 * f + e];
            len[2 * f + e] = l;
            uint8_t *ob = bases + (size_t)(2 * f + e) * (size_t)stride;
            uint8_t *oq = quals + (size_t)(2 * f + e) * (size_t)stride;
            memset(ob, 0, (size_t)stride);
            memset(oq, 0, (size_t)stride);
            if (l > 0) {
                memcpy(ob, r->fam_b[2 * f + e], (size_t)l);
                memcpy(oq, r->fam_q[2 * f + e], (size_t)l);
            }
        }
    }
}

void orc_get_ss(const orc_result *r, int32_t stride, int32_t *len, uint8_t *bases, uint8_t *quals, int32_t *depth,
                int32_t *err) {
    for (int64_t i = 0; i < 4 * r->nfam; i++) {
        const ssread *x = &r->fam_ss[i];
        len[i] = x->len;
        const size_t o = (size_t)i * (size_t)stride;
        memset(bases + o, 0, (size_t)stride);
        memset(quals + o, 0, (size_t)stride);
        memset(depth + o, 0, sizeof(int32_t) * (size_t)stride);
        memset(err + o, 0, sizeof(int32_t) * (size_t)stride);
        if (x->len > 0) {
            memcpy(bases + o, x->b, (size_t)x->len);
            memcpy(quals + o, x->q, (size_t)x->len);
            memcpy(depth + o, x->depth, sizeof(int32_t) * (size_t)x->len);
            memcpy(err + o, x->err, sizeof(int32_t) * (size_t)x->len);
        }
    }
}

void orc_sources_size(const orc_result *r, int64_t *n_reads, int64_t *n_bases) {
    int64_t nr = 0, nb = 0;
    for (int64_t f = 0; r->src_count && f < r->nfam; f++) {
        int32_t c = r->src_count[4 * f] + r->src_count[4 * f + 1] + r->src_count[4 * f + 2] + r->src_count[4 * f + 3];
        for (int32_t i = 0; i < c; i++) nb += r->src_len[f][i];
        nr += c;
    }
    *n_reads = nr;
    *n_bases = nb;
}

void orc_get_sources(const orc_result *r, int32_t *set_count, int32_t *len, uint8_t *bases, uint8_t *quals) {
    int64_t ri = 0, bi = 0;
    for (int64_t f = 0; r->src_count && f < r->nfam; f++) {
        int32_t c = 0;
        for (int s = 0; s < 4; s++) {
            set_count[4 * f + s] = r->src_count[4 * f + s];
            c += r->src_count[4 * f + s];
        }
        int64_t fb = 0;
        for (int32_t i = 0; i < c; i++) {
            len[ri++] = r->src_len[f][i];
            fb += r->src_len[f][i];
        }
        memcpy(bases + bi, r->src_b[f], (size_t)fb);
        memcpy(quals + bi, r->src_q[f], (size_t)fb);
        bi += fb;
    }
}

/* Exhaustive check of libbsdc's agreement-case tables against this restatement's arithmetic:
 * for every D in [0, dmax] (the best base's sum, every other base 0) the vote's Q equals
 * qlo[D >> 16] + (D >= dthr[qlo[D >> 16] + 1]).  Returns the first D that differs, or -1. */
int64_t orc_check_agree(const uint8_t *qlo, const int32_t *dthr, const float *thr, int64_t dmax) {
    int64_t bad = -1;
#pragma omp parallel for schedule(static) reduction(max : bad)
    for (int64_t blk = 0; blk <= dmax >> 16; blk++) {
        for (int64_t D = blk << 16; D < ((blk + 1) << 16) && D <= dmax; D++) {
            float S = 0.0f;
            for (int b = 0; b < 3; b++) {
                const float x = (float)((double)(0 - D) * LR_INV_SCALE);
                if (x < -80.0f) continue;
                S += orc_det_expf(x);
            }
            int Q = 0;
            for (int k = 1; k < 94; k++) {
                if (S <= thr[k])
                    Q = k;
                else
                    break;
            }
            const int64_t d = D < ((int64_t)1 << 27) ? D : ((int64_t)1 << 27) - 1;
            const int q0 = qlo[d >> 16];
            const int qt = q0 + (d >= dthr[q0 + 1] ? 1 : 0);
            if (qt != Q) {
                if (bad < 0 || D < bad) bad = D;
                break;
            }
        }
    }
    return bad;
}
