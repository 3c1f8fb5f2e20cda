// bsdc_host.cpp -- host-side family formation of the step-5 path in C++ (include/bsdc_host.h).
//
// The same record bookkeeping as batch.plan_families_py / materialize_py (the numpy statement of
// it, kept as the test restatement): which records the two tools keep, soft-clip stripping, tool
// 2's MI groups and 4-record pairing, fgbio TemplateCoordinate order and its runs of one MI, and
// then, for any contiguous range of families, the device batch of include/bsdc.h (record words,
// family images, cigars, read-through data, LDS buckets).  OpenMP over records and families; the
// TemplateCoordinate sort is a parallel comparison sort.
//   tool 1 dispatch      tools/1.convert_AG_to_CT.py:70-80
//   tool 2 grouping      tools/2.extend_gap.py:155-186 (4-record groups :112-140)
//   TemplateCoordinate   fgbio SortBam (main.snake.py:152) + the duplex caller's MI runs
//                        (parity unpinned)
#include "../../include/bsdc_host.h"

#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#endif

#include "../../include/bsdc.h"
#include "../../include/bsdc_layout.h"

namespace {

thread_local std::string g_err;
thread_local int64_t g_err_rec = -1;
int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };
inline bool ref_consuming(int op) { return op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X; }
inline bool is_clip(int op) { return op == OP_S || op == OP_H; }

// clips / reference length of a cigar as batch._clips_reflen reads them: a clip op leads while
// no non-clip op precedes it, trails while none follows (and it does not lead)
struct ClipRef {
    int64_t lead = 0, trail = 0, reflen = 0;
};
ClipRef clips_reflen(const uint32_t *c, int64_t n) {
    ClipRef r;
    if (n <= 0) return r;
    int64_t first_nc = -1, last_nc = -1;
    for (int64_t i = 0; i < n; i++) {
        const int op = (int)(c[i] & 0xF);
        const int64_t l = c[i] >> 4;
        if (ref_consuming(op)) r.reflen += l;
        if (!is_clip(op)) {
            if (first_nc < 0) first_nc = i;
            last_nc = i;
        }
    }
    for (int64_t i = 0; i < n; i++) {
        const int op = (int)(c[i] & 0xF);
        if (!is_clip(op)) continue;
        const bool lm = first_nc < 0 || i < first_nc;
        const bool tm = !lm && i > last_nc;
        if (lm) r.lead += c[i] >> 4;
        if (tm) r.trail += c[i] >> 4;
    }
    return r;
}
// the MC variant (batch._mc_clips_reflen): an all-clip cigar counts as leading AND trailing
ClipRef mc_clips_reflen(const uint32_t *c, int64_t n) {
    ClipRef r;
    if (n <= 0) return r;
    int64_t nonclip = 0;
    for (int64_t i = 0; i < n; i++) nonclip += !is_clip((int)(c[i] & 0xF));
    int64_t upto = 0;
    for (int64_t i = 0; i < n; i++) {
        const int op = (int)(c[i] & 0xF);
        const int64_t l = c[i] >> 4;
        if (ref_consuming(op)) r.reflen += l;
        const bool clip = is_clip(op);
        if (!clip) upto++;
        const int64_t before = upto - (clip ? 0 : 1), after = nonclip - upto;
        if (clip && before == 0) r.lead += l;
        if (clip && after == 0) r.trail += l;
    }
    return r;
}

inline uint32_t ref_nib(const bsdc_host_reference *ref, int64_t i) {
    const uint8_t b = ref->packed[i >> 1];
    return (i & 1) ? (b & 0xFu) : (b >> 4);
}

struct PlanOut {
    std::vector<int64_t> order, fam_off, t2_rank, partner_raw, sL, L, kfirst, kn;
    std::vector<int32_t> fam_mi;
    std::vector<uint8_t> conv, ext_right, ext_left, rd_in, fam_split;
};

}  // namespace

struct bsdc_plan {
    PlanOut p;
};

extern "C" {

const char *bsdc_host_last_error(void) { return g_err.c_str(); }
int64_t bsdc_host_error_record(void) { return g_err_rec; }

int32_t bsdc_plan_families(const bsdc_host_records *R, const bsdc_host_reference *ref, int32_t mode, int32_t tc_order,
                           int32_t n_threads, bsdc_plan **out) {
    if (!R || !out) return fail(BSDC_EINVAL, "null argument");
    *out = nullptr;
    if (mode != BSDC_PLAN_FULL && mode != BSDC_PLAN_VOTE) return fail(BSDC_EINVAL, "plan mode: full or vote");
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
    const int64_t n = R->n;
    const bool full = mode == BSDC_PLAN_FULL;
    auto *h = new bsdc_plan();
    PlanOut &P = h->p;
    P.conv.assign(n, 0);
    P.ext_right.assign(n, 0);
    P.ext_left.assign(n, 0);
    P.rd_in.assign(n, 0);
    P.partner_raw.assign(n, -1);
    P.sL.assign(n, 0);
    P.L.assign(n, 0);
    P.kfirst.assign(n, 0);
    P.kn.assign(n, 0);
    std::vector<uint8_t> keep2(n, 0);
    // ---- per record: tool-1 dispatch (:70-80), hard clips (:160-161), soft-clip strip (:30-52) ----
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; k++) {
        const uint32_t *c = R->cigar + R->cig_off[k];
        const int64_t nc = R->n_cig[k] > 0 ? R->n_cig[k] : 0;
        bool hasI = false, hasD = false, hasH = false;
        for (int64_t i = 0; i < nc; i++) {
            const int op = (int)(c[i] & 0xF);
            hasI |= op == OP_I;
            hasD |= op == OP_D;
            hasH |= op == OP_H;
        }
        const int f = R->flag[k];
        bool keep1 = true, cv = false;
        if (full) {
            const bool pas = f == 0 || f == 99 || f == 147;
            cv = (f == 1 || f == 83 || f == 163) && !(hasI || hasD || hasH);
            keep1 = pas || cv;
        }
        P.conv[k] = cv;
        keep2[k] = full ? (keep1 && !hasH) : keep1;
        if (full) {
            const bool fS = nc > 0 && (int)(c[0] & 0xF) == OP_S;
            const int64_t sl = fS ? (int64_t)(c[0] >> 4) : 0;
            const int64_t rem = nc - (fS ? 1 : 0);
            const bool lS = rem > 0 && (int)(c[nc - 1] & 0xF) == OP_S;
            const int64_t sr = lS ? (int64_t)(c[nc - 1] >> 4) : 0;
            const int64_t a = std::max<int64_t>(R->l_seq[k] - sl, 0);
            P.sL[k] = sl;
            P.L[k] = sr > 0 ? std::max<int64_t>(a - sr, 0) : a;
            P.kfirst[k] = fS ? 1 : 0;
            P.kn[k] = rem - (lS ? 1 : 0);
        } else {  // tool-2 output: no clips left, records as they are
            P.L[k] = R->l_seq[k];
            P.kn[k] = nc;
        }
    }
    for (int64_t k = 0; k < n; k++)
        if (keep2[k] && R->mi_id[k] < 0) {
            delete h;
            g_err = "record " + std::to_string(k) + " does not have MI tag.";
            g_err_rec = k;
            return BSDC_PLAN_EMISSING_MI;
        }
    // ---- tool-2 groups: MI in first-seen order, members in input order (:155-186) ----
    int32_t max_mi = -1;
    for (int64_t k = 0; k < n; k++)
        if (keep2[k] && R->mi_id[k] > max_mi) max_mi = R->mi_id[k];
    std::vector<int64_t> grank((size_t)max_mi + 1, -1);
    int64_t ng = 0;
    std::vector<int64_t> gcount;
    for (int64_t k = 0; k < n; k++) {
        if (!keep2[k]) continue;
        int64_t &g = grank[(size_t)R->mi_id[k]];
        if (g < 0) {
            g = ng++;
            gcount.push_back(0);
        }
        gcount[(size_t)g]++;
    }
    std::vector<int64_t> goff((size_t)ng + 1, 0);
    for (int64_t g = 0; g < ng; g++) goff[(size_t)g + 1] = goff[(size_t)g] + gcount[(size_t)g];
    std::vector<int64_t> members((size_t)goff[(size_t)ng]), fill(goff.begin(), goff.end() - 1);
    std::vector<int32_t> gmi((size_t)ng);
    for (int64_t k = 0; k < n; k++) {
        if (!keep2[k]) continue;
        const int64_t g = grank[(size_t)R->mi_id[k]];
        members[(size_t)fill[(size_t)g]++] = k;
        gmi[(size_t)g] = R->mi_id[k];
    }
    // 4-groups: order 163, 99, 83, 147 (the swapped return of process_read_pair, :124-126), other
    // flags dropped; extension roles (:58-110)
    std::vector<int64_t> gkeep(gcount);
    if (full) {
#pragma omp parallel for schedule(static)
        for (int64_t g = 0; g < ng; g++) {
            if (gcount[(size_t)g] != 4) continue;
            int64_t *M = members.data() + goff[(size_t)g];
            int slot[4];
            for (int i = 0; i < 4; i++) {
                const int f = R->flag[M[i]];
                slot[i] = f == 99 ? 0 : f == 163 ? 1 : f == 83 ? 2 : f == 147 ? 3 : 4;
            }
            int ord[4] = {0, 1, 2, 3};
            std::stable_sort(ord, ord + 4, [&](int a, int b) { return slot[a] < slot[b]; });
            int64_t outm[4];
            int outs[4], cnt[5] = {0, 0, 0, 0, 0};
            for (int i = 0; i < 4; i++) {
                outm[i] = M[ord[i]];
                outs[i] = slot[ord[i]];
                cnt[slot[i]]++;
            }
            int start[4];
            start[0] = 0;
            for (int s = 1; s < 4; s++) start[s] = start[s - 1] + cnt[s - 1];
            for (int s = 0; s < 4; s++) start[s] = std::min(start[s], 3);
            const bool p1 = cnt[0] > 0 && cnt[1] > 0, p2 = cnt[2] > 0 && cnt[3] > 0;
            const int64_t a_rec = outm[start[0]], b_rec = outm[start[1]];
            if (p1) {
                outm[start[0]] = b_rec;
                outm[start[1]] = a_rec;
            }
            const int64_t c_rec = outm[start[2]], d_rec = outm[start[3]];
            int nkeep = 0;
            for (int i = 0; i < 4; i++) nkeep += outs[i] < 4;
            if (p1) {  // LA = 1 always after tool 1 (:70-80)
                P.ext_right[a_rec] = 1;
                P.partner_raw[a_rec] = b_rec;
                P.ext_left[b_rec] = 1;
                P.partner_raw[b_rec] = a_rec;
            }
            if (p2) {
                P.ext_right[d_rec] = 1;
                P.partner_raw[d_rec] = c_rec;
                P.ext_left[c_rec] = 1;
                P.partner_raw[c_rec] = d_rec;
            }
            for (int i = 0; i < 4; i++) M[i] = outm[i];
            gkeep[(size_t)g] = nkeep;
        }
    }
    std::vector<int64_t> order;
    order.reserve(members.size());
    std::vector<int64_t> fam_sizes;
    fam_sizes.reserve((size_t)ng);
    for (int64_t g = 0; g < ng; g++) {
        for (int64_t i = 0; i < gkeep[(size_t)g]; i++) order.push_back(members[(size_t)(goff[(size_t)g] + i)]);
        fam_sizes.push_back(gkeep[(size_t)g]);
    }
    const int64_t nr = (int64_t)order.size();
    std::vector<int64_t> t2_rank(nr);
    std::iota(t2_rank.begin(), t2_rank.end(), 0);
    std::vector<int32_t> fam_mi(gmi);
    if (tc_order && nr > 0) {
        bool any_conv = false;
        for (int64_t i = 0; i < nr && full; i++) any_conv |= P.conv[order[i]] != 0;
        if (any_conv && !ref) {
            delete h;
            return fail(BSDC_EINVAL, "converting records needs the reference");
        }
        // ---- TemplateCoordinate keys of the tool-2 records (current positions; stale mates) ----
        struct Key {
            int64_t t1, t2, p1, p2, mi, nm;
            int32_t n1, n2, upper;
            int64_t ord;
        };
        std::vector<Key> keys(nr);
        const int64_t BIG = 2147483647;
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < nr; i++) {
            const int64_t k = order[i];
            const ClipRef own = clips_reflen(R->cigar + R->cig_off[k], R->n_cig[k]);
            const int64_t pos0 = R->pos[k];
            int64_t us, ue;
            if (full) {
                const bool cv = P.conv[k];
                bool rdp = false;
                if (cv) {  // tool 1's RD from the input's last base and two reference bases (batch.predict_rd)
                    const int64_t tid = R->tid[k];
                    const int64_t np0 = std::max<int64_t>(pos0 - 1, 0);
                    const bool okt = tid >= 0 && tid < ref->n_contig && ref->contig_off[tid] >= 0;
                    const int64_t coff = okt ? ref->contig_off[tid] : -1, clen = okt ? ref->contig_len[tid] : 0;
                    const int64_t Ls = P.L[k], Lp = Ls + 1;
                    const int64_t avail = coff >= 0 ? std::min(std::max<int64_t>(clen - np0, 0), Lp + 1) : 0;
                    auto refnib = [&](int64_t j) -> uint32_t { return j < avail ? ref_nib(ref, coff + np0 + j) : 15u; };
                    const uint32_t last = Ls > 0 ? R->seq[R->seq_off[k] + P.sL[k] + Ls - 1] : refnib(0);
                    rdp = last == 2 && refnib(Lp - 1) == 2 && refnib(Lp) == 4;
                }
                const bool er = P.ext_right[k], el = P.ext_left[k];
                const int64_t pos1 = cv ? std::max<int64_t>(pos0 - 1, 0) : (er ? pos0 - 1 : pos0);
                const int64_t rl1 = own.reflen + (cv ? 1 : 0) - ((cv && rdp) ? 1 : 0) + (er ? 1 : 0) + ((el && rdp) ? 1 : 0);
                us = pos1;
                ue = pos1 + rl1 - 1;
            } else {
                us = pos0 - own.lead;
                ue = pos0 + own.reflen - 1 + own.trail;
            }
            int64_t mus = R->next_pos[k], mue = R->next_pos[k];
            if (R->mc_off[k] >= 0) {  // batch.mate_unclipped: the record's own clip rule on MC
                const ClipRef mc = clips_reflen(R->mc_cigar + R->mc_off[k], R->mc_n[k]);
                mus = R->next_pos[k] - mc.lead;
                mue = R->next_pos[k] + mc.reflen - 1 + mc.trail;
            }
            const int f = R->flag[k];
            const int32_t neg = (f & 16) != 0;
            const int64_t t1 = R->tid[k], p1 = neg ? ue : us;
            const bool paired = (f & 1) && !(f & 8);
            const int32_t n2 = paired && (f & 32);
            const int64_t t2 = paired ? (int64_t)R->next_tid[k] : BIG;
            const int64_t p2 = paired ? (n2 ? mue : mus) : BIG;
            const bool lower = t1 < t2 || (t1 == t2 && (p1 < p2 || (p1 == p2 && neg <= n2)));
            Key &K = keys[i];
            K.t1 = lower ? t1 : t2;
            K.t2 = lower ? t2 : t1;
            K.p1 = lower ? p1 : p2;
            K.p2 = lower ? p2 : p1;
            K.n1 = lower ? neg : n2;
            K.n2 = lower ? n2 : neg;
            K.mi = R->mi_rank ? R->mi_rank[k] : R->mi_id[k];
            K.nm = R->name_rank ? R->name_rank[k] : R->name_id[k];
            K.upper = lower ? 0 : 1;
            K.ord = i;
        }
        auto less = [](const Key &a, const Key &b) {
            if (a.t1 != b.t1) return a.t1 < b.t1;
            if (a.t2 != b.t2) return a.t2 < b.t2;
            if (a.p1 != b.p1) return a.p1 < b.p1;
            if (a.p2 != b.p2) return a.p2 < b.p2;
            if (a.n1 != b.n1) return a.n1 < b.n1;
            if (a.n2 != b.n2) return a.n2 < b.n2;
            if (a.mi != b.mi) return a.mi < b.mi;
            if (a.nm != b.nm) return a.nm < b.nm;
            if (a.upper != b.upper) return a.upper < b.upper;
            return a.ord < b.ord;
        };
#ifdef _OPENMP
        __gnu_parallel::sort(keys.begin(), keys.end(), less);
#else
        std::sort(keys.begin(), keys.end(), less);
#endif
        std::vector<int64_t> o2(nr);
        for (int64_t i = 0; i < nr; i++) {
            o2[i] = order[keys[i].ord];
            t2_rank[i] = keys[i].ord;
        }
        order.swap(o2);
        fam_sizes.clear();
        fam_mi.clear();
        for (int64_t i = 0; i < nr; i++) {
            const int32_t mi = R->mi_id[order[i]];
            if (i == 0 || mi != R->mi_id[order[i - 1]]) {
                fam_sizes.push_back(0);
                fam_mi.push_back(mi);
            }
            fam_sizes.back()++;
        }
    }
    const int64_t nf = (int64_t)fam_sizes.size();
    P.fam_off.assign(nf + 1, 0);
    for (int64_t f = 0; f < nf; f++) P.fam_off[f + 1] = P.fam_off[f] + fam_sizes[f];
    // families whose records' tool-2 partners sit elsewhere (the fused launch is invalid there)
    P.fam_split.assign(nf, 0);
    if (nr > 0) {
        std::vector<int64_t> inv(n, -1), fam_of(nr);
        for (int64_t i = 0; i < nr; i++) inv[order[i]] = i;
        for (int64_t f = 0; f < nf; f++)
            for (int64_t i = P.fam_off[f]; i < P.fam_off[f + 1]; i++) fam_of[i] = f;
        for (int64_t i = 0; i < nr; i++) {
            const int64_t k = order[i];
            if (!(P.ext_right[k] || P.ext_left[k])) continue;
            const int64_t pb = inv[P.partner_raw[k]];
            const int64_t f = fam_of[i];
            if (pb < 0 || fam_of[pb] != f || pb - P.fam_off[f] > 3) {
                P.fam_split[f] = 1;
            }
        }
    }
    P.order.swap(order);
    P.t2_rank.swap(t2_rank);
    P.fam_mi.swap(fam_mi);
    *out = h;
    return 0;
}

void bsdc_plan_sizes(const bsdc_plan *h, int64_t *n_rec, int64_t *n_fam) {
    *n_rec = (int64_t)h->p.order.size();
    *n_fam = (int64_t)h->p.fam_mi.size();
}

void bsdc_plan_copy(const bsdc_plan *h, const bsdc_plan_arrays *a) {
    const PlanOut &P = h->p;
    auto cp = [](void *dst, const void *src, size_t bytes) {
        if (dst && bytes) std::memcpy(dst, src, bytes);
    };
    cp(a->order, P.order.data(), P.order.size() * 8);
    cp(a->fam_off, P.fam_off.data(), P.fam_off.size() * 8);
    cp(a->fam_mi, P.fam_mi.data(), P.fam_mi.size() * 4);
    cp(a->t2_rank, P.t2_rank.data(), P.t2_rank.size() * 8);
    cp(a->fam_split, P.fam_split.data(), P.fam_split.size());
    cp(a->conv, P.conv.data(), P.conv.size());
    cp(a->ext_right, P.ext_right.data(), P.ext_right.size());
    cp(a->ext_left, P.ext_left.data(), P.ext_left.size());
    cp(a->rd_in, P.rd_in.data(), P.rd_in.size());
    cp(a->partner_raw, P.partner_raw.data(), P.partner_raw.size() * 8);
    cp(a->sL, P.sL.data(), P.sL.size() * 8);
    cp(a->L, P.L.data(), P.L.size() * 8);
    cp(a->kfirst, P.kfirst.data(), P.kfirst.size() * 8);
    cp(a->kn, P.kn.data(), P.kn.size() * 8);
}

void bsdc_plan_free(bsdc_plan *h) { delete h; }

}  // extern "C"

// ------------------------------------------------------------------------------------------
// materialize: the device batch of plan families [f0, f1)
// ------------------------------------------------------------------------------------------
namespace {
constexpr uint32_t LINK_MATE_NONE = 0xFFFFu;
constexpr int kSmallBuckets[BSDC_SMALL_BUCKETS] = {3072, 4096, 5120, 6144, 8192, 12288, 16384, 24576};
}  // namespace

struct bsdc_batch {
    // inputs kept for the fill
    const bsdc_host_records *R;
    const bsdc_host_reference *ref;
    bsdc_host_plan_view pv;
    int64_t r0, r1, f0, f1;
    int32_t mode_full, small_cap;
    // layout
    std::vector<int64_t> fam_of, local, cap4, rec_off, img, fam_base;
    int64_t n_slots = 0, n_bases = 0, n_cigar = 0;
    int32_t max_len = 0;
};

extern "C" {

int32_t bsdc_materialize_prepare(const bsdc_host_records *R, const bsdc_host_reference *ref,
                                 const bsdc_host_plan_view *pv, int64_t f0, int64_t f1, int32_t mode_full,
                                 int32_t small_cap, int32_t n_threads, bsdc_batch **out, bsdc_batch_sizes *s) {
    if (!R || !pv || !out || !s || f0 < 0 || f1 < f0 || f1 > pv->n_fam) return fail(BSDC_EINVAL, "bad materialize range");
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
    auto *b = new bsdc_batch();
    b->R = R;
    b->ref = ref;
    b->pv = *pv;
    b->f0 = f0;
    b->f1 = f1;
    b->r0 = pv->fam_off[f0];
    b->r1 = pv->fam_off[f1];
    b->mode_full = mode_full;
    b->small_cap = small_cap;
    const int64_t nr = b->r1 - b->r0, nf = f1 - f0;
    b->fam_of.resize(nr);
    b->local.resize(nr);
    b->cap4.resize(nr);
    b->rec_off.resize(nr);
    b->img.resize(nf);
    b->fam_base.assign(nf + 1, 0);
    int64_t nb = 0, ncig = 0;
    int32_t ml = 0;
#pragma omp parallel for schedule(static) reduction(+ : nb, ncig) reduction(max : ml)
    for (int64_t f = 0; f < nf; f++) {
        const int64_t a = pv->fam_off[f0 + f] - b->r0, e = pv->fam_off[f0 + f + 1] - b->r0;
        int64_t span = 0;
        for (int64_t i = a; i < e; i++) {
            const int64_t k = pv->order[b->r0 + i];
            const int64_t L = pv->L[k];
            b->fam_of[i] = f;
            b->local[i] = i - a;
            b->cap4[i] = (L + 2 + 3) & ~int64_t(3);
            b->rec_off[i] = span;  // within the family for now
            span += b->cap4[i];
            nb += L;
            ml = std::max<int32_t>(ml, (int32_t)L);
            // kept cigar ops of complex records only (counted exactly in the fill)
            ncig += pv->kn[k];
        }
        b->img[f] = (span + 31) & ~int64_t(31);
    }
    for (int64_t f = 0; f < nf; f++) b->fam_base[f + 1] = b->fam_base[f] + b->img[f];
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nr; i++) b->rec_off[i] += b->fam_base[b->fam_of[i]];
    b->n_slots = b->fam_base[nf] + 64;
    b->n_bases = nb;
    b->n_cigar = ncig;  // an upper bound (simple records carry none)
    b->max_len = ml;
    if (ml > 0xFFFF - 8) {
        delete b;
        return fail(BSDC_EINVAL, "record longer than 65527 bases");
    }
    if (b->n_slots >= ((int64_t)1 << 32)) {
        delete b;
        return fail(BSDC_EINVAL, "batch too large for 32-bit offsets; split it");
    }
    s->n_rec = nr;
    s->n_fam = nf;
    s->n_slots = b->n_slots;
    s->n_bases = nb;
    s->n_cigar_max = ncig;
    s->max_len = ml;
    *out = b;
    return 0;
}

int32_t bsdc_materialize_fill(bsdc_batch *b, const bsdc_batch_arrays *o, int64_t *n_cigar_out) {
    const bsdc_host_records *R = b->R;
    const bsdc_host_plan_view &pv = b->pv;
    const int64_t nr = b->r1 - b->r0, nf = b->f1 - b->f0;
    const bool full = b->mode_full != 0;
    const int32_t max_len = b->max_len;
    // ---- per record: cigars (complex = any kept op not M/=/X), image copy, words ----
    std::vector<int64_t> nops(nr), reflen(nr);
    std::vector<uint8_t> cplx(nr);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t i = 0; i < nr; i++) {
        const int64_t k = pv.order[b->r0 + i];
        const uint32_t *c = R->cigar + R->cig_off[k] + pv.kfirst[k];
        const int64_t m = pv.kn[k];
        bool cx = false;
        int64_t rl = 0;
        for (int64_t j = 0; j < m; j++) {
            const int op = (int)(c[j] & 0xF);
            cx |= !(op == OP_M || op == OP_EQ || op == OP_X);
            if (ref_consuming(op)) rl += c[j] >> 4;
        }
        nops[i] = m;
        cplx[i] = cx;
        reflen[i] = (!full && !cx) ? pv.L[k] : rl;  // vote mode: a simple record's length (batch.py)
        if (cx && (m > 0xFFFF || rl > 0xFFFF)) bad |= 1;
        // the record's bases / quals: nibble / byte rec_off + 1 (odd) of the images; two records
        // never share a byte of the packed image (slots are 4-aligned).  Every byte from the slot
        // to the next record's slot (or the image end) is written here, the tools' room and the
        // family alignment as zeros, so the images need no zeroed (fresh) memory
        const int64_t L = pv.L[k], so = R->seq_off[k] + pv.sL[k], S = b->rec_off[i], d = S + 1;
        const int64_t end = i + 1 < nr ? b->rec_off[i + 1] : b->n_slots;
        o->qual[S] = 0;
        std::memcpy(o->qual + d, R->qual + so, (size_t)L);
        std::memset(o->qual + d + L, 0, (size_t)(end - d - L));
        const uint8_t *s = R->seq + so;
        uint8_t *p = o->seq + (S >> 1);
        int64_t j = 0;
        *p = L > 0 ? (uint8_t)(s[0] & 15) : 0;  // nibble S (room) and d, the low half of byte S / 2
        p++;
        j = 1;
        for (; j + 1 < L; j += 2) *p++ = (uint8_t)(((s[j] & 15) << 4) | (s[j + 1] & 15));
        if (j < L) *p++ = (uint8_t)((s[j] & 15) << 4);  // a high nibble, then zeros
        std::memset(p, 0, (size_t)(o->seq + (end >> 1) - p));
    }
    if (nr == 0) {
        std::memset(o->qual, 0, (size_t)b->n_slots);
        std::memset(o->seq, 0, (size_t)(b->n_slots >> 1));
    } else if (b->rec_off[0] > 0) {  // (leading empty families)
        std::memset(o->qual, 0, (size_t)b->rec_off[0]);
        std::memset(o->seq, 0, (size_t)(b->rec_off[0] >> 1));
    }
    if (bad) return fail(BSDC_EINVAL, "cigar too long");
    int64_t nc = 0;
    for (int64_t i = 0; i < nr; i++) {
        o->cig_off[i] = (uint32_t)nc;
        if (cplx[i]) nc += nops[i];
    }
    *n_cigar_out = nc;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nr; i++) {
        const int64_t k = pv.order[b->r0 + i];
        if (cplx[i]) {
            const uint32_t *c = R->cigar + R->cig_off[k] + pv.kfirst[k];
            for (int64_t j = 0; j < nops[i]; j++) o->cigar[o->cig_off[i] + j] = c[j];
            o->cig_info[i] = (uint32_t)(nops[i] | (reflen[i] << 16));
        } else {
            o->cig_info[i] = 0;
        }
    }
    // ---- link words: template mates (first usable R1 of a name -> first usable R2 of the name,
    // one family; both mapped, one contig), strand, roles; read-through data; windows ----
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t f = 0; f < nf; f++) {
        const int64_t a = pv.fam_off[b->f0 + f] - b->r0, e = pv.fam_off[b->f0 + f + 1] - b->r0;
        std::vector<std::pair<int32_t, int64_t>> r1s, r2s;
        for (int64_t i = a; i < e; i++) {
            const int64_t k = pv.order[b->r0 + i];
            const int fl = R->flag[k];
            const bool usable = (fl & 1) && !(fl & 0x900) && R->mi_strand[k] >= 0;
            uint32_t link = LINK_MATE_NONE;
            if (usable && (fl & 0x40)) r1s.emplace_back(R->name_id[k], i);
            if (usable && (fl & 0x80)) r2s.emplace_back(R->name_id[k], i);
            const int st = R->mi_strand[k];
            if (st == 0) link |= BSDC_LINK_AB;
            if (st == 1) link |= BSDC_LINK_BA;
            if (cplx[i]) link |= BSDC_LINK_COMPLEX;
            if (pv.conv[k]) link |= BSDC_LINK_CONVERT;
            if (pv.ext_right[k]) link |= BSDC_LINK_EXT_RIGHT;
            if (pv.ext_left[k]) link |= BSDC_LINK_EXT_LEFT;
            if (pv.rd_in[k]) link |= BSDC_LINK_RD_IN;
            if (usable) link |= BSDC_LINK_USABLE;
            o->rec[4 * i + 3] = link;
        }
        std::sort(r1s.begin(), r1s.end());
        std::sort(r2s.begin(), r2s.end());
        size_t q = 0;
        for (size_t p = 0; p < r1s.size(); p++) {
            if (p > 0 && r1s[p].first == r1s[p - 1].first) continue;  // the first R1 of a name
            while (q < r2s.size() && r2s[q].first < r1s[p].first) q++;
            if (q < r2s.size() && r2s[q].first == r1s[p].first) {
                const int64_t ia = r1s[p].second, ib = r2s[q].second;  // r2s sorted: the first R2 of the name
                const int64_t ka = pv.order[b->r0 + ia], kb = pv.order[b->r0 + ib];
                if (R->tid[ka] == R->tid[kb] && !(R->flag[ka] & 4) && !(R->flag[kb] & 4))
                    o->rec[4 * ia + 3] = (o->rec[4 * ia + 3] & ~LINK_MATE_NONE) | (uint32_t)b->local[ib];
            }
        }
    }
    // partners (family-local), windows, read-through, record words
    const bsdc_host_reference *ref = b->ref;
    bool need_ref = false;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t i = 0; i < nr; i++) {
        const int64_t k = pv.order[b->r0 + i];
        const int64_t L = pv.L[k];
        const int fl = R->flag[k];
        uint32_t link = o->rec[4 * i + 3];
        if (pv.ext_right[k] || pv.ext_left[k]) {
            // the partner's position in this family (plan.fam_split marks families where it is not)
            const int64_t fa = pv.fam_off[b->f0 + b->fam_of[i]] - b->r0, fe = pv.fam_off[b->f0 + b->fam_of[i] + 1] - b->r0;
            int64_t pl = 0;
            for (int64_t j = fa; j < fe; j++)
                if (pv.order[b->r0 + j] == pv.partner_raw[k]) {
                    pl = j - fa;
                    break;
                }
            if (pl < 0 || pl > 3) pl = 0;
            link |= (uint32_t)pl << BSDC_LINK_PARTNER_SHIFT;
        }
        // tool-1 reference window (tools/1.convert_AG_to_CT.py:103-117)
        uint32_t w0 = 0, w1 = 0;
        if (pv.conv[k]) {
            if (!ref) {
                bad |= 2;
            } else {
                const int64_t tid = R->tid[k];
                const int64_t np0 = std::max<int64_t>((int64_t)R->pos[k] - 1, 0);
                const bool okt = tid >= 0 && tid < ref->n_contig && ref->contig_off[tid] >= 0;
                if (okt) {
                    const int64_t coff = ref->contig_off[tid], clen = ref->contig_len[tid];
                    const int64_t st = coff + np0;
                    if (st >= ((int64_t)1 << 32)) bad |= 4;
                    w0 = (uint32_t)st;
                    w1 = (uint32_t)std::min(std::max<int64_t>(clen - np0, 0), L + 2);
                }
            }
        }
        o->rec_win[2 * i] = w0;
        o->rec_win[2 * i + 1] = w1;
        // read-through candidates (stale mate fields, MC tag)
        int32_t rt[4] = {0, 0, 0, 0};
        const bool usable = (link & BSDC_LINK_USABLE) != 0;
        if (usable && !(fl & 0xC) && R->next_tid[k] == R->tid[k] && R->mc_off[k] >= 0) {
            const ClipRef mc = mc_clips_reflen(R->mc_cigar + R->mc_off[k], R->mc_n[k]);
            const int64_t np_ = R->next_pos[k];
            const int64_t mus = np_ - mc.lead, mue = np_ + mc.reflen - 1 + mc.trail;
            const int64_t pos = R->pos[k];
            const int64_t rl = cplx[i] ? reflen[i] : L;
            const bool neg = fl & 16;
            const bool cand = neg ? pos - 2 < mus : pos + rl - 1 + 2 > mue;
            if (cand) {
                link |= BSDC_LINK_RT;
                rt[0] = (int32_t)np_;
                rt[1] = R->tlen[k];
                rt[2] = (int32_t)mus;
                rt[3] = (int32_t)mue;
            }
        }
        for (int j = 0; j < 4; j++) o->rt[4 * i + j] = rt[j];
        o->rec[4 * i] = (uint32_t)b->rec_off[i];
        o->rec[4 * i + 1] = (uint32_t)R->pos[k];
        o->rec[4 * i + 2] = (uint32_t)(L | ((int64_t)fl << 16));
        o->rec[4 * i + 3] = link;
        o->src[i] = k;
    }
    (void)need_ref;
    if (bad & 2) return fail(BSDC_EINVAL, "converting records needs the reference");
    if (bad & 4) return fail(BSDC_EINVAL, "reference too large for 32-bit nibble offsets");
    // ---- per family: offsets, list entry, arena needs, size class ----
#pragma omp parallel for schedule(static)
    for (int64_t f = 0; f < nf; f++) {
        const int64_t a = pv.fam_off[b->f0 + f] - b->r0, e = pv.fam_off[b->f0 + f + 1] - b->r0;
        const int64_t n = e - a;
        int64_t cops = 0, nconv = 0, mlf = 0;
        for (int64_t i = a; i < e; i++) {
            const int64_t k = pv.order[b->r0 + i];
            if (cplx[i]) cops += nops[i];
            nconv += pv.conv[k] ? 1 : 0;
            mlf = std::max<int64_t>(mlf, pv.L[k]);
        }
        o->fam_off[f] = (uint32_t)a;
        const int64_t img = b->img[f];
        o->fam_entry[4 * f] = (uint32_t)f;
        o->fam_entry[4 * f + 1] = (uint32_t)a;
        o->fam_entry[4 * f + 2] = (uint32_t)(n | ((img / 32) << 8));
        o->fam_entry[4 * f + 3] = (uint32_t)b->fam_base[f];
        const int64_t need_s = bsdc_layout::SmallLayout((int)std::min<int64_t>(n, 1 << 30), img, (int)nconv, cops, max_len).total;
        const int64_t need_l = bsdc_layout::ArenaLayout((int)std::min<int64_t>(n, 1 << 30), 2 * img, (int)mlf, cops).total;
        o->need_l[f] = need_l;
        o->img[f] = img;
        const bool small = n <= 64 && need_s <= b->small_cap && img / 32 < (1 << 24);
        int cls = -1;
        if (small) {
            int64_t lo = -1;
            for (int q = 0; q < BSDC_SMALL_BUCKETS; q++) {
                const int64_t cap = std::min<int64_t>(kSmallBuckets[q], b->small_cap);
                if (need_s > lo && need_s <= cap) {
                    cls = q;
                    break;
                }
                lo = cap;
                if (cap == b->small_cap) break;
            }
        } else {
            int64_t lo = -1;
            cls = BSDC_SMALL_BUCKETS + BSDC_LARGE_BUCKETS - 1;  // beyond the LDS classes: HBM scratch
            for (int q = 0; q < BSDC_LARGE_BUCKETS - 1; q++) {
                const int64_t cap = o->large_caps[q];
                if (need_l > lo && need_l <= cap) {
                    cls = BSDC_SMALL_BUCKETS + q;
                    break;
                }
                lo = cap;
            }
        }
        o->cls[f] = (int8_t)cls;
    }
    o->fam_off[nf] = (uint32_t)nr;
    return 0;
}

void bsdc_batch_free(bsdc_batch *b) { delete b; }

}  // extern "C"

// ------------------------------------------------------------------------------------------
// part mode: split families of the HBM-scratch bucket (include/bsdc_host.h)
// ------------------------------------------------------------------------------------------
namespace {
struct SplitPart {
    std::vector<int32_t> recs;   // family-local record indices
    std::vector<int32_t> lmate;  // part-local mate index of each (0xFFFF: none)
    int64_t img = 0;             // slot entries
};
// A part's records lie back to back in the family image (bsdc_split_fill lays them out), from an
// entry that need not be 32-aligned: the part stages the 32-entry chunks covering them, up to 31
// entries before its first and after its last, so its arena has room for 32 entries more
inline int64_t part_arena(int n, int64_t span, int32_t ml) {
    return bsdc_layout::ArenaLayout(n, 2 * (((span + 31) & ~int64_t(31)) + 32), ml, 0).total;
}
// The parts of one bucket entry: whole templates (an R1 and the R2 its mate link names, or a
// record no link joins) dealt in record order into parts grown while their arena fits; empty when
// the family is not cut.  A record's slot holds round4(len + 2) entries (include/bsdc.h).
std::vector<SplitPart> split_one(const uint32_t *rec, const uint32_t *e, int64_t part_cap, int32_t max_part_rec) {
    std::vector<SplitPart> parts;
    const int64_t r0 = e[1], n = e[2];
    if (n < 2 || n >= 65536) return parts;
    std::vector<int32_t> mate_of((size_t)n, -1);
    std::vector<uint8_t> is_target((size_t)n, 0);
    for (int64_t i = 0; i < n; i++) {
        const uint32_t link = rec[4 * (r0 + i) + 3];
        if (link & (BSDC_LINK_COMPLEX | BSDC_LINK_EXT_LEFT | BSDC_LINK_EXT_RIGHT)) return parts;
        const uint32_t m = link & BSDC_LINK_MATE_MASK;
        if (m == BSDC_LINK_MATE_MASK) continue;
        if ((int64_t)m >= n || (int64_t)m == i || is_target[m]) return parts;
        mate_of[(size_t)i] = (int32_t)m;
        is_target[(size_t)m] = 1;
    }
    auto len_of = [&](int64_t i) { return (int32_t)(rec[4 * (r0 + i) + 2] & 0xFFFF); };
    auto cap4 = [&](int64_t i) { return (int64_t)((len_of(i) + 2 + 3) & ~3); };
    SplitPart cur;
    int32_t ml = 0;
    int64_t span = 0;
    auto close = [&]() {
        cur.img = span;
        parts.push_back(std::move(cur));
        cur = SplitPart();
        ml = 0;
        span = 0;
    };
    for (int64_t i = 0; i < n; i++) {
        if (is_target[(size_t)i]) continue;  // (placed with its R1)
        const int64_t m = mate_of[(size_t)i];
        const int k = m >= 0 ? 2 : 1;
        const int64_t add = cap4(i) + (m >= 0 ? cap4(m) : 0);
        const int32_t ml2 = std::max(ml, std::max(len_of(i), m >= 0 ? len_of(m) : 0));
        const int64_t n2 = (int64_t)cur.recs.size() + k;
        const int64_t need = part_arena((int)n2, span + add, ml2);
        if (!cur.recs.empty() && (need > part_cap || n2 > max_part_rec)) close();
        {
            const int64_t n1 = (int64_t)cur.recs.size() + k;
            const int32_t ml1 = std::max(ml, std::max(len_of(i), m >= 0 ? len_of(m) : 0));
            if (part_arena((int)n1, span + add, ml1) > part_cap || n1 > max_part_rec) {  // one template alone does not fit
                parts.clear();
                return parts;
            }
        }
        const int32_t li = (int32_t)cur.recs.size();
        cur.recs.push_back((int32_t)i);
        cur.lmate.push_back(m >= 0 ? li + 1 : 0xFFFF);
        if (m >= 0) {
            cur.recs.push_back((int32_t)m);
            cur.lmate.push_back(0xFFFF);
        }
        span += add;
        ml = std::max(ml, std::max(len_of(i), m >= 0 ? len_of(m) : 0));
    }
    if (!cur.recs.empty()) close();
    if (parts.size() < 2) {
        parts.clear();
        return parts;
    }
    // the family's first record leads the family image (the whole-family fallback reads the image
    // from its slot): its part goes first, its template first in the part, and the record first in
    // its template (an R2 before its R1: the part-local mate links follow the order)
    size_t j0 = 0, q0 = 0;
    for (size_t j = 0; j < parts.size(); j++)
        for (size_t q = 0; q < parts[j].recs.size(); q++)
            if (parts[j].recs[q] == 0) j0 = j, q0 = q;
    if (j0 != 0) std::rotate(parts.begin(), parts.begin() + (int64_t)j0, parts.begin() + (int64_t)j0 + 1);
    SplitPart &P0 = parts[0];
    const size_t t0 = (q0 > 0 && P0.lmate[q0 - 1] == (int32_t)q0) ? q0 - 1 : q0;  // its template's first record
    const size_t tn = P0.lmate[t0] != 0xFFFF ? 2 : 1;
    std::vector<int32_t> order;
    order.push_back(0);
    if (tn == 2) order.push_back(P0.recs[t0] == 0 ? P0.recs[t0 + 1] : P0.recs[t0]);
    for (size_t q = 0; q < P0.recs.size(); q++)
        if (q < t0 || q >= t0 + tn) order.push_back(P0.recs[q]);
    std::vector<int32_t> pos((size_t)n, -1);
    for (size_t q = 0; q < order.size(); q++) pos[(size_t)order[q]] = (int32_t)q;
    std::vector<int32_t> lm(order.size(), 0xFFFF);
    for (size_t q = 0; q < order.size(); q++) {
        const int32_t m = mate_of[(size_t)order[q]];
        if (m >= 0) lm[q] = pos[(size_t)m];
    }
    P0.recs = std::move(order);
    P0.lmate = std::move(lm);
    return parts;
}
}  // namespace

extern "C" {

int64_t bsdc_split_count(const uint32_t *rec, const uint32_t *ents, int64_t n_ent, int64_t part_cap, int32_t max_part_rec,
                         int32_t *nparts, int64_t *nrecs, int32_t n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
    int64_t tot = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : tot)
    for (int64_t e = 0; e < n_ent; e++) {
        const auto pr = split_one(rec, ents + 4 * e, part_cap, max_part_rec);
        nparts[e] = (int32_t)pr.size();
        nrecs[e] = pr.empty() ? 0 : ents[4 * e + 2];
        tot += nparts[e];
    }
    return tot;
}

void bsdc_split_fill(const uint32_t *rec, const uint32_t *ents, int64_t n_ent, int64_t part_cap, int32_t max_part_rec,
                     const int64_t *first_part, const int64_t *first_rec, uint32_t *parts, uint32_t *part_recs,
                     int32_t n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t e = 0; e < n_ent; e++) {
        const uint32_t *en = ents + 4 * e;
        const auto pr = split_one(rec, en, part_cap, max_part_rec);
        const int64_t r0 = en[1];
        int64_t pk = first_rec[e];
        // the family image re-laid out part after part (bsdc_split_move moves the bytes): a part's
        // records back to back from `at`, staged as the 32-entry chunks from `at` rounded down
        uint32_t at = rec[4 * r0];  // (the family's first slot: the image base)
        for (size_t j = 0; j < pr.size(); j++) {
            uint32_t *o = parts + 4 * (first_part[e] + (int64_t)j);
            const uint32_t a0 = at & ~31u;
            o[0] = en[0];
            o[1] = (uint32_t)pk;
            o[2] = (uint32_t)pr[j].recs.size();
            o[3] = ((at - a0) + (uint32_t)pr[j].img + 31u) & ~31u;  // staged entries
            for (size_t q = 0; q < pr[j].recs.size(); q++, pk++) {
                const int64_t gi = r0 + pr[j].recs[q];
                uint32_t *w = part_recs + 4 * pk;
                w[0] = (uint32_t)gi;
                w[1] = at - a0;  // its slot in the part's staged image
                w[2] = (uint32_t)pr[j].lmate[q] | (rec[4 * gi + 2] & 0xFFFFu) << 16;  // | its length
                w[3] = at;       // its new slot in the batch image
                at += (uint32_t)(((rec[4 * gi + 2] & 0xFFFF) + 2 + 3) & ~3u);
            }
        }
    }
}


// The cut families' images re-laid out as bsdc_split_fill placed their records (include/bsdc_host.h).
void bsdc_split_move(uint8_t *seq, uint8_t *qual, uint32_t *rec_off, const uint32_t *split_fams, int64_t n_sf,
                     const uint32_t *parts, const uint32_t *part_recs, int32_t n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t f = 0; f < n_sf; f++) {
        const uint32_t *sf = split_fams + 8 * f;
        const uint32_t r0 = sf[1], img = sf[3], p0 = sf[4], np = sf[5];
        const uint32_t base = rec_off[r0];
        std::vector<uint8_t> tq(img), ts(img / 2 + 1);
        std::memcpy(tq.data(), qual + base, img);  // (entries no record holds keep their bytes)
        std::memcpy(ts.data(), seq + base / 2, img / 2);
        for (uint32_t p = p0; p < p0 + np; p++) {
            const uint32_t *pt = parts + 4 * (int64_t)p;
            for (uint32_t q = 0; q < (pt[2] & 0xFFu); q++) {
                const uint32_t *w = part_recs + 4 * ((int64_t)pt[1] + q);
                const uint32_t from = rec_off[w[0]], to = w[3];
                const uint32_t cap = ((w[2] >> 16) + 2 + 3) & ~3u;  // (slots start at even entries: whole bytes)
                std::memcpy(tq.data() + (to - base), qual + from, cap);
                std::memcpy(ts.data() + (to - base) / 2, seq + from / 2, cap / 2);
            }
        }
        std::memcpy(qual + base, tq.data(), img);
        std::memcpy(seq + base / 2, ts.data(), img / 2);
        for (uint32_t p = p0; p < p0 + np; p++) {
            const uint32_t *pt = parts + 4 * (int64_t)p;
            for (uint32_t q = 0; q < (pt[2] & 0xFFu); q++) {
                const uint32_t *w = part_recs + 4 * ((int64_t)pt[1] + q);
                rec_off[w[0]] = w[3];
            }
        }
    }
}

}  // extern "C"
