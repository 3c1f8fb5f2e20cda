// bsdc_io.cpp -- BAM/BGZF codec for the step-5 drop-in (include/bsdc_io.h).
//
// Reader: the file is read whole, its BGZF blocks are located by one scan of the block headers
// (BSIZE in the BC extra field), inflated in parallel straight into one buffer at their
// uncompressed offsets (raw deflate, CRC32 checked), then the records are found by one scan of
// block_size words and parsed in parallel into structure-of-arrays.  QNAMEs and MI bases are
// interned sequentially (hash maps over views into the buffer).
// Writer: record sizes -> prefix sums -> parallel encode into one buffer -> 0xff00-byte BGZF
// blocks deflated in parallel -> one write, then the 28-byte EOF block.
#include "../../include/bsdc_io.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <mutex>
#include <set>
#include <chrono>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#else  // a build without -fopenmp runs every parallel region on one thread
inline int omp_get_max_threads() { return 1; }
inline int omp_get_thread_num() { return 0; }
inline int omp_get_num_threads() { return 1; }
#endif

// Byte buffers that grow without zero-filling: every byte is written before it is read (inflate,
// record encode, deflate slots), and value-initialising gigabytes per chunk was serial memset time
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <class U>
    NoInit(const NoInit<U> &) {}
    template <class U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, NoInit<uint8_t>>;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
inline int32_t rdi32(const uint8_t *p) { return (int32_t)rd32(p); }
inline void wr16(uint8_t *p, uint16_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
inline void wr32(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}

// libdeflate (the system's libdeflate.so.0, loaded at run time; its published v1 C API) inflates,
// deflates and CRCs BGZF blocks 2-3x faster than zlib.  Without it (or with BSDC_ZLIB set) the
// codec uses zlib; both read every valid BGZF file, and each writes valid BGZF (the compressed
// bytes differ between the two).
struct Libdeflate {
    void *(*alloc_d)() = nullptr;
    void (*free_d)(void *) = nullptr;
    int (*decompress)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    void *(*alloc_c)(int) = nullptr;
    void (*free_c)(void *) = nullptr;
    size_t (*compress)(void *, const void *, size_t, void *, size_t) = nullptr;
    size_t (*bound)(void *, size_t) = nullptr;
    uint32_t (*crc)(uint32_t, const void *, size_t) = nullptr;
    bool ok = false;
    Libdeflate() {
        if (getenv("BSDC_ZLIB")) return;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc_d = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        free_d = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        decompress = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_deflate_decompress");
        alloc_c = (void *(*)(int))dlsym(h, "libdeflate_alloc_compressor");
        free_c = (void (*)(void *))dlsym(h, "libdeflate_free_compressor");
        compress = (size_t(*)(void *, const void *, size_t, void *, size_t))dlsym(h, "libdeflate_deflate_compress");
        bound = (size_t(*)(void *, size_t))dlsym(h, "libdeflate_deflate_compress_bound");
        crc = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
        ok = alloc_d && free_d && decompress && alloc_c && free_c && compress && bound && crc;
    }
};
const Libdeflate &libdeflate() {
    static const Libdeflate L;
    return L;
}
// one decompressor / compressor per thread, kept for the thread's life
struct DeflateState {
    void *d = nullptr, *c = nullptr;
    int level = -1;
    ~DeflateState() {
        if (d) libdeflate().free_d(d);
        if (c) libdeflate().free_c(c);
    }
};
DeflateState &deflate_state() {
    thread_local DeflateState s;
    return s;
}
uint32_t crc32_of(const uint8_t *p, int64_t n) {
    const Libdeflate &L = libdeflate();
    return L.ok ? L.crc(0, p, (size_t)n) : (uint32_t)crc32(0L, p, (uInt)n);
}
// raw deflate stream in[0, n) -> exactly `want` bytes at out; false on any error
bool raw_inflate(const uint8_t *in, int64_t n, uint8_t *out, int64_t want) {
    const Libdeflate &L = libdeflate();
    if (L.ok) {
        DeflateState &st = deflate_state();
        if (!st.d) st.d = L.alloc_d();
        size_t got = 0;
        return st.d && L.decompress(st.d, in, (size_t)n, out, (size_t)want, &got) == 0 && (int64_t)got == want;
    }
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = const_cast<uint8_t *>(in);
    zs.avail_in = (uInt)n;
    zs.next_out = out;
    zs.avail_out = (uInt)want;
    const int rc = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    return rc == Z_STREAM_END && (int64_t)zs.total_out == want;
}
// raw deflate of in[0, n) at `level` into out[0, cap) -> compressed size, 0 on failure
int64_t raw_deflate(const uint8_t *in, int64_t n, int level, uint8_t *out, int64_t cap) {
    const Libdeflate &L = libdeflate();
    if (L.ok && level > 0) {  // (stored blocks, level 0, through zlib)
        DeflateState &st = deflate_state();
        if (!st.c || st.level != level) {
            if (st.c) L.free_c(st.c);
            st.c = L.alloc_c(level);
            st.level = level;
        }
        return st.c ? (int64_t)L.compress(st.c, in, (size_t)n, out, (size_t)cap) : 0;
    }
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
    zs.next_in = const_cast<uint8_t *>(in);
    zs.avail_in = (uInt)n;
    zs.next_out = out;
    zs.avail_out = (uInt)cap;
    const int rc = deflate(&zs, Z_FINISH);
    deflateEnd(&zs);
    return rc == Z_STREAM_END ? (int64_t)zs.total_out : 0;
}

void set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

const char kCigarOps[] = "MIDNSHP=X";
inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// packed SEQ byte -> its two bases as one little-endian uint16 (high nibble first)
struct NibblePairs {
    uint16_t v[256];
    NibblePairs() {
        for (int b = 0; b < 256; b++) v[b] = (uint16_t)((b >> 4) | ((b & 15) << 8));
    }
};
const NibblePairs kNibblePairs;

// aux field size past the 3-byte tag+type header, or -1 if malformed
int64_t aux_value_size(const uint8_t *p, const uint8_t *end) {
    const char t = (char)p[2];
    const uint8_t *v = p + 3;
    switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'Z': case 'H': {
        const uint8_t *z = (const uint8_t *)memchr(v, 0, (size_t)(end - v));
        return z ? (int64_t)(z - v) + 1 : -1;
    }
    case 'B': {
        if (end - v < 5) return -1;
        const char sub = (char)v[0];
        const int64_t cnt = rd32(v + 1);
        int w;
        switch (sub) {
        case 'c': case 'C': w = 1; break;
        case 's': case 'S': w = 2; break;
        case 'i': case 'I': case 'f': w = 4; break;
        default: return -1;
        }
        return 5 + cnt * w;
    }
    default: return -1;
    }
}

int64_t aux_int(const uint8_t *p) {
    const uint8_t *v = p + 3;
    switch ((char)p[2]) {
    case 'c': return (int8_t)v[0];
    case 'C': return v[0];
    case 's': return (int16_t)rd16(v);
    case 'S': return rd16(v);
    case 'i': return rdi32(v);
    case 'I': return rd32(v);
    default: return -1;
    }
}

}  // namespace

// ids[k] = index of keys[k] among the distinct keys in first-seen order, appended to `uniq`; with
// `present`, a record whose present[k] is empty gets -1.  Hash-sharded, every pass parallel: the
// hashes, a stable counting scatter of the records by shard (per-thread histograms), one
// open-addressing table per shard, and the global ids as a prefix sum over the records that are
// their key's first occurrence.
static void intern(const std::vector<std::string_view> &keys, const std::vector<std::string_view> *present,
            std::vector<int32_t> &ids, std::vector<std::string_view> &uniq) {
    const int64_t n = (int64_t)keys.size();
    constexpr int S = 256;
    std::vector<uint32_t> shard((size_t)n);
    std::vector<uint64_t> hv((size_t)n);
    std::vector<int64_t> order((size_t)n);
    std::vector<int32_t> local((size_t)n);
    std::vector<uint8_t> is_first((size_t)n);
    std::vector<int64_t> start(S + 2, 0);
    std::vector<std::vector<int64_t>> first(S);
    const int T = omp_get_max_threads();
    std::vector<int64_t> cnt((size_t)T * (S + 1), 0);  // per thread and shard (S = absent)
    std::vector<int64_t> part((size_t)T + 1, 0);        // per thread: first occurrences in its block
#pragma omp parallel
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        int64_t *c = cnt.data() + (size_t)t * (S + 1);
        for (int64_t k = lo; k < hi; k++) {
            const bool ok = present == nullptr || !(*present)[(size_t)k].empty();
            const uint64_t h = std::hash<std::string_view>{}(keys[(size_t)k]);
            hv[(size_t)k] = h;
            const uint32_t sh = ok ? (uint32_t)(h % S) : (uint32_t)S;
            shard[(size_t)k] = sh;
            c[sh]++;
            is_first[(size_t)k] = 0;
        }
#pragma omp barrier
#pragma omp single
        {
            // shard s's records start after every smaller shard; within a shard, thread blocks
            // in order, so the scatter keeps each shard's records in ascending k
            int64_t run = 0;
            for (int sh = 0; sh <= S; sh++) {
                start[sh] = run;
                for (int u = 0; u < nt; u++) {
                    const int64_t v = cnt[(size_t)u * (S + 1) + sh];
                    cnt[(size_t)u * (S + 1) + sh] = run;
                    run += v;
                }
            }
            start[S + 1] = run;
        }
        for (int64_t k = lo; k < hi; k++) order[(size_t)c[shard[(size_t)k]]++] = k;
#pragma omp barrier
        // per shard: an open-addressing table (linear probing) of the shard's distinct keys
#pragma omp for schedule(dynamic, 4)
        for (int sh = 0; sh < S; sh++) {
            const int64_t m = start[sh + 1] - start[sh];
            size_t cap = 16;
            while ((int64_t)cap < 2 * m) cap <<= 1;
            std::vector<int32_t> slot(cap, -1);
            std::vector<int64_t> &fs = first[sh];
            for (int64_t i = start[sh]; i < start[sh + 1]; i++) {
                const int64_t k = order[(size_t)i];
                const std::string_view key = keys[(size_t)k];
                size_t pos = (size_t)(hv[(size_t)k] / S) & (cap - 1);
                while (slot[pos] >= 0 && keys[(size_t)fs[(size_t)slot[pos]]] != key) pos = (pos + 1) & (cap - 1);
                if (slot[pos] < 0) {
                    slot[pos] = (int32_t)fs.size();
                    fs.push_back(k);
                    is_first[(size_t)k] = 1;
                }
                local[(size_t)k] = slot[pos];
            }
        }
        // (implicit barrier) global ids: first occurrences ranked by record index
        int64_t f = 0;
        for (int64_t k = lo; k < hi; k++) f += is_first[(size_t)k];
        part[(size_t)t + 1] = f;
#pragma omp barrier
#pragma omp single
        {
            for (int u = 0; u < nt; u++) part[(size_t)u + 1] += part[(size_t)u];
            uniq.resize(uniq.size() + (size_t)part[(size_t)nt]);
            ids.resize((size_t)n);
        }
        const int64_t base = (int64_t)uniq.size() - part[(size_t)nt];
        int64_t g = base + part[(size_t)t];
        for (int64_t k = lo; k < hi; k++)
            if (is_first[(size_t)k]) {
                uniq[(size_t)g] = keys[(size_t)k];
                ids[(size_t)k] = (int32_t)g++;  // (a first occurrence's own id; the rest below)
            }
#pragma omp barrier
        for (int64_t k = lo; k < hi; k++) {
            const uint32_t sh = shard[(size_t)k];
            if (sh == (uint32_t)S)
                ids[(size_t)k] = -1;
            else if (!is_first[(size_t)k])
                ids[(size_t)k] = ids[(size_t)first[sh][(size_t)local[(size_t)k]]];
        }
    }
}

struct bsdc_bam {
    Bytes data;  // the uncompressed stream
    std::string header;
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_len;
    std::vector<int64_t> rec_start;  // offset of each record's block_size word
    // parsed
    std::vector<int32_t> name_id, mi_id;
    std::vector<int8_t> mi_strand;
    std::vector<std::string_view> names, mis;
    std::vector<int32_t> la, rd;
    std::vector<int64_t> mc_tag_off;  // offset of the MC string in data, -1 = none
    std::vector<int32_t> mc_n;
    int64_t n_bases = 0, n_cigar = 0, n_mc = 0, aux_bytes = 0;
    int64_t dn = 0;       // record bytes in data (a stream chunk before bsdc_bam_parse)
    bool parsed = true;   // false: a raw stream chunk (bsdc_bam_stream_next_raw)
};

extern "C" {

int32_t bsdc_io_abi_version(void) { return BSDC_IO_ABI_VERSION; }
const char *bsdc_io_last_error(void) { return g_err.c_str(); }

}  // extern "C"

namespace {

// Whole BGZF blocks of comp[0, n) inflated (in parallel) and appended to `out`; *used = the bytes
// of the whole blocks (a trailing partial block is left for the caller unless `final`, where it
// is an error).  Every block is CRC-checked.
int32_t inflate_blocks(const uint8_t *comp, int64_t n, bool final, Bytes &out, int64_t *used) {
    std::vector<int64_t> boff, bsz, uoff;
    int64_t o = 0, u = (int64_t)out.size();
    *used = 0;
    while (o < n) {
        const uint8_t *h = comp + o;
        if (n - o < 18) {
            if (!final) break;
            return fail(BSDC_IO_EFORMAT, "truncated BGZF block");
        }
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4))
            return fail(BSDC_IO_EFORMAT, "not a BGZF file (bad block header)");
        const int xlen = rd16(h + 10);
        if (n - o < 12 + xlen) {
            if (!final) break;
            return fail(BSDC_IO_EFORMAT, "truncated BGZF block");
        }
        int64_t bsize = -1;
        for (int x = 0; x + 4 <= xlen;) {
            const uint8_t *sf = h + 12 + x;
            const int slen = rd16(sf + 2);
            if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) bsize = rd16(sf + 4) + 1;
            x += 4 + slen;
        }
        if (bsize < 0) return fail(BSDC_IO_EFORMAT, "truncated BGZF block");
        if (o + bsize > n) {
            if (!final) break;
            return fail(BSDC_IO_EFORMAT, "truncated BGZF block");
        }
        boff.push_back(o);
        bsz.push_back(bsize);
        uoff.push_back(u);
        u += rd32(h + bsize - 4);
        o += bsize;
    }
    // (+8: the readers pad the stream for dword loads; geometric growth for the streaming buffer)
    if (out.capacity() < (size_t)u + 8) out.reserve(std::max((size_t)u + 8, 2 * out.capacity()));
    out.resize((size_t)u);
    const int64_t nb = (int64_t)boff.size();
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(| : bad)
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t *h = comp + boff[i];
        const int xlen = rd16(h + 10);
        const uint8_t *cdata = h + 12 + xlen;
        const int64_t clen = bsz[i] - 12 - xlen - 8;
        const uint32_t isize = rd32(h + bsz[i] - 4), crc = rd32(h + bsz[i] - 8);
        if (isize == 0) continue;
        if (clen < 0) {
            bad |= 1;
            continue;
        }
        if (!raw_inflate(cdata, clen, out.data() + uoff[i], isize) || crc32_of(out.data() + uoff[i], isize) != crc) bad |= 1;
    }
    if (bad) return fail(BSDC_IO_EFORMAT, "corrupt BGZF block (inflate or CRC32)");
    *used = o;
    return 0;
}

// The BAM header at the start of d[0, dn): text, references; *p = the first record's offset.
int32_t parse_header(const uint8_t *d, int64_t dn, bsdc_bam *b, int64_t *p_out) {
    if (dn < 12 || memcmp(d, "BAM\1", 4) != 0) return fail(BSDC_IO_EFORMAT, "missing BAM magic");
    int64_t p = 4;
    const int64_t l_text = rd32(d + p);
    p += 4;
    if (p + l_text + 4 > dn) return fail(BSDC_IO_EFORMAT, "truncated BAM header");
    b->header.assign((const char *)d + p, (size_t)l_text);
    b->header.resize(strnlen(b->header.c_str(), b->header.size()));
    p += l_text;
    const int32_t n_ref = rdi32(d + p);
    p += 4;
    for (int32_t i = 0; i < n_ref; i++) {
        if (p + 4 > dn) break;
        const int32_t ln = rdi32(d + p);
        p += 4;
        if (ln < 1 || p + ln + 4 > dn) return fail(BSDC_IO_EFORMAT, "truncated reference list");
        b->ref_names.emplace_back((const char *)d + p, (size_t)ln - 1);
        p += ln;
        b->ref_len.push_back(rd32(d + p));
        p += 4;
    }
    *p_out = p;
    return 0;
}

// The records of b->data from offset p to dn (whole records only): boundaries, tags, interning.
// (rec_start already filled: the records at those offsets, each whole inside [0, dn), as the
// streaming reader hands them over)
int32_t parse_records(bsdc_bam *b, int64_t p, int64_t dn) {
    const uint8_t *d = b->data.data();
    if (b->rec_start.empty()) {
        while (p + 4 <= dn) {
            const int64_t bs = rd32(d + p);
            if (bs < 32 || p + 4 + bs > dn) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
            b->rec_start.push_back(p);
            p += 4 + bs;
        }
        if (p != dn) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
    } else {
        for (const int64_t q : b->rec_start)
            if (q < 0 || q + 4 > dn || rd32(d + q) < 32 || q + 4 + (int64_t)rd32(d + q) > dn)
                return fail(BSDC_IO_EFORMAT, "truncated BAM record");
    }
    const int64_t nr = (int64_t)b->rec_start.size();
    // ---- per record: tags, sizes ----
    b->la.assign(nr, -1);
    b->rd.assign(nr, -1);
    b->mc_tag_off.assign(nr, -1);
    b->mc_n.assign(nr, 0);
    std::vector<std::string_view> mi_full(nr);
    int64_t nbases = 0, ncig = 0, nmc = 0, naux = 0;
    int badrec = 0;
#pragma omp parallel for schedule(static) reduction(+ : nbases, ncig, nmc, naux) reduction(| : badrec)
    for (int64_t k = 0; k < nr; k++) {
        const uint8_t *r = d + b->rec_start[k];
        const int64_t bs = rd32(r);
        const uint8_t *end = r + 4 + bs;
        const int l_name = r[12];
        const int n_cig = rd16(r + 16);
        const int32_t l_seq = rdi32(r + 20);
        // fixed part + name + cigar + seq + qual, in 64 bits (untrusted lengths)
        const int64_t body = 36 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + (int64_t)l_seq;
        if (l_seq < 0 || l_name < 1 || body > 4 + bs) {
            badrec |= 1;
            continue;
        }
        const uint8_t *aux = r + body;
        nbases += l_seq;
        ncig += n_cig;
        naux += end - aux;
        for (const uint8_t *a = aux; a + 3 <= end;) {
            const int64_t vs = aux_value_size(a, end);
            if (vs < 0 || vs > (end - a) - 3) {
                badrec |= 1;
                break;
            }
            if (a[0] == 'M' && a[1] == 'I' && a[2] == 'Z') {
                mi_full[k] = std::string_view((const char *)a + 3, (size_t)vs - 1);
            } else if (a[0] == 'M' && a[1] == 'C' && a[2] == 'Z') {
                const char *s = (const char *)a + 3;
                if (!(vs == 2 && s[0] == '*')) {
                    int cnt = 0;
                    for (int64_t i = 0; i < vs - 1; i++) cnt += strchr(kCigarOps, s[i]) != nullptr && !(s[i] >= '0' && s[i] <= '9');
                    b->mc_tag_off[k] = (int64_t)((const uint8_t *)s - d);
                    b->mc_n[k] = cnt;
                    nmc += cnt;
                }
            } else if (a[0] == 'L' && a[1] == 'A') {
                b->la[k] = (int32_t)aux_int(a);
            } else if (a[0] == 'R' && a[1] == 'D') {
                b->rd[k] = (int32_t)aux_int(a);
            }
            a += 3 + vs;
        }
    }
    if (badrec) return fail(BSDC_IO_EFORMAT, "malformed BAM record (lengths or aux)");
    b->n_bases = nbases;
    b->n_cigar = ncig;
    b->n_mc = nmc;
    b->aux_bytes = naux;
    // ---- interning: QNAME, MI base = MI up to the first '/'; ids in first-seen order ----
    b->name_id.resize(nr);
    b->mi_id.resize(nr);
    b->mi_strand.resize(nr);
    std::vector<std::string_view> nm(nr), mk(nr);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nr; k++) {
        const uint8_t *r = d + b->rec_start[k];
        const int l_name = r[12];
        nm[k] = std::string_view((const char *)r + 36, l_name > 0 ? (size_t)l_name - 1 : 0);
        const std::string_view mi = mi_full[k];
        const size_t L = mi.size();
        if (L) {
            const size_t slash = mi.find('/');
            mk[k] = slash == std::string_view::npos ? mi : mi.substr(0, slash);
        }
        b->mi_strand[k] = (L >= 2 && mi[L - 2] == '/' && mi[L - 1] == 'A') ? 0
                          : (L >= 2 && mi[L - 2] == '/' && mi[L - 1] == 'B') ? 1 : -1;
    }
    intern(nm, nullptr, b->name_id, b->names);
    intern(mk, &mi_full, b->mi_id, b->mis);
    return 0;
}

}  // namespace

extern "C" {

int32_t bsdc_bam_read(const char *path, int32_t n_threads, bsdc_bam **out) {
    *out = nullptr;
    set_threads(n_threads);
    FILE *f = fopen(path, "rb");
    if (!f) return fail(BSDC_IO_EIO, std::string("cannot open ") + path);
    Bytes comp;
    {
        fseek(f, 0, SEEK_END);
        const long sz = ftell(f);
        fseek(f, 0, SEEK_SET);
        comp.resize(sz > 0 ? (size_t)sz : 0);
        if (sz > 0 && fread(comp.data(), 1, comp.size(), f) != comp.size()) {
            fclose(f);
            return fail(BSDC_IO_EIO, std::string("short read on ") + path);
        }
        fclose(f);
    }
    auto *b = new bsdc_bam();
    int64_t used = 0, p = 0;
    int32_t rc = inflate_blocks(comp.data(), (int64_t)comp.size(), true, b->data, &used);
    const int64_t dn = (int64_t)b->data.size();
    if (rc == 0) rc = parse_header(b->data.data(), dn, b, &p);
    b->data.resize((size_t)dn + 8);
    memset(b->data.data() + dn, 0, 8);  // the pad (a no-init buffer)
    if (rc == 0) rc = parse_records(b, p, dn);
    if (rc != 0) {
        delete b;
        return rc;
    }
    *out = b;
    return 0;
}

// ------------------------------------------------------------------------------------------
// streaming reader: family-complete chunks of a coordinate-sorted BAM, in bounded memory
// ------------------------------------------------------------------------------------------
namespace {
// (contig, position) as one ordered coordinate; unmapped (tid -1) sorts last
inline int64_t coord(int32_t tid, int32_t pos) {
    return tid < 0 ? INT64_MAX / 4 : ((int64_t)tid << 32) + (int64_t)pos;
}
struct StreamRec {
    int64_t off, len;  // the record's bytes in bsdc_bam_stream::buf
    int32_t fam;       // its MI family (stream-wide index); -1: deferred (left for bsdc_bam_stream_spill)
    int64_t c, seq;    // its coordinate and its place in the file (the spill's sort key)
};
// a TemplateCoordinate key, coarsely: (lower end's contig << 32 | other end's contig, lower end's
// position); BIG (0x7FFFFFFF) for an unmapped or absent mate, as the key's mate contig
using TcKey = std::pair<int64_t, int64_t>;
constexpr int64_t kBigTid = 0x7FFFFFFF;
constexpr int64_t kKeyDelta = 4;  // |key position before tools 1 + 2 - after| <= 2, twice
// a family whose coarse keys come this close to a deferred key may interleave with it in the exact
// TemplateCoordinate order (both sides' keys move by up to kKeyDelta; a deferred template's two
// records may estimate its key kKeyDelta apart): it is deferred too
constexpr int64_t kDeferMargin = 3 * kKeyDelta;
constexpr int kFamShards = 64;
inline int fam_shard(uint64_t h) { return (int)(h >> 58); }
// A record's coordinate c, its reach e (max of its own and its mate's coordinate) and its coarse
// TemplateCoordinate key: the template's lower end's contig, then the other end's (BIG for an
// unpaired record or unmapped mate), then the lower end's unclipped 5' position -- from the
// input's cigar and MC, so within kKeyDelta of the key of the records tools 1 and 2 make (a
// prepended base, an appended one, the RD trim).  r: a whole record (block_size first); mc: its MC
// value (empty if absent).
struct RecKey {
    int64_t c, e;
    TcKey key;
    int64_t m;  // the mate's coordinate (c when the mate is unmapped or absent)
    bool own;   // the key is this record's own end (the template's lower end), not its mate's
};
inline RecKey rec_key(const uint8_t *r, std::string_view mc) {
    const int l_name = r[12];
    const int n_cig = rd16(r + 16);
    const int32_t tid = rdi32(r + 4), pos = rdi32(r + 8), ntid = rdi32(r + 24), npos = rdi32(r + 28);
    const int flag = rd16(r + 18);
    const int64_t c = coord(tid, pos);
    const uint8_t *cg = r + 36 + l_name;
    int64_t lead = 0, trail = 0, reflen = 0;
    {
        int first_nc = -1, last_nc = -1;
        for (int i = 0; i < n_cig; i++) {
            const uint32_t op = rd32(cg + 4 * i) & 15;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) reflen += rd32(cg + 4 * i) >> 4;
            if (op != 4 && op != 5) {
                if (first_nc < 0) first_nc = i;
                last_nc = i;
            }
        }
        for (int i = 0; i < n_cig; i++) {
            const uint32_t op = rd32(cg + 4 * i) & 15;
            if (op != 4 && op != 5) continue;
            if (first_nc < 0 || i < first_nc) lead += rd32(cg + 4 * i) >> 4;
            else if (i > last_nc) trail += rd32(cg + 4 * i) >> 4;
        }
    }
    const int64_t p_own = (flag & 16) ? pos + reflen - 1 + trail : pos - lead;
    int64_t p_mate = npos;
    if (!mc.empty() && !(mc.size() == 1 && mc[0] == '*')) {
        int64_t mlead = 0, mref = 0, num = 0, clip_run = 0;  // clip_run: clips since the last non-clip op
        bool seen_nc = false;
        for (char ch : mc) {
            if (ch >= '0' && ch <= '9') {
                num = num * 10 + (ch - '0');
                continue;
            }
            if (ch == 'M' || ch == 'D' || ch == 'N' || ch == '=' || ch == 'X') mref += num;
            if (ch == 'S' || ch == 'H') {
                if (!seen_nc) mlead += num;
                else clip_run += num;
            } else {
                seen_nc = true;
                clip_run = 0;
            }
            num = 0;
        }
        p_mate = (flag & 32) ? npos + mref - 1 + clip_run : npos - mlead;
    }
    const bool paired = (flag & 1) && !(flag & 8) && ntid >= 0;
    const int64_t t1 = tid < 0 ? kBigTid : tid;
    TcKey key;
    bool own = true;
    if (!paired) key = {(t1 << 32) | kBigTid, p_own};
    else if (tid == ntid) key = {(t1 << 32) | t1, std::min(p_own, p_mate)}, own = p_own <= p_mate;
    else if (tid >= 0 && tid < ntid) key = {(t1 << 32) | (int64_t)ntid, p_own};
    else key = {((int64_t)ntid << 32) | t1, p_mate}, own = false;
    const int64_t m = ntid >= 0 ? coord(ntid, npos) : c;
    return RecKey{c, std::max(c, m), key, m, own};
}
// A far record (bsdc_bam_stream_set_defer): its template's key is a cross key (the mate on another
// contig, unmapped or absent: the key sorts at its contig's end) or its mate lies more than `span`
// positions away on the same contig.
inline bool far_record(const RecKey &k, int64_t span) {
    if ((k.key.first >> 32) != (k.key.first & 0xFFFFFFFFll)) return true;
    return (k.m > k.c ? k.m - k.c : k.c - k.m) > span;
}
struct StreamFam {
    int64_t lo = INT64_MAX, hi = INT64_MIN;  // min own position, max own or mate position (coord)
    TcKey klo{INT64_MAX, INT64_MAX}, khi{INT64_MIN, INT64_MIN};  // bounds of its records' keys
    int64_t n = 0;                           // buffered records
    bool def = false;  // deferred by adjacency (set_defer): its records go to the spill
    bool live() const { return n > 0; }
};
}  // namespace

struct bsdc_bam_stream {
    FILE *f = nullptr;
    bsdc_bam hdr;                 // header text and references only
    Bytes comp;    // compressed bytes read but not yet inflated (a partial block)
    // buf = [buffered records (recs) | inflated bytes not yet split, from `tail`]; inflated blocks
    // land at its end and records are split in place (no copy); `spare` keeps the capacity the
    // kept records move to when a chunk goes out
    int64_t tail = 0;
    Bytes spare;
    bool eof = false;
    int64_t read_size = 0;
    // buffered records (file order) and their families
    Bytes buf;
    std::vector<StreamRec> recs;
    // hash of the MI base -> family, in kFamShards shards by the hash's top bits (the shards are
    // filled in parallel, one thread each)
    std::vector<std::unordered_map<uint64_t, int32_t>> fam_of = std::vector<std::unordered_map<uint64_t, int32_t>>(kFamShards);
    std::unordered_map<std::string, int32_t> fam_exact;  // MI bases whose hash another live family holds
    std::vector<std::string> fam_key;               // per family: its MI base
    std::vector<StreamFam> fams;
    std::vector<int32_t> free_fams;
    int64_t cursor = INT64_MIN;  // the last record's position
    int64_t par_min = 1 << 14;   // records per split from which families are assigned in parallel
    double prof[5] = {0, 0, 0, 0, 0};  // seconds: fill, split, select, emit, parse (BSDC_STREAM_PROF)
    // chunks handed out and not yet recycled, and their buffers coming back: a chunk may be parsed
    // and copied out on another thread while this one reads the next (bsdc_bam_stream_next_raw);
    // the stream is deleted once it is closed and every chunk is back
    std::mutex mu;
    std::vector<Bytes> pool;  // returned chunk buffers (at most 2 kept)
    int64_t outstanding = 0;
    bool closed = false;
    // MI-run chunks (bsdc_bam_stream_next_runs): the MI value of the last record scanned
    std::string run_mi;
    // a record range of the file (bsdc_bam_stream_open_range): reading starts at a BGZF block and
    // drops skip_head inflated bytes, and stops at file offset `limit` (-1: the end), dropping the
    // last block's drop_tail bytes; fpos = the file offset read so far
    int64_t fpos = 0, limit = -1, skip_head = 0, drop_tail = 0;
    int64_t hdr_len = 0;  // the header's uncompressed bytes (the first record's offset)
    // a rank's key interval (bsdc_bam_stream_set_owner): -1 = every record
    int32_t own_rank = -1;
    std::vector<TcKey> own_bounds;
    std::vector<int64_t> own_coord;
    int64_t own_slack = 0;
    bool own_stop = false;
    // deferred templates (bsdc_bam_stream_set_defer): span 0 = off
    int64_t defer_span = 0;
    Bytes spill;                     // (bsdc_bam_stream_spill) {coordinate, seq, record} entries
    std::set<TcKey> dset;            // deferred keys near the emitted output (adjacency test)
    std::set<TcKey> dreg;            // every far template key registered (its far record's check)
    std::vector<TcKey> pend;         // deferred keys not yet reported (bsdc_bam_stream_splices)
    std::vector<TcKey> splices;      // the keys reported with the last chunk
    TcKey reach{INT64_MIN, INT64_MIN};  // the largest key emitted so far
    int64_t seq = 0;                 // records split so far (file order)
    int64_t st_dropped = 0, st_foreign = 0, st_spilled = 0, st_deferred = 0;
    int64_t st_peak = 0;  // the most record bytes buffered at a chunk selection (the memory bound)
    // statistics of the records split so far: count, first coordinate, max reach, key bounds
    int64_t st_n = 0, st_c0 = 0;
};

int32_t bsdc_bam_stream_open(const char *path, int32_t n_threads, int64_t read_size, bsdc_bam_stream **out) {
    *out = nullptr;
    set_threads(n_threads);
    FILE *f = fopen(path, "rb");
    if (!f) return fail(BSDC_IO_EIO, std::string("cannot open ") + path);
    auto *s = new bsdc_bam_stream();
    s->f = f;
    s->read_size = read_size > 0 ? read_size : ((int64_t)64 << 20);
    if (const char *e = getenv("BSDC_STREAM_PAR_MIN")) s->par_min = atoll(e);  // (tests: 0 = always parallel)
    // inflate until the header is whole
    for (;;) {
        int64_t p = 0;
        bsdc_bam probe;
        const bool have = s->buf.size() >= 12 &&
                          parse_header(s->buf.data(), (int64_t)s->buf.size(), &probe, &p) == 0;
        if (have) {
            s->hdr.header = probe.header;
            s->hdr.ref_names = probe.ref_names;
            s->hdr.ref_len = probe.ref_len;
            s->buf.erase(s->buf.begin(), s->buf.begin() + p);
            s->tail = 0;
            s->hdr_len = p;
            break;
        }
        if (s->eof) {
            const int64_t dn = (int64_t)s->buf.size();
            const int32_t rc = parse_header(s->buf.data(), dn, &probe, &p);
            bsdc_bam_stream_close(s);
            return rc != 0 ? rc : fail(BSDC_IO_EFORMAT, "missing BAM header");
        }
        const int32_t rc = bsdc_bam_stream_fill(s);
        if (rc != 0) {
            bsdc_bam_stream_close(s);
            return rc;
        }
    }
    *out = s;
    return 0;
}

namespace {
// The BGZF block header at comp[0, n): its total size, or -1 if these bytes are no block header.
int64_t bgzf_block_size(const uint8_t *h, int64_t n) {
    if (n < 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return -1;
    const int xlen = rd16(h + 10);
    if (n < 12 + xlen) return -1;
    for (int x = 0; x + 4 <= xlen;) {
        const uint8_t *sf = h + 12 + x;
        const int slen = rd16(sf + 2);
        if (sf[0] == 'B' && sf[1] == 'C' && slen == 2) return (int64_t)rd16(sf + 4) + 1;
        x += 4 + slen;
    }
    return -1;
}
}  // namespace

// A record range of a coordinate-sorted BAM as a stream (see include/bsdc_io.h).
int32_t bsdc_bam_stream_open_range(const char *path, int32_t n_threads, int64_t read_size, int64_t start_block,
                                   int64_t start_off, int64_t end_block, int64_t end_off, bsdc_bam_stream **out) {
    *out = nullptr;
    bsdc_bam_stream *s = nullptr;
    int32_t rc = bsdc_bam_stream_open(path, n_threads, read_size, &s);
    if (rc != 0) return rc;
    if (start_block < 0 && end_block >= 0) {  // the first range: from the file start, past the header
        start_block = 0;
        start_off = s->hdr_len;
    }
    if (start_block >= 0) {  // drop what the header read buffered; start at the block
        if (fseeko(s->f, (off_t)start_block, SEEK_SET) != 0) {
            bsdc_bam_stream_close(s);
            return fail(BSDC_IO_EIO, "seek failed");
        }
        s->comp.clear();
        s->buf.clear();
        s->tail = 0;
        s->eof = false;
        s->fpos = start_block;
        s->skip_head = start_off;
    }
    if (end_block >= 0) {
        if (start_block >= 0 ? end_block < start_block : false) {
            bsdc_bam_stream_close(s);
            return fail(BSDC_IO_EFORMAT, "bad record range");
        }
        if (end_off == 0) {  // the range ends where that block starts
            s->limit = end_block;
        } else {
            uint8_t h[64];
            FILE *g = fopen(path, "rb");
            const bool ok = g && fseeko(g, (off_t)end_block, SEEK_SET) == 0 && fread(h, 1, sizeof h, g) >= 18;
            int64_t bs = ok ? bgzf_block_size(h, sizeof h) : -1;
            uint8_t foot[4];
            const bool ok2 = bs > 0 && fseeko(g, (off_t)(end_block + bs - 4), SEEK_SET) == 0 && fread(foot, 1, 4, g) == 4;
            if (g) fclose(g);
            if (!ok2 || end_off > (int64_t)rd32(foot)) {
                bsdc_bam_stream_close(s);
                return fail(BSDC_IO_EFORMAT, "bad record range end");
            }
            s->limit = end_block + bs;
            s->drop_tail = (int64_t)rd32(foot) - end_off;
        }
        if (s->fpos >= s->limit) {  // (a header read that went past a range end inside the first block)
            bsdc_bam_stream_close(s);
            return fail(BSDC_IO_EFORMAT, "record range ends inside the header read; open it from a block");
        }
    }
    *out = s;
    return 0;
}

void bsdc_bam_stream_range_stats(const bsdc_bam_stream *s, int64_t *st) {
    st[0] = s->st_n;
    st[1] = s->st_c0;
    st[2] = s->st_dropped;
    st[3] = s->st_foreign;
    st[4] = s->st_spilled;
    st[5] = s->st_deferred;
    st[6] = s->st_peak;
}

int32_t bsdc_bam_stream_set_defer(bsdc_bam_stream *s, int64_t span) {
    if (!s || span < 0) return fail(BSDC_IO_EINVAL, "bad defer span");
    s->defer_span = span;
    return 0;
}

int64_t bsdc_bam_stream_spill(bsdc_bam_stream *s, uint8_t *dst) {
    const int64_t n = (int64_t)s->spill.size();
    if (dst) {
        if (n) memcpy(dst, s->spill.data(), (size_t)n);
        s->spill.clear();
    }
    return n;
}

int64_t bsdc_bam_stream_splices(bsdc_bam_stream *s, int64_t *dst) {
    const int64_t n = (int64_t)s->splices.size();
    if (dst) {
        for (int64_t i = 0; i < n; i++) {
            dst[2 * i] = s->splices[(size_t)i].first;
            dst[2 * i + 1] = s->splices[(size_t)i].second;
        }
        s->splices.clear();
    }
    return n;
}

namespace {
// A record starts at d[p] (dn bytes follow the stream start d): its length fields, names and
// cigar are consistent, and its bin is the one its position and cigar give (mapped records).
bool plausible_record(const uint8_t *d, int64_t dn, int64_t p, int32_t n_ref, int64_t *next) {
    if (p + 36 > dn) return false;
    const uint8_t *r = d + p;
    const int64_t bs = rd32(r);
    if (bs < 32 || bs > (1 << 26) || p + 4 + bs > dn) return false;
    const int32_t tid = rdi32(r + 4), pos = rdi32(r + 8), ntid = rdi32(r + 24), npos = rdi32(r + 28);
    if (tid < -1 || tid >= n_ref || ntid < -1 || ntid >= n_ref || pos < -1 || npos < -1) return false;
    const int l_name = r[12];
    const int n_cig = rd16(r + 16);
    const int32_t l_seq = rdi32(r + 20);
    if (l_name < 1 || l_seq < 0) return false;
    const int64_t body = 36 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + (int64_t)l_seq;
    if (body > 4 + bs) return false;
    if (r[36 + l_name - 1] != 0) return false;
    for (int i = 0; i < l_name - 1; i++)
        if (r[36 + i] < 33 || r[36 + i] > 126) return false;
    const uint8_t *cg = r + 36 + l_name;
    int64_t rl = 0;
    for (int i = 0; i < n_cig; i++) {
        const uint32_t op = rd32(cg + 4 * i) & 15;
        if (op > 8) return false;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += rd32(cg + 4 * i) >> 4;
    }
    if (tid >= 0 && pos >= 0) {  // SAMv1 reg2bin of [pos, end)
        const int64_t beg = pos, end = (rl > 0 ? pos + rl : pos + 1) - 1;
        int bin;
        if (beg >> 14 == end >> 14) bin = (int)(((1 << 15) - 1) / 7 + (beg >> 14));
        else if (beg >> 17 == end >> 17) bin = (int)(((1 << 12) - 1) / 7 + (beg >> 17));
        else if (beg >> 20 == end >> 20) bin = (int)(((1 << 9) - 1) / 7 + (beg >> 20));
        else if (beg >> 23 == end >> 23) bin = (int)(((1 << 6) - 1) / 7 + (beg >> 23));
        else if (beg >> 26 == end >> 26) bin = (int)(((1 << 3) - 1) / 7 + (beg >> 26));
        else bin = 0;
        if (rd16(r + 14) != bin) return false;
    }
    *next = p + 4 + bs;
    return true;
}
}  // namespace

// A rank boundary of a coordinate-sorted BAM after a file offset (see include/bsdc_io.h).
int32_t bsdc_bam_find_cut(const char *path, int32_t n_threads, int64_t from, int64_t min_span, int64_t slack,
                          int64_t guard, int64_t max_bytes, int64_t *out) {
    for (int i = 0; i < 7; i++) out[i] = -1;
    out[7] = 0;
    set_threads(n_threads);
    int32_t n_ref = 0;
    {
        bsdc_bam_stream *hs = nullptr;
        const int32_t rc = bsdc_bam_stream_open(path, 1, 1 << 20, &hs);
        if (rc != 0) return rc;
        n_ref = (int32_t)hs->hdr.ref_names.size();
        bsdc_bam_stream_close(hs);
    }
    FILE *f = fopen(path, "rb");
    if (!f) return fail(BSDC_IO_EIO, std::string("cannot open ") + path);
    fseeko(f, 0, SEEK_END);
    const int64_t fsize = (int64_t)ftello(f);
    // the first BGZF block at or after `from`: a header whose chain of block sizes runs on (4
    // blocks, or to the end of the file)
    int64_t blk = -1;
    {
        const int64_t win = std::min<int64_t>(fsize - from, (int64_t)4 << 20);
        Bytes w((size_t)std::max<int64_t>(win, 0));
        fseeko(f, (off_t)from, SEEK_SET);
        if (win > 0 && fread(w.data(), 1, w.size(), f) != w.size()) {
            fclose(f);
            return fail(BSDC_IO_EIO, "read error");
        }
        for (int64_t p = 0; p + 18 <= win && blk < 0; p++) {
            int64_t q = p;
            int okn = 0;
            while (okn < 4 && q < win) {
                const int64_t bs = bgzf_block_size(w.data() + q, win - q);
                if (bs < 28) break;
                q += bs;
                okn++;
            }
            if (okn >= 4 || (okn >= 1 && from + q == fsize)) blk = from + p;
        }
    }
    if (blk < 0) {  // no block starts in the window: the end of the file
        fclose(f);
        return 0;
    }
    // inflate from there, a few MB at a time, with a map of the blocks' uncompressed offsets
    Bytes comp, data;
    std::vector<int64_t> boff, uoff;  // per block inflated: file offset, offset in `data`
    int64_t fo = blk;
    bool feof_ = false;
    auto more = [&]() -> int32_t {
        if (feof_ || fo - blk >= max_bytes) return 1;
        const int64_t want = std::min<int64_t>((int64_t)4 << 20, fsize - fo);
        const size_t have = comp.size();
        comp.resize(have + (size_t)std::max<int64_t>(want, 0));
        fseeko(f, (off_t)fo, SEEK_SET);
        const size_t got = want > 0 ? fread(comp.data() + have, 1, (size_t)want, f) : 0;
        comp.resize(have + got);
        const int64_t comp_base = fo - (int64_t)have;  // file offset of comp[0]
        fo += (int64_t)got;
        if (fo >= fsize) feof_ = true;
        int64_t o = 0;  // the whole blocks of comp, listed, then inflated
        std::vector<int64_t> nb_off, nb_u;
        int64_t u = (int64_t)data.size();
        while (o < (int64_t)comp.size()) {
            const int64_t bs = bgzf_block_size(comp.data() + o, (int64_t)comp.size() - o);
            if (bs < 0) {
                if ((int64_t)comp.size() - o >= 18 + 256) return -1;
                break;
            }
            if (o + bs > (int64_t)comp.size()) break;
            nb_off.push_back(o);
            nb_u.push_back(u);
            u += rd32(comp.data() + o + bs - 4);
            o += bs;
        }
        int64_t used = 0;
        Bytes part;
        const int32_t rc = inflate_blocks(comp.data(), o, true, part, &used);
        if (rc != 0) return -1;
        data.insert(data.end(), part.begin(), part.end());
        for (size_t i = 0; i < nb_off.size(); i++) {
            boff.push_back(comp_base + nb_off[i]);
            uoff.push_back(nb_u[i]);
        }
        comp.erase(comp.begin(), comp.begin() + o);
        return 0;
    };
    auto vofs = [&](int64_t p, int64_t *b_, int64_t *o_) {  // a record's block and offset in it
        const size_t b = (size_t)(std::upper_bound(uoff.begin(), uoff.end(), p) - uoff.begin()) - 1;
        *b_ = boff[b];
        *o_ = p - uoff[b];
    };
    int32_t mr = more();
    if (mr < 0) {
        fclose(f);
        return fail(BSDC_IO_EFORMAT, "corrupt BGZF data");
    }
    // the first record boundary: the smallest offset where 8 records (or all the data left) chain
    int64_t sync = -1;
    for (;;) {
        const int64_t dn = (int64_t)data.size();
        for (int64_t p0 = 0; p0 + 36 <= std::min<int64_t>(dn, (int64_t)1 << 20) && sync < 0; p0++) {
            int64_t p = p0, nx = 0;
            int k = 0;
            while (k < 8 && plausible_record(data.data(), dn, p, n_ref, &nx)) {
                p = nx;
                k++;
            }
            if (k >= 8 || (k >= 1 && p == dn && feof_)) sync = p0;
        }
        if (sync >= 0) break;
        mr = more();
        if (mr != 0) break;
    }
    if (sync < 0) {  // no record starts in reach (the end of the file, or a record larger than max_bytes)
        fclose(f);
        return 0;
    }
    // records from the sync point: their offsets, coordinates and same-contig template keys
    std::vector<int64_t> roff, rc_;
    std::vector<int64_t> keys;  // key positions of the sync contig's same-contig templates
    int64_t p = sync, ctid = -2, x = -1;
    for (;;) {
        int64_t nx = 0;
        const int64_t dn = (int64_t)data.size();
        if (p + 4 > dn || p + 4 + (int64_t)rd32(data.data() + p) > dn) {
            mr = more();
            if (mr < 0) {
                fclose(f);
                return fail(BSDC_IO_EFORMAT, "corrupt BGZF data");
            }
            if (mr > 0) break;  // the end of the file / of max_bytes: no boundary
            continue;
        }
        if (!plausible_record(data.data(), dn, p, n_ref, &nx)) {
            fclose(f);
            return fail(BSDC_IO_EFORMAT, "malformed BAM record");
        }
        const uint8_t *r = data.data() + p;
        std::string_view mc;
        {
            const int64_t bs = rd32(r);
            const uint8_t *end = r + 4 + bs;
            const int l_name = r[12];
            const int n_cig = rd16(r + 16);
            const int32_t l_seq = rdi32(r + 20);
            const int64_t body = 36 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + (int64_t)l_seq;
            for (const uint8_t *a = r + body; a + 3 <= end;) {
                const int64_t vs = aux_value_size(a, end);
                if (vs < 0 || vs > (end - a) - 3) break;
                if (a[0] == 'M' && a[1] == 'C' && a[2] == 'Z') mc = std::string_view((const char *)a + 3, (size_t)vs - 1);
                a += 3 + vs;
            }
        }
        const RecKey rk = rec_key(r, mc);
        if (ctid == -2) ctid = rk.c >= INT64_MAX / 4 ? -1 : (rk.c >> 32);
        if (ctid < 0 || (rk.c >> 32) != ctid || rk.c >= INT64_MAX / 4) break;  // (a boundary stays inside a contig)
        roff.push_back(p);
        rc_.push_back(rk.c & 0xFFFFFFFFll);
        if (rk.key.first == ((ctid << 32) | ctid)) keys.push_back(rk.key.second);
        // a boundary x: at least min_span past the first record, no same-contig key within guard of
        // it, and every record still unread at least slack past x + guard (an unread record's key
        // is at least its position - slack)
        const int64_t cur = rk.c & 0xFFFFFFFFll;
        if (cur > rc_[0] + min_span + 2 * guard + slack && (int64_t)keys.size() > 1) {
            std::vector<int64_t> ks(keys);
            std::sort(ks.begin(), ks.end());
            const int64_t lo = rc_[0] + min_span;
            for (size_t i = 0; i + 1 < ks.size(); i++) {
                const int64_t cand = std::max(ks[i] + guard + 1, lo);
                if (cand + guard >= ks[i + 1]) continue;  // no room between these two keys
                if (cand + guard + slack >= cur) break;   // too near the unread records
                x = cand;
                break;
            }
            if (x >= 0) break;
        }
        p = nx;
    }
    if (x < 0) {
        fclose(f);
        return 0;
    }
    // the next rank's window starts at the first record at or past x - slack; this one's ends at
    // the first record at or past x + slack (windows overlap: a template's records near x are
    // read by both ranks and kept by the owner of its key)
    const int64_t ws = std::lower_bound(rc_.begin(), rc_.end(), x - slack) - rc_.begin();
    const int64_t we = std::lower_bound(rc_.begin(), rc_.end(), x + slack) - rc_.begin();
    if (ws >= (int64_t)roff.size() || we >= (int64_t)roff.size() || rc_[0] > x - slack) {
        fclose(f);
        return 0;
    }
    vofs(roff[(size_t)ws], &out[0], &out[1]);
    vofs(roff[(size_t)we], &out[2], &out[3]);
    out[4] = (ctid << 32) | ctid;
    out[5] = x;
    out[6] = (ctid << 32) + x;
    out[7] = 1;
    fclose(f);
    return 0;
}

// A rank's share of its window (bsdc_bam_stream_set_owner): the records whose TemplateCoordinate
// key lies in [bounds[rank - 1], bounds[rank]); a dropped record another rank cannot see (its
// coordinate outside that rank's window) is counted as foreign.
int32_t bsdc_bam_stream_set_owner(bsdc_bam_stream *s, int32_t rank, const int64_t *bounds, int32_t n_bounds,
                                  int64_t slack, int32_t flags) {
    if (!s || rank < 0 || rank > n_bounds || n_bounds < 0) return fail(BSDC_IO_EFORMAT, "bad rank");
    s->own_rank = rank;
    s->own_bounds.clear();
    for (int32_t i = 0; i < n_bounds; i++) s->own_bounds.push_back(TcKey{bounds[3 * i], bounds[3 * i + 1]});
    s->own_coord.clear();
    for (int32_t i = 0; i < n_bounds; i++) s->own_coord.push_back(bounds[3 * i + 2]);
    s->own_slack = slack;
    s->own_stop = (flags & BSDC_OWN_STOP_FOREIGN) != 0;
    return 0;
}

// Reads read_size more compressed bytes and inflates the whole blocks onto the end of buf.
int32_t bsdc_bam_stream_fill(bsdc_bam_stream *s) {
    if (s->eof) return 0;
    const size_t have = s->comp.size();
    const int64_t want = s->limit >= 0 ? std::min<int64_t>(s->read_size, std::max<int64_t>(s->limit - s->fpos, 0)) : s->read_size;
    s->comp.resize(have + (size_t)want);
    const size_t got = want > 0 ? fread(s->comp.data() + have, 1, (size_t)want, s->f) : 0;
    s->comp.resize(have + got);
    s->fpos += (int64_t)got;
    if (got < (size_t)want || (s->limit >= 0 && s->fpos >= s->limit)) {
        if (ferror(s->f)) return fail(BSDC_IO_EIO, "read error");
        s->eof = true;
    }
    const size_t before = s->buf.size();
    int64_t used = 0;
    const int32_t rc = inflate_blocks(s->comp.data(), (int64_t)s->comp.size(), s->eof, s->buf, &used);
    if (rc != 0) return rc;
    s->comp.erase(s->comp.begin(), s->comp.begin() + used);
    if (s->skip_head > 0 && s->buf.size() > before) {  // a range's first block: the bytes before its first record
        const int64_t k = std::min<int64_t>(s->skip_head, (int64_t)(s->buf.size() - before));
        s->buf.erase(s->buf.begin() + (int64_t)before, s->buf.begin() + (int64_t)before + k);
        s->skip_head -= k;
    }
    if (s->eof && s->drop_tail > 0) {  // a range's last block: the bytes past its end
        if ((int64_t)s->buf.size() - s->tail < s->drop_tail) return fail(BSDC_IO_EFORMAT, "bad range end");
        s->buf.resize(s->buf.size() - (size_t)s->drop_tail);
        s->drop_tail = 0;
    }
    return 0;
}

namespace {
// The live family of an MI base, or -1 (no family is created)
int32_t find_fam(bsdc_bam_stream *s, std::string_view mi, uint64_t h) {
    if (!s->fam_exact.empty()) {
        auto ie = s->fam_exact.find(std::string(mi));
        if (ie != s->fam_exact.end() && s->fams[(size_t)ie->second].live()) return ie->second;
    }
    const auto &fm = s->fam_of[(size_t)fam_shard(h)];
    auto it = fm.find(h);
    if (it != fm.end() && s->fams[(size_t)it->second].live() && s->fam_key[(size_t)it->second] == mi) return it->second;
    return -1;
}
// A deferred key (bsdc_bam_stream_set_defer): kept for the adjacency test and reported as a splice
// point with the chunk whose keys reach past it.  A key at or behind what was already emitted (a far
// record whose template's lower record was never read) cannot be spliced: an error.
int32_t defer_key(bsdc_bam_stream *s, const TcKey &k) {
    if (k.first < s->reach.first || (k.first == s->reach.first && k.second <= s->reach.second + 2 * kKeyDelta))
        return fail(BSDC_IO_EFORMAT, "a template whose other end lies far away has its lower record missing or "
                                     "behind the output already written; read the file whole instead");
    if (s->dset.insert(k).second) s->pend.push_back(k);
    return 0;
}
// a spill entry: {coordinate, file sequence} (the pass-2 sort key), then the record
void spill_record(bsdc_bam_stream *s, const uint8_t *r, int64_t c, int64_t seq) {
    const int64_t len = 4 + (int64_t)rd32(r);
    const size_t at = s->spill.size();
    s->spill.resize(at + 16 + (size_t)len);
    memcpy(s->spill.data() + at, &c, 8);
    memcpy(s->spill.data() + at + 8, &seq, 8);
    memcpy(s->spill.data() + at + 16, r, (size_t)len);
    s->st_spilled++;
}
// Family m (buffered, complete, owned) turns deferred: its key range is registered; its records
// follow with spill_deferred.
int32_t defer_family(bsdc_bam_stream *s, int32_t m) {
    StreamFam &F = s->fams[(size_t)m];
    F.def = true;
    s->st_deferred++;
    const int32_t rc = defer_key(s, F.klo);
    if (rc == 0) s->dset.insert(F.khi);  // (the range's upper end: adjacency only, not a splice point)
    return rc;
}
// The buffered records s->recs[0, upto) of deferred families to the spill (they are owned: a rank
// drops the others before family assignment); they leave their families' counts.
void spill_deferred(bsdc_bam_stream *s, size_t upto) {
    for (size_t i = 0; i < upto; i++) {
        StreamRec &r = s->recs[i];
        if (r.fam < 0 || !s->fams[(size_t)r.fam].def) continue;
        spill_record(s, s->buf.data() + r.off, r.c, r.seq);
        s->fams[(size_t)r.fam].n--;
        r.fam = -1;
    }
}

// The whole records of buf's unsplit tail added to the buffered records, each with its MI family.  A record's family
// is its MI base (the MI up to the first '/', as the reader interns it); a record without MI is a
// family of its own.  With set_defer, a far record (far_record) -- and every record of its MI family,
// buffered or to come -- goes to the spill instead (a rank: the far records of its core coordinates,
// and the near ones it owns), and its keys are registered (defer_key).
int32_t stream_split(bsdc_bam_stream *s) {
    uint8_t *d = s->buf.data() + s->tail;
    const int64_t dn = (int64_t)s->buf.size() - s->tail;
    // record boundaries (sequential), then each record's family key and positions (parallel)
    std::vector<int64_t> starts;
    int64_t p = 0;
    while (p + 4 <= dn) {
        const int64_t bs = rd32(d + p);
        if (bs < 32) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
        if (p + 4 + bs > dn) break;
        starts.push_back(p);
        p += 4 + bs;
    }
    int64_t nr = (int64_t)starts.size();
    const bool defer = s->defer_span > 0;
    struct Parsed {
        std::string_view mi;
        uint64_t h;  // hash of mi
        int64_t c, e;
        TcKey key;
        int64_t seq;   // the record's place in the file (split order)
        uint8_t far;   // far_record (set_defer)
        uint8_t own;   // the key is the record's own end
    };
    std::vector<Parsed> P((size_t)nr);
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < nr; k++) {
        const uint8_t *r = d + starts[(size_t)k];
        const int64_t bs = rd32(r);
        const uint8_t *end = r + 4 + bs;
        const int l_name = r[12];
        const int n_cig = rd16(r + 16);
        const int32_t l_seq = rdi32(r + 20);
        const int64_t body = 36 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + (int64_t)l_seq;
        if (l_seq < 0 || l_name < 1 || body > 4 + bs) {
            bad |= 1;
            continue;
        }
        std::string_view mi, mc;
        for (const uint8_t *a = r + body; a + 3 <= end;) {
            const int64_t vs = aux_value_size(a, end);
            if (vs < 0 || vs > (end - a) - 3) {
                bad |= 1;
                break;
            }
            if (a[0] == 'M' && a[1] == 'I' && a[2] == 'Z') mi = std::string_view((const char *)a + 3, (size_t)vs - 1);
            if (a[0] == 'M' && a[1] == 'C' && a[2] == 'Z') mc = std::string_view((const char *)a + 3, (size_t)vs - 1);
            a += 3 + vs;
        }
        const size_t slash = mi.find('/');
        if (slash != std::string_view::npos) mi = mi.substr(0, slash);
        const RecKey rk = rec_key(r, mc);
        P[(size_t)k] = Parsed{mi, std::hash<std::string_view>{}(mi), rk.c, rk.e, rk.key, s->seq + k,
                              (uint8_t)(defer && far_record(rk, s->defer_span)), (uint8_t)rk.own};
    }
    if (bad) return fail(BSDC_IO_EFORMAT, "malformed BAM record (lengths or aux)");
    s->seq += nr;
    // per record: 0 buffered, 1 dropped (another rank's), 2 far (family marking; spilled if `core`)
    std::vector<uint8_t> cls((size_t)nr, 0), core((size_t)nr, 1), owned((size_t)nr, 1);
    if (s->own_rank >= 0 && nr > 0) {  // a rank: the records of its key interval only
        const auto &bd = s->own_bounds;
        // this rank's core coordinates (its own share of the file: the far records it spills)
        const int64_t core_lo = s->own_rank == 0 ? INT64_MIN : s->own_coord[(size_t)s->own_rank - 1];
        const int64_t core_hi = s->own_rank == (int)bd.size() ? INT64_MAX : s->own_coord[(size_t)s->own_rank];
        for (int64_t k = 0; k < nr; k++) {
            const Parsed &q = P[(size_t)k];
            const int owner = (int)(std::upper_bound(bd.begin(), bd.end(), q.key) - bd.begin());
            owned[(size_t)k] = owner == s->own_rank;
            if (q.far) {
                // a template reaching past the windows: every rank marks its MI family, the rank
                // whose core holds the record spills it, the key's owner registers the key
                cls[(size_t)k] = 2;
                core[(size_t)k] = q.c >= core_lo && q.c < core_hi;
                continue;
            }
            if (owned[(size_t)k]) continue;
            cls[(size_t)k] = 1;
            s->st_dropped++;
            // the owner reads the coordinates [its lower bound - slack, its upper bound + slack)
            const int64_t lo = owner == 0 ? INT64_MIN : s->own_coord[(size_t)owner - 1] - s->own_slack;
            const int64_t hi = owner == (int)bd.size() ? INT64_MAX : s->own_coord[(size_t)owner] + s->own_slack;
            if (q.c < lo || q.c >= hi) s->st_foreign++;
        }
        if (s->own_stop && s->st_foreign > 0)
            return fail(BSDC_IO_EFORMAT, "foreign record: a record another rank owns but never reads (its template "
                                         "reaches past the windows and deferral is off)");
    } else if (defer) {
        for (int64_t k = 0; k < nr; k++)
            if (P[(size_t)k].far) cls[(size_t)k] = 2;
    }
    int64_t call = INT64_MIN;  // (the cursor passes the dropped records too)
    for (int64_t k = 0; k < nr; k++) call = std::max(call, P[(size_t)k].c);
    if (nr > 0 && s->st_n == 0) s->st_c0 = P[0].c;  // (the range statistics: bsdc_bam_stream_range_stats)
    s->st_n += nr;
    bool any_drop = false;
    for (int64_t k = 0; k < nr && !any_drop; k++) any_drop = cls[(size_t)k] == 1;
    if (any_drop) {  // the other records moved together (a record's MI view moves with it)
        int64_t wp = 0, m = 0;
        for (int64_t k = 0; k < nr; k++) {
            if (cls[(size_t)k] == 1) continue;
            const int64_t st = starts[(size_t)k], len = 4 + (int64_t)rd32(d + st);
            const int64_t mo = P[(size_t)k].mi.empty() ? 0 : (const uint8_t *)P[(size_t)k].mi.data() - (d + st);
            if (wp != st) memmove(d + wp, d + st, (size_t)len);
            P[(size_t)m] = P[(size_t)k];
            cls[(size_t)m] = cls[(size_t)k];
            core[(size_t)m] = core[(size_t)k];
            owned[(size_t)m] = owned[(size_t)k];
            if (!P[(size_t)m].mi.empty()) P[(size_t)m].mi = std::string_view((const char *)d + wp + mo, P[(size_t)m].mi.size());
            starts[(size_t)m] = wp;
            wp += len;
            m++;
        }
        if (wp != p) {  // the partial record after them, and the buffer's end
            memmove(d + wp, d + p, (size_t)(dn - p));
            s->buf.resize((size_t)(s->tail + wp + (dn - p)));
        }
        nr = m;
        P.resize((size_t)m);
        starts.resize((size_t)m);
        p = wp;
        if (nr == 0) {
            s->cursor = std::max(s->cursor, call);
            return 0;
        }
    }
    // families (sequential: the MI map), then the records' bytes in one copy
    auto new_fam = [&]() {
        int32_t fam;
        if (!s->free_fams.empty()) {
            fam = s->free_fams.back();
            s->free_fams.pop_back();
            s->fams[(size_t)fam] = StreamFam();
        } else {
            fam = (int32_t)s->fams.size();
            s->fams.emplace_back();
            s->fam_key.emplace_back();
        }
        return fam;
    };
    // the family of an MI base: the map holds hashes and each family keeps its key; a key whose
    // hash a different live key holds (a 64-bit collision) goes to the exact map, looked up first
    auto fam_of_mi = [&](std::string_view mi, uint64_t h) {
        if (!s->fam_exact.empty()) {
            auto ie = s->fam_exact.find(std::string(mi));
            if (ie != s->fam_exact.end() && s->fams[(size_t)ie->second].live()) return ie->second;
        }
        auto &fm = s->fam_of[(size_t)fam_shard(h)];
        auto it = fm.find(h);
        if (it != fm.end() && s->fams[(size_t)it->second].live() && s->fam_key[(size_t)it->second] == mi)
            return it->second;
        const int32_t fam = new_fam();
        s->fam_key[(size_t)fam].assign(mi.data(), mi.size());
        if (it == fm.end()) fm.emplace(h, fam);
        else if (!s->fams[(size_t)it->second].live()) it->second = fam;
        else s->fam_exact[std::string(mi)] = fam;  // collision with a live family
        return fam;
    };
    const int64_t base = s->tail;
    std::vector<int32_t> famv((size_t)nr);
    if (nr > 0 && nr >= s->par_min && s->fam_exact.empty()) {
        // ---- the same in parallel: families by hash shard (a family's records all fall in one
        // shard), new families numbered in shard order, 64-bit collisions resolved serially ----
        int unsorted = 0;
#pragma omp parallel for schedule(static) reduction(| : unsorted)
        for (int64_t k = 0; k < nr; k++)
            unsorted |= P[(size_t)k].c < (k > 0 ? P[(size_t)k - 1].c : s->cursor);
        if (unsorted)
            return fail(BSDC_IO_EFORMAT, "input is not coordinate-sorted (the streaming step needs the "
                                         "coordinate order of the step-5 input; read it whole instead)");
        constexpr int S = kFamShards;  // + bucket S: records without MI; S + 1: far records (none)
        std::vector<int64_t> sstart(S + 3, 0);
        std::vector<uint8_t> shard_of((size_t)nr);
        for (int64_t k = 0; k < nr; k++) {
            const int sh = cls[(size_t)k] == 2 ? S + 1 : P[(size_t)k].mi.empty() ? S : fam_shard(P[(size_t)k].h);
            shard_of[(size_t)k] = (uint8_t)sh;
            sstart[(size_t)sh + 1]++;
            if (sh == S + 1) famv[(size_t)k] = -9;
        }
        for (int sh = 0; sh <= S + 1; sh++) sstart[(size_t)sh + 1] += sstart[(size_t)sh];
        std::vector<int64_t> sorder((size_t)nr), sfill(sstart.begin(), sstart.end() - 1);
        for (int64_t k = 0; k < nr; k++) sorder[(size_t)sfill[shard_of[(size_t)k]]++] = k;
        // fam[k]: >= 0 an existing family; -1 no MI; -2 a collision; <= -3 new family -3 - i of the shard
        std::vector<std::vector<int64_t>> newfirst(S + 1);
#pragma omp parallel for schedule(dynamic, 1)
        for (int sh = 0; sh <= S; sh++) {
            if (sh == S) {
                for (int64_t i = sstart[S]; i < sstart[S + 1]; i++) famv[(size_t)sorder[(size_t)i]] = -1;
                continue;
            }
            auto &fm = s->fam_of[(size_t)sh];
            std::unordered_map<uint64_t, int32_t> nw;
            std::vector<int64_t> &nf = newfirst[(size_t)sh];
            for (int64_t i = sstart[(size_t)sh]; i < sstart[(size_t)sh + 1]; i++) {
                const int64_t k = sorder[(size_t)i];
                const Parsed &q = P[(size_t)k];
                auto it = fm.find(q.h);
                if (it != fm.end() && s->fams[(size_t)it->second].live()) {
                    famv[(size_t)k] = s->fam_key[(size_t)it->second] == q.mi ? it->second : -2;
                    continue;
                }
                auto jt = nw.find(q.h);
                if (jt == nw.end()) {
                    nw.emplace(q.h, (int32_t)nf.size());
                    famv[(size_t)k] = -3 - (int32_t)nf.size();
                    nf.push_back(k);
                } else {
                    famv[(size_t)k] = P[(size_t)nf[(size_t)jt->second]].mi == q.mi ? -3 - jt->second : -2;
                }
            }
        }
        // new families get ids (free list first), shard by shard; then the records without MI and
        // the collisions, in file order (the exact map)
        std::vector<std::vector<int32_t>> gid(S);
        std::vector<uint8_t> fresh;  // families created by this split (live before their records count)
        auto mark_fresh = [&](int32_t f) {
            if ((size_t)f >= fresh.size()) fresh.resize((size_t)f + 1, 0);
            fresh[(size_t)f] = 1;
        };
        for (int sh = 0; sh < S; sh++)
            for (size_t i = 0; i < newfirst[(size_t)sh].size(); i++) {
                const int32_t f = new_fam();
                mark_fresh(f);
                gid[(size_t)sh].push_back(f);
            }
#pragma omp parallel for schedule(dynamic, 1)
        for (int sh = 0; sh < S; sh++) {  // their keys and map entries (a stale entry is taken over)
            auto &fm = s->fam_of[(size_t)sh];
            const std::vector<int64_t> &nf = newfirst[(size_t)sh];
            for (size_t i = 0; i < nf.size(); i++) {
                const Parsed &q = P[(size_t)nf[i]];
                const int32_t f = gid[(size_t)sh][i];
                s->fam_key[(size_t)f].assign(q.mi.data(), q.mi.size());
                fm[q.h] = f;
            }
        }
        for (int64_t k = 0; k < nr; k++) {
            if (famv[(size_t)k] == -1) {
                famv[(size_t)k] = new_fam();
                mark_fresh(famv[(size_t)k]);
            } else if (famv[(size_t)k] == -2) {
                const std::string key(P[(size_t)k].mi);
                auto ie = s->fam_exact.find(key);
                if (ie != s->fam_exact.end() &&
                    (s->fams[(size_t)ie->second].live() || ((size_t)ie->second < fresh.size() && fresh[(size_t)ie->second]))) {
                    famv[(size_t)k] = ie->second;
                } else {
                    const int32_t f = new_fam();
                    mark_fresh(f);
                    s->fam_key[(size_t)f] = key;
                    s->fam_exact[key] = f;
                    famv[(size_t)k] = f;
                }
            }
        }
        // ids and per-family bounds, shard by shard (disjoint families)
#pragma omp parallel for schedule(dynamic, 1)
        for (int sh = 0; sh <= S; sh++) {
            for (int64_t i = sstart[(size_t)sh]; i < sstart[(size_t)sh + 1]; i++) {
                const int64_t k = sorder[(size_t)i];
                int32_t &f = famv[(size_t)k];
                if (f <= -3) f = gid[(size_t)sh][(size_t)(-3 - f)];
                const Parsed &q = P[(size_t)k];
                StreamFam &F = s->fams[(size_t)f];
                F.lo = std::min(F.lo, q.c);
                F.hi = std::max(F.hi, q.e);
                F.klo = std::min(F.klo, q.key);
                F.khi = std::max(F.khi, q.key);
                F.n++;
            }
        }
    } else {
        for (int64_t k = 0; k < nr; k++) {
            const Parsed &q = P[(size_t)k];
            if (q.c < s->cursor)
                return fail(BSDC_IO_EFORMAT, "input is not coordinate-sorted (the streaming step needs the "
                                             "coordinate order of the step-5 input; read it whole instead)");
            s->cursor = std::max(s->cursor, q.c);
            if (cls[(size_t)k] == 2) continue;  // (a far record: its family, if any, below)
            const int32_t fam = !q.mi.empty() ? fam_of_mi(q.mi, q.h) : new_fam();  // (no MI: a family of its own)
            StreamFam &F = s->fams[(size_t)fam];
            F.lo = std::min(F.lo, q.c);
            F.hi = std::max(F.hi, q.e);
            F.klo = std::min(F.klo, q.key);
            F.khi = std::max(F.khi, q.key);
            F.n++;
            s->cursor = std::max(s->cursor, q.c);
            famv[(size_t)k] = fam;
        }
    }
    // the records, in file order: buffered with their family, or (a far record) deferred -- unless
    // its MI family is buffered (a molecule whose other templates are near): it joins that family,
    // so one MI never straddles the stream and the spill over a key gap it would not straddle in the
    // whole file's order
    for (int64_t k = 0; k < nr; k++) {
        const Parsed &q = P[(size_t)k];
        int32_t f = famv[(size_t)k];
        if (cls[(size_t)k] == 2) {
            f = q.mi.empty() ? -1 : find_fam(s, q.mi, q.h);
            if (f < 0) {
                // the template's key comes with its lower record (the other one finds it registered);
                // a record whose lower record never came registers it if still ahead of the output.
                // A rank registers no cross key (its lower record may lie in an earlier rank's core,
                // and the key sorts at its contig's end, past this rank's output by the time the
                // upper record comes): a rank's output is cut at every change of the key's contig
                // pair instead (bam._stream_step regions), which is where those families go.
                const bool cross = (q.key.first >> 32) != (q.key.first & 0xFFFFFFFFll);
                if (owned[(size_t)k] && !(cross && s->own_rank >= 0) && (q.own || !s->dreg.count(q.key))) {
                    const int32_t rc = defer_key(s, q.key);
                    if (rc != 0) return rc;
                    s->dreg.insert(q.key);
                }
                if (core[(size_t)k]) spill_record(s, d + starts[(size_t)k], q.c, q.seq);
                continue;
            }
            if (!owned[(size_t)k])  // (another rank's template whose MI this rank buffers: not a rank's to join)
                return fail(BSDC_IO_EFORMAT, "a far record of an MI family another rank owns");
            StreamFam &F = s->fams[(size_t)f];
            F.lo = std::min(F.lo, q.c);
            F.hi = std::max(F.hi, q.e);
            F.klo = std::min(F.klo, q.key);
            F.khi = std::max(F.khi, q.key);
            F.n++;
        }
        const int64_t len = (k + 1 < nr ? starts[(size_t)k + 1] : p) - starts[(size_t)k];
        s->recs.push_back(StreamRec{base + starts[(size_t)k], len, f, q.c, q.seq});
    }
    s->cursor = std::max(s->cursor, call);
    s->tail += p;
    return 0;
}
}  // namespace

// The next chunk (see include/bsdc_io.h): the buffered records of every family that is complete
// and whose TemplateCoordinate keys all sort before any key still to come, once they reach
// min_bytes (everything left at the end of the file).  Per family m: hi_m = its highest record
// or mate position; m is complete once the stream has passed hi_m + slack (a family's templates
// share their coordinates; slack > any read's reference span plus clips).  Its records' keys lie
// within [klo_m, khi_m] up to kKeyDelta in the position.  T = the least key a record not yet
// emitted can have: (cursor contig, cursor contig, cursor - slack) for the records still unread,
// klo_m - kKeyDelta of the incomplete families and of the complete ones kept back; a complete
// family goes out when khi_m + kKeyDelta < T.  (Templates whose mate is on another contig or unmapped sort after every
// template of their contig with both ends on it, so they wait for the contig's end.)
int32_t bsdc_bam_stream_next_raw(bsdc_bam_stream *s, int64_t min_bytes, int64_t slack, bsdc_bam **out) {
    *out = nullptr;
    std::vector<uint8_t> take;  // per buffered family: goes out now
    // room for a chunk, what stays behind and the fills in flight, reserved once (no regrowth,
    // no fresh pages per fill); a recycled chunk buffer serves when one is back
    const size_t want = (size_t)std::max<int64_t>(min_bytes, 0) * 5 / 4 + (size_t)s->read_size * 16;
    if (s->buf.capacity() < want) s->buf.reserve(want);
    if (s->spare.capacity() < want) {
        std::lock_guard<std::mutex> lk(s->mu);
        for (auto &v : s->pool)
            if (v.capacity() >= want) {
                s->spare.swap(v);
                break;
            }
    }
    if (s->spare.capacity() < want) s->spare.reserve(want);
    for (;;) {
        double t0 = now_s();
        int32_t rc = stream_split(s);
        if (rc != 0) return rc;
        s->prof[1] += now_s() - t0;
        t0 = now_s();
        const bool end = s->eof && s->comp.empty();
        if (end && s->tail < (int64_t)s->buf.size()) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
        if (!end && s->tail < min_bytes) {  // a chunk takes >= min_bytes of the buffered records:
            s->prof[2] += now_s() - t0;     // not there yet, so no selection until the next fill
            t0 = now_s();
            rc = bsdc_bam_stream_fill(s);
            if (rc != 0) return rc;
            s->prof[0] += now_s() - t0;
            continue;
        }
        {
            int64_t held = 0;
            for (const auto &r : s->recs) held += r.fam >= 0 ? r.len : 0;
            s->st_peak = std::max(s->st_peak, held);
        }
        take.assign(s->fams.size(), 0);
        int64_t bytes = 0;
        TcKey chunk_reach{INT64_MIN, INT64_MIN};
        if (end) {  // every family is complete and nothing is left to read
            for (size_t m = 0; m < s->fams.size(); m++) take[m] = s->fams[m].n > 0;
        } else if (s->cursor != INT64_MIN) {
            const int64_t ct = s->cursor >> 32, cp = s->cursor & 0xFFFFFFFFll;
            const int64_t ctid = s->cursor >= INT64_MAX / 4 ? kBigTid : ct;
            // records still unread start at or after the cursor: their keys' positions are at
            // least cursor - slack (a leading clip, a mate's reverse 5' end)
            TcKey T{(ctid << 32) | ctid, (s->cursor >= INT64_MAX / 4 ? 0 : cp) - slack};
            auto lo_of = [&](const StreamFam &F) { return TcKey{F.klo.first, F.klo.second - kKeyDelta}; };
            auto hi_of = [&](const StreamFam &F) { return TcKey{F.khi.first, F.khi.second + kKeyDelta}; };
            for (size_t m = 0; m < s->fams.size(); m++) {
                const StreamFam &F = s->fams[m];
                if (F.n > 0 && F.hi + slack >= s->cursor) T = std::min(T, lo_of(F));  // incomplete
            }
            for (bool moved = true; moved;) {  // complete ones kept back lower T in turn
                moved = false;
                for (size_t m = 0; m < s->fams.size(); m++) {
                    const StreamFam &F = s->fams[m];
                    if (F.n > 0 && F.hi + slack < s->cursor && !(hi_of(F) < T) && lo_of(F) < T) {
                        T = lo_of(F);
                        moved = true;
                    }
                }
            }
            for (size_t m = 0; m < s->fams.size(); m++) {
                const StreamFam &F = s->fams[m];
                take[m] = F.n > 0 && F.hi + slack < s->cursor && hi_of(F) < T;
            }
        }
        if (s->defer_span > 0 && !s->dset.empty()) {
            // a family whose keys come within kDeferMargin of a deferred key may interleave with it
            // in TemplateCoordinate order: it is deferred too (and its keys then defer its own
            // neighbours), so that the stream's and the spill's families are each whole
            std::vector<int32_t> nd;
            for (bool more = true; more;) {
                more = false;
                for (size_t m = 0; m < s->fams.size(); m++) {
                    if (!take[m]) continue;
                    const StreamFam &F = s->fams[m];
                    auto it = s->dset.lower_bound(TcKey{F.klo.first, F.klo.second - kDeferMargin});
                    if (it == s->dset.end() || TcKey{F.khi.first, F.khi.second + kDeferMargin} < *it) continue;
                    take[m] = 0;
                    const int32_t rc = defer_family(s, (int32_t)m);
                    if (rc != 0) return rc;
                    nd.push_back((int32_t)m);
                    more = true;
                }
            }
            if (!nd.empty()) {
                spill_deferred(s, s->recs.size());
                for (int32_t m : nd) {  // (their records are in the spill: the families are done)
                    s->fams[(size_t)m].def = false;
                    s->free_fams.push_back(m);
                }
            }
        }
        {
            // bounded chunks: of the families that may go, only a key prefix of about min_bytes,
            // cut between two families whose key ranges do not meet (the rest stays for the next
            // call, where it may go again)
            std::vector<int64_t> fb(s->fams.size(), 0);
            for (auto &r : s->recs)
                if (r.fam >= 0) fb[(size_t)r.fam] += take[(size_t)r.fam] ? r.len : 0;
            std::vector<int32_t> ord;
            for (size_t m = 0; m < s->fams.size(); m++)
                if (take[m]) ord.push_back((int32_t)m);
            std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return s->fams[(size_t)a].klo < s->fams[(size_t)b].klo; });
            TcKey reach{INT64_MIN, INT64_MIN};
            size_t i = 0;
            for (; i < ord.size(); i++) {
                const StreamFam &F = s->fams[(size_t)ord[i]];
                if (bytes > 0 && bytes >= min_bytes && reach < TcKey{F.klo.first, F.klo.second - 2 * kKeyDelta}) break;
                bytes += fb[(size_t)ord[i]];
                reach = std::max(reach, F.khi);
            }
            for (; i < ord.size(); i++) take[(size_t)ord[i]] = 0;
            chunk_reach = reach;
        }
        s->prof[2] += now_s() - t0;
        t0 = now_s();
        if (end || (bytes > 0 && bytes >= min_bytes)) {
            if (bytes == 0) {  // the end of the stream: every deferred key left is a splice after the last chunk
                std::sort(s->pend.begin(), s->pend.end());
                s->splices = s->pend;
                s->pend.clear();
                return 0;
            }
            // the deferred keys this chunk's families reach past: its output is cut before each
            if (chunk_reach > s->reach) s->reach = chunk_reach;
            std::sort(s->pend.begin(), s->pend.end());
            const size_t np = (size_t)(std::upper_bound(s->pend.begin(), s->pend.end(), s->reach) - s->pend.begin());
            s->splices.assign(s->pend.begin(), s->pend.begin() + (ptrdiff_t)np);
            s->pend.erase(s->pend.begin(), s->pend.begin() + (ptrdiff_t)np);
            // keys far enough behind the output cannot meet a family still to come
            s->dset.erase(s->dset.begin(), s->dset.lower_bound(TcKey{s->reach.first, s->reach.second - 4 * kDeferMargin}));
            auto *b = new bsdc_bam();
            b->header = s->hdr.header;
            b->ref_names = s->hdr.ref_names;
            b->ref_len = s->hdr.ref_len;
            // destinations by prefix sums (taken records to the chunk, the rest to `spare`, then
            // the unsplit tail after them), then the copies in parallel
            // the chunk takes the whole buffer (its records stay where they are, listed in file
            // order); the records kept back and the unsplit tail move to `spare`, the next buffer
            const int64_t nrec = (int64_t)s->recs.size();
            std::vector<int64_t> src_k;
            std::vector<StreamRec> krecs;
            b->rec_start.reserve((size_t)nrec);
            int64_t ok = 0;
            for (int64_t i = 0; i < nrec; i++) {
                const StreamRec &r = s->recs[(size_t)i];
                if (r.fam < 0) continue;  // (deferred: in the spill)
                if (take[(size_t)r.fam]) {
                    b->rec_start.push_back(r.off);
                } else {
                    src_k.push_back(r.off);
                    krecs.push_back(StreamRec{ok, r.len, r.fam, r.c, r.seq});
                    ok += r.len;
                }
            }
            const int64_t tail_n = (int64_t)s->buf.size() - s->tail;
            s->spare.resize((size_t)(ok + tail_n));
            const int64_t nk = (int64_t)krecs.size();
#pragma omp parallel for schedule(dynamic, 1024)
            for (int64_t i = 0; i < nk; i++)
                memcpy(s->spare.data() + krecs[(size_t)i].off, s->buf.data() + src_k[(size_t)i], (size_t)krecs[(size_t)i].len);
            if (tail_n > 0) memcpy(s->spare.data() + ok, s->buf.data() + s->tail, (size_t)tail_n);
            const int64_t dn = (int64_t)s->buf.size();
            b->data.swap(s->buf);
            b->data.resize((size_t)dn + 8);
    memset(b->data.data() + dn, 0, 8);  // the pad (a no-init buffer)
            for (size_t m = 0; m < s->fams.size(); m++)
                if (take[m]) {
                    s->fams[m].n = 0;
                    s->free_fams.push_back((int32_t)m);
                }
#pragma omp parallel for schedule(dynamic, 1)
            for (int sh = 0; sh < kFamShards; sh++) {  // forget the emitted MI bases
                auto &fm = s->fam_of[(size_t)sh];
                for (auto it = fm.begin(); it != fm.end();)
                    it = !s->fams[(size_t)it->second].live() ? fm.erase(it) : std::next(it);
            }
            for (auto it = s->fam_exact.begin(); it != s->fam_exact.end();)
                it = !s->fams[(size_t)it->second].live() ? s->fam_exact.erase(it) : std::next(it);
            s->buf.swap(s->spare);  // (spare is now the chunk's old, empty vector: reserved on the next call)
            s->tail = ok;
            s->recs.swap(krecs);
            s->prof[3] += now_s() - t0;
            b->dn = dn;
            b->parsed = false;
            {
                std::lock_guard<std::mutex> lk(s->mu);
                s->outstanding++;
            }
            *out = b;
            return 0;
        }
        rc = bsdc_bam_stream_fill(s);
        if (rc != 0) return rc;
        s->prof[0] += now_s() - t0;
    }
}

// The next chunk of a GroupReadsByUmi-ordered stream (include/bsdc_io.h): a prefix of the
// buffered records cut at the first record, at or past min_bytes, whose MI value differs from the
// one before it, so no run of one MI tag (fgbio CallMolecularConsensusReads' unit) straddles two
// chunks.  No family bookkeeping and no coordinate order: the records are listed by the parse.
// s->tail = the bytes of whole records scanned (all of them in one run with s->run_mi, when the
// scan did not find a cut).
int32_t bsdc_bam_stream_next_runs(bsdc_bam_stream *s, int64_t min_bytes, bsdc_bam **out) {
    *out = nullptr;
    if (!s->recs.empty()) return fail(BSDC_IO_EINVAL, "stream already cut by families (bsdc_bam_stream_next_raw)");
    const size_t want = (size_t)std::max<int64_t>(min_bytes, 0) * 5 / 4 + (size_t)s->read_size * 16;
    if (s->buf.capacity() < want) s->buf.reserve(want);
    if (s->spare.capacity() < want) {
        std::lock_guard<std::mutex> lk(s->mu);
        for (auto &v : s->pool)
            if (v.capacity() >= want) {
                s->spare.swap(v);
                break;
            }
    }
    if (s->spare.capacity() < want) s->spare.reserve(want);
    for (;;) {
        double t0 = now_s();
        const uint8_t *d = s->buf.data();
        const int64_t dn = (int64_t)s->buf.size();
        int64_t p = s->tail, cut = -1;
        while (p + 4 <= dn) {
            const int64_t bs = rd32(d + p);
            if (bs < 32) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
            if (p + 4 + bs > dn) break;
            const uint8_t *r = d + p, *end = r + 4 + bs;
            const int64_t body = 36 + (int64_t)r[12] + 4 * (int64_t)rd16(r + 16) + ((int64_t)rdi32(r + 20) + 1) / 2 +
                                 (int64_t)rdi32(r + 20);
            if (rdi32(r + 20) < 0 || r[12] < 1 || body > 4 + bs) return fail(BSDC_IO_EFORMAT, "malformed BAM record (lengths or aux)");
            std::string_view mi;
            for (const uint8_t *a = r + body; a + 3 <= end;) {
                const int64_t vs = aux_value_size(a, end);
                if (vs < 0 || vs > (end - a) - 3) return fail(BSDC_IO_EFORMAT, "malformed BAM record (lengths or aux)");
                if (a[0] == 'M' && a[1] == 'I' && a[2] == 'Z') mi = std::string_view((const char *)a + 3, (size_t)vs - 1);
                a += 3 + vs;
            }
            if (p > 0 && p >= min_bytes && mi != s->run_mi) {
                cut = p;
                break;
            }
            s->run_mi.assign(mi.data(), mi.size());
            p += 4 + bs;
        }
        s->prof[1] += now_s() - t0;
        const bool end = s->eof && s->comp.empty();
        if (cut < 0) {
            s->tail = p;
            if (end) {
                if (p < dn) return fail(BSDC_IO_EFORMAT, "truncated BAM record");
                if (p == 0) return 0;  // the end of the stream
                cut = p;
            }
        }
        if (cut >= 0) {  // records [0, cut) go out in the buffer; the rest moves to `spare`
            t0 = now_s();
            auto *b = new bsdc_bam();
            b->header = s->hdr.header;
            b->ref_names = s->hdr.ref_names;
            b->ref_len = s->hdr.ref_len;
            const int64_t kept = dn - cut;
            s->spare.resize((size_t)kept);
            if (kept > 0) memcpy(s->spare.data(), d + cut, (size_t)kept);
            b->data.swap(s->buf);
            b->data.resize((size_t)cut + 8);
            memset(b->data.data() + cut, 0, 8);
            s->buf.swap(s->spare);
            s->tail = 0;  // rescan the kept bytes (the first one opens a new run)
            b->dn = cut;
            b->parsed = false;
            s->prof[3] += now_s() - t0;
            {
                std::lock_guard<std::mutex> lk(s->mu);
                s->outstanding++;
            }
            *out = b;
            return 0;
        }
        t0 = now_s();
        const int32_t rc = bsdc_bam_stream_fill(s);
        if (rc != 0) return rc;
        s->prof[0] += now_s() - t0;
    }
}

// Spill entries (bsdc_bam_stream_spill; several streams' concatenated) -> their records in file
// order (see include/bsdc_io.h).
int64_t bsdc_spill_sort(const uint8_t *data, int64_t n, uint8_t *out, int64_t *n_rec) {
    struct E {
        int64_t c, q, off, len;
    };
    std::vector<E> es;
    int64_t p = 0, total = 0;
    while (p < n) {
        if (p + 20 > n) return fail(BSDC_IO_EFORMAT, "truncated spill");
        E e;
        memcpy(&e.c, data + p, 8);
        memcpy(&e.q, data + p + 8, 8);
        e.off = p + 16;
        e.len = 4 + (int64_t)rd32(data + p + 16);
        if (e.off + e.len > n) return fail(BSDC_IO_EFORMAT, "truncated spill");
        es.push_back(e);
        total += e.len;
        p = e.off + e.len;
    }
    if (n_rec) *n_rec = (int64_t)es.size();
    if (!out) return total;
    std::stable_sort(es.begin(), es.end(), [](const E &x, const E &y) { return x.c != y.c ? x.c < y.c : x.q < y.q; });
    std::vector<int64_t> dst(es.size() + 1, 0);
    for (size_t i = 0; i < es.size(); i++) dst[i + 1] = dst[i] + es[i].len;
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t i = 0; i < (int64_t)es.size(); i++) memcpy(out + dst[(size_t)i], data + es[(size_t)i].off, (size_t)es[(size_t)i].len);
    return total;
}

// The coarse TemplateCoordinate key of every record of b, in record order (see include/bsdc_io.h).
int32_t bsdc_bam_rec_keys(const bsdc_bam *b, int64_t *out) {
    const int64_t n = (int64_t)b->rec_start.size();
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < n; k++) {
        const uint8_t *r = b->data.data() + b->rec_start[(size_t)k];
        const int64_t bs = rd32(r);
        const uint8_t *end = r + 4 + bs;
        const int64_t body = 36 + (int64_t)r[12] + 4 * (int64_t)rd16(r + 16) + ((int64_t)rdi32(r + 20) + 1) / 2 +
                             (int64_t)rdi32(r + 20);
        std::string_view mc;
        for (const uint8_t *a = r + body; a + 3 <= end;) {
            const int64_t vs = aux_value_size(a, end);
            if (vs < 0 || vs > (end - a) - 3) {
                bad |= 1;
                break;
            }
            if (a[0] == 'M' && a[1] == 'C' && a[2] == 'Z') mc = std::string_view((const char *)a + 3, (size_t)vs - 1);
            a += 3 + vs;
        }
        const RecKey rk = rec_key(r, mc);
        out[2 * k] = rk.key.first;
        out[2 * k + 1] = rk.key.second;
    }
    return bad ? fail(BSDC_IO_EFORMAT, "malformed BAM record (aux)") : 0;
}

// Parses a raw chunk (records, tags, interned names and MI bases); a no-op for a parsed one.
int32_t bsdc_bam_parse(bsdc_bam *b, int32_t n_threads) {
    if (b->parsed) return 0;
    set_threads(n_threads);
    const int32_t rc = parse_records(b, 0, b->dn);
    if (rc == 0) b->parsed = true;
    return rc;
}

int32_t bsdc_bam_stream_next(bsdc_bam_stream *s, int64_t min_bytes, int64_t slack, bsdc_bam **out) {
    const int32_t rc = bsdc_bam_stream_next_raw(s, min_bytes, slack, out);
    if (rc != 0 || *out == nullptr) return rc;
    const double t0 = now_s();
    const int32_t pc = parse_records(*out, 0, (*out)->dn);
    s->prof[4] += now_s() - t0;
    if (pc != 0) {
        bsdc_bam_stream_recycle(s, *out);
        *out = nullptr;
        return pc;
    }
    (*out)->parsed = true;
    return 0;
}

void bsdc_bam_stream_recycle(bsdc_bam_stream *s, bsdc_bam *b) {
    if (!s) {
        delete b;
        return;
    }
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        if (b) {
            if (s->pool.size() < 2 && b->data.capacity() > 0) {
                b->data.clear();
                s->pool.push_back(std::move(b->data));
            }
            s->outstanding--;
        }
        last = s->closed && s->outstanding == 0;
    }
    delete b;
    if (last) delete s;
}

// The stream's header and references as a record-less bsdc_bam.
int32_t bsdc_bam_stream_header(const bsdc_bam_stream *s, bsdc_bam **out) {
    auto *b = new bsdc_bam();
    b->header = s->hdr.header;
    b->ref_names = s->hdr.ref_names;
    b->ref_len = s->hdr.ref_len;
    b->data.assign(8, 0);
    *out = b;
    return 0;
}

void bsdc_bam_stream_close(bsdc_bam_stream *s) {
    if (!s) return;
    if (s->f) fclose(s->f);
    s->f = nullptr;
    if (getenv("BSDC_STREAM_PROF"))
        fprintf(stderr, "bsdc stream s: fill %.3f split %.3f select %.3f emit %.3f parse %.3f\n", s->prof[0], s->prof[1],
                s->prof[2], s->prof[3], s->prof[4]);
    bool last;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        s->closed = true;
        last = s->outstanding == 0;
    }
    if (last) delete s;  // else the last bsdc_bam_stream_recycle deletes it
}

void bsdc_bam_sizes_of(const bsdc_bam *b, bsdc_bam_sizes *s) {
    memset(s, 0, sizeof *s);
    s->n_rec = (int64_t)b->rec_start.size();
    s->n_bases = b->n_bases;
    s->n_cigar = b->n_cigar;
    s->n_mc = b->n_mc;
    s->aux_bytes = b->aux_bytes;
    s->n_names = (int64_t)b->names.size();
    for (auto &x : b->names) s->name_bytes += (int64_t)x.size();
    s->n_mi = (int64_t)b->mis.size();
    for (auto &x : b->mis) s->mi_bytes += (int64_t)x.size();
    s->header_bytes = (int64_t)b->header.size();
    s->n_ref = (int32_t)b->ref_names.size();
    for (auto &x : b->ref_names) s->ref_name_bytes += (int64_t)x.size();
}

int32_t bsdc_bam_copy(const bsdc_bam *b, const bsdc_bam_arrays *a) {
    if (!b->parsed) return fail(BSDC_IO_EFORMAT, "stream chunk not parsed (bsdc_bam_parse)");
    const int64_t nr = (int64_t)b->rec_start.size();
    const uint8_t *d = b->data.data();
    // running offsets (sequential prefix sums)
    std::vector<int64_t> so(nr + 1), co(nr + 1), ao(nr + 1), mo(nr + 1);
    for (int64_t k = 0; k < nr; k++) {
        const uint8_t *r = d + b->rec_start[k];
        const int64_t bs = rd32(r);
        const int l_name = r[12];
        const int n_cig = rd16(r + 16);
        const int32_t l_seq = rdi32(r + 20);
        const int64_t auxlen = 4 + bs - (36 + l_name + 4 * n_cig + (l_seq + 1) / 2 + l_seq);
        so[k + 1] = so[k] + l_seq;
        co[k + 1] = co[k] + n_cig;
        ao[k + 1] = ao[k] + auxlen;
        mo[k + 1] = mo[k] + b->mc_n[k];
    }
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nr; k++) {
        const uint8_t *r = d + b->rec_start[k];
        const int64_t bs = rd32(r);
        const int l_name = r[12];
        const int n_cig = rd16(r + 16);
        const int32_t l_seq = rdi32(r + 20);
        a->tid[k] = rdi32(r + 4);
        a->pos[k] = rdi32(r + 8);
        a->mapq[k] = r[13];
        a->flag[k] = rd16(r + 18);
        a->l_seq[k] = l_seq;
        a->next_tid[k] = rdi32(r + 24);
        a->next_pos[k] = rdi32(r + 28);
        a->tlen[k] = rdi32(r + 32);
        a->seq_off[k] = so[k];
        a->cig_off[k] = co[k];
        a->n_cig[k] = n_cig;
        const uint8_t *c = r + 36 + l_name;
        for (int i = 0; i < n_cig; i++) a->cigar[co[k] + i] = rd32(c + 4 * i);
        const uint8_t *sq = c + 4 * n_cig;
        uint8_t *dst = a->seq + so[k];
        for (int32_t i = 0; i < l_seq >> 1; i++) memcpy(dst + 2 * i, &kNibblePairs.v[sq[i]], 2);
        if (l_seq & 1) dst[l_seq - 1] = (uint8_t)(sq[l_seq >> 1] >> 4);
        memcpy(a->qual + so[k], sq + (l_seq + 1) / 2, (size_t)l_seq);
        const uint8_t *aux = sq + (l_seq + 1) / 2 + l_seq;
        memcpy(a->aux + ao[k], aux, (size_t)(ao[k + 1] - ao[k]));
        a->aux_off[k] = ao[k];
        a->name_id[k] = b->name_id[k];
        a->mi_id[k] = b->mi_id[k];
        a->mi_strand[k] = b->mi_strand[k];
        a->la[k] = b->la[k];
        a->rd[k] = b->rd[k];
        a->mc_n[k] = b->mc_n[k];
        a->mc_off[k] = b->mc_tag_off[k] >= 0 ? mo[k] : -1;
        if (b->mc_tag_off[k] >= 0) {
            const char *s = (const char *)d + b->mc_tag_off[k];
            int64_t w = mo[k];
            uint32_t num = 0;
            for (; *s; s++) {
                if (*s >= '0' && *s <= '9') {
                    num = num * 10 + (uint32_t)(*s - '0');
                } else {
                    const char *q = strchr(kCigarOps, *s);
                    if (q) a->mc_cigar[w++] = (num << 4) | (uint32_t)(q - kCigarOps);
                    num = 0;
                }
            }
        }
        (void)bs;
    }
    a->aux_off[nr] = ao[nr];
    int64_t o = 0;
    for (size_t i = 0; i < b->names.size(); i++) {
        a->name_off[i] = o;
        memcpy(a->name_buf + o, b->names[i].data(), b->names[i].size());
        o += (int64_t)b->names[i].size();
    }
    a->name_off[b->names.size()] = o;
    o = 0;
    for (size_t i = 0; i < b->mis.size(); i++) {
        a->mi_off[i] = o;
        memcpy(a->mi_buf + o, b->mis[i].data(), b->mis[i].size());
        o += (int64_t)b->mis[i].size();
    }
    a->mi_off[b->mis.size()] = o;
    memcpy(a->header, b->header.data(), b->header.size());
    o = 0;
    for (size_t i = 0; i < b->ref_names.size(); i++) {
        a->ref_len[i] = b->ref_len[i];
        a->ref_name_off[i] = o;
        memcpy(a->ref_name_buf + o, b->ref_names[i].data(), b->ref_names[i].size());
        o += (int64_t)b->ref_names[i].size();
    }
    a->ref_name_off[b->ref_names.size()] = o;
    return 0;
}

void bsdc_bam_free(bsdc_bam *b) { delete b; }

}  // extern "C"

namespace {
// SAM spec reg2bin (0-based, end exclusive)
int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}
constexpr int64_t kBlock = 0xff00;  // uncompressed bytes per BGZF block (htslib's size)
// BGZF framing of an uncompressed buffer: 0xff00-byte blocks deflated in parallel (each a gzip
// member, so the file is also plain multi-member gzip), one write, then the 28-byte EOF block.
// BGZF blocks of src[0, total) (kBlock uncompressed bytes each, the last one shorter), deflated
// in parallel and written to f.
int32_t deflate_write(FILE *f, const uint8_t *src0, int64_t total, int32_t level) {
    const int64_t nb = (total + kBlock - 1) / kBlock;
    // each block compresses into its own 64 KiB slot of one buffer (BSIZE <= 65536 by format)
    Bytes slots((size_t)std::max<int64_t>(nb, 1) << 16);
    std::vector<int32_t> bsz((size_t)std::max<int64_t>(nb, 1));
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(| : bad)
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t *src = src0 + i * kBlock;
        const int64_t len = std::min(kBlock, total - i * kBlock);
        uint8_t *h = slots.data() + ((size_t)i << 16);
        // a block that does not shrink to fit BSIZE (incompressible) is stored (level 0; a stored
        // 0xff00-byte block is 0xff05 bytes of deflate, inside the slot)
        int64_t clen = raw_deflate(src, len, level, h + 18, 65536 - 26);
        if (clen <= 0) clen = raw_deflate(src, len, 0, h + 18, 65536 - 26);
        if (clen <= 0 || 18 + clen + 8 > 65536) {
            bad |= 1;
            continue;
        }
        const int64_t bsize = 18 + clen + 8;
        const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0};
        memcpy(h, hdr, 16);
        wr16(h + 16, (uint16_t)(bsize - 1));
        wr32(h + 18 + clen, crc32_of(src, len));
        wr32(h + 18 + clen + 4, (uint32_t)len);
        bsz[(size_t)i] = (int32_t)bsize;
    }
    if (bad) return fail(BSDC_IO_EFORMAT, "deflate failed");
    for (int64_t i = 0; i < nb; i++)
        if (fwrite(slots.data() + ((size_t)i << 16), 1, (size_t)bsz[(size_t)i], f) != (size_t)bsz[(size_t)i])
            return fail(BSDC_IO_EIO, "BGZF write failed");
    return 0;
}

const uint8_t kBgzfEof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

int32_t write_bgzf(const char *path, const Bytes &buf, int32_t level) {
    FILE *f = fopen(path, "wb");
    if (!f) return fail(BSDC_IO_EIO, std::string("cannot create ") + path);
    int32_t rc = deflate_write(f, buf.data(), (int64_t)buf.size(), level);
    if (rc == 0 && fwrite(kBgzfEof, 1, 28, f) != 28) rc = fail(BSDC_IO_EIO, std::string("write failed on ") + path);
    if (fclose(f) != 0 && rc == 0) rc = fail(BSDC_IO_EIO, std::string("write failed on ") + path);
    return rc;
}

// BAM header bytes (magic, text, references)
void encode_header(Bytes &head, const char *header_text, int64_t header_len, int32_t n_ref,
                   const int64_t *ref_name_off, const char *ref_name_buf, const int64_t *ref_len) {
    auto put32 = [&](uint32_t v) {
        uint8_t t[4];
        wr32(t, v);
        head.insert(head.end(), t, t + 4);
    };
    head.insert(head.end(), {'B', 'A', 'M', 1});
    put32((uint32_t)header_len);
    head.insert(head.end(), header_text, header_text + header_len);
    put32((uint32_t)n_ref);
    for (int32_t i = 0; i < n_ref; i++) {
        const int64_t l = ref_name_off[i + 1] - ref_name_off[i];
        put32((uint32_t)(l + 1));
        head.insert(head.end(), ref_name_buf + ref_name_off[i], ref_name_buf + ref_name_off[i] + l);
        head.push_back(0);
        put32((uint32_t)ref_len[i]);
    }
}

// The records' BAM bytes appended to buf (encoded in parallel)
int32_t encode_records(const bsdc_bam_records *r, Bytes &buf) {
    const int64_t nr = r->n_rec;
    std::vector<int64_t> off(nr + 1);
    off[0] = (int64_t)buf.size();
    for (int64_t k = 0; k < nr; k++) {
        const int64_t l_name = r->name_off[k + 1] - r->name_off[k] + 1;
        const int64_t n_cig = r->cig_off[k + 1] - r->cig_off[k];
        const int64_t l_seq = r->seq_off[k + 1] - r->seq_off[k];
        const int64_t l_aux1 = r->aux_off[k + 1] - r->aux_off[k];
        const int64_t l_aux = l_aux1 + (r->aux2_off ? r->aux2_off[k + 1] - r->aux2_off[k] : 0);
        if (l_name > 254 || n_cig > 0xFFFF) return fail(BSDC_IO_EFORMAT, "record name or cigar too long for BAM");
        off[k + 1] = off[k] + 4 + 32 + l_name + 4 * n_cig + (l_seq + 1) / 2 + l_seq + l_aux;
    }
    buf.resize((size_t)off[nr]);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nr; k++) {
        uint8_t *p = buf.data() + off[k];
        const int64_t l_name = r->name_off[k + 1] - r->name_off[k] + 1;
        const int64_t n_cig = r->cig_off[k + 1] - r->cig_off[k];
        const int64_t l_seq = r->seq_off[k + 1] - r->seq_off[k];
        const int64_t l_aux1 = r->aux_off[k + 1] - r->aux_off[k];
        const int64_t l_aux = l_aux1 + (r->aux2_off ? r->aux2_off[k + 1] - r->aux2_off[k] : 0);
        const uint32_t *cg = r->cigar + r->cig_off[k];
        int64_t reflen = 0;
        for (int64_t i = 0; i < n_cig; i++) {
            const uint32_t op = cg[i] & 0xF;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) reflen += cg[i] >> 4;
        }
        const int64_t pos = r->pos[k];
        const int bin = pos < 0 ? 4680 : reg2bin(pos, pos + (reflen > 0 ? reflen : 1));
        wr32(p, (uint32_t)(off[k + 1] - off[k] - 4));
        wr32(p + 4, (uint32_t)r->tid[k]);
        wr32(p + 8, (uint32_t)pos);
        p[12] = (uint8_t)l_name;
        p[13] = r->mapq[k];
        wr16(p + 14, (uint16_t)bin);
        wr16(p + 16, (uint16_t)n_cig);
        wr16(p + 18, r->flag[k]);
        wr32(p + 20, (uint32_t)l_seq);
        wr32(p + 24, (uint32_t)r->next_tid[k]);
        wr32(p + 28, (uint32_t)r->next_pos[k]);
        wr32(p + 32, (uint32_t)r->tlen[k]);
        uint8_t *q = p + 36;
        memcpy(q, r->name_buf + r->name_off[k], (size_t)(l_name - 1));
        q[l_name - 1] = 0;
        q += l_name;
        for (int64_t i = 0; i < n_cig; i++) wr32(q + 4 * i, cg[i]);
        q += 4 * n_cig;
        const uint8_t *s = r->seq + r->seq_off[k];
        for (int64_t i = 0; i < l_seq; i += 2) q[i >> 1] = (uint8_t)((s[i] << 4) | (i + 1 < l_seq ? s[i + 1] : 0));
        q += (l_seq + 1) / 2;
        memcpy(q, r->qual + r->seq_off[k], (size_t)l_seq);
        q += l_seq;
        memcpy(q, r->aux + r->aux_off[k], (size_t)l_aux1);
        if (r->aux2_off) memcpy(q + l_aux1, r->aux2 + r->aux2_off[k], (size_t)(l_aux - l_aux1));
    }
    return 0;
}
}  // namespace

extern "C" int32_t bsdc_bam_write(const char *path, const char *header_text, int64_t header_len, int32_t n_ref,
                                  const int64_t *ref_name_off, const char *ref_name_buf, const int64_t *ref_len,
                                  const bsdc_bam_records *r, int32_t level, int32_t n_threads) {
    set_threads(n_threads);
    Bytes buf;
    encode_header(buf, header_text, header_len, n_ref, ref_name_off, ref_name_buf, ref_len);
    const int32_t rc = encode_records(r, buf);
    if (rc != 0) return rc;
    return write_bgzf(path, buf, level);
}

// ------------------------------------------------------------------------------------------
// streaming writer: the same bytes as bsdc_bam_write of all the records at once (whole kBlock
// blocks are deflated as they fill; the rest waits for the next records or the close)
// ------------------------------------------------------------------------------------------
struct bsdc_bam_writer {
    FILE *f = nullptr;
    int32_t level = 6;
    Bytes tail;
    bool no_eof = false;  // a fragment (bsdc_bam_writer_fragment): no EOF block at the close
};

extern "C" int32_t bsdc_bam_writer_open(const char *path, const char *header_text, int64_t header_len, int32_t n_ref,
                                        const int64_t *ref_name_off, const char *ref_name_buf, const int64_t *ref_len,
                                        int32_t level, bsdc_bam_writer **out) {
    *out = nullptr;
    FILE *f = fopen(path, "wb");
    if (!f) return fail(BSDC_IO_EIO, std::string("cannot create ") + path);
    auto *w = new bsdc_bam_writer();
    w->f = f;
    w->level = level;
    encode_header(w->tail, header_text, header_len, n_ref, ref_name_off, ref_name_buf, ref_len);
    *out = w;
    return 0;
}

extern "C" int32_t bsdc_bam_writer_add(bsdc_bam_writer *w, const bsdc_bam_records *r, int32_t n_threads) {
    set_threads(n_threads);
    int32_t rc = encode_records(r, w->tail);
    if (rc != 0) return rc;
    const int64_t whole = ((int64_t)w->tail.size() / kBlock) * kBlock;
    if (whole > 0) {
        rc = deflate_write(w->f, w->tail.data(), whole, w->level);
        if (rc != 0) return rc;
        w->tail.erase(w->tail.begin(), w->tail.begin() + whole);
    }
    return 0;
}

// The GPU-compressed write path (bsdc_bgzf_deflate in libbsdc): encode, move the whole blocks out
// to the caller's (pinned) buffer with their CRC32s, let the caller compress them on the GPU while
// the next records encode, then hand the compressed blocks back to be finished and written.
extern "C" int64_t bsdc_bam_writer_encode(bsdc_bam_writer *w, const bsdc_bam_records *r, int32_t n_threads,
                                          const uint8_t **data) {
    set_threads(n_threads);
    const int32_t rc = encode_records(r, w->tail);
    if (rc != 0) return rc;
    *data = w->tail.data();
    return ((int64_t)w->tail.size() / kBlock) * kBlock;
}

namespace {
// The first nblk whole blocks of an encoded tail leave it: copied to dst (nblk * 65280 bytes) with
// each block's CRC32 in crc[b] (one pass over the bytes, the blocks in parallel).
int32_t take_blocks(Bytes &tail, int64_t nblk, uint8_t *dst, uint32_t *crc) {
    if (nblk < 0 || nblk * kBlock > (int64_t)tail.size()) return fail(BSDC_IO_EFORMAT, "more blocks than encoded bytes");
    const uint8_t *src0 = tail.data();
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; b++) {
        memcpy(dst + b * kBlock, src0 + b * kBlock, (size_t)kBlock);
        crc[b] = crc32_of(dst + b * kBlock, kBlock);
    }
    tail.erase(tail.begin(), tail.begin() + nblk * kBlock);
    return 0;
}

// nblk taken blocks back compressed: block b's BGZF bytes are packed[off_b .. off_b + sizes[b])
// (off = running sum of sizes), complete but for CRC32 and ISIZE, which are filled in here from
// crc[b]; a block of size 0 did not fit and is deflated here from raw (the taken bytes; stored when
// incompressible).  Then the blocks are written in order.
int32_t put_blocks(FILE *f, int32_t level, int64_t nblk, uint8_t *packed, const int32_t *sizes, const uint32_t *crc,
                   const uint8_t *raw) {
    int64_t off = 0;
    for (int64_t b = 0; b < nblk; b++) {
        const int32_t bs = sizes[b];
        int32_t rc = 0;
        if (bs > 0) {
            if (bs < 26 || bs > 65536) return fail(BSDC_IO_EFORMAT, "bad compressed block size");
            uint8_t *h = packed + off;
            wr32(h + bs - 8, crc[b]);
            wr32(h + bs - 4, (uint32_t)kBlock);
            if (fwrite(h, 1, (size_t)bs, f) != (size_t)bs) rc = fail(BSDC_IO_EIO, "BGZF write failed");
            off += bs;
        } else {
            rc = deflate_write(f, raw + b * kBlock, kBlock, level);
        }
        if (rc != 0) return rc;
    }
    return 0;
}
}  // namespace

extern "C" int32_t bsdc_bam_writer_take(bsdc_bam_writer *w, int64_t nblk, uint8_t *dst, uint32_t *crc,
                                        int32_t n_threads) {
    set_threads(n_threads);
    return take_blocks(w->tail, nblk, dst, crc);
}

extern "C" int32_t bsdc_bam_writer_put(bsdc_bam_writer *w, int64_t nblk, uint8_t *packed, const int32_t *sizes,
                                       const uint32_t *crc, const uint8_t *raw, int32_t n_threads) {
    set_threads(n_threads);
    return put_blocks(w->f, w->level, nblk, packed, sizes, crc, raw);
}

extern "C" int32_t bsdc_bam_writer_close(bsdc_bam_writer *w, int32_t n_threads) {
    if (!w) return 0;
    set_threads(n_threads);
    int32_t rc = deflate_write(w->f, w->tail.data(), (int64_t)w->tail.size(), w->level);
    if (rc == 0 && !w->no_eof && fwrite(kBgzfEof, 1, 28, w->f) != 28) rc = fail(BSDC_IO_EIO, "BGZF write failed");
    if (fclose(w->f) != 0 && rc == 0) rc = fail(BSDC_IO_EIO, "BGZF close failed");
    delete w;
    return rc;
}

// Everything added so far leaves as BGZF blocks (the last one short), so the file can be cut here.
extern "C" int32_t bsdc_bam_writer_flush(bsdc_bam_writer *w, int32_t n_threads) {
    set_threads(n_threads);
    const int32_t rc = deflate_write(w->f, w->tail.data(), (int64_t)w->tail.size(), w->level);
    w->tail.clear();
    return rc;
}

extern "C" int64_t bsdc_bam_writer_tell(bsdc_bam_writer *w) { return (int64_t)ftello(w->f); }

// Raw BAM records (block_size-prefixed, as a stream chunk holds them) appended as they are.
extern "C" int32_t bsdc_bam_writer_raw(bsdc_bam_writer *w, const uint8_t *data, int64_t n, int32_t n_threads) {
    set_threads(n_threads);
    w->tail.insert(w->tail.end(), data, data + n);
    const int64_t whole = ((int64_t)w->tail.size() / kBlock) * kBlock;
    if (whole > 0) {
        const int32_t rc = deflate_write(w->f, w->tail.data(), whole, w->level);
        if (rc != 0) return rc;
        w->tail.erase(w->tail.begin(), w->tail.begin() + whole);
    }
    return 0;
}

// A writer of one piece of a BAM whose pieces are concatenated later: header or not (keep_header:
// the first piece), no EOF block at the close (the assembler appends one).
extern "C" int32_t bsdc_bam_writer_fragment(bsdc_bam_writer *w, int32_t keep_header) {
    if (!w) return fail(BSDC_IO_EFORMAT, "no writer");
    if (!keep_header) w->tail.clear();  // (nothing but the header is encoded at the open)
    w->no_eof = true;
    return 0;
}

namespace {
// the RX value of one record's aux block (empty view if absent)
std::string_view find_rx(const uint8_t *a, const uint8_t *end) {
    while (a + 3 <= end) {
        const int64_t vs = aux_value_size(a, end);
        if (vs < 0 || vs > (end - a) - 3) break;
        if (a[0] == 'R' && a[1] == 'X' && a[2] == 'Z') return std::string_view((const char *)a + 3, (size_t)vs - 1);
        a += 3 + vs;
    }
    return {};
}
}  // namespace

extern "C" int64_t bsdc_rx_consensus(int64_t n_fam, const int64_t *fam_rec_off, const int64_t *rec, const int8_t *strand,
                                     const int64_t *aux_off, const uint8_t *aux, char *out, int32_t *out_len,
                                     int32_t n_threads) {
    set_threads(n_threads);
    const int64_t nrec = fam_rec_off[n_fam];
    if (!out) {
        int64_t w = 0;
#pragma omp parallel for schedule(static) reduction(max : w)
        for (int64_t i = 0; i < nrec; i++) {
            const int64_t k = rec[i];
            w = std::max<int64_t>(w, (int64_t)find_rx(aux + aux_off[k], aux + aux_off[k + 1]).size());
        }
        return w;
    }
    int64_t width = 0;
    for (int64_t i = 0; i < nrec; i++) {
        const int64_t k = rec[i];
        width = std::max<int64_t>(width, (int64_t)find_rx(aux + aux_off[k], aux + aux_off[k + 1]).size());
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t f = 0; f < n_fam; f++) {
        std::vector<std::string> v;
        for (int64_t i = fam_rec_off[f]; i < fam_rec_off[f + 1]; i++) {
            const int64_t k = rec[i];
            const std::string_view rx = find_rx(aux + aux_off[k], aux + aux_off[k + 1]);
            if (rx.empty()) continue;
            std::string s(rx);
            const size_t dash = s.find('-');
            if (strand[k] == 1 && dash != std::string::npos)  // B strand: U2-U1 -> U1-U2
                s = s.substr(dash + 1) + "-" + s.substr(0, dash);
            v.push_back(std::move(s));
        }
        char *o = out + f * width;
        if (v.empty()) {
            out_len[f] = 0;
            continue;
        }
        // the most common length (the first seen on a tie)
        size_t L = v[0].size();
        int best = 0;
        for (auto &a : v) {
            int c = 0;
            for (auto &b2 : v) c += b2.size() == a.size();
            if (c > best) {
                best = c;
                L = a.size();
            }
        }
        for (size_t j = 0; j < L; j++) {
            int cnt[256] = {0};
            for (auto &a : v)
                if (a.size() == L) cnt[(uint8_t)a[j]]++;
            int top = 0, ties = 0, ch = 'N';
            for (int c = 0; c < 256; c++) {
                if (cnt[c] > top) {
                    top = cnt[c];
                    ch = c;
                    ties = 0;
                } else if (cnt[c] == top && top > 0) {
                    ties++;
                }
            }
            o[j] = (char)(ties ? 'N' : ch);
        }
        out_len[f] = (int32_t)L;
    }
    return width;
}

namespace {
const char kNt16[] = "=ACMGRSVTWYHKDBN";
const char kNt16Comp[] = "=TGKCYSBAWRDMHVN";

// BAM aux writer: sizes only when p == nullptr.  Integers take the smallest BAM type that holds
// them (htsjdk's encoding of an Int attribute).
struct AuxOut {
    uint8_t *p;
    int64_t n = 0;
    void bytes(const void *src, int64_t k) {
        if (p) memcpy(p + n, src, (size_t)k);
        n += k;
    }
    void head(const char *tag, char type) {
        const uint8_t h[3] = {(uint8_t)tag[0], (uint8_t)tag[1], (uint8_t)type};
        bytes(h, 3);
    }
    void integer(const char *tag, int64_t v) {
        uint8_t b[4];
        if (v >= 0 && v <= 255) {
            head(tag, 'C');
            b[0] = (uint8_t)v;
            bytes(b, 1);
        } else if (v >= 0 && v <= 65535) {
            head(tag, 'S');
            wr16(b, (uint16_t)v);
            bytes(b, 2);
        } else if (v >= -128 && v < 0) {
            head(tag, 'c');
            b[0] = (uint8_t)(int8_t)v;
            bytes(b, 1);
        } else if (v >= -32768 && v < 0) {
            head(tag, 's');
            wr16(b, (uint16_t)(int16_t)v);
            bytes(b, 2);
        } else {
            head(tag, v < 0 ? 'i' : 'I');
            wr32(b, (uint32_t)v);
            bytes(b, 4);
        }
    }
    void real(const char *tag, float v) {
        head(tag, 'f');
        uint32_t u;
        memcpy(&u, &v, 4);
        uint8_t b[4];
        wr32(b, u);
        bytes(b, 4);
    }
    void shorts(const char *tag, const int32_t *v, int32_t len) {
        head(tag, 'B');
        uint8_t b[5] = {'s'};
        wr32(b + 1, (uint32_t)len);
        bytes(b, 5);
        if (p)
            for (int32_t i = 0; i < len; i++) wr16(p + n + 2 * i, (uint16_t)(int16_t)v[i]);
        n += 2 * (int64_t)len;
    }
    void text(const char *tag, const uint8_t *v, int32_t len, const char *map, int add) {
        head(tag, 'Z');
        if (p)
            for (int32_t i = 0; i < len; i++) p[n + i] = map ? (uint8_t)map[v[i] & 15] : (uint8_t)(v[i] + add);
        n += len;
        const uint8_t z = 0;
        bytes(&z, 1);
    }
};

struct SsView {  // one single-strand consensus read, truncated to `len`: depths / errors as the
                 // kernels' bytes, or a wide family's exact u16 values (w16 set)
    const uint8_t *b, *q;
    const uint8_t *d8, *e8;
    const uint16_t *d16, *e16;
    int32_t len;
    int64_t d(int32_t i) const { return d16 ? (int64_t)d16[i] : (int64_t)d8[i]; }
    int64_t e(int32_t i) const { return e16 ? (int64_t)e16[i] : (int64_t)e8[i]; }
};

// D (max depth), M (min depth), E (errors / depth) of one read; depth(i), err(i) per column
template <class Dep, class Err>
void per_read(AuxOut &o, const char *tD, const char *tM, const char *tE, Dep depth, Err err, int32_t len) {
    int64_t mx = 0, mn = len ? INT64_MAX : 0, sd = 0, se = 0;
    for (int32_t i = 0; i < len; i++) {
        const int64_t d = depth(i);
        mx = std::max<int64_t>(mx, d);
        mn = std::min<int64_t>(mn, d);
        sd += d;
        se += err(i);
    }
    o.integer(tD, mx);
    o.integer(tM, mn);
    o.real(tE, (float)se / (float)sd);
}

// a B:s array of the kernels' counts: a wide family's u16 values as they are (the same 16 bits as
// the int16 value), the bytes widened
void shorts16(AuxOut &o, const char *tag, const uint8_t *v8, const uint16_t *v16, int32_t len) {
    o.head(tag, 'B');
    uint8_t b[5] = {'s'};
    wr32(b + 1, (uint32_t)len);
    o.bytes(b, 5);
    if (v16) {
        o.bytes(v16, 2 * (int64_t)len);  // (little-endian host)
        return;
    }
    if (o.p)
        for (int32_t i = 0; i < len; i++) wr16(o.p + o.n + 2 * i, (uint16_t)v8[i]);
    o.n += 2 * (int64_t)len;
}
}  // namespace

// fgbio's consensus tags of one output record (DuplexConsensusCaller / VanillaUmiConsensusCaller
// createSamRecord, restated: PARITY UNPINNED), from the single-strand reads the kernels wrote with
// BSDC_MODE_TAGS.  See include/bsdc_io.h.
extern "C" int64_t bsdc_consensus_tags(int64_t n, const int64_t *row_a, const int64_t *row_b, const int32_t *out_len,
                                       int32_t kind, int32_t stride, const uint8_t *ss_base, const uint8_t *ss_qual,
                                       const uint8_t *ss_depth, const uint8_t *ss_err, const int32_t *ss_wide,
                                       const uint16_t *ss_wdepth, const uint16_t *ss_werr, int64_t *off, uint8_t *buf,
                                       int32_t n_threads) {
    set_threads(n_threads);
    auto one = [&](int64_t k, uint8_t *p) -> int64_t {
        AuxOut o{p};
        const int32_t L = out_len[k];
        auto view = [&](int64_t row) {
            const size_t at = (size_t)row * (size_t)stride;
            SsView v{ss_base + at, ss_qual + at, ss_depth + at, ss_err + at, nullptr, nullptr, L};
            const int32_t w = ss_wide ? ss_wide[row >> 2] : -1;
            if (w >= 0) {
                const size_t aw = (4 * (size_t)w + (size_t)(row & 3)) * (size_t)stride;
                v.d16 = ss_wdepth + aw;
                v.e16 = ss_werr + aw;
            }
            return v;
        };
        const SsView a = view(row_a[k]);
        auto ad = [&](int32_t i) { return a.d(i); };
        auto ae = [&](int32_t i) { return a.e(i); };
        if (kind == 1) {  // molecular: cD cM cE, cd ce
            per_read(o, "cD", "cM", "cE", ad, ae, L);
            shorts16(o, "cd", a.d8, a.d16, L);
            shorts16(o, "ce", a.e8, a.e16, L);
            return o.n;
        }
        const bool two = row_b[k] >= 0;
        const SsView b = two ? view(row_b[k]) : SsView{};
        if (two) {
            // the duplex call before its N mask; errors counted against it: a strand whose call
            // agrees contributes its errors, one that disagrees all of its reads
            auto td = [&](int32_t i) { return a.d(i) + b.d(i); };
            auto te = [&](int32_t i) {
                const uint8_t ab = a.b[i] & 15, bb = b.b[i] & 15;
                const uint8_t raw = ab == bb ? ab : a.q[i] > b.q[i] ? ab : b.q[i] > a.q[i] ? bb : ab;
                return (ab == raw ? a.e(i) : a.d(i)) + (bb == raw ? b.e(i) : b.d(i));
            };
            per_read(o, "cD", "cM", "cE", td, te, L);
        } else {
            per_read(o, "cD", "cM", "cE", ad, ae, L);
        }
        per_read(o, "aD", "aM", "aE", ad, ae, L);
        if (two) {
            auto bdf = [&](int32_t i) { return b.d(i); };
            auto bef = [&](int32_t i) { return b.e(i); };
            per_read(o, "bD", "bM", "bE", bdf, bef, L);
        }
        shorts16(o, "ad", a.d8, a.d16, L);
        shorts16(o, "ae", a.e8, a.e16, L);
        o.text("ac", a.b, L, kNt16, 0);
        o.text("aq", a.q, L, nullptr, 33);
        if (two) {
            shorts16(o, "bd", b.d8, b.d16, L);
            shorts16(o, "be", b.e8, b.e16, L);
            o.text("bc", b.b, L, kNt16, 0);
            o.text("bq", b.q, L, nullptr, 33);
        }
        return o.n;
    };
    if (!buf) {
#pragma omp parallel for schedule(dynamic, 256)
        for (int64_t k = 0; k < n; k++) off[k + 1] = one(k, nullptr);
        off[0] = 0;
        for (int64_t k = 0; k < n; k++) off[k + 1] += off[k];
        return off[n];
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t k = 0; k < n; k++) one(k, buf + off[k]);
    return off[n];
}

namespace {
// Paired FASTQ text of records appended to buf[0] (first of pair) / buf[1] (second), as
// bsdc_fastq_write formats it; the pairing checks of include/bsdc_io.h.
int32_t format_fastq(const bsdc_bam_records *r, Bytes *buf) {
    const int64_t nr = r->n_rec;
    // record k -> its file (0: first of pair, 1: second) or -1 (not written); pairs must be adjacent
    std::vector<int8_t> dst((size_t)nr, -1);
    for (int64_t k = 0; k < nr; k++) {
        const uint16_t fl = r->flag[k];
        if (fl & (0x100 | 0x800 | 0x200)) continue;  // secondary, supplementary, QC-fail
        if (!(fl & 1)) return fail(BSDC_IO_EFORMAT, "unpaired record in a paired FASTQ write");
        dst[(size_t)k] = (fl & 0x40) ? 0 : 1;
    }
    int64_t want = 0, first = -1;
    for (int64_t k = 0; k < nr; k++) {
        if (dst[(size_t)k] < 0) continue;
        if (dst[(size_t)k] != want) return fail(BSDC_IO_EFORMAT, "records are not in first/second-of-pair order");
        if (want == 0) {
            first = k;
        } else {
            const int64_t l0 = r->name_off[first + 1] - r->name_off[first], l1 = r->name_off[k + 1] - r->name_off[k];
            if (l0 != l1 || memcmp(r->name_buf + r->name_off[first], r->name_buf + r->name_off[k], (size_t)l0) != 0)
                return fail(BSDC_IO_EFORMAT, "mates of a pair have different names");
        }
        want ^= 1;
    }
    if (want) return fail(BSDC_IO_EFORMAT, "a first-of-pair record has no mate");
    // "@name/N\nSEQ\n+\nQUAL\n" per record, sizes -> offsets per file -> parallel format
    std::vector<int64_t> off[2] = {std::vector<int64_t>((size_t)nr + 1), std::vector<int64_t>((size_t)nr + 1)};
    int64_t tot[2] = {(int64_t)buf[0].size(), (int64_t)buf[1].size()};
    for (int64_t k = 0; k < nr; k++) {
        off[0][(size_t)k] = tot[0];
        off[1][(size_t)k] = tot[1];
        const int d = dst[(size_t)k];
        if (d < 0) continue;
        const int64_t ln = r->name_off[k + 1] - r->name_off[k], ls = r->seq_off[k + 1] - r->seq_off[k];
        tot[d] += 1 + ln + 2 + 1 + ls + 1 + 2 + ls + 1;
    }
    buf[0].resize((size_t)tot[0]);
    buf[1].resize((size_t)tot[1]);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < nr; k++) {
        const int d = dst[(size_t)k];
        if (d < 0) continue;
        uint8_t *p = buf[d].data() + off[d][(size_t)k];
        const int64_t ln = r->name_off[k + 1] - r->name_off[k], ls = r->seq_off[k + 1] - r->seq_off[k];
        const bool rev = r->flag[k] & 0x10;  // SamToFastq writes reads in sequencing orientation
        const uint8_t *s = r->seq + r->seq_off[k], *q = r->qual + r->seq_off[k];
        *p++ = '@';
        memcpy(p, r->name_buf + r->name_off[k], (size_t)ln);
        p += ln;
        *p++ = '/';
        *p++ = d == 0 ? '1' : '2';
        *p++ = '\n';
        for (int64_t i = 0; i < ls; i++) *p++ = rev ? kNt16Comp[s[ls - 1 - i] & 15] : kNt16[s[i] & 15];
        *p++ = '\n';
        *p++ = '+';
        *p++ = '\n';
        for (int64_t i = 0; i < ls; i++) *p++ = (uint8_t)(33 + (rev ? q[ls - 1 - i] : q[i]));
        *p++ = '\n';
    }
    return 0;
}
}  // namespace

extern "C" int32_t bsdc_fastq_write(const char *path1, const char *path2, const bsdc_bam_records *r, int32_t level,
                                    int32_t n_threads) {
    set_threads(n_threads);
    Bytes buf[2];
    const int32_t rc = format_fastq(r, buf);
    if (rc != 0) return rc;
    for (int d = 0; d < 2; d++) {
        const int32_t rc2 = write_bgzf(d == 0 ? path1 : path2, buf[d], level);
        if (rc2 != 0) return rc2;
    }
    return 0;
}

// streaming paired-FASTQ writer: the bytes of bsdc_fastq_write over all the records at once
struct bsdc_fastq_writer {
    FILE *f[2] = {nullptr, nullptr};
    int32_t level = 6;
    Bytes tail[2];
    bool no_eof = false;  // a fragment: no EOF block at the close
};

extern "C" int32_t bsdc_fastq_writer_open(const char *path1, const char *path2, int32_t level, bsdc_fastq_writer **out) {
    *out = nullptr;
    auto *w = new bsdc_fastq_writer();
    w->level = level;
    for (int d = 0; d < 2; d++) {
        w->f[d] = fopen(d == 0 ? path1 : path2, "wb");
        if (!w->f[d]) {
            if (d == 1) fclose(w->f[0]);
            delete w;
            return fail(BSDC_IO_EIO, std::string("cannot create ") + (d == 0 ? path1 : path2));
        }
    }
    *out = w;
    return 0;
}

extern "C" int32_t bsdc_fastq_writer_add(bsdc_fastq_writer *w, const bsdc_bam_records *r, int32_t n_threads) {
    set_threads(n_threads);
    int32_t rc = format_fastq(r, w->tail);
    if (rc != 0) return rc;
    for (int d = 0; d < 2; d++) {
        const int64_t whole = ((int64_t)w->tail[d].size() / kBlock) * kBlock;
        if (whole > 0) {
            rc = deflate_write(w->f[d], w->tail[d].data(), whole, w->level);
            if (rc != 0) return rc;
            w->tail[d].erase(w->tail[d].begin(), w->tail[d].begin() + whole);
        }
    }
    return 0;
}

// The same with the whole blocks compressed by the caller (bsdc_bam_writer_encode / take / put for
// the two files): whole[d] = the bytes of whole blocks now at the front of file d's tail.
extern "C" int32_t bsdc_fastq_writer_encode(bsdc_fastq_writer *w, const bsdc_bam_records *r, int32_t n_threads,
                                            int64_t *whole) {
    set_threads(n_threads);
    const int32_t rc = format_fastq(r, w->tail);
    if (rc != 0) return rc;
    for (int d = 0; d < 2; d++) whole[d] = ((int64_t)w->tail[d].size() / kBlock) * kBlock;
    return 0;
}

extern "C" int32_t bsdc_fastq_writer_take(bsdc_fastq_writer *w, int32_t which, int64_t nblk, uint8_t *dst, uint32_t *crc,
                                          int32_t n_threads) {
    set_threads(n_threads);
    if (which != 0 && which != 1) return fail(BSDC_IO_EFORMAT, "no such FASTQ file");
    return take_blocks(w->tail[which], nblk, dst, crc);
}

extern "C" int32_t bsdc_fastq_writer_put(bsdc_fastq_writer *w, int32_t which, int64_t nblk, uint8_t *packed,
                                         const int32_t *sizes, const uint32_t *crc, const uint8_t *raw,
                                         int32_t n_threads) {
    set_threads(n_threads);
    if (which != 0 && which != 1) return fail(BSDC_IO_EFORMAT, "no such FASTQ file");
    return put_blocks(w->f[which], w->level, nblk, packed, sizes, crc, raw);
}

extern "C" int32_t bsdc_fastq_writer_close(bsdc_fastq_writer *w, int32_t n_threads) {
    if (!w) return 0;
    set_threads(n_threads);
    int32_t rc = 0;
    for (int d = 0; d < 2; d++) {
        if (rc == 0) rc = deflate_write(w->f[d], w->tail[d].data(), (int64_t)w->tail[d].size(), w->level);
        if (rc == 0 && !w->no_eof && fwrite(kBgzfEof, 1, 28, w->f[d]) != 28) rc = fail(BSDC_IO_EIO, "BGZF write failed");
        if (fclose(w->f[d]) != 0 && rc == 0) rc = fail(BSDC_IO_EIO, "BGZF close failed");
    }
    delete w;
    return rc;
}

extern "C" int32_t bsdc_fastq_writer_fragment(bsdc_fastq_writer *w) {
    if (!w) return fail(BSDC_IO_EFORMAT, "no writer");
    w->no_eof = true;
    return 0;
}

extern "C" int32_t bsdc_fastq_writer_flush(bsdc_fastq_writer *w, int32_t n_threads) {
    set_threads(n_threads);
    for (int d = 0; d < 2; d++) {
        const int32_t rc = deflate_write(w->f[d], w->tail[d].data(), (int64_t)w->tail[d].size(), w->level);
        w->tail[d].clear();
        if (rc != 0) return rc;
    }
    return 0;
}

extern "C" void bsdc_fastq_writer_tell(bsdc_fastq_writer *w, int64_t *out) {
    for (int d = 0; d < 2; d++) out[d] = (int64_t)ftello(w->f[d]);
}

// Packed byte tables (entry r of a table = buf[off[r], off[r + 1])): per entry, the concatenation
// of k parts (a table, or a constant: off NULL, buf const_len bytes).  out_buf NULL: fills out_off
// [n + 1] and returns the total; else fills out_buf in parallel.
extern "C" int64_t bsdc_table_concat(int64_t n, int32_t k, const int64_t *const *offs, const uint8_t *const *bufs,
                                     const int64_t *const_len, int64_t *out_off, uint8_t *out_buf, int32_t n_threads) {
    set_threads(n_threads);
    if (!out_buf) {
        int64_t t = 0;
        for (int64_t r = 0; r < n; r++) {
            out_off[r] = t;
            for (int32_t j = 0; j < k; j++) t += offs[j] ? offs[j][r + 1] - offs[j][r] : const_len[j];
        }
        out_off[n] = t;
        return t;
    }
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; r++) {
        uint8_t *d = out_buf + out_off[r];
        for (int32_t j = 0; j < k; j++) {
            const int64_t l = offs[j] ? offs[j][r + 1] - offs[j][r] : const_len[j];
            memcpy(d, offs[j] ? bufs[j] + offs[j][r] : bufs[j], (size_t)l);
            d += l;
        }
    }
    return out_off[n];
}

// rank[i] = byte-order rank of entry i of a packed table among its entries (equal entries share a
// rank): the TemplateCoordinate key's MI and name components (batch.lex_rank).
extern "C" void bsdc_table_rank(int64_t n, const int64_t *off, const uint8_t *buf, int64_t *rank, int32_t n_threads) {
    set_threads(n_threads);
    std::vector<int64_t> ord((size_t)n);
    for (int64_t i = 0; i < n; i++) ord[(size_t)i] = i;
    auto sv = [&](int64_t i) { return std::string_view((const char *)buf + off[i], (size_t)(off[i + 1] - off[i])); };
    auto less = [&](int64_t a, int64_t b) { return sv(a) < sv(b); };
#ifdef _OPENMP
    __gnu_parallel::sort(ord.begin(), ord.end(), less);
#else
    std::sort(ord.begin(), ord.end(), less);
#endif
    int64_t r = -1;
    for (int64_t k = 0; k < n; k++) {
        if (k == 0 || sv(ord[(size_t)k]) != sv(ord[(size_t)k - 1])) r++;
        rank[ord[(size_t)k]] = r;
    }
}

// Entries idx[0], idx[1], ... of a packed table; two-phase as bsdc_table_concat.
extern "C" int64_t bsdc_table_take(int64_t n, const int64_t *idx, const int64_t *off, const uint8_t *buf, int64_t *out_off,
                                   uint8_t *out_buf, int32_t n_threads) {
    set_threads(n_threads);
    if (!out_buf) {
        int64_t t = 0;
        for (int64_t r = 0; r < n; r++) {
            out_off[r] = t;
            t += off[idx[r] + 1] - off[idx[r]];
        }
        out_off[n] = t;
        return t;
    }
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; r++) memcpy(out_buf + out_off[r], buf + off[idx[r]], (size_t)(off[idx[r] + 1] - off[idx[r]]));
    return out_off[n];
}

extern "C" void bsdc_unpack_nibbles(int64_t n_bytes, const uint8_t *in, uint8_t *out, int32_t n_threads) {
    set_threads(n_threads);
    const int64_t nb = (n_bytes + 4095) / 4096;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nb; b++) {
        const int64_t e = std::min(n_bytes, (b + 1) * 4096);
        for (int64_t i = b * 4096; i < e; i++) {
            out[2 * i] = in[i] >> 4;
            out[2 * i + 1] = in[i] & 15;
        }
    }
}

extern "C" void bsdc_rows_gather(int64_t n, const int64_t *row, const int32_t *len, int64_t stride, const uint8_t *src,
                                 const int64_t *out_off, uint8_t *out, int32_t n_threads) {
    set_threads(n_threads);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) memcpy(out + out_off[i], src + row[i] * stride, (size_t)len[i]);
}

extern "C" int32_t bsdc_family_image(int64_t n_rec, const int64_t *src_off, const int64_t *len, const int64_t *dst_off,
                                     const uint8_t *seq, const uint8_t *qual, int64_t n_slots, uint8_t *packed,
                                     uint8_t *qual_out, int32_t n_threads) {
    set_threads(n_threads);
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(| : bad)
    for (int64_t r = 0; r < n_rec; r++) {
        const int64_t d = dst_off[r] + 1, l = len[r];
        if (dst_off[r] < 0 || (dst_off[r] & 1) || d + l > n_slots) {
            bad |= 1;
            continue;
        }
        const uint8_t *s = seq + src_off[r];
        memcpy(qual_out + d, qual + src_off[r], (size_t)l);
        // nibble d (odd) is the low half of byte d / 2; then whole bytes, then a last high nibble
        uint8_t *p = packed + (d >> 1);
        int64_t j = 0;
        if (l > 0) {
            *p = (uint8_t)((*p & 0xF0) | (s[0] & 15));
            p++;
            j = 1;
        }
        for (; j + 1 < l; j += 2) *p++ = (uint8_t)(((s[j] & 15) << 4) | (s[j + 1] & 15));
        if (j < l) *p = (uint8_t)(((s[j] & 15) << 4) | (*p & 0x0F));
    }
    if (bad) return fail(BSDC_IO_EFORMAT, "family image: record slot out of range or misaligned");
    return 0;
}
