/* bsdc_io.h -- host-side BAM/BGZF codec for the step-5 drop-in (libbsdc_io.so, C++/zlib/OpenMP).
 *
 * Replaces the file I/O around the step: the reference's tools read and write BAM
 * through pysam (tools/1.convert_AG_to_CT.py:86-99, tools/2.extend_gap.py:147-190) and fgbio
 * through htsjdk (main.snake.py:152,163).  The reader hands the step the structure-of-arrays
 * record stream the family builder consumes (bsseqconsensusreads_amd.records.RawRecords): MI tags
 * interned to MI-base ids with the /A|/B strand, QNAMEs interned, MC parsed to cigar ops, LA/RD
 * pulled out, everything else kept as raw aux bytes.  The writer encodes records and BGZF-deflates
 * blocks in parallel.
 *
 * Conventions: 0 on success, a negative code on failure (message in bsdc_io_last_error(), per
 * thread); caller-owned output arrays, sized from bsdc_bam_sizes. */
#ifndef BSDC_IO_H
#define BSDC_IO_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define BSDC_IO_ABI_VERSION 12
#define BSDC_IO_EFORMAT (-10) /* not BGZF/BAM, truncated, bad CRC */
#define BSDC_IO_EIO (-11)     /* open/read/write failed */
#define BSDC_IO_EINVAL (-22)  /* bad argument */

typedef struct bsdc_bam bsdc_bam; /* a decoded BAM held in host memory */

typedef struct {
    int64_t n_rec;
    int64_t n_bases;      /* sum of l_seq */
    int64_t n_cigar;      /* cigar ops */
    int64_t n_mc;         /* MC-tag cigar ops */
    int64_t aux_bytes;
    int64_t n_names, name_bytes; /* distinct QNAMEs */
    int64_t n_mi, mi_bytes;      /* distinct MI bases (MI up to the first '/') */
    int64_t header_bytes;        /* SAM header text */
    int32_t n_ref;
    int64_t ref_name_bytes;
} bsdc_bam_sizes;

/* Output arrays (caller-allocated; n = n_rec).  seq is one nt16 code per byte. */
typedef struct {
    uint16_t *flag;
    int32_t *tid, *pos;
    uint8_t *mapq;
    int32_t *l_seq;
    int64_t *seq_off;
    uint8_t *seq, *qual;
    int64_t *cig_off;
    int32_t *n_cig;
    uint32_t *cigar;
    int32_t *next_tid, *next_pos, *tlen;
    int32_t *name_id;
    int64_t *name_off; /* [n_names + 1] */
    char *name_buf;
    int32_t *mi_id;     /* -1: no (or empty) MI tag */
    int8_t *mi_strand;  /* 0 "/A", 1 "/B", -1 neither */
    int64_t *mi_off;    /* [n_mi + 1] */
    char *mi_buf;
    int64_t *mc_off;    /* -1: no MC tag */
    int32_t *mc_n;
    uint32_t *mc_cigar;
    int32_t *la, *rd;   /* -1: tag absent */
    int64_t *aux_off;   /* [n + 1] */
    uint8_t *aux;
    char *header;
    int64_t *ref_len;       /* [n_ref] */
    int64_t *ref_name_off;  /* [n_ref + 1] */
    char *ref_name_buf;
} bsdc_bam_arrays;

int32_t bsdc_io_abi_version(void);
const char *bsdc_io_last_error(void);

/* Reads and decodes a whole BAM (BGZF blocks inflated in parallel, records parsed in parallel). */
int32_t bsdc_bam_read(const char *path, int32_t n_threads, bsdc_bam **out);
void bsdc_bam_sizes_of(const bsdc_bam *b, bsdc_bam_sizes *s);
int32_t bsdc_bam_copy(const bsdc_bam *b, const bsdc_bam_arrays *a);
void bsdc_bam_free(bsdc_bam *b);

/* Streaming reader (bounded memory): the file's records as a sequence of decoded chunks
 * (bsdc_bam objects, read with bsdc_bam_sizes_of / bsdc_bam_copy, freed with bsdc_bam_free; names
 * and MI ids are chunk-local).  A chunk holds at least min_bytes of record bytes (the rest of the
 * file at its end) and ends where a cut is safe for a coordinate-sorted file: every record before
 * the cut, and its mate, lies more than `slack` positions before the next record on that record's
 * contig, or on an earlier contig.  Templates and MI families (which share their template's
 * coordinates) then never straddle chunks, and each chunk's TemplateCoordinate keys sort before
 * the next chunk's, so the chunks' family plans concatenate to the whole file's (tests/test_stream.py).
 * read_size: compressed bytes read (and inflated in parallel) per refill.  *out = NULL at the end. */
typedef struct bsdc_bam_stream bsdc_bam_stream;
int32_t bsdc_bam_stream_open(const char *path, int32_t n_threads, int64_t read_size, bsdc_bam_stream **out);
int32_t bsdc_bam_stream_fill(bsdc_bam_stream *s);
int32_t bsdc_bam_stream_next(bsdc_bam_stream *s, int64_t min_bytes, int64_t slack, bsdc_bam **out);
int32_t bsdc_bam_stream_header(const bsdc_bam_stream *s, bsdc_bam **out); /* header only, no records */
void bsdc_bam_stream_close(bsdc_bam_stream *s);
/* bsdc_bam_free for a chunk of this stream that has been copied out: its buffer goes back to the
 * stream for the next chunk (no fresh pages per chunk).  Any thread may recycle a chunk while the
 * stream reads the next one; a closed stream is deleted when its last chunk comes back. */
void bsdc_bam_stream_recycle(bsdc_bam_stream *s, bsdc_bam *b);
/* The next chunk unparsed (records listed, not decoded): bsdc_bam_parse it, on any thread, before
 * bsdc_bam_sizes_of / bsdc_bam_copy.  bsdc_bam_stream_next = next_raw + parse.  Lets one thread cut
 * the next chunk while another decodes this one (bam.step5_stream). */
int32_t bsdc_bam_stream_next_raw(bsdc_bam_stream *s, int64_t min_bytes, int64_t slack, bsdc_bam **out);
int32_t bsdc_bam_parse(bsdc_bam *b, int32_t n_threads);
/* Step 1's chunks (rule call_consensus_reads_molecular, main.snake.py:46-55): the input is in
 * GroupReadsByUmi order, where fgbio CallMolecularConsensusReads' unit -- a run of consecutive
 * records with one MI value -- is contiguous.  The next chunk unparsed: the buffered records up to
 * the first record at or past min_bytes whose MI value differs from its predecessor's (the rest of
 * the file at its end), so no run straddles two chunks and the chunks' runs concatenate to the
 * whole file's.  No coordinate order is needed.  A stream is cut either this way or by
 * bsdc_bam_stream_next_raw, not both.  *out = NULL at the end. */
int32_t bsdc_bam_stream_next_runs(bsdc_bam_stream *s, int64_t min_bytes, bsdc_bam **out);

/* Rank-parallel step 5 over one coordinate-sorted BAM (IO ABI 9; bsseqconsensusreads_amd/ranks.py).
 * Rank r owns the templates whose TemplateCoordinate key lies in [X_r, X_r+1): it decodes the
 * record window around that interval and keeps the records it owns, so the ranks' outputs, in
 * rank order, are the one stream's.  A boundary X sits in a gap of the keys (no family straddles
 * it), so it exists inside a contig even where every position is covered by templates.
 * bsdc_bam_find_cut: from the first BGZF block at or after file offset `from`, the first record
 * boundary (8 consecutive records that parse, bins included), then on that record's contig the
 * first position x >= its coordinate + min_span with no same-contig template key within `guard`
 * positions of x among the records read, and the records read reaching x + guard + slack (an
 * unread record's key is at least its position - slack).  out[8] = {block file offset, offset in
 * the block's uncompressed bytes} of the first record at or past x - slack (where the next rank's
 * window starts), the same of the first record at or past x + slack (where this rank's window
 * ends), then X = {contig << 32 | contig, x}, the coordinate contig << 32 | x, and 1 -- or -1s and
 * 0: no boundary within max_bytes of compressed data on that contig.
 * bsdc_bam_stream_open_range: a stream of the records from (start_block, start_off) -- start_block
 * -1: the first record after the header -- up to (end_block, end_off) exclusive -- end_block -1:
 * the end of the file.  bsdc_bam_stream_set_owner (before the first chunk): keep only the records
 * whose key k has bounds[rank - 1] <= k < bounds[rank], bounds = n_bounds triples {key first,
 * key second, coordinate} (find_cut's out[4..6]), and count as foreign the dropped records whose
 * coordinate lies outside their owner's window [its lower coordinate - slack, its upper + slack)
 * (a mate on another contig, or unmapped: the owner never reads them; ranks.py then falls back to
 * one range); flags BSDC_OWN_STOP_FOREIGN: the first one fails the stream (BSDC_IO_EFORMAT,
 * "foreign record ...").  With bsdc_bam_stream_set_defer no record is foreign: a far record (below)
 * is spilled by the rank whose core coordinates [its lower bound, its upper bound) hold it and its
 * key registered by the key's owner.  bsdc_bam_stream_range_stats: {records read, first coordinate,
 * dropped, foreign, spilled, deferred families, the most record bytes buffered at a chunk
 * selection}. */
int32_t bsdc_bam_find_cut(const char *path, int32_t n_threads, int64_t from, int64_t min_span, int64_t slack,
                          int64_t guard, int64_t max_bytes, int64_t *out);
int32_t bsdc_bam_stream_open_range(const char *path, int32_t n_threads, int64_t read_size, int64_t start_block,
                                   int64_t start_off, int64_t end_block, int64_t end_off, bsdc_bam_stream **out);
#define BSDC_OWN_STOP_FOREIGN 1   /* set_owner flags: the first foreign record fails the stream */
int32_t bsdc_bam_stream_set_owner(bsdc_bam_stream *s, int32_t rank, const int64_t *bounds, int32_t n_bounds,
                                  int64_t slack, int32_t flags);
void bsdc_bam_stream_range_stats(const bsdc_bam_stream *s, int64_t *st);
/* (IO ABI 12) Deferred templates: bounded memory whatever the inserts.  A template whose other end
 * lies more than `span` positions away (bsdc_bam_stream_set_defer, before the first chunk; 0 = off)
 * or on another contig, unmapped or absent (a cross key: it sorts at its contig's end) would hold
 * every family after its key until the stream reaches that end.  Its records (a "far" record: its
 * own mate fields say so) leave the stream for the spill instead, unless its MI family is buffered
 * (a molecule whose other templates are near: the record joins it), and its key is registered.  A
 * buffered family whose coarse keys come within 3 x 4 positions of a registered key may interleave
 * with it in TemplateCoordinate order: it is spilled too, and its keys registered.  So the chunks'
 * families and the spill's are each whole, and the output is the chunks' outputs with the spill's
 * families spliced in at the registered keys (bam.py: a second pass over the spill, then
 * assembly).  A far record whose key lies at or behind the output already cut (its template's lower
 * record is missing) fails the stream (BSDC_IO_EFORMAT).
 * bsdc_bam_stream_spill: the spilled entries so far -- per record an int64 coordinate (contig << 32
 * | position, unmapped last), an int64 sequence number (its place in the stream's file order), then
 * the record (block_size-prefixed) -- returns their bytes; with dst, copies them there and forgets
 * them.  Sorted by (coordinate, sequence) they are in file order.
 * bsdc_bam_stream_splices: the registered keys the last chunk reported (2 int64 each, ascending;
 * after the last chunk, at the end of the stream, every key left): its output is cut before its
 * first family whose key exceeds each, and the spill's families of that key go there.  Returns
 * their count; with dst, copies them there and forgets them.
 * bsdc_bam_rec_keys: the coarse TemplateCoordinate key of every record of a chunk or file (raw or
 * parsed), in record order: out[2k] = lower end's contig << 32 | other end's contig (0x7FFFFFFF:
 * unmapped or absent), out[2k + 1] = the lower end's unclipped 5' position, from the input's
 * cigar and MC; within 4 positions of the key of the records tools 1 and 2 make. */
int32_t bsdc_bam_stream_set_defer(bsdc_bam_stream *s, int64_t span);
int64_t bsdc_bam_stream_spill(bsdc_bam_stream *s, uint8_t *dst);
int64_t bsdc_bam_stream_splices(bsdc_bam_stream *s, int64_t *dst);
int32_t bsdc_bam_rec_keys(const bsdc_bam *b, int64_t *out);
/* Spill entries (bsdc_bam_stream_spill's bytes, several streams' concatenated) -> their records,
 * sorted by (coordinate, sequence) -- file order -- into out (stable for equal pairs); returns the
 * records' bytes (out NULL: the size only) and their count in *n_rec (if not NULL), < 0 on a
 * malformed spill. */
int64_t bsdc_spill_sort(const uint8_t *data, int64_t n, uint8_t *out, int64_t *n_rec);

/* Records to write (n_rec entries; every *_off array has n_rec + 1 entries). */
typedef struct {
    int64_t n_rec;
    const uint16_t *flag;
    const int32_t *tid, *pos;
    const uint8_t *mapq;
    const int32_t *next_tid, *next_pos, *tlen;
    const int64_t *name_off;
    const char *name_buf;
    const int64_t *cig_off;
    const uint32_t *cigar;
    const int64_t *seq_off;  /* l_seq = seq_off[k+1] - seq_off[k] */
    const uint8_t *seq;      /* nt16 codes, one per byte */
    const uint8_t *qual;
    const int64_t *aux_off;
    const uint8_t *aux;
    const int64_t *aux2_off; /* optional (NULL = none): more aux bytes written after aux (the consensus
                                tags, so they are never concatenated to the per-family tags first) */
    const uint8_t *aux2;
} bsdc_bam_records;

/* Writes header + records as BGZF (blocks deflated in parallel at `level`), with the EOF block. */
int32_t bsdc_bam_write(const char *path, const char *header_text, int64_t header_len, int32_t n_ref,
                       const int64_t *ref_name_off, const char *ref_name_buf, const int64_t *ref_len,
                       const bsdc_bam_records *r, int32_t level, int32_t n_threads);

/* Streaming writer: the bytes bsdc_bam_write writes for all the records at once, written as
 * records are added (whole BGZF blocks deflated in parallel as they fill). */
typedef struct bsdc_bam_writer bsdc_bam_writer;
int32_t bsdc_bam_writer_open(const char *path, const char *header_text, int64_t header_len, int32_t n_ref,
                             const int64_t *ref_name_off, const char *ref_name_buf, const int64_t *ref_len,
                             int32_t level, bsdc_bam_writer **out);
int32_t bsdc_bam_writer_add(bsdc_bam_writer *w, const bsdc_bam_records *r, int32_t n_threads);
/* The same with the whole blocks compressed by the caller (on the GPU: bsdc_bgzf_deflate in
 * libbsdc): encode returns the byte count of whole 65280-byte blocks now at the front of the tail
 * (*data: valid until the next call); take moves the first nblk of them to dst with their CRC32s;
 * put writes nblk taken blocks back compressed -- block b's BGZF bytes packed back to back,
 * sizes[b] each with the CRC32 / ISIZE bytes still to fill (from crc[b]), 0 = deflate it here from
 * raw (what take copied) -- in order.  Takes and puts come in the same order. */
int64_t bsdc_bam_writer_encode(bsdc_bam_writer *w, const bsdc_bam_records *r, int32_t n_threads, const uint8_t **data);
int32_t bsdc_bam_writer_take(bsdc_bam_writer *w, int64_t nblk, uint8_t *dst, uint32_t *crc, int32_t n_threads);
int32_t bsdc_bam_writer_put(bsdc_bam_writer *w, int64_t nblk, uint8_t *packed, const int32_t *sizes,
                            const uint32_t *crc, const uint8_t *raw, int32_t n_threads);
int32_t bsdc_bam_writer_close(bsdc_bam_writer *w, int32_t n_threads);
/* A writer of one piece of a BAM assembled later (ranks.py): keep_header 0 drops the header
 * encoded at the open; no EOF block at the close.  Call right after the open. */
int32_t bsdc_bam_writer_fragment(bsdc_bam_writer *w, int32_t keep_header);
/* (IO ABI 11) flush: everything added so far leaves as BGZF blocks (the last one short), so the
 * file may be cut at tell() (its bytes written); raw: block_size-prefixed BAM records appended as
 * they are (a spill file). */
int32_t bsdc_bam_writer_flush(bsdc_bam_writer *w, int32_t n_threads);
int64_t bsdc_bam_writer_tell(bsdc_bam_writer *w);
int32_t bsdc_bam_writer_raw(bsdc_bam_writer *w, const uint8_t *data, int64_t n, int32_t n_threads);

/* Paired FASTQ of records, as picard SamToFastq F=path1 F2=path2 writes them (the step after the
 * duplex call, main.snake.py:167-177; parity unpinned): "@name/1" or "/2", SEQ, "+", QUAL+33,
 * reverse-strand records reverse-complemented; secondary, supplementary and QC-fail records
 * skipped.  The written records must come as adjacent first/second-of-pair mates of one name
 * (an error otherwise, as picard raises on an unpaired mate).  Each file is BGZF-framed gzip. */
int32_t bsdc_fastq_write(const char *path1, const char *path2, const bsdc_bam_records *r, int32_t level,
                         int32_t n_threads);

/* Streaming paired-FASTQ writer: the bytes bsdc_fastq_write writes for all the records at once
 * (each add must hold whole pairs). */
typedef struct bsdc_fastq_writer bsdc_fastq_writer;
int32_t bsdc_fastq_writer_open(const char *path1, const char *path2, int32_t level, bsdc_fastq_writer **out);
int32_t bsdc_fastq_writer_add(bsdc_fastq_writer *w, const bsdc_bam_records *r, int32_t n_threads);
/* The FASTQ pair's whole blocks compressed by the caller, as for the BAM writer above: encode
 * reports whole[d], the bytes of whole 65280-byte blocks at the front of file d's tail (d = 0, 1);
 * take / put move and write file `which`'s blocks like bsdc_bam_writer_take / _put. */
int32_t bsdc_fastq_writer_encode(bsdc_fastq_writer *w, const bsdc_bam_records *r, int32_t n_threads, int64_t *whole);
int32_t bsdc_fastq_writer_take(bsdc_fastq_writer *w, int32_t which, int64_t nblk, uint8_t *dst, uint32_t *crc,
                               int32_t n_threads);
int32_t bsdc_fastq_writer_put(bsdc_fastq_writer *w, int32_t which, int64_t nblk, uint8_t *packed, const int32_t *sizes,
                              const uint32_t *crc, const uint8_t *raw, int32_t n_threads);
int32_t bsdc_fastq_writer_close(bsdc_fastq_writer *w, int32_t n_threads);
int32_t bsdc_fastq_writer_fragment(bsdc_fastq_writer *w);
int32_t bsdc_fastq_writer_flush(bsdc_fastq_writer *w, int32_t n_threads);
void bsdc_fastq_writer_tell(bsdc_fastq_writer *w, int64_t *out);  /* out[2]: bytes written per file */ /* no EOF blocks at the close */

/* Packed byte tables (entry r = buf[off[r], off[r + 1])), for the output records: per entry the
 * concatenation of k parts (a table, or a constant when offs[j] is NULL: bufs[j], const_len[j]
 * bytes), and a gather of entries.  Two phases: out_buf NULL fills out_off [n + 1] and returns the
 * total bytes; then the bytes, in parallel. */
int64_t bsdc_table_concat(int64_t n, int32_t k, const int64_t *const *offs, const uint8_t *const *bufs,
                          const int64_t *const_len, int64_t *out_off, uint8_t *out_buf, int32_t n_threads);
void bsdc_table_rank(int64_t n, const int64_t *off, const uint8_t *buf, int64_t *rank, int32_t n_threads);
int64_t bsdc_table_take(int64_t n, const int64_t *idx, const int64_t *off, const uint8_t *buf, int64_t *out_off,
                        uint8_t *out_buf, int32_t n_threads);
/* Fixed-stride rows -> a packed table: out[out_off[i], + len[i]) = src[row[i] * stride, + len[i])
 * (the consensus rows of the emitted families, in record order; len[i] <= stride). */
/* Packed nt16 (two per byte, high nibble first) -> one code per byte: out[2i] = in[i] >> 4,
 * out[2i + 1] = in[i] & 15 (the consensus rows the kernels write). */
void bsdc_unpack_nibbles(int64_t n_bytes, const uint8_t *in, uint8_t *out, int32_t n_threads);
void bsdc_rows_gather(int64_t n, const int64_t *row, const int32_t *len, int64_t stride, const uint8_t *src,
                      const int64_t *out_off, uint8_t *out, int32_t n_threads);

/* Host side of the family batch (bsseqconsensusreads_amd/batch.py, include/bsdc.h layout): record r's
 * len[r] bases and quals, from seq/qual (nt16 codes and phred, one per byte) at src_off[r], go to
 * nibble / byte dst_off[r] + 1 of the image (dst_off even; the caller zeroes both outputs):
 * packed holds n_slots nibbles, two per byte, high nibble first; qual_out n_slots bytes. */
int32_t bsdc_family_image(int64_t n_rec, const int64_t *src_off, const int64_t *len, const int64_t *dst_off,
                          const uint8_t *seq, const uint8_t *qual, int64_t n_slots, uint8_t *packed,
                          uint8_t *qual_out, int32_t n_threads);

/* Consensus RX per family for the duplex output records (fgbio's consensus
 * UMI, parity unpinned): every family record's RX, a /B-strand record's two '-'-separated halves
 * swapped, then per position the most common character over the RX values of the most common
 * length (a tie -> 'N').  Families with no RX get an empty string.  Output: width = longest RX
 * (call with out = NULL to get it), out[f * width ...] and out_len[f]. */
int64_t bsdc_rx_consensus(int64_t n_fam, const int64_t *fam_rec_off, const int64_t *rec, const int8_t *strand,
                          const int64_t *aux_off, const uint8_t *aux, char *out, int32_t *out_len,
                          int32_t n_threads);

/* fgbio consensus tags of n output records, BAM aux bytes (replaces the tag block of fgbio
 * DuplexConsensusCaller.createSamRecord (kind 0) / VanillaUmiConsensusCaller.createSamRecord
 * (kind 1), main.snake.py:54,163; fgbio unvendored: PARITY UNPINNED).  Record k's consensus has
 * out_len[k] columns; row_a[k] / row_b[k] are its single-strand reads' rows of the ss_* arrays
 * libbsdc writes with BSDC_MODE_TAGS (row_b = -1: one strand; kind 1 uses row_a only): depths and
 * errors as bytes, a family f with ss_wide[f] = w >= 0 read from rows (w, s) of the exact u16
 * ss_wdepth / ss_werr instead (include/bsdc.h; ss_wide NULL: none; IO ABI 10).
 *   kind 0: cD cM cE, aD aM aE, [bD bM bE], ad ae ac aq, [bd be bc bq]
 *   kind 1: cD cM cE, cd ce
 * Call with buf = NULL to fill off[0..n] (prefix sums of the sizes), then with buf. Returns the
 * total bytes. */
int64_t bsdc_consensus_tags(int64_t n, const int64_t *row_a, const int64_t *row_b, const int32_t *out_len,
                            int32_t kind, int32_t stride, const uint8_t *ss_base, const uint8_t *ss_qual,
                            const uint8_t *ss_depth, const uint8_t *ss_err, const int32_t *ss_wide,
                            const uint16_t *ss_wdepth, const uint16_t *ss_werr, int64_t *off, uint8_t *buf,
                            int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
