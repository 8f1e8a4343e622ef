/*
 * micall_hip.h -- C-ABI of libmicall_hip.so, the MI355X (gfx950) drop-in for
 * MiCall-Lite's iterative remap hot path.
 *
 * The reference crosses two boundaries on this path; every entry point below
 * replaces one of them (file:line into the reference):
 *
 *   1. the bowtie2 / bowtie2-build process boundary, reached through
 *      micall/utils/externals.py:106-125 (CommandWrapper.yield_output) and
 *      :185-203 (Bowtie2Build.build):
 *        bowtie2-build-s ... -f <fasta> <template>   prelim_map.py:106,
 *                                                    remap.py:695
 *          -> mh_index_build
 *        bowtie2 ... -1 R1 -2 R2 | -U R [--local]    prelim_map.py:134,
 *                                                    remap.py:734
 *          -> mh_reads_load / mh_reads_load_fastq (FASTQ ingest, once),
 *             mh_map (one mapping pass), mh_alns_fetch / mh_format_rows
 *             (the SAM lines bowtie2 would print), mh_map_counts (the
 *             per-line tallies remap.py:743-755 and :485-515 make);
 *   2. the pileup the reference runs in Python on the SAM text,
 *      remap.py:141-306 (sam_to_conseqs -> merge_reads -> apply_cigar /
 *      merge_pairs / merge_inserts -> update_counts)
 *          -> mh_rows_load (SAM rows read back from prelim.csv),
 *             mh_pileup, mh_pileup_fetch / mh_pileup_events,
 *             mh_pileup_export / mh_pileup_import (RCCL all-reduce between
 *             ranks, done by the caller on device buffers);
 *   3. the _gotoh2 C-extension boundary, micall/alignment/src/_gotoh2.c:544-607
 *      (align_wrapper, "ssiiisO")
 *          -> mh_gotoh_align;
 *   4. (next stage) sam2aln's Python merge of remap.csv,
 *      micall/core/sam2aln.py:395-478
 *          -> mh_sam2aln_csv, mh_sam2aln_output;
 *   5. (the stage before) censor_fastq.censor's per-base
 *      Python loop, micall/core/censor_fastq.py:32-102
 *          -> mh_censor_fastq / mh_censor_staged, mh_censor_output /
 *             mh_censor_write;
 *   6. (the stage after sam2aln) aln2counts' per-read loops,
 *      SequenceReport._count_reads (micall/core/aln2counts.py:115-172) and
 *      InsertionWriter.write (:748-811)
 *          -> mh_a2c_load_csv / mh_a2c_load_rows, mh_a2c_counts,
 *             mh_a2c_inserts.
 *
 * Conventions: every function returns 0 on success, -1 on traceback failure
 * (mh_gotoh_align only), -2 on out-of-memory, -3 on a bad argument, -4 on a
 * HIP runtime error, -5 when the HIP device or kernels are unavailable.
 * mh_last_error() describes the last failure of the calling thread.  No C++
 * exception and no exit() crosses this boundary.  All host buffers are owned
 * by the caller; device buffers are owned by the context.  One context per
 * device; calls on one context are not thread-safe, calls on different
 * contexts are independent (ctypes releases the GIL around each call).
 */
#ifndef MICALL_HIP_H
#define MICALL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_MAXOPS 128

enum { MH_E2E = 0, MH_LOCAL = 1 };          /* bowtie2 default / --local */
enum { MH_OP_M = 0, MH_OP_I = 1, MH_OP_D = 2, MH_OP_S = 4 };

/* Scoring knobs MiCall passes to bowtie2 (prelim_map.py:27-30,114-131). */
typedef struct {
    int mode;                 /* MH_E2E (prelim_map) or MH_LOCAL (remap) */
    int rdg_open, rdg_ext;    /* --rdg 10,3 */
    int rfg_open, rfg_ext;    /* --rfg 10,3 */
    int maxins;               /* -X 1200 */
} mh_params;

/* One SAM record of one read, fields as bowtie2 prints them.  Layout is
 * identical to oracle/og_mapper.h og_aln. */
typedef struct {
    int32_t ref, pos, rev, score, secbest, flag, mapq, rnext, pnext, tlen;
    int32_t sam_ref, sam_pos, xm, xo, xg, nm, ys, yt, yf, n_cigar;
    uint32_t cigar[MH_MAXOPS];   /* (len << 4) | op */
} mh_aln;

typedef struct mh_ctx mh_ctx;

int mh_version(void);
int mh_last_error(char *buf, size_t cap);
int mh_device_count(int *n);

int mh_ctx_create(int device, mh_ctx **out);
int mh_ctx_destroy(mh_ctx *ctx);
int mh_ctx_sync(mh_ctx *ctx);
/* the hipStream_t the context launches on (as an opaque handle) */
int mh_ctx_stream(mh_ctx *ctx, void **stream);

/* ---- reference set: replaces bowtie2-build ---------------------------- */
int mh_index_build(mh_ctx *ctx, int n_refs, const char *const *seqs, int seedlen);

/* ---- reads: replaces bowtie2's FASTQ input (-1/-2/-U) ------------------ */
/* Reads back to back; paired: reads 2p and 2p+1 are mates 1 and 2.  Kept
 * resident on the device (2-bit bases + N mask + qualities) across passes. */
int mh_reads_load(mh_ctx *ctx, int64_t n_reads, int paired, const uint8_t *seq,
                  const uint8_t *qual, const int64_t *offsets, const int32_t *lens);
/* Parse (gzip or plain) FASTQ files and load them; path2 may be NULL.
 * Keeps the read names (bowtie2 QNAME rules) for mh_format_rows. */
int mh_reads_load_fastq(mh_ctx *ctx, const char *path1, const char *path2, int64_t *n_reads);
/* One rank's block of a sharded run: the same parse (raw line count of the
 * whole file included), but only units (pairs, or reads when unpaired)
 * [U*part/parts, U*(part+1)/parts) of the U in the files stay resident;
 * *first_unit receives the block's first unit.  parts = 1 is
 * mh_reads_load_fastq. */
int mh_reads_load_fastq_part(mh_ctx *ctx, const char *path1, const char *path2, int part, int parts,
                             int64_t *n_reads, int64_t *first_unit);
int mh_reads_count(mh_ctx *ctx, int64_t *n_reads, int *paired);

/* ---- sharded FASTQ ingest (host only; replaces each rank's decode of the
 * whole file: the reference streams the FASTQ once per pass,
 * prelim_map.py:114-134 / censor_fastq.py:58-96) ---------------------------
 * mh_fastq_open_part decodes part `part` of `parts` of a FASTQ file (path,
 * or an open descriptor when path is NULL): with parts > 1 the gzip members
 * starting in the part's byte range (mode 1), the byte range of a plain file
 * (mode 2); the whole file otherwise (mode 0; also with parts == 1).
 * info[10]: mode, first and end file offset read, decoded bytes, newlines in
 * them, ends with '\n', starts with '\n', file bytes decoded, file size,
 * wall time (microseconds). */
typedef struct mh_fastq mh_fastq;
int mh_fastq_open_part(const char *path, int fd, int part, int parts, mh_fastq **out, int64_t *info);
/* The ranks' test for a single gzip member: info[3] = is gzip, file size,
 * 1 if a gzip member starts inside part `part`'s byte range (past offset
 * 0).  Scans 1/parts of the file; no decode. */
int mh_fastq_scan_part(const char *path, int fd, int part, int parts, int64_t *info);
/* Part `part` of `parts` of a FASTQ file that is one gzip member (bcl2fastq's
 * layout), decoded without any other part's bytes (the reference reads the
 * file once per pass, prelim_map.py:114-134; censor_fastq.py:58-96):
 *   open    info[7]: this part's first deflate block start (bit; -1 if its
 *           share of the compressed bytes holds none: not splittable), the
 *           stream's end bit, the trailer's CRC-32 and size, spans, file
 *           size, microseconds;
 *   decode  up to end_bit (the next part's first block start, or the
 *           stream's end bit for the last part); info[2]: text bytes (-1:
 *           not decodable this way), microseconds;
 *   tail    with `window` = the previous part's last 32768 text bytes (NULL
 *           for part 0), this part's last 32768 text bytes into tail[32768]
 *           (the next part's window);
 *   finish  the rest of the text resolved; info[11]: the mh_fastq_open_part
 *           fields with mode 3 and file offsets c0 / c1 as given, then the
 *           CRC-32 of this part's text (the caller checks the combined CRC
 *           and size against the trailer).
 * Each returns 0, -1 (not resolvable: fall back), -2 out of memory, -3 bad
 * arguments. */
int mh_fastq_member_open(const char *path, int fd, int part, int parts, mh_fastq **out, int64_t *info);
int mh_fastq_member_decode(mh_fastq *fq, int64_t end_bit, int64_t *info);
int mh_fastq_member_tail(mh_fastq *fq, const char *window, char *tail);
int mh_fastq_member_finish(mh_fastq *fq, const char *window, int64_t c0, int64_t c1, int64_t *info);
/* Record starts of the held text, a record being four lines: line0 = lines
 * of the file before its first byte, starts_line = 1 if that byte starts a
 * line.  out[5]: offset of the first record start (the size if none),
 * record starts, that start's line number in the file (-1 if none), 1 if a
 * blank line sits where a record starts (the ingest's parser would skip it),
 * 1 if the text ends in an unterminated record-start line that is only a
 * '\r'. */
int mh_fastq_frame(mh_fastq *fq, int64_t line0, int starts_line, int64_t *out5);
/* byte offset of framed record k (k = the record count: the text's size) */
int mh_fastq_record_offset(mh_fastq *fq, int64_t k, int64_t *off);
/* the held text becomes front + text[lo, hi) + back (framing is dropped) */
int mh_fastq_splice(mh_fastq *fq, int64_t lo, int64_t hi, const char *front, int64_t flen,
                    const char *back, int64_t blen);
/* the held text (valid until the handle changes or is closed) */
int mh_fastq_view(mh_fastq *fq, const char **data, int64_t *len);
int mh_fastq_close(mh_fastq *fq);
/* Host-only parse of staged FASTQ text (fq2 NULL: unpaired) as the loader
 * parses it (records, bowtie2 QNAMEs, SEQ / QUAL; the texts are kept): the
 * QNAMEs '\n'-terminated in names, the bases and qualities concatenated,
 * the lengths per read (mates interleaved).  With names, seq, qual or lens
 * NULL only the sizes are returned.  For tests of the ingest without a
 * device. */
int mh_fastq_parse(mh_fastq *fq1, mh_fastq *fq2, char *names, size_t names_cap, uint8_t *seq,
                   uint8_t *qual, size_t bases_cap, int32_t *lens, int64_t reads_cap, int64_t *n_reads,
                   int64_t *n_bases, size_t *names_used);
/* Load the reads of staged FASTQ text: units [range[0], range[1]) of fq1's
 * records and [range[2], range[3]) of fq2's (-1, -1: all of them; the two
 * counts must agree), mates interleaved when fq2 is given.  The records are
 * parsed as mh_reads_load_fastq parses a file; the texts are moved into the
 * context (the handles are left empty).  fastq_lines1 is the newline count
 * of the whole FASTQ 1 (mh_reads_fastq_lines, raw_count). */
int mh_reads_load_staged(mh_ctx *ctx, mh_fastq *fq1, mh_fastq *fq2, const int64_t *range4,
                         int64_t fastq_lines1, int64_t *n_reads);
/* newlines in FASTQ 1 of the last mh_reads_load_fastq (the `gunzip -c | wc
 * -l` of LineCounter, externals.py:206-231; raw_count = lines / 2). */
int mh_reads_fastq_lines(mh_ctx *ctx, int64_t *lines1);

/* ---- one mapping pass: replaces `bowtie2 [--local] ...` ---------------- */
int mh_map(mh_ctx *ctx, const mh_params *par);
int mh_alns_fetch(mh_ctx *ctx, int64_t first, int64_t n, mh_aln *out);
/* Per-reference tallies of the last pass (n_refs entries each):
 *   lines[r]     SAM lines with RNAME r           (prelim count, remap.py:494)
 *   filtered[r]  mapped lines with a >50-base M run (remap.py:500-506)
 *   mapped[r]    mapped lines with RNAME r        (new_counts, remap.py:755)
 *   first_row[r] first line index with RNAME r, -1 if none
 *   first_mapped[r] first mapped line with RNAME r (Counter order), -1 if none
 * and *unmapped = unmapped lines (remap.py:743-753); star_lines / star_first =
 * number of / first line with RNAME '*'. */
int mh_map_counts(mh_ctx *ctx, int64_t *lines, int64_t *filtered, int64_t *mapped,
                  int64_t *first_row, int64_t *first_mapped, int64_t *unmapped,
                  int64_t *star_lines, int64_t *star_first);
/* Work done by the last mh_map: out[0] reads, out[1] banded extensions
 * (candidates aligned by the DP, up to 31 diagonals x read length cells each,
 * mate rescues included), out[2] CIGAR pool words reserved (per-wave
 * chunks), out[3] extensions resolved by the ungapped fast path (no DP),
 * out[4] mate-rescue extensions. */
int mh_map_stats(mh_ctx *ctx, int64_t *out5);
/* Test entry point (not a tuning knob): start the grow-and-retry buffers of
 * every later call at these capacities (0 = the library's own sizing):
 * the CIGAR pool of mh_map (uint32 words), the pileup's insertion-token
 * events and their bytes (mh_pileup), the distinct-token bytes of the token
 * aggregation (mh_pileup_events, mh_pileup_fetch).  A pass that needs more
 * takes the retry path, which the parity tests then check bit for bit.  The
 * call drops the buffers (and the last pass's records) so the next call
 * sizes them again. */
int mh_test_set_capacities(mh_ctx *ctx, int64_t cigar_pool_words, int64_t pileup_events,
                           int64_t pileup_event_bytes, int64_t token_bytes);
/* Retries taken so far by those paths: out4[0] CIGAR pool (a mapping pass
 * run again from k_seed), out4[1] pileup events, out4[2] token bytes,
 * out4[3] Gotoh batches run again after a strip's wait timed out. */
int mh_retry_counts(mh_ctx *ctx, int64_t *out4);
/* Test entry point: k_gotoh's first attempt of every later batch gives up a
 * neighbour wait after `ticks` of the 100 MHz real-time clock (0: the
 * default 20 s), so the timeout-and-retry path of mh_gotoh_align_batch runs. */
int mh_test_set_gotoh_wait(mh_ctx *ctx, int64_t ticks);
/* The 20 int32 header fields of mh_aln (no CIGAR) for reads [first, first+n). */
int mh_recs_fetch(mh_ctx *ctx, int64_t first, int64_t n, int32_t *out20);
/* Fields [field0, field0 + nfields) of records [first, first + n) (the
 * mh_recs_fetch field order), nfields int32 per record. */
int mh_recs_fetch_fields(mh_ctx *ctx, int64_t first, int64_t n, int field0, int nfields, int32_t *out);
/* SAM text for reads order[first .. first+n) (order NULL: reads first ..
 * first+n-1): style 0 = tab-separated SAM with
 * optional tags, style 1 = the 11 CSV columns prelim.csv / remap.csv hold
 * (csv.QUOTE_MINIMAL).  Needs names from mh_reads_load_fastq or
 * mh_reads_set_names.  *used = bytes written; -2 if cap is too small.
 * buf NULL: a size query; *used = the text's size, and the text is kept
 * for the next call with the same arguments (a copy into buf, no
 * reformatting).  Rows are formatted on host threads. */
int mh_reads_set_names(mh_ctx *ctx, int64_t n, const char *const *names);
int mh_format_rows(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                   const char *const *refnames, char *buf, size_t cap, size_t *used);
/* Rows order[0 .. n) (order NULL: reads 0 .. n - 1) formatted as style 0 /
 * 1 text (as mh_format_rows) in n_seg segments, segment s being rows
 * seg_rows[s] .. seg_rows[s + 1] (ascending, seg_rows[n_seg] <= n).  The
 * text is kept; seg_bytes[s] = its size per segment.  A sharded run
 * all-gathers the sizes to place every rank's segments in one file. */
int mh_format_segments(mh_ctx *ctx, int style, const int64_t *order, int64_t n,
                       const char *const *refnames, int n_seg, const int64_t *seg_rows,
                       int64_t *seg_bytes);
/* Write the text of the last mh_format_segments to fd, segment s at file
 * offset seg_off[s] (pwrite on host threads; the file position is not
 * used); crc[s] = crc32 of segment s (crc NULL: none).  Frees the text. */
int mh_write_segments(mh_ctx *ctx, int fd, const int64_t *seg_off, uint32_t *crc);
/* crc32 (zlib's) of A then B, from crc32(A), crc32(B) and B's length */
uint32_t mh_crc32_combine(uint32_t a, uint32_t b, int64_t len_b);
/* crc32 of a whole open file and its size (a read-back check) */
int mh_file_crc32(int fd, int64_t *size, uint32_t *crc);
/* Host wall time (ms) per phase of the file path since the last reset:
 * MH_PHASE_INFLATE (FASTQ gunzip), _PARSE (record scan, names, copies),
 * _UPLOAD (H2D + 2-bit packing), _FORMAT (SAM / CSV text), _WRITE (pwrite).
 * ms[MH_PHASES]; reset != 0 zeroes them after the copy. */
enum { MH_PHASE_INFLATE = 0, MH_PHASE_PARSE = 1, MH_PHASE_UPLOAD = 2, MH_PHASE_FORMAT = 3,
       MH_PHASE_WRITE = 4, MH_PHASES = 5 };
int mh_phase_times(mh_ctx *ctx, double *ms, int reset);
/* The same rows written straight to an open file descriptor at `offset`
 * (pwrite from the formatting threads, no copy through the caller):
 * *written bytes.  The caller moves its file position past them. */
int mh_write_rows(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                  const char *const *refnames, int fd, int64_t offset, int64_t *written);
/* mh_write_rows that also returns the crc32 of the bytes written (crc NULL:
 * none).  The rows are formatted in chunks on host threads while one
 * thread writes the finished chunks in order. */
int mh_write_rows_crc(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                      const char *const *refnames, int fd, int64_t offset, int64_t *written,
                      uint32_t *crc);
/* (crc32 << 32) | adler32 of a whole open file (zlib's, computed over
 * chunks on host threads) and its size: remap() checks with it that
 * prelim.csv is the file prelim_map() wrote. */
int mh_file_checksum(int fd, int64_t *size, uint64_t *sum);

/* ---- pileup: replaces sam_to_conseqs' counting (remap.py:141-306) ------ */
/* External SAM rows (e.g. prelim.csv read back, remap.py:474-498).
 * units: n_units pairs of row indices as matchmaker (remap.py:853-889)
 * yields them, -1 for a missing mate.  seq/qual as printed in SAM. */
int mh_rows_load(mh_ctx *ctx, int64_t n_rows, const int32_t *flag, const int32_t *ref,
                 const int32_t *pos, const int32_t *cigar_off, const int32_t *n_cigar,
                 const uint32_t *cigar, const uint8_t *seq, const uint8_t *qual,
                 const int64_t *offsets, const int32_t *lens, int64_t n_units,
                 const int64_t *unit_rows);
/* prelim.csv text (prelim_map.py:142-151) read back as remap() does
 * (remap.py:474-498): csv quoting, rname -> index into refnames (the @SQ
 * set), matchmaker pairing by qname, upload as rows.  mh_rows_info then
 * gives per row: name id (>= 0 index into refnames, < 0 other names such
 * as '*'), flag, longest M run (is_short_read, remap.py:70-83), ref index. */
int mh_rows_load_csv(mh_ctx *ctx, const char *text, int64_t len, int n_refs,
                     const char *const *refnames, int64_t *n_rows, int64_t *n_units,
                     int32_t *n_present);
/* out4 per row: name id, flag, longest M run, compact ref id; present[k] =
 * @SQ index of compact ref k; unknown = '\n'-joined names outside @SQ. */
int mh_rows_info(mh_ctx *ctx, int32_t *out4, int32_t *present, char *unknown, size_t cap);
/* source 0 = alignments of the last mh_map (units = pairs / reads),
 * source 1 = rows from mh_rows_load.  n_refs/ref_lens size the dense
 * counters (positions 1..ref_lens[r] + MH_PILEUP_SLACK). */
#define MH_PILEUP_SLACK 2048
int mh_pileup(mh_ctx *ctx, int source, int q_cutoff, int n_refs, const int32_t *ref_lens);
/* mh_pileup counting only the references sel[0 .. n_sel) (n_sel < 0: all):
 * the units mapped to any other are skipped and its counters, read count
 * and positions stay empty.  The prelim pass builds only the seed-group
 * winners' consensuses (remap.py:531-541 keeps those of build_conseqs'
 * output), so their pileup alone is needed; every reference is counted
 * independently of the others, so theirs are the same. */
int mh_pileup_only(mh_ctx *ctx, int source, int q_cutoff, int n_refs, const int32_t *ref_lens, int n_sel,
                   const int32_t *sel);
/* dense: n_refs x cap x 4 int32 counts of A,C,G,T at positions 1..cap;
 * nflag/dflag: n_refs x cap bytes ('N' seen -> count -1, '-' seen -> -2);
 * read_counts: merged pairs per ref; first_unit: first merged unit index
 * per ref (-1 if none); max_pos: largest position touched per ref. */
int mh_pileup_dims(mh_ctx *ctx, int *n_refs, int32_t *cap, int64_t *n_events,
                   int64_t *event_bytes);
int mh_pileup_fetch(mh_ctx *ctx, int32_t *dense, uint8_t *nflag, uint8_t *dflag,
                    int64_t *read_counts, int64_t *first_unit, int32_t *max_pos);
/* The dense / nflag / dflag rows of one reference (cap positions each):
 * fetching only the references that received pairs keeps a pileup over many
 * seeds from copying every seed's counters. */
int mh_pileup_fetch_ref(mh_ctx *ctx, int ref, int32_t *dense, uint8_t *nflag, uint8_t *dflag);
/* The counter rows of n_sel references in one call (one stream
 * synchronisation): dense / nflag / dflag are the whole (n_refs x cap [x 4])
 * arrays, and reference refs[k]'s rows 0 .. max_pos - 1 are written (its
 * positions 1 .. max_pos; past its last counted position every row is zero,
 * and those rows are left as the caller zeroed them). */
int mh_pileup_fetch_refs(mh_ctx *ctx, int n_sel, const int32_t *refs, int32_t *dense, uint8_t *nflag,
                         uint8_t *dflag);
/* Sparse tokens (base + insertion with len % 3 == 0), aggregated over the
 * pileup: n_events (mh_pileup_dims) distinct (ref, pos, token) entries in
 * (ref, pos, token) order, each with the number of merged pairs that voted
 * for it; the token is pool[tok_off[e] .. tok_off[e] + tok_len[e]). */
int mh_pileup_events(mh_ctx *ctx, int32_t *ref, int32_t *pos, int32_t *tok_off,
                     int32_t *tok_len, int64_t *count, char *pool);
/* Multi-GPU: the caller all-reduces three device buffers with RCCL after
 * mh_pileup_export and hands them to mh_pileup_import.  Only the rows of the
 * n_sel references in sel (the same list on every rank: those with data on
 * any rank) travel:
 *   sum   int32, SUM: dense rows of sel, then read_counts of every ref
 *   max   int32, MAX: max_pos of every ref, then -(first_unit + unit_base)
 *         (unit_base = this rank's first unit index: the MAX yields the
 *         global first unit, i.e. the reference's refmap order)
 *   flags uint8, MAX: nflag rows, then dflag rows of sel (0/1: MAX = OR)
 * mh_pileup_exchange_bytes gives the three sizes. */
int mh_pileup_exchange_bytes(mh_ctx *ctx, int n_sel, int64_t *sum_bytes, int64_t *max_bytes,
                             int64_t *flag_bytes);
int mh_pileup_export(mh_ctx *ctx, int n_sel, const int32_t *sel, int64_t unit_base,
                     void *dev_sum, void *dev_max, void *dev_flags);
int mh_pileup_import(mh_ctx *ctx, int n_sel, const int32_t *sel, const void *dev_sum,
                     const void *dev_max, const void *dev_flags);
/* Insertion-token events across ranks (the sparse side table of the pileup):
 * mh_pileup_event_bytes gives this rank's raw event count and pool bytes;
 * mh_pileup_events_export copies them (4 int32 per event, then the bytes)
 * into caller device buffers; after an all-gather of those buffers,
 * mh_pileup_events_import replaces the rank's events by the concatenation of
 * `parts` parts (part p at dev_events + p * events_stride int32 words and
 * dev_pool + p * pool_stride bytes), so mh_pileup_events aggregates every
 * rank's tokens. */
int mh_pileup_event_bytes(mh_ctx *ctx, int64_t *n_events, int64_t *pool_bytes);
int mh_pileup_events_export(mh_ctx *ctx, void *dev_events, void *dev_pool);
int mh_pileup_events_import(mh_ctx *ctx, int parts, const int64_t *n_events,
                            const int64_t *pool_bytes, const void *dev_events,
                            int64_t events_stride, const void *dev_pool, int64_t pool_stride);

/* ---- sam2aln: replaces sam2aln.sam2aln (sam2aln.py:395-478) ----------- */
/* remap.csv text (the SAM columns remap() writes) read as DictReader does,
 * paired by qname (matchmaker, sam2aln.py:291-312), every pair merged on the
 * device (parse_sam, :315-391: apply_cigar, merge_pairs at q_cutoff, the
 * prop_N > max_prop_n test) and identical merged sequences counted per rname
 * (:449-456).  MiCall passes q_cutoff 15 and max_prop_n 0.5
 * (SAM2ALN_Q_CUTOFFS, MAX_PROP_N).  Fails (-3, message as the reference's
 * RuntimeError) on a CIGAR apply_cigar rejects.  *n_units = matchmaker pairs. */
int mh_sam2aln_csv(mh_ctx *ctx, const char *text, int64_t len, int q_cutoff, double max_prop_n,
                   int64_t *n_units);
/* CSV text of the last mh_sam2aln_csv: which 0 = aligned.csv, 1 =
 * insert.csv, 2 = failed.csv (DictWriter, '\n' line ends, with header).
 * buf NULL: only *used = bytes needed. */
int mh_sam2aln_output(mh_ctx *ctx, int which, char *buf, size_t cap, size_t *used);
/* mh_sam2aln_csv on the whole of a regular file (fd, mmap'd from offset 0):
 * 0, or 1 when the file holds '\r' (a text-mode read would translate it;
 * the caller reads the file itself), or an error. */
int mh_sam2aln_file(mh_ctx *ctx, int fd, int q_cutoff, double max_prop_n, int64_t *n_units);
/* Output `which` (as mh_sam2aln_output) written to fd at offset with
 * pwrite (the descriptor's own offset is not used); *written = its size.
 * Not sized before (no mh_sam2aln_output size query), it is formatted and
 * written in one pass, the writes overlapping the formatting. */
int mh_sam2aln_write(mh_ctx *ctx, int which, int fd, int64_t offset, int64_t *written);
/* out[0] pairs, out[1] pairs merged on the device, out[2] distinct merged
 * sequences, out[3] failed pairs. */
int mh_sam2aln_stats(mh_ctx *ctx, int64_t *out4);
/* Host wall time (ms) of the last call: [0] CSV parse + matchmaker, [1]
 * upload + device merge/group + fetch, [2..4] formatting of the three
 * outputs (0 until formatted). */
int mh_sam2aln_timing(mh_ctx *ctx, double *ms5);

/* ---- sam2aln split over the ranks of a job (same reference call,
 * sam2aln.py:395-478; the bytes move between ranks through the caller's
 * collectives, torch.distributed in sam2aln._sam2aln_sharded).  Rank `part`
 * of `parts`:
 *   mh_sam2aln_part       parses its share of remap.csv (fd, mmap'd): the
 *                         record at or after byte part/parts of the body, a
 *                         cut between the two rows of one qname moved past
 *                         the second, and merges its pairs on its device.
 *                         0, or 1 = not split (a line with an odd number of
 *                         '"', no qname column, '\r' in the file: every rank
 *                         gets 1 and the caller runs mh_sam2aln_file on one).
 *                         info[0..5] = units, pair units, reference names,
 *                         distinct merged sequences, share bytes, file bytes.
 *   mh_sam2aln_part_units qname hash (n = info[0]) and leftover flag per
 *                         unit: the caller checks that no leftover qname
 *                         has rows on two ranks (matchmaker, :291-312, pairs
 *                         across the whole file), else falls back.
 *   mh_sam2aln_part_names this rank's reference names ('\n' after each) and
 *                         the first unit of each; _set_names gives each its
 *                         job-wide id (the names in first-appearance order,
 *                         the order of groups in aligned.csv, :449-478).
 *   mh_sam2aln_records    step 0: distinct sequences as records, one buffer
 *                         per owner rank (hash % parts), sizes[parts];
 *                         step 1: up to per_name evenly spaced records of
 *                         every name of the owner's merged order, sizes[1];
 *                         step 2 (after mh_sam2aln_splitters): the owner's
 *                         records to the rank of their range, sizes[parts].
 *                         *data = the concatenated buffers (valid until the
 *                         next call on ctx).
 *   mh_sam2aln_records_merge  stage 0: the records every rank sent this
 *                         owner, equal ones added up (:446-452), sorted as
 *                         aligned.csv lists them (:466-470); stage 1: the
 *                         records of this rank's ranges, sorted.
 *   mh_sam2aln_splitters  all ranks' samples -> the splitters of each name.
 *   mh_sam2aln_range_counts   rows of this rank's range per job-wide name.
 *   mh_sam2aln_range_text aligned.csv rows of this rank's range (:471-478),
 *                         one segment per name, row numbers ("rank" column)
 *                         from base[name] (the rows of ranks before it).
 *   mh_sam2aln_part_text  insert.csv (which 1) / failed.csv (which 2) rows
 *                         of this rank's pair units (seg 0) or leftover
 *                         units (seg 1), with the header when head != 0; the
 *                         caller writes segments segment-major by rank. */
int mh_sam2aln_part(mh_ctx *ctx, int fd, int part, int parts, int q_cutoff, double max_prop_n,
                    int64_t *info);
int mh_sam2aln_part_units(mh_ctx *ctx, uint64_t *qhash, uint8_t *leftover);
int mh_sam2aln_part_names(mh_ctx *ctx, char *buf, size_t cap, size_t *used, int64_t *first_unit);
int mh_sam2aln_part_set_names(mh_ctx *ctx, const int32_t *gid, int n);
int mh_sam2aln_records(mh_ctx *ctx, int step, int parts, int per_name, int64_t *sizes,
                       const uint8_t **data);
int mh_sam2aln_records_merge(mh_ctx *ctx, int stage, const uint8_t *data, int64_t len);
int mh_sam2aln_splitters(mh_ctx *ctx, const uint8_t *data, int64_t len, int parts);
int mh_sam2aln_range_counts(mh_ctx *ctx, int n_names, int64_t *counts);
int mh_sam2aln_range_text(mh_ctx *ctx, int n_names, const char *const *names, const int64_t *base,
                          int64_t *seg_bytes, const uint8_t **data);
int mh_sam2aln_part_text(mh_ctx *ctx, int which, int seg, int head, int64_t *bytes,
                         const uint8_t **data);

/* ---- censor: replaces censor_fastq.censor (censor_fastq.py:32-102) ---- */
/* One FASTQ file (src, gzip when src_gzip) censored on the device: bases /
 * qualities at the bad (tile, cycle) pairs (tiles[k], cycles[k]; negative
 * cycles = reverse reads) become 'N' / '#', a trailing run of bad cycles is
 * dropped as the reference drops it, header and '+' lines are kept
 * verbatim.  *base_count / *score_sum = number and sum (Phred) of all
 * quality characters, for the summary row (:94-102).  The censored file
 * (gzip when dst_gzip: independent deflate members, level 1) is then
 * copied out with mh_censor_output (buf NULL: *used = size). */
int mh_censor_fastq(mh_ctx *ctx, const uint8_t *src, int64_t len, int src_gzip, int n_bad,
                    const char *const *tiles, const int32_t *cycles, int dst_gzip,
                    int64_t *base_count, int64_t *score_sum);
/* The same on the text a staged FASTQ holds (mh_fastq_open_part: the whole
 * file, or a rank's block of records of a sharded job; gzip already
 * inflated).  The text is taken (the handle keeps an empty one).
 * *out_bytes = size of the censored output held for mh_censor_output /
 * mh_censor_write. */
int mh_censor_staged(mh_ctx *ctx, mh_fastq *fq, int n_bad, const char *const *tiles,
                     const int32_t *cycles, int dst_gzip, int64_t *out_bytes,
                     int64_t *base_count, int64_t *score_sum);
int mh_censor_output(mh_ctx *ctx, char *buf, size_t cap, size_t *used);
/* The held censored output written to fd at offset (pwrite; the descriptor's
 * own offset is not used); *written = its size.  The output is released. */
int mh_censor_write(mh_ctx *ctx, int fd, int64_t offset, int64_t *written);
/* mh_censor_staged, the output written to fd from offset (pwrite) while it
 * is made: each gzip member (or text block) as soon as it and those before
 * it are done; *written = bytes written.  Nothing is kept for
 * mh_censor_output / mh_censor_write.  Replaces the same censor_fastq.py:
 * 32-102 call as mh_censor_staged + mh_censor_write. */
int mh_censor_staged_write(mh_ctx *ctx, mh_fastq *fq, int n_bad, const char *const *tiles,
                           const int32_t *cycles, int dst_gzip, int fd, int64_t offset,
                           int64_t *written, int64_t *base_count, int64_t *score_sum);
/* Host wall ms of the last call: [0] gunzip + record split, [1] upload +
 * k_censor + download, [2] rewrite + gzip. */
int mh_censor_timing(mh_ctx *ctx, double *ms3);

/* ---- aln2counts: replaces the per-read loops of aln2counts.py ---------- */
/* aligned.csv text (refname, qcut, count, offset, seq columns) read as
 * csv.DictReader reads it; consecutive rows with equal (refname, qcut) form a
 * group (itertools.groupby, aln2counts.py:884-887).  Every row is counted on
 * the device in the three reading frames of _count_reads (:147-169): per
 * codon the 21 amino acids of AMINO_ALPHABET and, per codon position, the
 * bases A C G T N - (an 'n' is not counted, :642-645), each counter with the
 * first row of its group that touched it (the Counter insertion order that
 * most_common() breaks ties by).  codon_chars = the translations of the 216
 * codons over A C G T N - (translation.py:40-142), index 36 c0 + 6 c1 + c2.
 * slot 0..3 selects one of four independent row tables of the context.
 * Rejects (-3) seq characters outside A C G T N - n, offsets outside
 * 0..2^28 and counts outside 0..2^32-1.  *n_groups = number of groups. */
int mh_a2c_load_csv(mh_ctx *ctx, int slot, const char *text, int64_t len,
                    const char *codon_chars, int64_t *n_groups);
/* mh_a2c_load_csv on the whole of a regular file (fd, mmap'd): 0, or 1 when
 * the file holds '\r' (the caller reads it in text mode instead). */
int mh_a2c_load_file(mh_ctx *ctx, int slot, int fd, const char *codon_chars, int64_t *n_groups);
/* The same from rows in memory: row r's seq is pool[seq_off[r] ..
 * seq_off[r] + seq_len[r]); group g = rows group_first[g] ..
 * group_first[g + 1] - 1 (group names are empty). */
int mh_a2c_load_rows(mh_ctx *ctx, int slot, int64_t n_rows, const char *pool, int64_t pool_len,
                     const int64_t *seq_off, const int32_t *seq_len, const int64_t *offset,
                     const int64_t *count, int64_t n_groups, const int64_t *group_first,
                     const char *codon_chars);
/* info5 = first row, rows, and the SeedAmino list length of frames 0, 1, 2;
 * names = refname '\0' qcut (names NULL: only *used = bytes needed). */
int mh_a2c_group(mh_ctx *ctx, int slot, int64_t g, int64_t *info5, char *names, size_t cap,
                 size_t *used);
/* Counters of group g, frame 0..2, codons 0 .. info5[2 + frame] - 1:
 * aa_count / aa_first [codon][21], nuc_count / nuc_first [codon][3][6]
 * (position in the codon, base A C G T N -); first = 0xffffffff when never
 * touched (the Counter has no such key). */
int mh_a2c_counts(mh_ctx *ctx, int slot, int64_t g, int frame, uint32_t *aa_count,
                  uint32_t *aa_first, uint32_t *nuc_count, uint32_t *nuc_first);
/* InsertionWriter.write's read loop (:779-795) over the rows of group g for
 * the codon ranges [left[k], right[k]) in reading frame `frame`: distinct
 * amino-acid strings per range with their summed counts, in (range, first
 * row) order.  *n_entries = number of strings; fetch them with
 * mh_a2c_insert_entries (aminos: one string per line). */
int mh_a2c_inserts(mh_ctx *ctx, int slot, int64_t g, int frame, int n_ranges,
                   const int32_t *left, const int32_t *right, int64_t *n_entries);
int mh_a2c_insert_entries(mh_ctx *ctx, int slot, int32_t *range, int64_t *count,
                          uint32_t *first, char *aminos, size_t cap, size_t *used);
/* The insertion report rows (aln2counts InsertionWriter.write) of the last
 * mh_a2c_inserts: per entry, lead + (left[range] + 1) + ',' + its amino-acid
 * string + ',' + its count + ',' + target[range] (blank for INT32_MIN) +
 * eol.  buf NULL: formats and sets *used; then copies into buf. */
int mh_a2c_insert_rows(mh_ctx *ctx, int slot, const char *lead, int n_ranges, const int32_t *left,
                       const int32_t *target, const char *eol, char *buf, size_t cap, size_t *used);
/* Host wall ms: [0] parse of the last load, [1] its upload + k_a2c_count +
 * fetch, [2] mh_a2c_inserts since the last call of this function. */
int mh_a2c_timing(mh_ctx *ctx, int slot, double *ms3);

/* ---- aln2counts counting split over the ranks of a job (the same
 * aln2counts.py:115-172 loops; the counters are sums and a first row is a
 * minimum, so each rank counts its share and the caller reduces them) ----
 *   mh_a2c_part_open     rank `part` of `parts` parses the rows of its share
 *                        of aligned.csv (fd, mmap'd; cuts at line starts).
 *                        0, or 1 = not split (a quoted field in the share or
 *                        '\r' in the file: the caller loads it whole).
 *                        info3 = rows, local groups, share bytes.
 *   mh_a2c_part_groups   its runs of (refname, qcut): keys "refname\x1fqcut\n"
 *                        each (keys NULL: *used only), rows, the codon
 *                        extent of frames 0..2 (ncod3[3 g + f]) and the
 *                        summed count of each.
 *   mh_a2c_part_count    the job's groups (n_groups keys as above, the codon
 *                        extents the maximum over ranks), gid[k] = the job
 *                        group of local run k (increasing), row_base[k] = rows
 *                        of that group on the ranks before; counts on the
 *                        device.  *cells = counter cells (aa + nuc, all
 *                        groups and frames), as mh_a2c_counts lays them out.
 *   mh_a2c_part_counters set 0: copies the cells' counts and first rows out;
 *                        set 1: takes the reduced ones (counts summed, first
 *                        rows the minimum) back, after which mh_a2c_group /
 *                        mh_a2c_counts read the job's counters.
 *   mh_a2c_insert_export the entries of the last mh_a2c_inserts as bytes
 *                        (buf NULL: *used only);
 *   mh_a2c_insert_merge  every rank's exports of one call concatenated:
 *                        equal (range, string) added up, first row the least,
 *                        in (range, first row) order (InsertionWriter.write,
 *                        :779-795), for mh_a2c_insert_entries / _rows. */
int mh_a2c_part_open(mh_ctx *ctx, int slot, int fd, int part, int parts, const char *codon_chars,
                     int64_t *info3);
int mh_a2c_part_groups(mh_ctx *ctx, int slot, char *keys, size_t cap, size_t *used, int64_t *rows,
                       int32_t *ncod3, int64_t *total);
int mh_a2c_part_count(mh_ctx *ctx, int slot, int64_t n_groups, const char *keys, const int64_t *gid,
                      const int32_t *ncod3, const int64_t *row_base, int64_t *cells);
int mh_a2c_part_counters(mh_ctx *ctx, int slot, int set, uint32_t *cnt, uint32_t *first);
int mh_a2c_insert_export(mh_ctx *ctx, int slot, uint8_t *buf, size_t cap, size_t *used);
int mh_a2c_insert_merge(mh_ctx *ctx, int slot, const uint8_t *buf, int64_t len, int64_t *n_entries);

/* ---- Gotoh: replaces _gotoh2.align (_gotoh2.c:544-607) ---------------- */
/* seq1/seq2 already cleaned (gotoh2.py:70-72).  out1/out2 need
 * strlen(seq1)+strlen(seq2)+1 bytes (cap). */
int mh_gotoh_align(mh_ctx *ctx, const char *seq1, const char *seq2, int gop, int gep,
                   int is_global, const char *alphabet, const int *matrix, char *out1,
                   char *out2, int cap, int *score);

/* Many alignments with the same scoring in one launch (one workgroup each):
 * the consensus-distance filter's K x K alignments (remap.py:244-263) and
 * aln2counts' coordinate alignments.  status[t] = 0, or -1 where
 * _gotoh2.align would raise "Traceback failed"; the call itself returns
 * -3 / -2 / -4 for a bad argument / out of memory / a HIP error. */
int mh_gotoh_align_batch(mh_ctx *ctx, int count, const char *const *seq1,
                         const char *const *seq2, int gop, int gep, int is_global,
                         const char *alphabet, const int *matrix, char *const *out1,
                         char *const *out2, const int *cap, int *score, int *status);

/* The consensus-distance filter's edit distances (remap.py:247-251) as one
 * device batch: alignment t is mh_gotoh_align_batch's (seq1[t], seq2[t])
 * and dist[t] = Levenshtein.distance(extract_relevant_seed(aligned seq2,
 * aligned seq1), text[t]) (remap.py:129-138, :251), computed on the device
 * from the alignment (k_lev_prep, k_lev); only the distances are fetched.
 * status[t] = 0, -1 where the traceback fails, or -2 where the aligned
 * seq2 has no non-gap column (the reference's match is None); score[t] is
 * the alignment score.  Replaces remap.py:249-251's per-pair aligner.align +
 * extract_relevant_seed + Levenshtein.distance calls. */
int mh_gotoh_distance_batch(mh_ctx *ctx, int count, const char *const *seq1,
                            const char *const *seq2, const char *const *text, int gop, int gep,
                            int is_global, const char *alphabet, const int *matrix, int *dist,
                            int *score, int *status);

/* Per-kernel device time measured with HIP events on the context's stream
 * (k_seed, k_dp, k_pair, k_pileup).  mh_profile(ctx, 1) enables and resets. */
int mh_profile(mh_ctx *ctx, int enable);
int mh_profile_get(mh_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches);

/* Diagnostics (tests only; no reference counterpart): for n caller-given
 * extensions items[4t..4t+3] = (read index, strand, ref, centre diagonal) of
 * the loaded reads against the built index, run both k_dp paths on the same
 * staged tables: out[8t..8t+7] = (fast path taken, its best score, row, band
 * lane; the band half; the full banded DP's best score, row, band lane).
 * Whenever the fast path is taken its cell must equal the full DP's. */
int mh_probe_extend(mh_ctx *ctx, const mh_params *par, int n, const int32_t *items, int32_t *out);

/* Host side of counts_to_conseqs (remap.py:309-333 with find_top_token
 * :892-902 and the seed prefill :195-197) for one reference's fetched
 * pileup rows, positions 1..length (rows past `rows` count as empty): tok[i]
 * = the top base-like token of position i+1 -- the first of A < C < G < T
 * with the largest positive count, else the seed's character (count 0),
 * else 'N' (-1), else '-' (-2), else 0 (no token).  Insertion tokens are
 * merged in by the caller.  *any_positive: some row holds a positive count.
 * Replaces the reference's per-position Counter walk. */
int mh_top_tokens(int32_t length, int32_t rows, const int32_t *dense, const uint8_t *nflag,
                  const uint8_t *dflag, const char *seed, int32_t seed_len, uint8_t *tok,
                  int32_t *any_positive);

/* counts_to_conseqs (remap.py:309-333, find_top_token :892-902, seed
 * prefill :195-197) for n_sel references of a fetched pileup in one call
 * (host code): reference k is row rows_of[k] of dense ([rows][cap][4]
 * int32) / nflag / dflag ([rows][cap] bytes), positions 1..lengths[k], its
 * seed seeds[k] (seed_lens[k] bytes, may be 0); the insertion tokens are
 * n_ev events (row, pos, token = pool[off .. off+len), merged pairs).  Per
 * position the top of the reference's Counter, then the deletion-run rule;
 * consensus k is out[out_off[k] .. out_off[k+1]) and present[k] = 0 when no
 * count is positive (no consensus).  out_cap >= sum(lengths) + sum(ev_len)
 * always suffices.  Returns -2 when out_cap is too small. */
int mh_conseqs_build(int n_sel, const int32_t *rows_of, const int32_t *lengths, const char *const *seeds,
                     const int32_t *seed_lens, int32_t cap, const int32_t *dense, const uint8_t *nflag,
                     const uint8_t *dflag, int64_t n_ev, const int32_t *ev_row, const int32_t *ev_pos,
                     const int64_t *ev_off, const int32_t *ev_len, const int64_t *ev_cnt, const char *pool,
                     char *out, int64_t out_cap, int64_t *out_off, int32_t *present);

/* Unit-cost edit distance (Levenshtein.distance, remap.py:251). */
int mh_levenshtein(const char *a, const char *b);
/* out[t] = mh_levenshtein(a[t], b[t]) for count pairs, on host threads. */
int mh_levenshtein_batch(int count, const char *const *a, const char *const *b, int *out);

#ifdef __cplusplus
}
#endif
#endif
