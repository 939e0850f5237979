/*
 * kmer_spans.h -- C ABI of the MI355X-native k-mer span scanner
 * (libkmerspans.so, built from kmer_spans_amd/csrc/).
 *
 * This is the drop-in boundary for the span-scan path of lmjakt/kmer_spans
 * (reference snapshot /root/reference, 2025-03-21).  Every entry point is plain
 * C: pointers, sizes and status codes; no torch or HIP types in signatures
 * (HIP streams travel as void*).  The R `.Call` shim
 * (kmer_spans_amd/rcall/kmer_spans_call.c) maps the reference's six
 * registered routines (kmer_spans.c:795-808) onto these functions; see
 * INTEGRATION.md for that binding and for the ctypes binding Python uses.
 *
 * Conventions
 *  - Sequences are byte strings given as (pointer, length); like R CHARSXPs
 *    they contain no NUL.  Bytes N/n split runs; every other byte is encoded
 *    as (c >> 1) & 3 (A/a=0, C/c=1, T/t=2, G/g=3), kmer_spans.c:34-35.
 *  - k-mer codes: first base in the most significant bits, 4^k entries in
 *    the internal A,C,T,G order (kmer_spans.c:41, kmer_seq :161-171).
 *  - 1 <= k <= 15.  The reference admits k = 16 in kmer_counts (UB shift,
 *    Q2), has no lower bound in kmer_regions_r (k = 0 loops forever on an N)
 *    and no check in kmer_low_comp_regions (Q7); those are errors here.
 *  - Every function validates all arguments before touching the device and
 *    returns KS_OK or an error code; ks_last_error() returns the message
 *    (the reference's error() strings where one exists).
 *  - Output regions are allocated by the library; free with ks_regions_free.
 *  - Results are bit-exact with the reference: region triples and their
 *    order, scores (FP64, 0 ulp), counts and visit histograms.
 */
#ifndef KMER_SPANS_H
#define KMER_SPANS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t ks_status;
#define KS_OK 0
#define KS_ERR_ARG 1         /* invalid argument (reference: error()) */
#define KS_ERR_DEVICE 2      /* HIP runtime failure */
#define KS_ERR_NOMEM 3       /* host or device allocation failed */
#define KS_ERR_INTERNAL 4    /* internal consistency check failed */

#define KS_MAX_K 15

/* Thread-local message of the last failing call. */
const char *ks_last_error(void);
/* Library version string, e.g. "kmer_spans_amd 0.2 gfx950 build 1a2b3c4d5e6f"
 * (the build id is a hash of the library's sources, see csrc/Makefile). */
const char *ks_version(void);

/* Region list in the reference's record layout (seq_regions, kmer_spans.c:
 * 46-58): per region (seq_id, beg, end) int32 and score double; the second
 * double the reference stores ("entropy") is always 0.0 and is not kept.
 * Regions are ordered by (seq_id, beg), the reference's emission order. */
/* The four arrays live in one library-allocated block: seq_id, beg, end are
 * consecutive (a column-major 3 x n int32 matrix, the reference's `pos`
 * before kmer_spans.R:76 transposes it), score is followed by n zeros (the
 * 2 x n `score` matrix, second row 0.0, kmer_spans.c:280). */
typedef struct ks_regions {
  int64_t n;
  int32_t *seq_id; /* 0-based index into the input sequences (:536, :610) */
  int32_t *beg;    /* scan index of the first positive k-mer (:272)       */
  int32_t *end;    /* scan index of the first maximum (:289)              */
  double *score;   /* maximum score (:280, :302)                          */
} ks_regions;
void ks_regions_free(ks_regions *r);

/* Execution context: one GPU, one HIP stream, a grow-only device workspace.
 * Created lazily per process (fork-safe: never touches HIP until first use,
 * test.R:550-567 forks with mclapply).  One call at a time per context, like
 * the reference on R's main thread: a call entered from a second thread while
 * another is inside one on the same context returns KS_ERR_ARG ("in use by
 * another thread"); use one context per thread. */
typedef struct ks_ctx ks_ctx;
ks_status ks_ctx_create(int32_t device, ks_ctx **out);
void ks_ctx_destroy(ks_ctx *ctx);
/* Run the ctx's work on an external HIP stream (hipStream_t as void*).
 * NULL is HIP's default (null) stream, e.g. torch's default stream; a new
 * ctx starts on a non-blocking stream of its own. */
ks_status ks_ctx_set_stream(ks_ctx *ctx, void *hip_stream);
/* Process-wide default context on device 0 (what the .Call shim uses). */
ks_ctx *ks_default_ctx(void);

/* ---------------------------------------------------------------------
 * Host-buffer entry points: one per reference .Call routine on the path.
 * Sequences are host pointers; the library stages them to the device.
 * --------------------------------------------------------------------- */

/* kmer_counts(seq_r, k_r) -- replaces kmer_spans.c:453-487.
 * counts: int32[4^k] (overwritten), *n_words: words counted over sequences
 * with length >= k (sequence_kmer_count :135-155, incl. quirk Q1). */
ks_status ks_kmer_counts(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                         int32_t nseq, int32_t k, int32_t *counts, double *n_words);

/* kmer_regions_r(seq_r, k_r, kmer_w_r, min_width_r, min_score_r) -- replaces
 * kmer_spans.c:490-546.  w: double[4^k] in internal order; threshold 0.
 * visits: int32[4^k] visit histogram incl. restart re-visits (Q6), may be NULL
 * to skip it; *n_bases: total length of sequences with length >= k. */
ks_status ks_kmer_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                          int32_t nseq, int32_t k, const double *w, int64_t w_len,
                          int32_t min_width, double min_score, int32_t *visits,
                          double *n_bases, ks_regions *out);

/* kmer_low_comp_regions(seq_r, k_r, min_width_r, min_score_r, threshold_r) --
 * replaces kmer_spans.c:548-621: count -> weighted rank (rank_kmers_w
 * :189-202, stable (count, index) order) -> scan with threshold thr in (0,1).
 * counts int32[4^k], ranks double[4^k], n[2] = {#words, 0} (Q8). */
ks_status ks_low_comp_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                              int32_t nseq, int32_t k, int32_t min_width, double min_score,
                              double thr, int32_t *counts, double *ranks, double *n,
                              ks_regions *out);

/* tr_lr_regions_r(seq_r, params_r = (k, min_length), kmers_r, kmer_scores_r,
 * trans_scores_r) -- replaces kmer_spans.c:649-713 (find_kmer_tr_lr_regions
 * :329-395).  kmers[i] spells the k-mer of entry i of kmer_scores and
 * trans_scores (n_scores = 4^k entries, user order); they are remapped to
 * 2-bit code order as the reference does (:677-690; entries no string maps
 * to are 0 here, uninitialised there).  spectra (optional, 2 x 4^k,
 * column-major) receives the remapped kmer then transition scores.  Regions
 * are 1-based like the reference's: seq_id = sequence index + 1, beg and end
 * = 1 + region begin / max position, score = region maximum. */
ks_status ks_tr_lr_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq,
                           int32_t k, int32_t min_length, const char *const *kmers,
                           const double *kmer_scores, const double *trans_scores, int64_t n_scores,
                           double *spectra, ks_regions *out);

/* ---------------------------------------------------------------------
 * Several GPUs of one node behind the same entry points.  With a device list
 * of two or more entries, ks_kmer_counts, ks_kmer_regions and
 * ks_low_comp_regions called with ctx == NULL (what the .Call shim does)
 * spread the call: the sequences -- a sequence longer than half a fair share
 * cut in the middle of its N gaps of >= 1000 bases when whole sequences leave
 * a part more than 0.5 % above the fair share -- are dealt to the devices by LPT on length, each device
 * stages, counts and scans its share on a context of its own from a host
 * thread of its own, counts and visit histograms are added exactly (uint32
 * wrap-around), kmer_low_comp_regions builds every device's weighted-rank
 * table from the summed counts, and the regions come back in the caller's
 * coordinates and (seq_id, beg) order: the results equal the one-device
 * call's.  The list may repeat a device (two contexts on one card).  A call
 * with an explicit ctx runs on that ctx's device only.  A call owns every
 * context of the list from its start to its end; a second thread's
 * multi-device call meanwhile returns KS_ERR_ARG (busy).  The reference runs
 * these routines on R's main thread (kmer_spans.c:452-621); this replaces the
 * mclapply-over-sequences pattern of test.R:550-567 inside one call. */
/* devices: n device ordinals (n = 0: device 0 alone, the default).  Read from
 * KS_DEVICES ("0,1,2,3") at first use unless set here. */
ks_status ks_set_devices(const int32_t *devices, int32_t n);
/* The list's length; its first cap entries into devices. */
int32_t ks_get_devices(int32_t *devices, int32_t cap);
/* The shard plan (host only, no device): the pieces nparts devices take, rows
 * (part, sequence, lo, hi) of int64 in out[4 * cap], each part's rows ordered
 * by (sequence, lo); returns the number of pieces (> cap: only cap written),
 * -1 on a bad argument. */
int64_t ks_shard_plan(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t nparts,
                      int64_t *out, int64_t cap);
/* Phases of the last multi-device call (ms, host wall clock), into out[cap]:
 * [0] whole call, [1] the parts' first phase (kmer_counts / kmer_regions: the
 * whole per-device body; low_comp: staging + count), [2] the host-side sum of
 * the count / visit histograms, [3] low_comp: rank table + scan, [4] region
 * merge, [5] parts P, then per part p: [6 + 4p] body, [7 + 4p] staging +
 * count, [8 + 4p] score-table upload + compression, [9 + 4p] scan
 * (kmer_regions only).  Returns the number of values available. */
int32_t ks_multi_last_stats(double *out, int32_t cap);
/* Merge of the parts' regions (parts[p] in the coordinates of part p's pieces
 * passed as sequences in plan order, as a call on them returns them) into the
 * caller's coordinates and (seq_id, beg) order (host only). */
ks_status ks_merge_parts(const int64_t *plan, int64_t npieces, int32_t nparts, const ks_regions *parts,
                         ks_regions *out);

/* kmer_seq_r(k_r) -- replaces kmer_spans.c:623-639.  out: 4^k * (k+1) bytes,
 * NUL-terminated k-char strings in internal code order. Host only. */
ks_status ks_kmer_seq(int32_t k, char *out, size_t out_len);

/* ---------------------------------------------------------------------
 * Score-table builders (host, exact).  The reference computes the weighted
 * rank in C (rank_kmers_w :189-202) and leaves log2(f/f_med) and +-1 to user
 * R code (README.md:27-42, kmer.counts()$f kmer_spans.R:25).
 * --------------------------------------------------------------------- */
ks_status ks_rank_table(const int32_t *counts, int32_t k, double total, double *ranks);
ks_status ks_log2_table(const int32_t *counts, int32_t k, double *w);
ks_status ks_pm1_table(const int32_t *counts, int32_t k, double *w);

/* ---------------------------------------------------------------------
 * Device-resident entry points (inputs already in HBM).  Used by bench.py,
 * the multi-GPU driver and callers that keep a genome resident.
 * --------------------------------------------------------------------- */

/* A batch of sequences concatenated in one device buffer.
 * seq: device bytes; offsets_host/offsets_dev: nseq+1 int64 offsets (host
 * and device copies of the same array); sequence q is
 * seq[offsets[q] .. offsets[q+1]). */
typedef struct ks_dev_seqs {
  const uint8_t *seq;
  const int64_t *offsets_host;
  const int64_t *offsets_dev;
  int32_t nseq;
} ks_dev_seqs;

/* A score table resident on the device, s = w[code] - thr precomputed
 * bitwise as the reference computes it (kmer_spans.c:268).  Flags:
 *  KS_TABLE_COMPRESS  if the table has at most 65536 distinct values, store
 *                     it as a uint16 code table plus an FP64 value LUT
 *                     (exact: the LUT holds the very same doubles);
 *  KS_TABLE_EXPAND    also build an expanded table, so the scan issues one
 *                     random read per J scan indices (up to 128 GiB of the
 *                     GPU's HBM; skipped when it does not fit):
 *                     k = 8..13: a line table, one 64-B line per m-mer (m =
 *                     k + own - 1 <= 15) holding the codes / values of its
 *                     own k-mers and of every one- and two-base (FP64: one-
 *                     base) continuation, J = own + 2 (own + 1); at k = 12,
 *                     13 with <= 7168 distinct values, 128-B lines with
 *                     13-bit codes and the three-base continuations as
 *                     11-bit codes (escape to the base table), J = own + 3
 *                     (6 at k = 13);
 *                     other k: one entry per (k+J-1)-mer holding the J
 *                     codes / values of its J consecutive k-mers (J <= 5;
 *                     J = 5 with 12-bit codes and an escape). */
#define KS_TABLE_COMPRESS 1
#define KS_TABLE_EXPAND 2
typedef struct ks_table ks_table;
ks_status ks_table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                          int32_t flags, ks_table **out);
/* As ks_table_create, with the k-mer counts of the sequences to be scanned
 * (device pointer, 4^k int32; NULL = none) as a position-frequency hint:
 * it only decides which values get the short codes of the expanded table,
 * never the results. */
ks_status ks_table_create_hint(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                               int32_t flags, const int32_t *freq_dev, ks_table **out);
/* Score table built on the device from device-resident k-mer counts
 * (counts_dev: int32[4^k], e.g. ks_count_dev's), with no 4^k-sized host
 * round trip.  score:
 *   KS_SCORE_LOG2  w = log2(f / f_med), f = counts / sum(counts), f_med = R
 *                  median(f) (README.md:27-42, kmer.counts()$f kmer_spans.R:25)
 *   KS_SCORE_PM1   w = f >= f_med ? 1 : -1 (README.md:37-42)
 *   KS_SCORE_RANK  w = rank_kmers_w(counts, total) (kmer_spans.c:189-202;
 *                  total = the word count, as kmer_low_comp_regions :600-602)
 * total is ignored for LOG2 / PM1.  The table holds s = w - thr; it is
 * bitwise the table ks_table_create_hint(ks_log2_table / ks_pm1_table /
 * ks_rank_table(...), thr, flags, counts_dev) builds: log2 and +-1 are
 * evaluated once per distinct count on the host (glibc log2), the ranks by
 * a closed-form exact evaluation of the sequential FP64 prefix.  counts_dev
 * also serves as the position-frequency hint.  max_ext_bytes caps the
 * expanded table (<= 0: the default cap).  w_dev: optional device
 * double[4^k] receiving w.  In ks_table_info, ms_upload is the sort + value
 * phase and ms_compress the code/value mapping. */
#define KS_SCORE_LOG2 1
#define KS_SCORE_PM1 2
#define KS_SCORE_RANK 3
ks_status ks_table_from_counts(ks_ctx *ctx, const int32_t *counts_dev, int32_t k, int32_t score,
                               double total, double thr, int32_t flags, int64_t max_ext_bytes,
                               double *w_dev, ks_table **out);
void ks_table_destroy(ks_table *t);
/* The library keeps the buffer of the last destroyed expanded table (one
 * per device) for the next table that fits in it: a fresh 32-128 GiB
 * hipMalloc can take seconds (the driver clears new VRAM).  Like a caching
 * allocator, it stays allocated after the call that destroyed the table
 * returns (up to 128 GiB at k = 13 for a device-API table, 32 GiB for the
 * host entry points' J = 4 tables).  This returns it to the driver; so does
 * ks_ctx_destroy for its device; environment KS_EXT_POOL=0 disables the
 * pool.  Workspace retained by a context (scan scratch, the table builder's
 * sort scratch of ~20 B x 4^k) is freed by ks_ctx_destroy.  The last two freed region
 * output blocks of >= 1 MiB (ks_regions_free) are kept for reuse and freed here too. */
void ks_release_cache(void);
/* Memory policy of the host-buffer entry points (ks_kmer_counts,
 * ks_kmer_regions, ks_low_comp_regions, ks_tr_lr_regions, ks_windowed_dist,
 * ks_kmers_to_file): what happens to a call's device memory -- the context's
 * workspace and the pooled table buffer -- when it ends.
 *   keep = 2 (the default): kept while calls keep coming, returned once the
 *            context has been idle for the idle time (ks_set_host_cache_idle,
 *            20 s by default; a library thread returns it), so a session that
 *            calls kmer_regions_r in a loop pays for fresh VRAM once (the
 *            driver clears new VRAM: seconds for tens of GiB) and one that
 *            called it once gets its VRAM back shortly after;
 *   keep = 0: returned when the call ends (VRAM at its pre-call level on
 *            return; every call allocates again);
 *   keep = 1: kept until ks_release_cache() or ks_ctx_destroy.
 * Environment KS_HOST_CACHE=0/1/2 and KS_HOST_CACHE_SECONDS set them at first
 * use.  The pinned host staging buffer is kept either way. */
ks_status ks_set_host_cache(int32_t keep);
ks_status ks_set_host_cache_idle(double seconds);

/* Fork broker (mclapply after use, test.R:351 then :554-565).  On: right
 * before this process's first HIP use the library forks a broker process (a
 * copy that never touched HIP; not started if HIP is already open in the
 * process, e.g. by torch); children forked later send their host-buffer calls
 * (ks_kmer_counts, ks_kmer_regions, ks_low_comp_regions, ks_tr_lr_regions,
 * ks_windowed_dist, ks_kmers_to_file) to it over a Unix socket instead of
 * being refused.  Off by default (KS_FORK_BROKER=1 turns it on); the R shim's
 * R_init_kmer_spans turns it on.  Call before the first HIP use. */
ks_status ks_set_fork_broker(int32_t on);
/* 1 if the table is stored compressed (uint16 codes + LUT), else 0. */
int32_t ks_table_is_compressed(const ks_table *t);
int64_t ks_table_distinct(const ks_table *t);
/* Scan indices served per random table read (J of the expanded table, 1 if
 * it was not built). */
int32_t ks_table_positions_per_read(const ks_table *t);
/* Bits per value code in the expanded table (12, 13 for 128-B lines, 16),
 * 16 for a compressed table without one, 64 for an FP64 table. */
int32_t ks_table_code_bits(const ks_table *t);
/* Share of positions (by the hint, else by k-mer multiplicity) whose value
 * escapes the short codes: the 12-bit codes (code bits 12, every index) or
 * the 11-bit three-base continuations of 128-B lines (code bits 13, one
 * index per line); 0 otherwise. */
double ks_table_escape_fraction(const ks_table *t);

/* Shape and setup cost of a device table (host wall clock around the
 * synchronised device work of ks_table_create*, milliseconds). */
typedef struct ks_table_info {
  int32_t k, compressed, positions_per_read, code_bits;
  int64_t distinct, ext_bytes;
  double escape_fraction;
  double ms_upload;    /* w to the device, s = w - thr, finiteness scan          */
  double ms_compress;  /* distinct values (radix sort + unique), uint16 codes    */
  double ms_codes12;   /* 12-bit code choice: position-weight histogram, renumber */
  double ms_ext_alloc; /* hipMalloc of the expanded table                        */
  double ms_ext_build; /* expanded-table build kernel                            */
  double ms_total;
  int32_t line_kind;   /* 0: no line table; 1: uint16 64-B lines, 2: FP64 64-B lines, 3: 128-B lines */
  int32_t line_own;    /* own k-mers per line (m = k + line_own - 1)              */
} ks_table_info;
ks_status ks_table_get_info(const ks_table *t, ks_table_info *out);

/* Scan statistics of the last ks_scan_dev call (device time of each phase,
 * measured with hipEvents on the ctx stream). */
typedef struct ks_scan_stats {
  double ms_total;      /* whole scan (runs + kernels + compaction) */
  double ms_runs;       /* run segmentation */
  double ms_scan;       /* dominant scan kernel(s) */
  double ms_rescan;     /* rescan rounds */
  double ms_finish;     /* region ordering + D2H */
  int64_t n_bases;      /* bytes of sequences with length >= k */
  int64_t n_scored;     /* top-level scored positions */
  int64_t n_runs;       /* N-free runs with scored positions */
  int64_t n_regions;
  int64_t n_rescan;     /* rescan ranges processed */
  int32_t scan_algo;    /* 0 = lane per run, 1 = chunked carry scan */
  int64_t n_replay;     /* chunks whose carry needed an exact replay */
  /* chunked scan (scan_algo 1) phases inside the step; ms_scan is P1 */
  double ms_layout;     /* chunk table (k_make_chunks) */
  double ms_predict;    /* P2: approximate carry scan, segment marks, binade summaries */
  double ms_carry;      /* P3/P4: exact carry, heads */
  double ms_stitch;     /* P5: excursion stitch, candidates */
} ks_scan_stats;

/* Span scan of device-resident sequences (the hot path).  visits_dev: device
 * int32[4^k] accumulated (caller zeroes), or NULL.  Regions are returned in
 * host memory.  stats may be NULL. */
ks_status ks_scan_dev(ks_ctx *ctx, const ks_dev_seqs *seqs, int32_t k, const ks_table *table,
                      int32_t min_width, double min_score, int32_t *visits_dev,
                      ks_regions *out, ks_scan_stats *stats);

/* tr_lr scan of device-resident sequences: trans = transition scores, init
 * = first-k-mer scores, both ks_tables in 2-bit code order built with
 * threshold 0 (init without KS_TABLE_COMPRESS).  Tables with non-finite
 * values are scanned by the literal per-run kernel (the reference keeps NaN
 * through its clamp); all others by the chunked scan. */
ks_status ks_tr_lr_dev(ks_ctx *ctx, const ks_dev_seqs *seqs, int32_t k, const ks_table *trans,
                       const ks_table *init, int32_t min_length, ks_regions *out, ks_scan_stats *stats);

/* k-mer counting of device-resident sequences into counts_dev (int32[4^k],
 * accumulated: the caller zeroes it).  *n_words as in ks_kmer_counts. */
ks_status ks_count_dev(ks_ctx *ctx, const ks_dev_seqs *seqs, int32_t k, int32_t *counts_dev,
                       double *n_words);

/* ---------------------------------------------------------------------
 * Ingest: sequence files -> device-resident records,
 * batched multi-k counting and the reference's binary count files.
 * --------------------------------------------------------------------- */

/* Records of a FASTA file resident on the device.  The reference reads
 * sequence files with Biostrings::readDNAStringSet (kmers.to.file,
 * kmer_spans.R:127-160); here the raw bytes go to HBM and are parsed there
 * (description lines '>', ';' comments, one '\r' before '\n' dropped, empty
 * lines skipped, IUPAC DNA letters of either case plus '-', '+', '.'; other
 * bytes, or sequence before the first description line, are errors).  Kept
 * bytes are upper-cased (as.character(DNAStringSet)).  seqs can be passed to
 * ks_scan_dev / ks_tr_lr_dev / ks_count_dev directly. */
typedef struct ks_fasta {
  ks_dev_seqs seqs;   /* records with length >= min_len, device bytes + offsets */
  char **names;       /* seqs.nseq descriptions (the line after '>')            */
  int64_t n_records;  /* records in the file                                    */
  int64_t bases_all;  /* bases of all records (seq.size, kmer_spans.R:139)      */
  int64_t bases_kept; /* bases of the kept records (seq.fsize, :141)            */
  int32_t device;
  double ms_upload;   /* host read + H2D (overlapped)                           */
  double ms_parse;    /* device parse + record selection                        */
} ks_fasta;
/* path: plain or gzip FASTA.  Keeps records with length >= min_len (:141). */
ks_status ks_fasta_load(ks_ctx *ctx, const char *path, int64_t min_len, ks_fasta *out);
/* The same from an in-memory FASTA text of n bytes. */
ks_status ks_fasta_parse(ks_ctx *ctx, const char *buf, int64_t n, int64_t min_len, ks_fasta *out);
/* Copy the kept records' bytes (offsets_host[nseq] bytes) to host memory. */
ks_status ks_fasta_copy_seqs(const ks_fasta *f, uint8_t *dst);
void ks_fasta_free(ks_fasta *f);

/* k-mer counting for several k in one pass over device-resident sequences
 * (kmer.counts per k, kmer_spans.R:149-151).  counts_dev[i]: device
 * int32[4^ks[i]] accumulated (caller zeroes); n_words[i] as ks_kmer_counts. */
ks_status ks_count_multi_dev(ks_ctx *ctx, const ks_dev_seqs *seqs, const int32_t *ks, int32_t nk,
                             int32_t *const *counts_dev, double *n_words);

/* Count file of kmers.to.file / read.kmers (kmer_spans.R:113-186): int32
 * magic, int32 n, n x int32 4^k, then the n count vectors (int32, native
 * order). */
ks_status ks_count_file_write(const char *path, int32_t magic, int32_t nk, const int32_t *ks,
                              const int32_t *const *counts);
typedef struct ks_count_file {
  int32_t valid;      /* 0: wrong magic or n < 1 (read.kmers returns FALSE)   */
  int32_t nk;
  int32_t *k;         /* as.integer(log2(4^k) / 2) (:184); -1 for length 0    */
  int64_t *lens;      /* entries actually read (readBin stops at EOF)         */
  int32_t **counts;
} ks_count_file;
ks_status ks_count_file_read(const char *path, int32_t magic, ks_count_file *out);
void ks_count_file_free(ks_count_file *f);

/* kmers.to.file(seq.f, out.prefix, k, min.l, magic) -- kmer_spans.R:127-160:
 * load, drop records shorter than min_l, count every k (ks_count_multi_dev),
 * write <out_prefix>counts_<k1>_<k2>...bin.  A file that cannot be read, a
 * bad k, or no record left is the reference's NA result: KS_OK with
 * written = 0 and the reason in message. */
typedef struct ks_kmer_file_info {
  int32_t written;
  double seq_size, seq_fsize, seq_fl; /* :139-142 */
  char out_path[4096];
  char message[512];
} ks_kmer_file_info;
ks_status ks_kmers_to_file(ks_ctx *ctx, const char *seq_path, const char *out_prefix, const int32_t *ks,
                           int32_t nk, double min_l, int32_t magic, ks_kmer_file_info *info);

/* ---------------------------------------------------------------------
 * Windowed k-mer count distributions.
 * --------------------------------------------------------------------- */

/* windowed_kmer_count_distributions_r(seq_r, kmers_r, k_r, window_r,
 * ret_flag_r) -- replaces kmer_spans.c:717-793 (window.kmer.dist,
 * kmer_spans.R:103-118).  In every N-free run of every sequence longer than
 * window, each window of `window` bases holds window - k + 1 k-mers; for
 * query k-mer i (kmers[i], k characters, coded by init_kmer :757-758)
 * dist[i * (window + 1) + c] counts the windows holding it c times
 * (column-major (window + 1) x kmer_n, overwritten).  seq_included[q] = 1 if
 * lens[q] > window.  ret_flag & 1: scores[q] (int32 [lens[q] x kmer_n],
 * column-major, for included q; may be NULL to skip one) receives the count
 * at every window start, 0 elsewhere.  1 <= k <= 15, window >= 2k. */
ks_status ks_windowed_dist(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq,
                           const char *const *kmers, int32_t kmer_n, int32_t k, int32_t window, int32_t ret_flag,
                           int32_t *dist, int32_t *seq_included, int32_t *const *scores);
/* Device-resident form: kmer_codes are 2-bit codes (< 4^k); dist_dev
 * accumulated (caller zeroes); included_dev may be NULL; scores_dev (NULL =
 * none, zeroed by the caller) holds per sequence q the [len_q x kmer_n]
 * matrix at element offset kmer_n * offsets[q]. */
ks_status ks_windowed_dev(ks_ctx *ctx, const ks_dev_seqs *seqs, const uint32_t *kmer_codes, int32_t kmer_n,
                          int32_t k, int32_t window, int32_t *dist_dev, int32_t *included_dev, int32_t *scores_dev);

/* Scan algorithm selection (testing/benchmarking): -1 auto, 0 lane-per-run,
 * 1 chunked carry scan. */
ks_status ks_ctx_set_scan_algo(ks_ctx *ctx, int32_t algo);

#ifdef __cplusplus
}
#endif
#endif /* KMER_SPANS_H */
