/*
 * ks_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the lmjakt/kmer_spans span-scan path (reference snapshot
 * 2025-03-21, /root/reference/src/kmer_spans.c).  It is the parity checker for
 * the HIP product path (kmer_spans_amd/libkmerspans.so) and the "port" CPU
 * baseline timed by bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Parity pinning: the reference cannot be built here (it includes R.h /
 * Rinternals.h and R is absent; stand-in headers are not allowed), so this
 * restatement is pinned by (1) the test.R known-answer comments and (2) the
 * reference outputs recorded in SURVEY.md section 8(c) during the survey, both
 * committed as tests/golden/ fixtures.  See DESIGN.md "Oracle".
 */
#ifndef KS_ORACLE_H
#define KS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Region records, column layout of seq_regions (kmer_spans.c:46-58):
 * ints (seq_id, beg, end), doubles (score, 0.0). */
typedef struct {
  int64_t n, cap;
  int32_t *seq_id, *beg, *end;
  double *score;
} orc_regions;

void orc_regions_free(orc_regions *r);

/* kmer_counts (.Call, kmer_spans.c:453-487).  counts: int32[4^k], zeroed by
 * the callee.  *n_words = sum over sequences with len >= k of the words
 * counted (as double, :483).  Returns 0 or a negative error code. */
int orc_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq,
                    int32_t k, int32_t *counts, double *n_words);

/* kmer_regions_r (.Call, kmer_spans.c:490-546): threshold 0, visit histogram
 * (visits: int32[4^k], zeroed by the callee, may be NULL), n = sum of lengths
 * of sequences with len >= k (:535). */
int orc_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq,
                     int32_t k, const double *w, int32_t min_width,
                     double min_score, int32_t *visits, double *n_bases,
                     orc_regions *out);

/* Generic scan used by both .Call paths: kmer_regions (kmer_spans.c:243-307)
 * over every sequence with len >= k, threshold thr, optional visit histogram
 * (accumulated, not zeroed). */
int orc_scan(const char *const *seqs, const int64_t *lens, int32_t nseq,
             int32_t k, const double *w, double thr, int32_t min_width,
             double min_score, int32_t *visits, orc_regions *out);

/* kmer_low_comp_regions (.Call, kmer_spans.c:548-621).  counts int32[4^k],
 * ranks double[4^k], n[2] = {#words, 0} (Q8). */
int orc_low_comp(const char *const *seqs, const int64_t *lens, int32_t nseq,
                 int32_t k, int32_t min_width, double min_score, double thr,
                 int32_t *counts, double *ranks, double *n, orc_regions *out);

/* rank_kmers_w (kmer_spans.c:189-202) with a stable (count, index) order and
 * ranks[idx[0]] = 0 (the reference's zero-filled-allocation behaviour, Q3). */
int orc_rank_table(const int32_t *counts, int32_t k, double total, double *ranks);

/* Score tables of README.md:27-42 as the R user code builds them from
 * kmer.counts()$f (kmer_spans.R:25): f = counts / sum(counts); f_med = R
 * median(f); log2(f / f_med) or ifelse(f >= f_med, 1, -1). */
int orc_log2_table(const int32_t *counts, int32_t k, double *w);
int orc_pm1_table(const int32_t *counts, int32_t k, double *w);

/* kmer_seq_r (kmer_spans.c:623-639): 4^k strings of k chars in internal
 * A,C,T,G code order, written as out[i*(k+1) .. ] NUL-terminated. */
int orc_kmer_seq(int32_t k, char *out);

/* tr_lr_regions_r (kmer_spans.c:649-713, find_kmer_tr_lr_regions :329-395):
 * orc_trlr_remap maps the user-ordered tables (kmers[i] spells entry i) to
 * 2-bit code order; orc_tr_lr_regions scans with those tables.  Regions are
 * 1-based (seq_id, beg, end) with the region maximum as score. */
int orc_trlr_remap(const char *const *kmers, int32_t k, const double *ks_in, const double *tr_in,
                   double *ks_out, double *tr_out);
int orc_tr_lr_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                      int32_t min_len, const double *ks, const double *tr, orc_regions *out);
void orc_trlr_one(const char *s, int64_t len, int32_t seq_id, int32_t k, int32_t min_len,
                  const double *ks, const double *tr, orc_regions *out);

/* FASTA reading as kmers.to.file uses it (kmer_spans.R:136-148:
 * Biostrings::readDNAStringSet, nchar filter, as.character).  Biostrings is
 * absent here (an R/Bioconductor package, not vendored), so this restates
 * its documented FASTA rules line by line: a line ends at '\n' with one '\r'
 * before it dropped; empty lines are skipped; ';' lines are comments; '>'
 * starts a record whose description is the rest of the line; other lines are
 * sequence, each byte an IUPAC DNA letter (either case) or '-', '+', '.'.
 * Returns 0, -1 (invalid byte at *err_pos) or -2 (sequence before the
 * first description, *err_pos = its first byte).  Records shorter than
 * min_len are dropped from seq/offs/names (bases_all counts them).
 * Parity for this function is unpinned against Biostrings itself. */
typedef struct {
  int64_t n_records, nseq, bases_all, err_pos;
  uint8_t *seq;      /* kept bytes, upper-cased */
  int64_t *offs;     /* nseq + 1 */
  char **names;      /* nseq */
} orc_fasta;
int orc_fasta_parse(const char *buf, int64_t n, int64_t min_len, orc_fasta *out);
void orc_fasta_free(orc_fasta *f);

/* windowed_kmer_count_distributions_r (.Call, kmer_spans.c:717-793) and
 * windowed_kmer_count_distributions (:413-449).  kmers: kmer_n strings of
 * length k (their codes via init_kmer, :757-758); dist: int32
 * [(window + 1) x kmer_n] column-major, zeroed by the callee;
 * seq_included[nseq]: 1 if len > window (:776-779); pos (may be NULL):
 * per sequence an int32 [len x kmer_n] column-major matrix, zeroed by the
 * caller, receiving the window counts at each window start (:443-444).
 * Returns 0, -1 (k >= 16 or k < 1), -2 (a k-mer string of another length) or
 * -3 (window < 2k), the reference's error() conditions (:729-742). */
int orc_windowed_dist(const char *const *seqs, const int64_t *lens, int32_t nseq, const char *const *kmers,
                      int32_t kmer_n, int32_t k, int32_t window, int32_t *dist, int32_t *seq_included,
                      int32_t *const *pos);

/* Single-sequence primitives (exposed for tests). */
uint64_t orc_count_one(const char *s, int64_t len, int32_t k, int32_t *counts);
void orc_scan_one(const char *s, int64_t len, int32_t seq_id, int32_t k,
                  const double *w, double thr, int32_t min_width,
                  double min_score, int32_t *visits, orc_regions *out);

#ifdef __cplusplus
}
#endif
#endif
