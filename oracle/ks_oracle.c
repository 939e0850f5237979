/*
 * ks_oracle.c -- TEST INFRASTRUCTURE ONLY (see ks_oracle.h).
 *
 * A from-scratch CPU restatement of the span-scan path of lmjakt/kmer_spans
 * (/root/reference/src/kmer_spans.c, snapshot 2025-03-21).  Every function
 * cites the reference lines whose observable behaviour it reproduces,
 * including the quirks catalogued in SURVEY.md section 8(a):
 *   Q1  a window that ends exactly at the end of the string is not counted
 *       (sequence_kmer_count, :142-144),
 *   Q3  rank of the least frequent k-mer is 0 (zeroed R allocation, :198),
 *   Q5  the last k-mer of every N-free run is never scored (:265-296),
 *   Q6  the visit histogram counts restarted re-visits (:266-267),
 *   Q8  kmer_low_comp_regions n[1] is always 0 (:613),
 *   plus strict '>' first-argmax (:287), size_t min_width compare (:279),
 *   NaN -> 0 clamp (:270) and int32 wrap of histograms.
 * Inputs are (pointer, length) byte strings without NUL bytes, as R CHARSXPs
 * are; the reference's NUL terminator is the position `len`.
 */
#include "ks_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_K 15 /* MAX_K is 16 in the reference (:37) but 1<<32 is UB (Q2) */

static inline int orc_is_n(unsigned char c) { return (c | 0x20) == 'n'; } /* LC(c)=='n' :35 */
static inline uint64_t orc_code(unsigned char c) { return (c >> 1) & 3u; } /* UPDATE_OFFSET :34 */

/* ------------------------------------------------------------------ regions */

void orc_regions_free(orc_regions *r) {
  free(r->seq_id); free(r->beg); free(r->end); free(r->score);
  memset(r, 0, sizeof(*r));
}

/* seq_regions_push (:80-101): append one record, doubling capacity. */
static void orc_push(orc_regions *r, int32_t id, int64_t beg, int64_t end, double score) {
  if (r->n == r->cap) {
    int64_t cap = r->cap ? r->cap * 2 : 100; /* REG_N (:38) */
    r->seq_id = (int32_t *)realloc(r->seq_id, cap * sizeof(int32_t));
    r->beg = (int32_t *)realloc(r->beg, cap * sizeof(int32_t));
    r->end = (int32_t *)realloc(r->end, cap * sizeof(int32_t));
    r->score = (double *)realloc(r->score, cap * sizeof(double));
    r->cap = cap;
  }
  r->seq_id[r->n] = id;
  r->beg[r->n] = (int32_t)beg; /* size_t -> int argument conversion (:81) */
  r->end[r->n] = (int32_t)end;
  r->score[r->n] = score;
  r->n++;
}

/* ------------------------------------------------------------ k-mer priming */

/* init_kmer + skip_n (:111-132).  From position i, skip N runs and encode the
 * first window of k consecutive non-N bases into *code.  Returns the index
 * just past that window, or `len` when the string ends first (then *code holds
 * a partial window, exactly as the reference leaves it). */
static int64_t orc_prime(const unsigned char *s, int64_t len, int64_t i, int k, uint64_t *code) {
  int64_t j = 0;
  while (i < len) {
    uint64_t c = 0;
    for (j = 0; j < k && i + j < len && !orc_is_n(s[i + j]); ++j) c = (c << 2) | orc_code(s[i + j]);
    *code = c;
    if (i + j >= len || j == k) break;
    i += j;
    while (i < len && orc_is_n(s[i])) ++i; /* skip_n */
    j = 0;
  }
  return i + j;
}

/* ----------------------------------------------------------------- counting */

/* sequence_kmer_count (:135-155).  Adds every k-mer of every N-free run to
 * counts (mod 2^32), except Q1.  Returns the number of words counted. */
uint64_t orc_count_one(const char *str, int64_t len, int32_t k, int32_t *counts) {
  const unsigned char *s = (const unsigned char *)str;
  const uint64_t mask = (((uint64_t)1) << (2 * k)) - 1;
  uint32_t *cnt = (uint32_t *)counts; /* wrap like the reference's int++ */
  uint64_t words = 0, code = 0;
  int64_t i = 0;
  while (i < len) {
    i = orc_prime(s, len, i, k, &code);
    if (i >= len) break; /* Q1: the primed window is dropped at end of string */
    cnt[code & mask]++; ++words;
    for (; i < len && !orc_is_n(s[i]); ++i) {
      code = (code << 2) | orc_code(s[i]);
      cnt[code & mask]++; ++words;
    }
  }
  return words;
}

/* --------------------------------------------------------------------- scan */

/* kmer_regions (:243-307).  At scan index i the k-mer ending at i-1 is scored
 * (so a run's last k-mer never is, Q5).  S = max(S_prev + (w - thr), 0) with
 * NaN -> 0; an excursion opens where S turns positive (beg = max_pos = i),
 * keeps the first strict maximum, and ends where S returns to 0 or at the end
 * of the run.  An ended excursion with (size_t)(max_pos-beg) >= min_width and
 * max >= min_score is emitted and the scan restarts with fresh state at
 * max_pos+1 (re-priming the k-mer that ends at max_pos).  visits[k-mer] is
 * incremented at every scored index, re-visits included (Q6). */
void orc_scan_one(const char *str, int64_t len, int32_t seq_id, int32_t k,
                  const double *w, double thr, int32_t min_width,
                  double min_score, int32_t *visits, orc_regions *out) {
  const unsigned char *s = (const unsigned char *)str;
  const uint64_t mask = (((uint64_t)1) << (2 * k)) - 1;
  const uint64_t mw = (uint64_t)(int64_t)min_width; /* int -> size_t (:536) */
  uint32_t *vis = (uint32_t *)visits;
  uint64_t code = 0;
  int64_t i = 0, beg = 0, arg = 0;
  while (i < len) {
    i = orc_prime(s, len, i, k, &code);
    double S = 0.0, prev = 0.0, best = 0.0;
    int restarted = 0;
    for (; i < len && !orc_is_n(s[i]); ++i) {
      const uint64_t idx = code & mask;
      if (vis) vis[idx]++;
      const double t = prev + (w[idx] - thr);
      S = t > 0 ? t : 0.0; /* NaN fails the compare -> 0 */
      if (prev == 0 && S > 0) { beg = i; arg = i; best = S; }
      if (S == 0 && prev > 0) {
        if ((uint64_t)(arg - beg) >= mw && best >= min_score) {
          orc_push(out, seq_id, beg, arg, best);
          i = arg + 1 - k; /* restart (:281) */
          restarted = 1;
          break;
        }
        best = 0; arg = i;
      }
      if (S > best) { best = S; arg = i; }
      prev = S;
      code = (code << 2) | orc_code(s[i]);
    }
    if (restarted) continue;
    if (S > 0 && (uint64_t)(arg - beg) >= mw && best >= min_score) { /* :298-305 */
      orc_push(out, seq_id, beg, arg, best);
      i = arg + 1 - k;
    }
  }
}

/* -------------------------------------------------------- .Call equivalents */

int orc_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq,
                    int32_t k, int32_t *counts, double *n_words) {
  if (nseq < 1) return -1;                    /* :454-455 */
  if (k < 1 || k > ORC_MAX_K) return -2;      /* :461-462 (k=16 rejected, Q2) */
  memset(counts, 0, sizeof(int32_t) * ((size_t)1 << (2 * k)));
  double n = 0;
  for (int32_t q = 0; q < nseq; ++q) {
    if (lens[q] < k) continue;                /* :478-479 */
    n += (double)orc_count_one(seqs[q], lens[q], k, counts);
  }
  *n_words = n;
  return 0;
}

int orc_scan(const char *const *seqs, const int64_t *lens, int32_t nseq,
             int32_t k, const double *w, double thr, int32_t min_width,
             double min_score, int32_t *visits, orc_regions *out) {
  for (int32_t q = 0; q < nseq; ++q) {
    if (lens[q] < k) continue;                /* :533-534, :608-609 */
    orc_scan_one(seqs[q], lens[q], q, k, w, thr, min_width, min_score, visits, out);
  }
  return 0;
}

int orc_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq,
                     int32_t k, const double *w, int32_t min_width,
                     double min_score, int32_t *visits, double *n_bases,
                     orc_regions *out) {
  if (nseq < 1) return -1;                    /* :491-492 */
  if (k < 1 || k > ORC_MAX_K) return -2;      /* :504-505 (k<1 would hang the reference) */
  if (visits) memset(visits, 0, sizeof(int32_t) * ((size_t)1 << (2 * k)));
  double n = 0;
  for (int32_t q = 0; q < nseq; ++q)
    if (lens[q] >= k) n += (double)lens[q];   /* :535 */
  *n_bases = n;
  return orc_scan(seqs, lens, nseq, k, w, 0.0, min_width, min_score, visits, out);
}

/* glibc msort (stable top-down merge sort) with the reference comparator
 * comp_index_int (:177-184): int difference of the two counts. */
static int orc_cmp(const int32_t *v, uint32_t a, uint32_t b) {
  return (int32_t)((uint32_t)v[a] - (uint32_t)v[b]);
}
static void orc_msort(uint32_t *b, uint32_t *tmp, size_t n, const int32_t *v) {
  if (n <= 1) return;
  size_t n1 = n / 2, n2 = n - n1;
  uint32_t *b1 = b, *b2 = b + n1;
  orc_msort(b1, tmp, n1, v);
  orc_msort(b2, tmp, n2, v);
  uint32_t *t = tmp;
  while (n1 > 0 && n2 > 0) {
    if (orc_cmp(v, *b1, *b2) <= 0) { *t++ = *b1++; --n1; }
    else { *t++ = *b2++; --n2; }
  }
  if (n1 > 0) memcpy(t, b1, n1 * sizeof(uint32_t));
  memcpy(b, tmp, (n - n2) * sizeof(uint32_t));
}

int orc_rank_table(const int32_t *counts, int32_t k, double total, double *ranks) {
  if (k < 1 || k > ORC_MAX_K) return -2;
  const size_t n = (size_t)1 << (2 * k);
  uint32_t *idx = (uint32_t *)malloc(n * sizeof(uint32_t));
  uint32_t *tmp = (uint32_t *)malloc(n * sizeof(uint32_t));
  if (!idx || !tmp) { free(idx); free(tmp); return -3; }
  for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  orc_msort(idx, tmp, n, counts);
  /* Zeroed allocation + ranks[0]=0 (:198) == ranks[idx[0]] = 0 (Q3). */
  ranks[idx[0]] = 0.0;
  for (size_t i = 1; i < n; ++i)             /* :199-200 */
    ranks[idx[i]] = ranks[idx[i - 1]] + ((double)counts[idx[i - 1]] / total);
  free(idx); free(tmp);
  return 0;
}

int orc_low_comp(const char *const *seqs, const int64_t *lens, int32_t nseq,
                 int32_t k, int32_t min_width, double min_score, double thr,
                 int32_t *counts, double *ranks, double *n, orc_regions *out) {
  if (nseq < 1) return -1;                    /* :549-550 */
  if (!(thr > 0 && thr < 1)) {                /* :567-568 (NaN passes there; rejected here) */
    if (thr <= 0 || thr >= 1) return -4;
  }
  if (k < 1 || k > ORC_MAX_K) return -2;      /* no check in the reference (Q7) */
  double words = 0;
  int rc = orc_kmer_counts(seqs, lens, nseq, k, counts, &words); /* :592-601 */
  if (rc) return rc;
  n[0] = words;
  rc = orc_rank_table(counts, k, words, ranks); /* :602 */
  if (rc) return rc;
  rc = orc_scan(seqs, lens, nseq, k, ranks, thr, min_width, min_score, NULL, out); /* :605-612 */
  n[1] = 0;                                   /* Q8 (:613) */
  return rc;
}

/* R mean() of two doubles (summary.c real_mean: long double sum, divide,
 * one correction pass). */
static double orc_r_mean2(double a, double b) {
  long double s = (long double)a + (long double)b;
  s /= 2;
  long double t = ((long double)a - s) + ((long double)b - s);
  s += t / 2;
  return (double)s;
}

/* f = counts / sum(counts) and R median(f) (kmer_spans.R:25; README.md:27-32).
 * sum(counts) is taken exactly in 64 bits (R >= 3.5 accumulates integer sums
 * in a 64-bit integer).  4^k is even, so the median is mean of the two middle
 * order statistics.  Returns f (malloc'd) and *fmed. */
static int cmp_double(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}
static double *orc_freqs(const int32_t *counts, int32_t k, double *fmed) {
  const size_t n = (size_t)1 << (2 * k);
  int64_t tot = 0;
  for (size_t i = 0; i < n; ++i) tot += counts[i];
  const double total = (double)tot;
  double *f = (double *)malloc(n * sizeof(double));
  double *srt = (double *)malloc(n * sizeof(double));
  if (!f || !srt) { free(f); free(srt); return NULL; }
  int has_nan = 0;
  for (size_t i = 0; i < n; ++i) { f[i] = (double)counts[i] / total; srt[i] = f[i]; has_nan |= isnan(f[i]); }
  if (has_nan) {
    *fmed = NAN; /* median() of a vector with NA is NA */
  } else {
    qsort(srt, n, sizeof(double), cmp_double);
    *fmed = orc_r_mean2(srt[n / 2 - 1], srt[n / 2]);
  }
  free(srt);
  return f;
}

int orc_log2_table(const int32_t *counts, int32_t k, double *w) {
  if (k < 1 || k > ORC_MAX_K) return -2;
  double fmed;
  double *f = orc_freqs(counts, k, &fmed);
  if (!f) return -3;
  const size_t n = (size_t)1 << (2 * k);
  for (size_t i = 0; i < n; ++i) w[i] = log2(f[i] / fmed); /* README.md:27-29 */
  free(f);
  return 0;
}

int orc_pm1_table(const int32_t *counts, int32_t k, double *w) {
  if (k < 1 || k > ORC_MAX_K) return -2;
  double fmed;
  double *f = orc_freqs(counts, k, &fmed);
  if (!f) return -3;
  const size_t n = (size_t)1 << (2 * k);
  for (size_t i = 0; i < n; ++i) /* README.md:37-42, f_t = f_med; NA -> NaN */
    w[i] = (isnan(f[i]) || isnan(fmed)) ? NAN : (f[i] >= fmed ? 1.0 : -1.0);
  free(f);
  return 0;
}

int orc_kmer_seq(int32_t k, char *out) {
  static const char nuc[4] = {'A', 'C', 'T', 'G'}; /* NUC (:41) */
  if (k < 1 || k > ORC_MAX_K) return -2;            /* :627-628 */
  const size_t n = (size_t)1 << (2 * k);
  for (size_t i = 0; i < n; ++i) {                  /* kmer_seq (:161-171) */
    char *o = out + i * (size_t)(k + 1);
    size_t c = i;
    for (int p = k - 1; p >= 0; --p) { o[p] = nuc[c & 3]; c >>= 2; }
    o[k] = 0;
  }
  return 0;
}

/* ---------------------------------------------------------- tr_lr regions */

/* tr_lr_regions_r's k-mer remap (kmer_spans.c:677-690): entry i of the input
 * tables belongs to the k-mer spelled by kmers[i]; it is stored at the code
 * init_kmer computes for that string (N-skipping, possibly short).  Entries
 * never assigned are zero here (uninitialised in the reference).  Returns the
 * number of strings whose primed length is not k (the reference prints them). */
int orc_trlr_remap(const char *const *kmers, int32_t k, const double *ks_in, const double *tr_in,
                   double *ks_out, double *tr_out) {
  const size_t n = (size_t)1 << (2 * k);
  memset(ks_out, 0, n * sizeof(double));
  memset(tr_out, 0, n * sizeof(double));
  int bad = 0;
  for (size_t i = 0; i < n; ++i) {
    const unsigned char *s = (const unsigned char *)kmers[i];
    const int64_t len = (int64_t)strlen(kmers[i]);
    uint64_t code = 0;
    const int64_t ii = orc_prime(s, len, 0, k, &code);
    if (ii != k) ++bad;
    ks_out[code] = ks_in[i];
    tr_out[code] = tr_in[i];
  }
  return bad;
}

/* find_kmer_tr_lr_regions (kmer_spans.c:329-395) for one sequence.  Per
 * N-free run: the first k-mer's kmer score, clamped at 0 (`s < 0 ? 0 : s`,
 * NaN kept), is attributed to the position just past it; then at each later
 * position the k-mer ending there adds its transition score.  The maximum is
 * tested before the clamp; a region opens where the score turns positive;
 * when it returns to 0 the region is pushed if (max_pos - begin) >=
 * min_length and the scan ALWAYS restarts at max_pos + 1 with fresh state.
 * A region still open at the end of the run is pushed without a restart.
 * The run is skipped when the string ends within one base after its first
 * k-mer (:341).  Records are 1-based: (seq_id, 1 + begin, 1 + max_pos). */
void orc_trlr_one(const char *str, int64_t len, int32_t seq_id, int32_t k, int32_t min_len,
                  const double *ks, const double *tr, orc_regions *out) {
  const unsigned char *s = (const unsigned char *)str;
  const uint64_t mask = (((uint64_t)1) << (2 * k)) - 1;
  uint64_t code = 0;
  int64_t i = 0;
  while (i < len) {
    i = orc_prime(s, len, i, k, &code);
    if (i >= len || i + 1 >= len) break;
    code &= mask;
    double last, best = 0.0, score = ks[code];
    int64_t best_pos = 0, beg = 0;
    score = score < 0 ? 0 : score;
    if (score > 0) { best = score; best_pos = i; beg = i; }
    last = score;
    while (i < len && !orc_is_n(s[i])) {
      code = mask & ((code << 2) | orc_code(s[i]));
      score = last + tr[code];
      if (score > best) { best = score; best_pos = i; }
      score = score < 0 ? 0 : score;
      if (last == 0 && score > 0) { best = score; best_pos = i; beg = i; }
      if (score == 0 && last > 0) {
        if (best_pos - beg >= min_len) orc_push(out, seq_id, 1 + beg, 1 + best_pos, best);
        i = best_pos;
        score = last = best = 0;
        beg = i;
        best_pos = 0;
        orc_prime(s, len, 1 + i - k, k, &code); /* k-mer ending at i */
      }
      last = score;
      ++i;
    }
    if (best > 0 && best_pos - beg >= min_len) orc_push(out, seq_id, 1 + beg, 1 + best_pos, best);
  }
}

/* tr_lr_regions_r (.Call, kmer_spans.c:649-713) given the remapped tables
 * (2-bit code order): seq_id is 1-based (i + 1). */
int orc_tr_lr_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                      int32_t min_len, const double *ks, const double *tr, orc_regions *out) {
  if (nseq < 1) return -1;
  if (k < 1 || k > ORC_MAX_K) return -2;
  if (min_len < 0) return -3;
  for (int32_t q = 0; q < nseq; ++q) orc_trlr_one(seqs[q], lens[q], q + 1, k, min_len, ks, tr, out);
  return 0;
}

/* ---------------------------------------------------------------- FASTA */

static int orc_dna_byte(unsigned char c) {
  return c && strchr("ACGTMRWSYKVHDBNacgtmrwsykvhdbn-+.", c) != NULL;
}

void orc_fasta_free(orc_fasta *f) {
  if (!f) return;
  for (int64_t q = 0; f->names && q < f->nseq; ++q) free(f->names[q]);
  free(f->names);
  free(f->seq);
  free(f->offs);
  memset(f, 0, sizeof(*f));
}

int orc_fasta_parse(const char *buf, int64_t n, int64_t min_len, orc_fasta *out) {
  memset(out, 0, sizeof(*out));
  out->err_pos = -1;
  /* pass 1: every record's bytes (kept after the filter below) */
  int64_t cap = 16, nrec = 0;
  int64_t *roff = malloc(sizeof(int64_t) * (cap + 1));
  int64_t *hbeg = malloc(sizeof(int64_t) * cap), *hlen = malloc(sizeof(int64_t) * cap);
  uint8_t *all = malloc((size_t)n + 1);
  int64_t nall = 0;
  roff[0] = 0;
  int64_t i = 0;
  while (i < n) {
    int64_t e = i;
    while (e < n && buf[e] != '\n') ++e;   /* line [i, e) */
    int64_t le = e;
    if (le > i && buf[le - 1] == '\r') --le;
    if (le > i) {
      if (buf[i] == '>') {
        if (nrec == cap) {
          cap *= 2;
          roff = realloc(roff, sizeof(int64_t) * (cap + 1));
          hbeg = realloc(hbeg, sizeof(int64_t) * cap);
          hlen = realloc(hlen, sizeof(int64_t) * cap);
        }
        roff[nrec] = nall;
        hbeg[nrec] = i + 1;
        hlen[nrec] = le - i - 1;
        ++nrec;
      } else if (buf[i] != ';') {
        for (int64_t j = i; j < le; ++j) {
          const unsigned char c = (unsigned char)buf[j];
          if (!nrec) { out->err_pos = j; goto fail2; }
          if (!orc_dna_byte(c)) { out->err_pos = j; goto fail1; }
          all[nall++] = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
        }
      }
    }
    i = e + 1;
  }
  roff[nrec] = nall;
  out->n_records = nrec;
  out->bases_all = nall;
  out->seq = malloc((size_t)nall + 1);
  out->offs = malloc(sizeof(int64_t) * (nrec + 1));
  out->names = calloc((size_t)nrec + 1, sizeof(char *));
  out->offs[0] = 0;
  for (int64_t r = 0; r < nrec; ++r) {
    const int64_t len = roff[r + 1] - roff[r];
    if (len < min_len) continue;
    memcpy(out->seq + out->offs[out->nseq], all + roff[r], (size_t)len);
    out->offs[out->nseq + 1] = out->offs[out->nseq] + len;
    char *nm = malloc((size_t)hlen[r] + 1);
    memcpy(nm, buf + hbeg[r], (size_t)hlen[r]);
    nm[hlen[r]] = 0;
    out->names[out->nseq++] = nm;
  }
  free(roff); free(hbeg); free(hlen); free(all);
  return 0;
fail1:
  free(roff); free(hbeg); free(hlen); free(all);
  return -1;
fail2:
  free(roff); free(hbeg); free(hlen); free(all);
  return -2;
}

/* ------------------------------------------------------- windowed counts */

/* windowed_kmer_count_distributions (:413-449), one sequence: per N-free
 * run, slide a window of `window` bases; at each window start record, for
 * every query k-mer, how many of the window's k-mers equal it. */
static void orc_windowed_one(const unsigned char *s, int64_t len, const uint64_t *kmers, int32_t kmer_n,
                             uint32_t *kmer_counts, int32_t k, int32_t window, int32_t *dist, int32_t *pos) {
  const uint64_t mask = ((uint64_t)1 << (2 * k)) - 1;
  int64_t left = 0, right = 0;
  uint64_t right_offset = 0, left_offset = 0;
  while (right < len) {                                          /* :420 */
    memset(kmer_counts, 0, sizeof(uint32_t) << (2 * k));
    right = orc_prime(s, len, right, k, &right_offset);          /* :422 */
    if (right >= len) break;                                     /* :423-424 */
    left = right;
    left_offset = right_offset;
    kmer_counts[right_offset & mask]++;                          /* :427 */
    while (right < len && !orc_is_n(s[right])) {                 /* :428 */
      right_offset = (right_offset << 2) | orc_code(s[right]);
      kmer_counts[right_offset & mask]++;
      ++right;
      if ((uint64_t)window > (uint64_t)(right - (left - k))) continue;  /* :432-433 */
      for (int32_t i = 0; i < kmer_n; ++i) {
        const uint32_t c = kmer_counts[kmers[i] & mask];
        dist[(int64_t)i * (window + 1) + c]++;
        if (pos) pos[(int64_t)i * len + (left - k)] = (int32_t)c;
      }
      kmer_counts[left_offset & mask]--;                         /* :446 */
      left_offset = (left_offset << 2) | orc_code(s[left]);
      ++left;
    }
  }
}

int orc_windowed_dist(const char *const *seqs, const int64_t *lens, int32_t nseq, const char *const *kmers,
                      int32_t kmer_n, int32_t k, int32_t window, int32_t *dist, int32_t *seq_included,
                      int32_t *const *pos) {
  if (k >= 16 || k < 1) return -1;                              /* :730-731 (MAX_K = 16) */
  for (int32_t i = 0; i < kmer_n; ++i)
    if ((int64_t)strlen(kmers[i]) != k) return -2;               /* :733-736 */
  if (window < 2 * k) return -3;                                 /* :738-739 */
  uint64_t *codes = calloc((size_t)(kmer_n > 0 ? kmer_n : 1), sizeof(uint64_t));
  for (int32_t i = 0; i < kmer_n; ++i)
    orc_prime((const unsigned char *)kmers[i], k, 0, k, codes + i);  /* :757-758 */
  uint32_t *kc = malloc(sizeof(uint32_t) << (2 * k));
  memset(dist, 0, sizeof(int32_t) * (size_t)(window + 1) * (size_t)kmer_n);
  for (int32_t q = 0; q < nseq; ++q) {
    seq_included[q] = 0;
    if (lens[q] <= window) continue;                             /* :776-777 */
    seq_included[q] = 1;
    orc_windowed_one((const unsigned char *)seqs[q], lens[q], codes, kmer_n, kc, k, window, dist,
                     pos ? pos[q] : NULL);
  }
  free(kc);
  free(codes);
  return 0;
}
