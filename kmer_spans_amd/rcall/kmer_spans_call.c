/*
 * kmer_spans_call.c -- the R .Call entry points of lmjakt/kmer_spans
 * (kmer_spans.c:452-808) re-implemented over the C ABI of libkmerspans
 * (include/kmer_spans.h).  Build with R CMD SHLIB (see Makevars) into
 * src/kmer_spans.so next to kmer_spans.R; kmer_spans.R then works unchanged.
 *
 * Every routine keeps the reference's name, arity, argument checks, error
 * strings and return layout; the span scan, counting and table work runs on
 * the GPU through ks_*().  Arguments are validated completely before any
 * allocation because error() longjmps (kmer_spans.c:454-457, 491-511,
 * 549-568, 624-628).  HIP is initialised lazily inside the calling process,
 * so forked workers (parallel::mclapply, test.R:550-567) each get their own
 * context.
 */
#include <R.h>
#include <R_ext/Rdynload.h>
#include <Rinternals.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "kmer_spans.h"

#define MAX_K 16 /* the reference's MAX_K (kmer_spans.c:37); 16 itself is rejected by ks_* */

/* Marshal a STRSXP into (pointer, length) arrays; R strings hold no NUL. */
typedef struct {
  const char **ptrs;
  int64_t *lens;
  int n;
} seq_view;

static seq_view view_seqs(SEXP seq_r) {
  seq_view v;
  v.n = length(seq_r);
  v.ptrs = (const char **)R_alloc((size_t)v.n, sizeof(char *));
  v.lens = (int64_t *)R_alloc((size_t)v.n, sizeof(int64_t));
  for (int i = 0; i < v.n; ++i) {
    SEXP s = STRING_ELT(seq_r, i);
    v.ptrs[i] = CHAR(s);
    v.lens[i] = (int64_t)length(s);
  }
  return v;
}

static void ks_check(ks_status st) {
  if (st != KS_OK) error("%s", ks_last_error());
}

/* Copy a ks_regions into R's (3 x n int, 2 x n double) matrices. */
static void regions_to_r(ks_regions *reg, SEXP ret, int i_ints, int i_dbls) {
  SET_VECTOR_ELT(ret, i_ints, allocMatrix(INTSXP, 3, (int)reg->n));
  SET_VECTOR_ELT(ret, i_dbls, allocMatrix(REALSXP, 2, (int)reg->n));
  int *ip = INTEGER(VECTOR_ELT(ret, i_ints));
  double *dp = REAL(VECTOR_ELT(ret, i_dbls));
  for (int64_t j = 0; j < reg->n; ++j) {
    ip[3 * j] = reg->seq_id[j];
    ip[3 * j + 1] = reg->beg[j];
    ip[3 * j + 2] = reg->end[j];
    dp[2 * j] = reg->score[j];
    dp[2 * j + 1] = 0.0;
  }
  ks_regions_free(reg);
}

/* kmer_counts(seq_r, k_r)  -- kmer_spans.c:453-487 */
SEXP kmer_counts(SEXP seq_r, SEXP k_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r must be a character vector of length at least one");
  if (TYPEOF(k_r) != INTSXP || length(k_r) < 1)
    error("k_r must be an integer vector of length at least one");
  int k = INTEGER(k_r)[0];
  if (k < 1 || k > MAX_K)
    error("k must be a positive integer less than 1+MAX_K");
  if (k > KS_MAX_K) error("k must be a positive integer less than 1+MAX_K");
  seq_view v = view_seqs(seq_r);
  size_t counts_size = (size_t)1 << (2 * k);
  SEXP ret = PROTECT(allocVector(VECSXP, 2));
  SET_VECTOR_ELT(ret, 0, allocVector(REALSXP, 1));
  SET_VECTOR_ELT(ret, 1, allocVector(INTSXP, (R_xlen_t)counts_size));
  double n = 0;
  ks_status st = ks_kmer_counts(NULL, v.ptrs, v.lens, v.n, k, INTEGER(VECTOR_ELT(ret, 1)), &n);
  if (st != KS_OK) { UNPROTECT(1); ks_check(st); }
  REAL(VECTOR_ELT(ret, 0))[0] = n;
  UNPROTECT(1);
  return ret;
}

/* kmer_regions_r(seq_r, k_r, kmer_w_r, min_width_r, min_score_r)  -- :490-546 */
SEXP kmer_regions_r(SEXP seq_r, SEXP k_r, SEXP kmer_w_r, SEXP min_width_r, SEXP min_score_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r must be a character vector of length at least one");
  if (TYPEOF(k_r) != INTSXP || length(k_r) < 1)
    error("k_r must be an integer vector of length at least one");
  if (TYPEOF(kmer_w_r) != REALSXP)
    error("kmer_w_r must be a double vector of length k^4");
  if (TYPEOF(min_width_r) != INTSXP || length(min_width_r) != 1)
    error("the minimum width must be an integer vector of length 1");
  if (TYPEOF(min_score_r) != REALSXP || length(min_score_r) != 1)
    error("the minimum score must be a REAL vector of length 1");
  int k = INTEGER(k_r)[0];
  if (k >= MAX_K)
    error("kmer sizes larger than or equal to %d not currently supported", MAX_K);
  if (k < 1) error("k must be a positive integer");
  int kmer_n = length(kmer_w_r);
  if ((unsigned int)kmer_n != (1u << (2 * k)))
    error("kmer_w contains %d elements but should have %d", kmer_n, (1 << (2 * k)));
  seq_view v = view_seqs(seq_r);
  SEXP ret = PROTECT(allocVector(VECSXP, 4));
  SET_VECTOR_ELT(ret, 0, allocVector(REALSXP, 1));
  SET_VECTOR_ELT(ret, 1, allocVector(INTSXP, kmer_n));
  double n = 0;
  ks_regions reg;
  ks_status st = ks_kmer_regions(NULL, v.ptrs, v.lens, v.n, k, REAL(kmer_w_r), kmer_n,
                                 INTEGER(min_width_r)[0], REAL(min_score_r)[0],
                                 INTEGER(VECTOR_ELT(ret, 1)), &n, &reg);
  if (st != KS_OK) { UNPROTECT(1); ks_check(st); }
  REAL(VECTOR_ELT(ret, 0))[0] = n;
  regions_to_r(&reg, ret, 2, 3);
  UNPROTECT(1);
  return ret;
}

/* kmer_low_comp_regions(seq_r, k_r, min_width_r, min_score_r, threshold_r) -- :548-621 */
SEXP kmer_low_comp_regions(SEXP seq_r, SEXP k_r, SEXP min_width_r, SEXP min_score_r, SEXP threshold_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r must be a character vector of length at least one");
  if (TYPEOF(k_r) != INTSXP || length(k_r) < 1)
    error("k_r must be an integer vector of length at least one");
  if (TYPEOF(min_width_r) != INTSXP || length(min_width_r) != 1)
    error("the minimum width must be an integer vector of length 1");
  if (TYPEOF(min_score_r) != REALSXP || length(min_score_r) != 1)
    error("the minimum score must be a REAL vector of length 1");
  if (TYPEOF(threshold_r) != REALSXP || length(threshold_r) != 1)
    error("the threshold must be a REAL vector of length 1");
  int k = INTEGER(k_r)[0];
  double threshold = REAL(threshold_r)[0];
  if (threshold <= 0 || threshold >= 1)
    error("the threshold must be between 0 and 1");
  if (k < 1 || k > KS_MAX_K) /* unchecked in the reference (Q7) */
    error("k must be a positive integer less than 1+MAX_K");
  seq_view v = view_seqs(seq_r);
  size_t counts_size = (size_t)1 << (2 * k);
  SEXP ret = PROTECT(allocVector(VECSXP, 5));
  SET_VECTOR_ELT(ret, 0, allocVector(REALSXP, 2));
  SET_VECTOR_ELT(ret, 1, allocVector(INTSXP, (R_xlen_t)counts_size));
  SET_VECTOR_ELT(ret, 2, allocVector(REALSXP, (R_xlen_t)counts_size));
  ks_regions reg;
  ks_status st = ks_low_comp_regions(NULL, v.ptrs, v.lens, v.n, k, INTEGER(min_width_r)[0],
                                     REAL(min_score_r)[0], threshold, INTEGER(VECTOR_ELT(ret, 1)),
                                     REAL(VECTOR_ELT(ret, 2)), REAL(VECTOR_ELT(ret, 0)), &reg);
  if (st != KS_OK) { UNPROTECT(1); ks_check(st); }
  regions_to_r(&reg, ret, 3, 4);
  UNPROTECT(1);
  return ret;
}

/* kmer_seq_r(k_r)  -- :623-639 */
SEXP kmer_seq_r(SEXP k_r) {
  if (TYPEOF(k_r) != INTSXP || length(k_r) != 1)
    error("k_r should be an integer of length 1");
  unsigned int k = (unsigned int)(INTEGER(k_r)[0]);
  if (k > MAX_K || k < 1)
    error("k_r (%d) should be smaller than MAX_K (%d) and larger than 0", k, MAX_K);
  if (k > KS_MAX_K) error("k_r (%d) should be smaller than MAX_K (%d) and larger than 0", k, MAX_K);
  size_t n = (size_t)1 << (2 * k);
  char *buf = (char *)malloc(n * (k + 1));
  if (!buf) error("out of memory");
  ks_status st = ks_kmer_seq((int32_t)k, buf, n * (k + 1));
  if (st != KS_OK) { free(buf); ks_check(st); }
  SEXP ret = PROTECT(allocVector(STRSXP, (R_xlen_t)n));
  for (size_t i = 0; i < n; ++i) SET_STRING_ELT(ret, (R_xlen_t)i, mkChar(buf + i * (k + 1)));
  free(buf);
  UNPROTECT(1);
  return ret;
}

/* tr_lr_regions_r(seq_r, params_r, kmers_r, kmer_scores_r, trans_scores_r)
 * -- :649-713.  Returns list(spectra (4^k x 2: the remapped kmer and
 * transition scores), pos (3 x n: 1-based seq_id, beg, end), scores (2 x n)).
 * trans_scores_r is type-checked here (the reference reads it unchecked). */
SEXP tr_lr_regions_r(SEXP seq_r, SEXP params_r, SEXP kmers_r, SEXP kmer_scores_r, SEXP trans_scores_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r should be a character vector of of positive length");
  if (TYPEOF(params_r) != INTSXP || length(params_r) != 2)
    error("params_r should have two integers (k, and min_length)");
  if (TYPEOF(kmers_r) != STRSXP)
    error("kmers_r should be a character vector");
  if (TYPEOF(kmer_scores_r) != REALSXP || TYPEOF(trans_scores_r) != REALSXP)
    error("freq_a and freq_b should be double vectors");
  int k = INTEGER(params_r)[0];
  int min_length = INTEGER(params_r)[1];
  if (k < 1 || k > MAX_K)
    error("k should be a positive value less than MAX_K");
  if (min_length < 0)
    error("min_length should be a positive integer");
  if (k > KS_MAX_K) error("k should be a positive value less than MAX_K");
  size_t kmers_size = (size_t)1 << (2 * k);
  if ((size_t)length(kmers_r) != kmers_size || (size_t)length(kmer_scores_r) != kmers_size ||
      (size_t)length(trans_scores_r) != kmers_size)
    error("kmers_r, freq_a, freq_b should all be 4^k long");
  seq_view v = view_seqs(seq_r);
  const char **kmers = (const char **)R_alloc(kmers_size, sizeof(char *));
  for (size_t i = 0; i < kmers_size; ++i) kmers[i] = CHAR(STRING_ELT(kmers_r, (R_xlen_t)i));
  SEXP ret = PROTECT(allocVector(VECSXP, 3));
  SET_VECTOR_ELT(ret, 0, allocMatrix(REALSXP, (int)kmers_size, 2));
  ks_regions reg;
  ks_status st = ks_tr_lr_regions(NULL, v.ptrs, v.lens, v.n, k, min_length, kmers, REAL(kmer_scores_r),
                                  REAL(trans_scores_r), (int64_t)kmers_size, REAL(VECTOR_ELT(ret, 0)), &reg);
  if (st != KS_OK) { UNPROTECT(1); ks_check(st); }
  regions_to_r(&reg, ret, 1, 2);
  UNPROTECT(1);
  return ret;
}

/* windowed_kmer_count_distributions_r(seq_r, kmers_r, k_r, window_r, ret_flag_r)
 * -- :717-793.  Returns list(dist ((window + 1) x kmer_n int), seq.i (int per
 * sequence: 1 if longer than window), scores (ret_flag & 1: per sequence a
 * length x kmer_n int matrix, NULL for excluded sequences; else NULL)). */
SEXP windowed_kmer_count_distributions_r(SEXP seq_r, SEXP kmers_r, SEXP k_r, SEXP window_r, SEXP ret_flag_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r should be a character vector with at least one element");
  if (TYPEOF(kmers_r) != STRSXP || length(kmers_r) < 1)
    error("kmers_r should be a character vector with at least one element");
  if (TYPEOF(k_r) != INTSXP || length(k_r) != 1)
    error("k_r should be an integer vector with one element");
  if (TYPEOF(window_r) != INTSXP || length(window_r) != 1)
    error("window_r should be an integer vector with one element");
  if (TYPEOF(ret_flag_r) != INTSXP || length(ret_flag_r) != 1)
    error("ret_flag_r should a single integer");
  unsigned int k = (unsigned int)asInteger(k_r);
  if (k >= MAX_K)
    error("kmer sizes larger than or equal to %d not currently supported", MAX_K);
  for (int i = 0; i < length(kmers_r); ++i)
    if ((unsigned int)length(STRING_ELT(kmers_r, i)) != k)
      error("All kmers specified must be of the same length");
  int window = asInteger(window_r);
  if (window < 2 * (int)k)
    error("The window size must be at least two times k");
  unsigned int ret_flag = (unsigned int)asInteger(ret_flag_r);
  int kmer_n = length(kmers_r);
  seq_view v = view_seqs(seq_r);
  const char **kmers = (const char **)R_alloc((size_t)kmer_n, sizeof(char *));
  for (int i = 0; i < kmer_n; ++i) kmers[i] = CHAR(STRING_ELT(kmers_r, i));
  SEXP ret = PROTECT(allocVector(VECSXP, 3));
  SET_VECTOR_ELT(ret, 0, allocMatrix(INTSXP, window + 1, kmer_n));
  SET_VECTOR_ELT(ret, 1, allocVector(INTSXP, v.n));
  int32_t **scores = NULL;
  if (ret_flag & 1) {
    SET_VECTOR_ELT(ret, 2, allocVector(VECSXP, v.n));
    scores = (int32_t **)R_alloc((size_t)v.n, sizeof(int32_t *));
    for (int i = 0; i < v.n; ++i) {
      scores[i] = NULL;
      if (v.lens[i] <= window) continue;
      SET_VECTOR_ELT(VECTOR_ELT(ret, 2), i, allocMatrix(INTSXP, (int)v.lens[i], kmer_n));
      scores[i] = INTEGER(VECTOR_ELT(VECTOR_ELT(ret, 2), i));
    }
  }
  ks_status st = ks_windowed_dist(NULL, v.ptrs, v.lens, v.n, kmers, kmer_n, (int32_t)k, window, (int32_t)ret_flag,
                                  INTEGER(VECTOR_ELT(ret, 0)), INTEGER(VECTOR_ELT(ret, 1)), scores);
  if (st != KS_OK) { UNPROTECT(1); ks_check(st); }
  UNPROTECT(1);
  return ret;
}

/* kmers_to_file_r(seq_f, out_prefix, k, min_l, magic) -- the body of
 * kmers.to.file (kmer_spans.R:127-160) as one routine over ks_kmers_to_file:
 * list(seq.f, out.f or NA, seq.size, seq.fsize, seq.fl). */
SEXP kmers_to_file_r(SEXP seq_f_r, SEXP out_prefix_r, SEXP k_r, SEXP min_l_r, SEXP magic_r) {
  if (TYPEOF(seq_f_r) != STRSXP || length(seq_f_r) != 1) error("seq.f must be a single file name");
  if (TYPEOF(out_prefix_r) != STRSXP || length(out_prefix_r) != 1) error("out.prefix must be a single string");
  if (TYPEOF(k_r) != INTSXP) error("k must be an integer vector");
  if (TYPEOF(min_l_r) != REALSXP || length(min_l_r) != 1) error("min.l must be a single number");
  if (TYPEOF(magic_r) != INTSXP || length(magic_r) != 1) error("magic must be a single integer");
  ks_kmer_file_info info;
  ks_status st = ks_kmers_to_file(NULL, CHAR(STRING_ELT(seq_f_r, 0)), CHAR(STRING_ELT(out_prefix_r, 0)),
                                  INTEGER(k_r), length(k_r), REAL(min_l_r)[0], INTEGER(magic_r)[0], &info);
  ks_check(st);
  SEXP ret = PROTECT(allocVector(VECSXP, 5));
  SET_VECTOR_ELT(ret, 0, seq_f_r);
  if (info.written) {
    SET_VECTOR_ELT(ret, 1, allocVector(STRSXP, 1));
    SET_STRING_ELT(VECTOR_ELT(ret, 1), 0, mkChar(info.out_path));
  } else {
    SET_VECTOR_ELT(ret, 1, ScalarLogical(NA_LOGICAL));
  }
  SET_VECTOR_ELT(ret, 2, ScalarReal(info.seq_size));
  SET_VECTOR_ELT(ret, 3, ScalarReal(info.seq_fsize));
  SET_VECTOR_ELT(ret, 4, ScalarReal(info.seq_fl));
  UNPROTECT(1);
  return ret;
}

static const R_CallMethodDef callMethods[] = {
    {"kmer_counts", (DL_FUNC)&kmer_counts, 2},
    {"kmer_regions_r", (DL_FUNC)&kmer_regions_r, 5},
    {"kmer_low_comp_regions", (DL_FUNC)&kmer_low_comp_regions, 5},
    {"kmer_seq_r", (DL_FUNC)&kmer_seq_r, 1},
    {"tr_lr_regions_r", (DL_FUNC)&tr_lr_regions_r, 5},
    {"windowed_kmer_count_distributions_r", (DL_FUNC)&windowed_kmer_count_distributions_r, 5},
    {"kmers_to_file_r", (DL_FUNC)&kmers_to_file_r, 5},
    {NULL, NULL, 0}};

void R_init_kmer_spans(DllInfo *info) {
  R_registerRoutines(info, NULL, callMethods, NULL, NULL);
  /* mclapply workers forked after a call in the R session (test.R:351 then
     :554-565) reach the GPU through the broker (ks_broker.cpp) */
  ks_set_fork_broker(1);
}
