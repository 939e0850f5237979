// ks_tables.cpp -- host score-table builders (exact FP64).
//
// rank: rank_kmers_w (kmer_spans.c:189-202).  The reference sorts the 4^k
//   indices with qsort_r and comp_index_int (:177-184); glibc's qsort_r is a
//   stable merge sort, so the order is (count ascending, index ascending).
//   Here an LSD radix sort over the count bits gives that order in O(4^k)
//   (the reference spends 7.6 s sorting at k=13).  The prefix
//   r[idx[i]] = r[idx[i-1]] + count[idx[i-1]] / total is kept sequential so
//   every rounding matches; r[idx[0]] = 0 (zeroed allocation, quirk Q3).
// log2 / +-1: README.md:27-42 with f = counts / sum(counts) as kmer.counts
//   builds it (kmer_spans.R:25) and f_med = R median(f); 4^k is even, so the
//   median is R mean() of the two middle order statistics.  f is monotone in
//   the count, so those are found with nth_element on the counts.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ks_internal.h"

namespace ks {

ks_status rank_table_host(const int32_t *counts, int k, double total, double *ranks) {
  const size_t n = (size_t)1 << (2 * k);
  std::vector<uint32_t> idx(n), tmp(n);
  for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  // signed order of the int32 counts, stable: 4 LSD passes of 8 bits
  uint32_t or_all = 0, and_all = 0xffffffffu;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t key = (uint32_t)counts[i] ^ 0x80000000u;
    or_all |= key;
    and_all &= key;
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int sh = 8 * pass;
    if ((((or_all ^ and_all) >> sh) & 0xffu) == 0) continue;  // byte constant: skip
    size_t hist[257] = {0};
    for (size_t i = 0; i < n; ++i) hist[(((uint32_t)counts[idx[i]] ^ 0x80000000u) >> sh & 0xffu) + 1]++;
    for (int d = 0; d < 256; ++d) hist[d + 1] += hist[d];
    for (size_t i = 0; i < n; ++i) {
      const uint32_t d = ((uint32_t)counts[idx[i]] ^ 0x80000000u) >> sh & 0xffu;
      tmp[hist[d]++] = idx[i];
    }
    idx.swap(tmp);
  }
  ranks[idx[0]] = 0.0;
  for (size_t i = 1; i < n; ++i) ranks[idx[i]] = ranks[idx[i - 1]] + ((double)counts[idx[i - 1]] / total);
  return KS_OK;
}

namespace {

// R mean() of two doubles: long double sum, divide, one correction pass
// (summary.c real_mean).
double r_mean2(double a, double b) {
  long double s = (long double)a + (long double)b;
  s /= 2;
  long double t = ((long double)a - s) + ((long double)b - s);
  s += t / 2;
  return (double)s;
}

// f_med of f = counts / total; returns total via *tot.
double median_freq(const int32_t *counts, size_t n, double *tot) {
  int64_t sum = 0;
  for (size_t i = 0; i < n; ++i) sum += counts[i];
  const double total = (double)sum;
  *tot = total;
  if (sum == 0) return std::nan("");  // f is all NaN -> median NA
  std::vector<int32_t> c(counts, counts + n);
  std::nth_element(c.begin(), c.begin() + n / 2, c.end());
  const int32_t hi = c[n / 2];
  const int32_t lo = *std::max_element(c.begin(), c.begin() + n / 2);
  return r_mean2((double)lo / total, (double)hi / total);
}

}  // namespace

ks_status log2_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  for (size_t i = 0; i < n; ++i) w[i] = std::log2(((double)counts[i] / total) / fmed);
  return KS_OK;
}

ks_status pm1_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  for (size_t i = 0; i < n; ++i) {
    const double f = (double)counts[i] / total;
    w[i] = (std::isnan(f) || std::isnan(fmed)) ? std::nan("") : (f >= fmed ? 1.0 : -1.0);
  }
  return KS_OK;
}

}  // namespace ks
