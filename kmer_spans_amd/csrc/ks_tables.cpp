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
#include <climits>
#include <cstring>
#include <thread>
#include <vector>

#include "ks_internal.h"

namespace ks {

namespace {

// Worker threads for the embarrassingly parallel loops of the table builds.
int n_workers() {
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
}

template <typename F>
void parallel_for(size_t n, F f) {
  const int nt = n < ((size_t)1 << 16) ? 1 : n_workers();
  if (nt == 1) { f(0, n); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    const size_t a = n * t / nt, b = n * (t + 1) / nt;
    th.emplace_back([=] { f(a, b); });
  }
  for (auto &x : th) x.join();
}

template <typename F>
void parallel_for_t(int nt, F f) {
  if (nt == 1) { f(0); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back([=] { f(t); });
  for (auto &x : th) x.join();
}

}  // namespace


ks_status rank_table_host(const int32_t *counts, int k, double total, double *ranks) {
  const size_t n = (size_t)1 << (2 * k);
  int32_t cmin = INT32_MAX, cmax = INT32_MIN;
  for (size_t i = 0; i < n; ++i) {
    cmin = std::min(cmin, counts[i]);
    cmax = std::max(cmax, counts[i]);
  }
  const uint64_t span = (uint64_t)((int64_t)cmax - (int64_t)cmin) + 1;
  if (span <= ((uint64_t)1 << 22)) {
    // Counting sort without materialising the order: the sorted count
    // sequence comes from the histogram, so the sequential prefix
    // rs[j] = rs[j-1] + c_(j-1) / total (sorted position j) reads nothing
    // at random; element i then takes rs[start[c_i] + #earlier equal counts]
    // (stable order = index ascending).  Threads split the indices and get
    // their starting cursors from per-thread histograms.
    const int nt = n < ((size_t)1 << 20) ? 1 : std::min(n_workers(), (int)std::max<uint64_t>(1, ((uint64_t)1 << 26) / span));
    std::vector<std::vector<uint64_t>> th(nt, std::vector<uint64_t>(span, 0));
    parallel_for_t(nt, [&](int t) {
      const size_t a = n * t / nt, b = n * (t + 1) / nt;
      for (size_t i = a; i < b; ++i) ++th[t][(uint64_t)((int64_t)counts[i] - cmin)];
    });
    std::vector<double> rs(n);
    std::vector<uint64_t> start(span);
    uint64_t pos = 0;
    double r = 0.0, d_prev = 0.0;
    bool first = true;
    for (uint64_t v = 0; v < span; ++v) {
      uint64_t hv = 0;
      for (int t = 0; t < nt; ++t) hv += th[t][v];
      start[v] = pos;
      if (!hv) continue;
      const double d = (double)((int64_t)cmin + (int64_t)v) / total;
      for (uint64_t j = 0; j < hv; ++j) {
        if (first) { r = 0.0; first = false; }  // r[idx[0]] = 0 (quirk Q3)
        else r = r + d_prev;
        rs[pos++] = r;
        d_prev = d;
      }
    }
    // per-thread cursors: start[v] + elements with count v in earlier threads
    std::vector<std::vector<uint64_t>> cur(nt, std::vector<uint64_t>(span));
    for (uint64_t v = 0; v < span; ++v) {
      uint64_t c = start[v];
      for (int t = 0; t < nt; ++t) { cur[t][v] = c; c += th[t][v]; }
    }
    parallel_for_t(nt, [&](int t) {
      const size_t a = n * t / nt, b = n * (t + 1) / nt;
      std::vector<uint64_t> &cu = cur[t];
      for (size_t i = a; i < b; ++i) ranks[i] = rs[cu[(uint64_t)((int64_t)counts[i] - cmin)]++];
    });
    return KS_OK;
  }
  // wide count range: stable LSD radix sort over the signed count bits
  std::vector<uint32_t> idx(n), tmp(n);
  for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
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

// f_med of f = counts / total; returns total via *tot.  The two middle
// order statistics of the counts come from a count histogram when the count
// range is small (else nth_element).
double median_freq(const int32_t *counts, size_t n, double *tot) {
  int64_t sum = 0;
  int32_t cmin = INT32_MAX, cmax = INT32_MIN;
  for (size_t i = 0; i < n; ++i) {
    sum += counts[i];
    cmin = std::min(cmin, counts[i]);
    cmax = std::max(cmax, counts[i]);
  }
  const double total = (double)sum;
  *tot = total;
  if (sum == 0) return std::nan("");  // f is all NaN -> median NA
  int32_t lo, hi;  // order statistics n/2 - 1 and n/2
  const uint64_t span = (uint64_t)((int64_t)cmax - (int64_t)cmin) + 1;
  if (span <= ((uint64_t)1 << 26)) {
    std::vector<uint64_t> h(span, 0);
    for (size_t i = 0; i < n; ++i) ++h[(uint64_t)((int64_t)counts[i] - cmin)];
    auto kth = [&](uint64_t r) {  // value of order statistic r (0-based)
      uint64_t acc = 0;
      for (uint64_t v = 0; v < span; ++v) {
        acc += h[v];
        if (acc > r) return (int32_t)((int64_t)cmin + (int64_t)v);
      }
      return cmax;
    };
    lo = kth(n / 2 - 1);
    hi = kth(n / 2);
  } else {
    std::vector<int32_t> c(counts, counts + n);
    std::nth_element(c.begin(), c.begin() + n / 2, c.end());
    hi = c[n / 2];
    lo = *std::max_element(c.begin(), c.begin() + n / 2);
  }
  return r_mean2((double)lo / total, (double)hi / total);
}

// w[i] = g(counts[i]) for a per-count function g, evaluated once per distinct
// count when the count range is small.
template <typename G>
void map_counts(const int32_t *counts, size_t n, double *w, G g) {
  int32_t cmin = INT32_MAX, cmax = INT32_MIN;
  for (size_t i = 0; i < n; ++i) {
    cmin = std::min(cmin, counts[i]);
    cmax = std::max(cmax, counts[i]);
  }
  const uint64_t span = (uint64_t)((int64_t)cmax - (int64_t)cmin) + 1;
  if (span <= ((uint64_t)1 << 24)) {
    std::vector<uint8_t> seen(span, 0);
    for (size_t i = 0; i < n; ++i) seen[(uint64_t)((int64_t)counts[i] - cmin)] = 1;
    std::vector<double> lut(span, 0.0);
    for (uint64_t v = 0; v < span; ++v)
      if (seen[v]) lut[v] = g((int32_t)((int64_t)cmin + (int64_t)v));
    parallel_for(n, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; ++i) w[i] = lut[(uint64_t)((int64_t)counts[i] - cmin)];
    });
  } else {
    parallel_for(n, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; ++i) w[i] = g(counts[i]);
    });
  }
}

}  // namespace

ks_status log2_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  map_counts(counts, n, w, [&](int32_t c) { return std::log2(((double)c / total) / fmed); });
  return KS_OK;
}

ks_status pm1_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  map_counts(counts, n, w, [&](int32_t c) {
    const double f = (double)c / total;
    return (std::isnan(f) || std::isnan(fmed)) ? std::nan("") : (f >= fmed ? 1.0 : -1.0);
  });
  return KS_OK;
}

}  // namespace ks
