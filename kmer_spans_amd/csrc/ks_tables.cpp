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
    std::vector<int32_t> dv;
    std::vector<int64_t> dm;
    uint64_t pos = 0;
    for (uint64_t v = 0; v < span; ++v) {
      uint64_t hv = 0;
      for (int t = 0; t < nt; ++t) hv += th[t][v];
      start[v] = pos;
      if (!hv) continue;
      dv.push_back((int32_t)((int64_t)cmin + (int64_t)v));
      dm.push_back((int64_t)hv);
      pos += hv;
    }
    const std::vector<RankPiece> pcs = rank_pieces(dv.data(), dm.data(), (int64_t)dv.size(), total);
    if (!pcs.empty()) {  // closed-form pieces, positions filled in parallel
      parallel_for(n, [&](size_t a, size_t b) {
        size_t q = (size_t)(std::upper_bound(pcs.begin(), pcs.end(), (int64_t)a,
                                             [](int64_t j, const RankPiece &p) { return j < p.j0; }) -
                            pcs.begin()) - 1;
        for (size_t j = a; j < b; ++j) {
          while (q + 1 < pcs.size() && pcs[q + 1].j0 <= (int64_t)j) ++q;
          rs[j] = rank_piece_value(pcs[q], (int64_t)j);
        }
      });
    } else {  // negative (wrapped) counts: the sequential prefix
      double r = 0.0, d_prev = 0.0;
      size_t j = 0;
      for (size_t v = 0; v < dv.size(); ++v) {
        const double d = (double)dv[v] / total;
        for (int64_t t = 0; t < dm[v]; ++t) {
          if (j == 0) r = 0.0;  // r[idx[0]] = 0 (quirk Q3)
          else r = r + d_prev;
          rs[j++] = r;
          d_prev = d;
        }
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

std::vector<RankPiece> rank_pieces(const int32_t *vals, const int64_t *mult, int64_t nu, double total) {
  std::vector<RankPiece> P;
  for (int64_t v = 0; v < nu; ++v)
    if (vals[v] < 0) return P;
  auto bits = [](double x) { int64_t i; memcpy(&i, &x, 8); return i; };
  const int64_t M52 = (int64_t)1 << 52, M53 = (int64_t)1 << 53;
  int64_t j = 0;
  double R = 0.0;  // R_0 = 0: r[idx[0]] of the zeroed allocation (quirk Q3)
  for (int64_t v = 0; v < nu; ++v) {
    const double d = (double)vals[v] / total;
    int64_t rem = mult[v];
    while (rem > 0) {
      const double R1 = R + d;
      if (bits(R1) == bits(R)) {  // R absorbs d (d = 0, NaN R, ...): constant to the end of the run
        P.push_back({j, R, 0, 0, 0, 0});
        j += rem;
        break;
      }
      bool closed = false;
      if (std::isnormal(R) && R > 0 && std::isfinite(d) && d > 0) {
        const int e = std::ilogb(R);
        const int64_t m = (bits(R) & (M52 - 1)) | M52;
        const double y = std::ldexp(d, 52 - e);  // exact
        if (y < 2251799813685248.0) {            // 2^51
          const double q = std::floor(y), f = y - q;
          const int64_t qi = (int64_t)q;
          int64_t inc1, inc;
          if (f > 0.5) inc1 = inc = qi + 1;
          else if (f < 0.5) inc1 = inc = qi;
          else {  // exact half: the first step rounds to an even m, every later step adds the even increment
            inc1 = ((m + qi) & 1) ? qi + 1 : qi;
            inc = (qi & 1) ? qi + 1 : qi;
          }
          const int64_t m1 = m + inc1;
          if (m1 <= M53 - 1) {
            const int64_t T = inc > 0 ? 1 + (M53 - 1 - m1) / inc : INT64_MAX;  // steps inside the binade
            P.push_back({j, R, inc1, inc, e, 1});
            if (T >= rem) {
              const int64_t mt = m + inc1 + (rem - 1) * inc;
              int64_t b = ((int64_t)(e + 1023) << 52) | (mt - M52);
              memcpy(&R, &b, 8);
              j += rem;
              rem = 0;
            } else {  // T + 1 positions in this binade, then the crossing step in FP64
              const int64_t mt = m + inc1 + (T - 1) * inc;
              int64_t b = ((int64_t)(e + 1023) << 52) | (mt - M52);
              double Rt;
              memcpy(&Rt, &b, 8);
              R = Rt + d;
              j += T + 1;
              rem -= T + 1;
            }
            closed = true;
          }
        }
      }
      if (!closed) {  // one position, one FP64 step
        P.push_back({j, R, 0, 0, 0, 0});
        R = R1;
        j += 1;
        rem -= 1;
      }
    }
  }
  return P;
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

// The per-count scores of README.md:27-42 (f = c / total, f_med = R median).
static double log2_score(int32_t c, double total, double fmed) { return std::log2(((double)c / total) / fmed); }
static double pm1_score(int32_t c, double total, double fmed) {
  const double f = (double)c / total;
  return (std::isnan(f) || std::isnan(fmed)) ? std::nan("") : (f >= fmed ? 1.0 : -1.0);
}

ks_status log2_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  map_counts(counts, n, w, [&](int32_t c) { return log2_score(c, total, fmed); });
  return KS_OK;
}

ks_status pm1_table_host(const int32_t *counts, int k, double *w) {
  const size_t n = (size_t)1 << (2 * k);
  double total = 0;
  const double fmed = median_freq(counts, n, &total);
  map_counts(counts, n, w, [&](int32_t c) { return pm1_score(c, total, fmed); });
  return KS_OK;
}

void score_of_counts(int score, const int32_t *vals, const int64_t *mult, int64_t nu, double *w) {
  int64_t sum = 0, n = 0;
  for (int64_t v = 0; v < nu; ++v) {
    sum += (int64_t)vals[v] * mult[v];
    n += mult[v];
  }
  const double total = (double)sum;
  double fmed = std::nan("");  // f all NaN -> median NA
  if (sum != 0 && n >= 2) {
    auto kth = [&](int64_t r) {  // order statistic r (0-based) of the counts
      int64_t acc = 0;
      for (int64_t v = 0; v < nu; ++v) {
        acc += mult[v];
        if (acc > r) return vals[v];
      }
      return vals[nu - 1];
    };
    fmed = r_mean2((double)kth(n / 2 - 1) / total, (double)kth(n / 2) / total);
  }
  for (int64_t v = 0; v < nu; ++v)
    w[v] = score == 1 ? log2_score(vals[v], total, fmed) : pm1_score(vals[v], total, fmed);
}

}  // namespace ks
