// ks_table.hip -- device score tables.
//
// s[code] = w[code] - thr is formed on the device with the very FP64
// subtraction the reference performs per base (kmer_spans.c:268), once per
// table instead of once per base.  If the table has <= 65536 distinct values
// (bitwise), it is re-expressed exactly as a uint16 code table + FP64 LUT:
// log2(f/f_med) and +-1 tables depend only on the k-mer count, so at k=13 the
// 512 MiB FP64 table becomes a 128 MiB code table that stays resident in the
// 256 MiB Infinity Cache while the sequence streams past.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "ks_internal.h"

namespace ks {
namespace {

__global__ void k_sub_thr(const double *__restrict__ w, double thr, double *__restrict__ s,
                          unsigned long long *__restrict__ bits, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = w[i] - thr;
    s[i] = v;
    if (bits) bits[i] = (unsigned long long)__double_as_longlong(v);
  }
}

// max |s| over the finite values (as the bits of a non-negative double) and
// a flag for NaN or +Inf (-Inf only ever clamps to 0).
__global__ void k_absmax(const double *__restrict__ s, int64_t n, unsigned long long *__restrict__ out) {
  unsigned long long m = 0, bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = s[i];
    if (isfinite(v)) m = max(m, (unsigned long long)__double_as_longlong(fabs(v)));
    else if (!(v < 0)) bad = 1;  // NaN or +Inf
  }
  for (int d = 32; d >= 1; d >>= 1) {
    m = max(m, (unsigned long long)__shfl_down(m, d, 64));
    bad |= __shfl_down(bad, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], m);
    if (bad) atomicOr(&out[1], 1ull);
  }
}

__global__ void k_assign_codes(const double *__restrict__ s, const unsigned long long *__restrict__ uniq,
                               int64_t nu, uint16_t *__restrict__ codes, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = (unsigned long long)__double_as_longlong(s[i]);
    int64_t lo = 0, hi = nu - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (uniq[mid] < key) lo = mid + 1; else hi = mid;
    }
    codes[i] = (uint16_t)lo;
  }
}

// Expanded table, uint16 codes: entry for the (k+J-1)-mer x packs the codes of
// its J k-mers (first k-mer in the low 16 bits).  Consecutive entries share
// their k-mers, so the base-table reads are cached and the build is a stream.
template <int J, typename E>
__global__ void k_build_ext_u16(const uint16_t *__restrict__ codes, int k, uint64_t nent, E *__restrict__ ext) {
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nent;
       e += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v = 0;
#pragma unroll
    for (int t = 0; t < J; ++t) v |= (uint64_t)codes[(e >> (2 * (J - 1 - t))) & mk] << (16 * t);
    ext[e] = (E)v;
  }
}

// Position weight of every uint16 code: number of k-mers with that code, or
// (with a frequency hint) the number of positions scoring them.
__global__ void k_code_hist(const uint16_t *__restrict__ codes, const int32_t *__restrict__ freq, int64_t n,
                            unsigned long long *__restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long wgt = freq ? (unsigned long long)(uint32_t)freq[i] : 1ull;
    if (wgt) atomicAdd(&hist[codes[i]], wgt);
  }
}

// Expanded table, 12-bit codes: J = 5 codes per uint64 entry (rank12 maps a
// uint16 code to its 12-bit code or the escape 0xFFF).
__global__ void k_build_ext_c12(const uint16_t *__restrict__ codes, const uint16_t *__restrict__ rank12, int k,
                                uint64_t nent, uint64_t *__restrict__ ext) {
  constexpr int J = 5;
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nent;
       e += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t v = 0;
#pragma unroll
    for (int t = 0; t < J; ++t) v |= (uint64_t)rank12[codes[(e >> (2 * (J - 1 - t))) & mk]] << (12 * t);
    ext[e] = v;
  }
}

// Expanded table, FP64 values: J values per entry (double2 / double4).
template <int J>
__global__ void k_build_ext_f64(const double *__restrict__ vals, int k, uint64_t nent, double *__restrict__ ext) {
  constexpr int W = (J <= 2) ? 2 : 4;
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nent;
       e += (uint64_t)gridDim.x * blockDim.x) {
    double v[W];
#pragma unroll
    for (int t = 0; t < W; ++t) v[t] = (t < J) ? vals[(e >> (2 * (J - 1 - t))) & mk] : 0.0;
    if (W == 2) {
      reinterpret_cast<double2 *>(ext)[e] = make_double2(v[0], v[1]);
    } else {
      reinterpret_cast<double2 *>(ext)[2 * e] = make_double2(v[0], v[1]);
      reinterpret_cast<double2 *>(ext)[2 * e + 1] = make_double2(v[2], v[3]);
    }
  }
}

}  // namespace

// Entry bytes of an expanded table with J values per entry.
static size_t ext_entry_bytes(bool u16, int J) {
  if (u16) return J <= 2 ? 4 : 8;
  return J <= 2 ? 16 : 32;
}

// 12-bit code assignment for J = 5: the 4095 heaviest uint16 codes (by
// position weight) get codes 0..4094, the rest escape.  Returns false if the
// escape share is above max_escape.
static ks_status assign_code12(ks_ctx *ctx, ks_table *t, const int32_t *freq_dev, double max_escape, bool *use) {
  *use = false;
  hipStream_t st = ctx->stream;
  const int64_t n = (int64_t)1 << (2 * t->k);
  const int64_t nu = t->distinct;
  unsigned long long *d_hist = nullptr;
  KS_HIP(hipMalloc(&d_hist, 65536 * 8));
  KS_HIP(hipMemsetAsync(d_hist, 0, 65536 * 8, st));
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cus * 16);
  hipLaunchKernelGGL(k_code_hist, dim3(grid), dim3(256), 0, st, t->d_codes, freq_dev, n, d_hist);
  std::vector<unsigned long long> h(65536);
  std::vector<double> lut(nu);
  KS_HIP(hipMemcpyAsync(h.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(lut.data(), t->d_lut, nu * 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  KS_HIP(hipFree(d_hist));
  std::vector<int32_t> order(nu);
  for (int64_t i = 0; i < nu; ++i) order[i] = (int32_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return h[a] > h[b]; });
  const int64_t ndirect = std::min<int64_t>(nu, 4095);
  long double tot = 0, cov = 0;
  for (int64_t i = 0; i < nu; ++i) tot += h[order[i]];
  for (int64_t i = 0; i < ndirect; ++i) cov += h[order[i]];
  t->escape_frac = tot > 0 ? (double)(1.0L - cov / tot) : 0.0;
  if (t->escape_frac > max_escape) return KS_OK;
  std::vector<uint16_t> rank12(65536, 0xFFF), map12(4096, 0);
  std::vector<double> lut12(4096, 0.0);
  for (int64_t i = 0; i < ndirect; ++i) {
    rank12[order[i]] = (uint16_t)i;
    map12[i] = (uint16_t)order[i];
    lut12[i] = lut[order[i]];
  }
  KS_HIP(hipMalloc(&t->d_map12, 4096 * 2));
  KS_HIP(hipMalloc(&t->d_lut12, 4096 * 8));
  KS_HIP(hipMemcpyAsync(t->d_map12, map12.data(), 4096 * 2, hipMemcpyHostToDevice, st));
  KS_HIP(hipMemcpyAsync(t->d_lut12, lut12.data(), 4096 * 8, hipMemcpyHostToDevice, st));
  uint16_t *d_rank = nullptr;
  KS_HIP(hipMalloc(&d_rank, 65536 * 2));
  KS_HIP(hipMemcpyAsync(d_rank, rank12.data(), 65536 * 2, hipMemcpyHostToDevice, st));
  KS_HIP(hipStreamSynchronize(st));
  t->d_rank12_tmp = d_rank;
  *use = true;
  return KS_OK;
}

ks_status table_expand(ks_ctx *ctx, ks_table *t, size_t max_bytes, const int32_t *freq_dev) {
  if (t->d_ext || t->ext_J > 1) return KS_OK;
  const bool u16 = t->compressed;
  size_t free_b = 0, total_b = 0;
  KS_HIP(hipMemGetInfo(&free_b, &total_b));
  // leave room for the sequences and the scan workspace
  const size_t reserve = std::max<size_t>((size_t)32 << 30, total_b / 4);
  const size_t budget = std::min(max_bytes, free_b > reserve ? free_b - reserve : (size_t)0);
  // candidates, best first: (J, code bits); (k+J-1)-mer indices up to 34 bits
  struct Cand { int J, bits; };
  const Cand cands_u16[] = {{5, 12}, {4, 16}, {3, 16}, {2, 16}};
  const Cand cands_f64[] = {{4, 64}, {3, 64}, {2, 64}};
  const Cand *cands = u16 ? cands_u16 : cands_f64;
  const int ncand = u16 ? 4 : 3;
  const char *jmax_env = getenv("KS_EXT_MAX_J");  // tests: cap J to exercise every table form
  const int jmax = jmax_env ? atoi(jmax_env) : 5;
  const char *esc_env = getenv("KS_EXT_ESCAPE_MAX");
  const double max_escape = esc_env ? atof(esc_env) : 0.01;
  int J = 0, bits = 16;
  for (int i = 0; i < ncand; ++i) {
    const Cand c = cands[i];
    if (c.J > jmax) continue;
    const int kx = t->k + c.J - 1;
    if (kx > 17) continue;
    if (!u16 && kx > 16) continue;
    const size_t bytes = ((size_t)1 << (2 * kx)) * ext_entry_bytes(u16, c.J);
    if (bytes > budget) continue;
    if (c.bits == 12) {
      if (getenv("KS_NO_CODE12")) continue;
      bool use = false;
      KS_TRY(assign_code12(ctx, t, freq_dev, max_escape, &use));
      if (!use) continue;
    }
    J = c.J;
    bits = c.bits;
    break;
  }
  if (J == 0) return KS_OK;
  const int kx = t->k + J - 1;
  const uint64_t nent = (uint64_t)1 << (2 * kx);
  const size_t bytes = nent * ext_entry_bytes(u16, J);
  hipStream_t st = ctx->stream;
  void *ext = nullptr;
  if (hipMalloc(&ext, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return KS_OK;
  }
  hipEvent_t a, b;
  KS_HIP(hipEventCreate(&a));
  KS_HIP(hipEventCreate(&b));
  KS_HIP(hipEventRecord(a, st));
  const unsigned grid = (unsigned)std::min<uint64_t>((nent + 255) / 256, (uint64_t)ctx->num_cus * 32);
  if (u16 && bits == 12) {
    hipLaunchKernelGGL(k_build_ext_c12, dim3(grid), dim3(256), 0, st, t->d_codes, t->d_rank12_tmp, t->k, nent,
                       (uint64_t *)ext);
  } else if (u16) {
    if (J == 4) hipLaunchKernelGGL((k_build_ext_u16<4, uint64_t>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint64_t *)ext);
    else if (J == 3) hipLaunchKernelGGL((k_build_ext_u16<3, uint64_t>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint64_t *)ext);
    else hipLaunchKernelGGL((k_build_ext_u16<2, uint32_t>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint32_t *)ext);
  } else {
    if (J == 4) hipLaunchKernelGGL(k_build_ext_f64<4>, dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
    else if (J == 3) hipLaunchKernelGGL(k_build_ext_f64<3>, dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
    else hipLaunchKernelGGL(k_build_ext_f64<2>, dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
  }
  KS_HIP(hipGetLastError());
  KS_HIP(hipEventRecord(b, st));
  KS_HIP(hipEventSynchronize(b));
  float ms = 0;
  KS_HIP(hipEventElapsedTime(&ms, a, b));
  KS_HIP(hipEventDestroy(a));
  KS_HIP(hipEventDestroy(b));
  if (t->d_rank12_tmp) {
    KS_HIP(hipFree(t->d_rank12_tmp));
    t->d_rank12_tmp = nullptr;
  }
  if (bits != 12) {  // a 12-bit assignment that was not used
    if (t->d_map12) (void)hipFree(t->d_map12);
    if (t->d_lut12) (void)hipFree(t->d_lut12);
    t->d_map12 = nullptr;
    t->d_lut12 = nullptr;
  }
  t->d_ext = ext;
  t->ext_J = J;
  t->ext_bits = bits;
  t->ext_bytes = bytes;
  t->ms_ext = ms;
  return KS_OK;
}

}  // namespace ks

using namespace ks;

extern "C" ks_status ks_table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                     int32_t flags, ks_table **out) {
  return ks_table_create_hint(ctx, w_host, k, thr, flags, nullptr, out);
}

extern "C" ks_status ks_table_create_hint(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                          int32_t flags, const int32_t *freq_dev, ks_table **out) {
  const int32_t allow_compress = flags & KS_TABLE_COMPRESS;
  if (!ctx || !w_host || !out) return fail(KS_ERR_ARG, "ks_table_create: null argument");
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  KS_TRY(activate(ctx));
  const int64_t n = (int64_t)1 << (2 * k);
  hipStream_t st = ctx->stream;
  ks_table *t = new ks_table();
  t->ctx = ctx;
  t->k = k;
  t->thr = thr;
  double *d_w = nullptr;
  unsigned long long *d_bits = nullptr, *d_sorted = nullptr;
  void *d_tmp = nullptr;
  int64_t *d_nu = nullptr;
  auto cleanup = [&]() {
    if (d_w) (void)hipFree(d_w);
    if (d_bits) (void)hipFree(d_bits);
    if (d_sorted) (void)hipFree(d_sorted);
    if (d_tmp) (void)hipFree(d_tmp);
    if (d_nu) (void)hipFree(d_nu);
  };
#define KS_TBL_HIP(call)                                                               \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      cleanup();                                                                       \
      ks_table_destroy(t);                                                             \
      return fail(KS_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_));      \
    }                                                                                  \
  } while (0)
  KS_TBL_HIP(hipMalloc(&d_w, n * sizeof(double)));
  KS_TBL_HIP(hipMalloc(&t->d_vals, n * sizeof(double)));
  if (allow_compress) KS_TBL_HIP(hipMalloc(&d_bits, n * sizeof(unsigned long long)));
  KS_TBL_HIP(hipMemcpyAsync(d_w, w_host, n * sizeof(double), hipMemcpyHostToDevice, st));
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_sub_thr, dim3(grid), dim3(256), 0, st, d_w, thr, t->d_vals, d_bits, n);
  KS_TBL_HIP(hipGetLastError());
  {  // finiteness and magnitude (tr_lr decides between the chunked and the literal path)
    unsigned long long *d_am = nullptr, h_am[2] = {0, 0};
    KS_TBL_HIP(hipMalloc(&d_am, 16));
    KS_TBL_HIP(hipMemsetAsync(d_am, 0, 16, st));
    hipLaunchKernelGGL(k_absmax, dim3(grid), dim3(256), 0, st, t->d_vals, n, d_am);
    KS_TBL_HIP(hipMemcpyAsync(h_am, d_am, 16, hipMemcpyDeviceToHost, st));
    KS_TBL_HIP(hipStreamSynchronize(st));
    KS_TBL_HIP(hipFree(d_am));
    t->no_nan_posinf = h_am[1] == 0;
    double ma = 0;
    memcpy(&ma, &h_am[0], 8);
    t->max_abs = ma;
  }
  t->distinct = -1;
  if (allow_compress) {
    KS_TBL_HIP(hipMalloc(&d_sorted, n * sizeof(unsigned long long)));
    KS_TBL_HIP(hipMalloc(&d_nu, sizeof(int64_t)));
    size_t b1 = 0, b2 = 0;
    KS_TBL_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, d_bits, d_sorted, (int)n, 0, 64, st));
    KS_TBL_HIP(hipcub::DeviceSelect::Unique(nullptr, b2, d_sorted, d_bits, d_nu, (int)n, st));
    KS_TBL_HIP(hipMalloc(&d_tmp, std::max(b1, b2)));
    KS_TBL_HIP(hipcub::DeviceRadixSort::SortKeys(d_tmp, b1, d_bits, d_sorted, (int)n, 0, 64, st));
    KS_TBL_HIP(hipcub::DeviceSelect::Unique(d_tmp, b2, d_sorted, d_bits, d_nu, (int)n, st));
    int64_t nu = 0;
    KS_TBL_HIP(hipMemcpyAsync(&nu, d_nu, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    KS_TBL_HIP(hipStreamSynchronize(st));
    t->distinct = nu;
    if (nu >= 1 && nu <= 65536) {
      KS_TBL_HIP(hipMalloc(&t->d_codes, n * sizeof(uint16_t)));
      KS_TBL_HIP(hipMalloc(&t->d_lut, nu * sizeof(double)));
      KS_TBL_HIP(hipMemcpyAsync(t->d_lut, d_bits, nu * sizeof(double), hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(k_assign_codes, dim3(grid), dim3(256), 0, st, t->d_vals, d_bits, nu,
                         t->d_codes, n);
      KS_TBL_HIP(hipGetLastError());
      KS_TBL_HIP(hipStreamSynchronize(st));
      t->compressed = true;
      (void)hipFree(t->d_vals);
      t->d_vals = nullptr;
    }
  }
  KS_TBL_HIP(hipStreamSynchronize(st));
#undef KS_TBL_HIP
  cleanup();
  if (flags & KS_TABLE_EXPAND) {
    const ks_status rc = table_expand(ctx, t, (size_t)160 << 30, freq_dev);
    if (rc != KS_OK) { ks_table_destroy(t); return rc; }
  }
  *out = t;
  return KS_OK;
}

extern "C" void ks_table_destroy(ks_table *t) {
  if (!t) return;
  if (t->d_vals) (void)hipFree(t->d_vals);
  if (t->d_codes) (void)hipFree(t->d_codes);
  if (t->d_lut) (void)hipFree(t->d_lut);
  if (t->d_ext) (void)hipFree(t->d_ext);
  if (t->d_map12) (void)hipFree(t->d_map12);
  if (t->d_lut12) (void)hipFree(t->d_lut12);
  if (t->d_rank12_tmp) (void)hipFree(t->d_rank12_tmp);
  delete t;
}

extern "C" int32_t ks_table_is_compressed(const ks_table *t) { return t && t->compressed ? 1 : 0; }
extern "C" int64_t ks_table_distinct(const ks_table *t) { return t ? t->distinct : -1; }
extern "C" int32_t ks_table_positions_per_read(const ks_table *t) { return t ? t->ext_J : 0; }
extern "C" int32_t ks_table_code_bits(const ks_table *t) {
  if (!t) return 0;
  if (t->ext_J > 1 && t->compressed) return t->ext_bits;
  return t->compressed ? 16 : 64;
}
extern "C" double ks_table_escape_fraction(const ks_table *t) {
  return (t && t->ext_bits == 12) ? t->escape_frac : 0.0;
}
