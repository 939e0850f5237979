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

ks_status table_expand(ks_ctx *ctx, ks_table *t, size_t max_bytes) {
  if (t->d_ext || t->ext_J > 1) return KS_OK;
  const bool u16 = t->compressed;
  int J = 0;
  for (int cand = 4; cand >= 2; --cand) {
    const int kx = t->k + cand - 1;
    if (kx > 16) continue;  // (k+J-1)-mer codes are 32-bit
    const size_t bytes = ((size_t)1 << (2 * kx)) * ext_entry_bytes(u16, cand);
    if (bytes <= max_bytes) { J = cand; break; }
  }
  if (J == 0) return KS_OK;
  const int kx = t->k + J - 1;
  const uint64_t nent = (uint64_t)1 << (2 * kx);
  const size_t bytes = nent * ext_entry_bytes(u16, J);
  size_t free_b = 0, total_b = 0;
  KS_HIP(hipMemGetInfo(&free_b, &total_b));
  if (bytes > free_b / 10 * 4) return KS_OK;  // leave room for the scan workspace
  hipStream_t st = ctx->stream;
  void *ext = nullptr;
  if (hipMalloc(&ext, bytes) != hipSuccess) { (void)hipGetLastError(); return KS_OK; }
  hipEvent_t a, b;
  KS_HIP(hipEventCreate(&a));
  KS_HIP(hipEventCreate(&b));
  KS_HIP(hipEventRecord(a, st));
  const unsigned grid = (unsigned)std::min<uint64_t>((nent + 255) / 256, (uint64_t)ctx->num_cus * 32);
  if (u16) {
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
  t->d_ext = ext;
  t->ext_J = J;
  t->ext_bytes = bytes;
  t->ms_ext = ms;
  return KS_OK;
}

}  // namespace ks

using namespace ks;

extern "C" ks_status ks_table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                     int32_t flags, ks_table **out) {
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
    const ks_status rc = table_expand(ctx, t, (size_t)32 << 30);
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
  delete t;
}

extern "C" int32_t ks_table_is_compressed(const ks_table *t) { return t && t->compressed ? 1 : 0; }
extern "C" int64_t ks_table_distinct(const ks_table *t) { return t ? t->distinct : -1; }
extern "C" int32_t ks_table_positions_per_read(const ks_table *t) { return t ? t->ext_J : 0; }
