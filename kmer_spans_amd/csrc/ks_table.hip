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

}  // namespace
}  // namespace ks

using namespace ks;

extern "C" ks_status ks_table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                     int32_t allow_compress, ks_table **out) {
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
  *out = t;
  return KS_OK;
}

extern "C" void ks_table_destroy(ks_table *t) {
  if (!t) return;
  if (t->d_vals) (void)hipFree(t->d_vals);
  if (t->d_codes) (void)hipFree(t->d_codes);
  if (t->d_lut) (void)hipFree(t->d_lut);
  delete t;
}

extern "C" int32_t ks_table_is_compressed(const ks_table *t) { return t && t->compressed ? 1 : 0; }
extern "C" int64_t ks_table_distinct(const ks_table *t) { return t ? t->distinct : -1; }
