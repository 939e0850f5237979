// cu_mask_bench.hip -- does the random-line request wall need every CU?
// Random 128-B (and 64-B) lines read by coalesced lane groups (line_bench's
// k_group) on a stream restricted to a fraction of the CUs
// (hipExtStreamCreateWithCUMask), alone and next to an LDS-atomic-bound
// kernel (a 2,048-bucket LDS histogram: the count's k_part shape) on the
// complementary CUs.  Decides whether config 5's count/table of the next
// genome can run beside the current genome's pass 1 on disjoint CUs.
// Also: the same line reads from an L2-sized (2 MiB) table.
// Prints one JSON line per case.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

template <int kPer, int U>
__global__ void __launch_bounds__(256) k_group(const uint4 *__restrict__ tab, uint64_t line_mask, int64_t nlines,
                                               uint32_t *out) {
  uint32_t acc = 0;
  const int g = threadIdx.x % kPer;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x / kPer) * U;
  const int64_t grp = (int64_t)blockIdx.x * (blockDim.x / kPer) + threadIdx.x / kPer;
  for (int64_t p = grp * U; p < nlines; p += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[(mix(p + u) & line_mask) * kPer + g];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].w;
  }
  if (acc == 0x12345u) out[0] = acc;
}

// LDS histogram of 2,048 buckets over hashed items (no memory traffic): the
// count passes' LDS-atomic shape
__global__ void __launch_bounds__(1024) k_ldshist(int64_t n, uint32_t *out) {
  __shared__ uint32_t h[2048];
  for (int i = threadIdx.x; i < 2048; i += 1024) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) {
    const uint64_t x = mix(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(&h[(x >> (11 * j)) & 2047], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 1024)
    if (h[i] == 0x7fffffffu) out[1] = h[i];
}

static int g_ncu = 256;

// mask of `take` CUs of every 8 consecutive logical CUs (kind 0) or the first
// frac of the CUs (kind 1); inv: the complement
static std::vector<uint32_t> make_mask(double frac, int kind, bool inv) {
  std::vector<uint32_t> m((g_ncu + 31) / 32, 0);
  const int take8 = (int)(frac * 8 + 0.5);
  const int takeN = (int)(frac * g_ncu + 0.5);
  for (int c = 0; c < g_ncu; ++c) {
    bool on = kind == 0 ? (c % 8) < take8 : c < takeN;
    if (inv) on = !on;
    if (on) m[c / 32] |= 1u << (c % 32);
  }
  return m;
}

int main(int argc, char **argv) {
  const size_t mib = (size_t)1 << 20;
  const size_t big = (argc > 1 ? (size_t)atoll(argv[1]) : 16384) * mib;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  g_ncu = prop.multiProcessorCount;
  printf("# CUs %d\n", g_ncu);
  void *tab = nullptr;
  if (hipExtMallocWithFlags(&tab, big, hipDeviceMallocContiguous) != hipSuccess) {
    (void)hipGetLastError();
    CK(hipMalloc(&tab, big));
  }
  CK(hipMemsetD32Async((hipDeviceptr_t)tab, 0x01010101, big / 4, nullptr));
  uint32_t *out;
  CK(hipMalloc(&out, 64));
  CK(hipDeviceSynchronize());
  const int64_t nl = (int64_t)1 << 30;  // line reads per launch
  const int64_t nh = (int64_t)1 << 31;  // hashed items per histogram launch (x4 atomics)
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1)); CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1));
  auto lines = [&](hipStream_t s, size_t bytes, int per) {
    if (per == 8)
      hipLaunchKernelGGL((k_group<8, 8>), dim3(8192), dim3(256), 0, s, (const uint4 *)tab, bytes / 128 - 1, nl, out);
    else
      hipLaunchKernelGGL((k_group<4, 8>), dim3(8192), dim3(256), 0, s, (const uint4 *)tab, bytes / 64 - 1, nl, out);
  };
  auto hist = [&](hipStream_t s) { hipLaunchKernelGGL(k_ldshist, dim3(2048), dim3(1024), 0, s, nh, out); };
  // L2-sized and big tables on the whole chip
  for (size_t bytes : {(size_t)2 * mib, (size_t)64 * mib, big}) {
    for (int per : {8, 4}) {
      lines(0, bytes, per);
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(a0, 0)); lines(0, bytes, per); CK(hipEventRecord(a1, 0)); CK(hipEventSynchronize(a1));
        float ms; CK(hipEventElapsedTime(&ms, a0, a1)); if (ms < best) best = ms;
      }
      printf("{\"case\":\"lines_all_cus\",\"table_MiB\":%zu,\"line_B\":%d,\"G_lines_per_s\":%.2f}\n", bytes / mib,
             16 * per, nl / (best * 1e6));
    }
  }
  {
    hist(0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a0, 0)); hist(0); CK(hipEventRecord(a1, 0)); CK(hipEventSynchronize(a1));
    float ms; CK(hipEventElapsedTime(&ms, a0, a1));
    printf("{\"case\":\"ldshist_all_cus\",\"G_atomics_per_s\":%.1f,\"ms\":%.3f}\n", 4.0 * nh / (ms * 1e6), ms);
  }
  for (int kind : {0, 1}) {
    for (double f : {0.75, 0.625, 0.5, 0.375, 0.25}) {
      auto mA = make_mask(f, kind, false), mB = make_mask(f, kind, true);
      hipStream_t sA, sB;
      CK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)mA.size(), mA.data()));
      CK(hipExtStreamCreateWithCUMask(&sB, (uint32_t)mB.size(), mB.data()));
      lines(sA, big, 8); hist(sB);
      CK(hipDeviceSynchronize());
      // alone
      CK(hipEventRecord(a0, sA)); lines(sA, big, 8); CK(hipEventRecord(a1, sA)); CK(hipEventSynchronize(a1));
      float la; CK(hipEventElapsedTime(&la, a0, a1));
      CK(hipEventRecord(b0, sB)); hist(sB); CK(hipEventRecord(b1, sB)); CK(hipEventSynchronize(b1));
      float ha; CK(hipEventElapsedTime(&ha, b0, b1));
      // together
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a0, sA)); CK(hipEventRecord(b0, sB));
      lines(sA, big, 8); hist(sB);
      CK(hipEventRecord(a1, sA)); CK(hipEventRecord(b1, sB));
      CK(hipDeviceSynchronize());
      float lt, ht; CK(hipEventElapsedTime(&lt, a0, a1)); CK(hipEventElapsedTime(&ht, b0, b1));
      printf("{\"case\":\"masked\",\"kind\":\"%s\",\"lines_cu_frac\":%.3f,\"lines_alone_G_per_s\":%.2f,"
             "\"hist_alone_G_per_s\":%.1f,\"lines_together_G_per_s\":%.2f,\"hist_together_G_per_s\":%.1f}\n",
             kind == 0 ? "interleaved" : "contiguous", f, nl / (la * 1e6), 4.0 * nh / (ha * 1e6), nl / (lt * 1e6),
             4.0 * nh / (ht * 1e6));
      fflush(stdout);
      CK(hipStreamDestroy(sA)); CK(hipStreamDestroy(sB));
    }
  }
  return 0;
}
