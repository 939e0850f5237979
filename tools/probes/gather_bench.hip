// gather_bench.hip -- measures the random-access rates that bound the span
// scan on MI355X: random gathers from tables of the sizes the score tables
// take (k=13: FP64 512 MiB, uint16 codes 128 MiB; k=11: FP64 32 MiB), random
// uint32 atomics into count histograms, and the sequential byte stream.
// Prints one JSON object per measurement.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}

template <typename T, int U>
__global__ void k_gather(const T *__restrict__ tab, uint32_t mask, int64_t n, double *out) {
  double acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; p < n; p += stride) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix(p + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (double)v[u];
  }
  if (acc == 12345.678) out[0] = acc;
}

// sequential-code pattern: each thread walks a contiguous chunk, rolling a
// k-mer code over pseudo-random bases (the scan's real address stream)
template <typename T, int U>
__global__ void k_gather_roll(const T *__restrict__ tab, int k, int64_t n, int64_t chunk, double *out) {
  const uint32_t mask = (1u << (2 * k)) - 1;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p0 = t * chunk;
  if (p0 >= n) return;
  uint32_t code = mix(p0) & mask;
  double acc = 0;
  for (int64_t p = p0; p < p0 + chunk; p += U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      code = ((code << 2) | (mix(p + u) & 3)) & mask;
      v[u] = tab[code];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (double)v[u];
  }
  if (acc == 12345.678) out[0] = acc;
}

__global__ void k_atomic(uint32_t *__restrict__ tab, uint32_t mask, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride)
    atomicAdd(&tab[mix(p) & mask], 1u);
}

__global__ void k_stream(const uint4 *__restrict__ a, int64_t n16, uint32_t *out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <typename T, int U>
void run_gather(const char *name, int log2n, int64_t n) {
  const size_t entries = (size_t)1 << log2n;
  T *tab;
  CK(hipMalloc(&tab, entries * sizeof(T)));
  CK(hipMemset(tab, 1, entries * sizeof(T)));
  double *out;
  CK(hipMalloc(&out, 8));
  const int grid = 256 * 16;
  float ms = time_it([&] { hipLaunchKernelGGL((k_gather<T, U>), dim3(grid), dim3(256), 0, 0, tab,
                                              (uint32_t)(entries - 1), n, out); }, 3);
  printf("{\"test\":\"gather_hash\",\"name\":\"%s\",\"table_MiB\":%.1f,\"unroll\":%d,\"Gaccess_per_s\":%.2f,\"ms\":%.3f}\n",
         name, entries * sizeof(T) / 1048576.0, U, n / (ms * 1e6), ms);
  // rolled codes, 4^k table (log2n = 2k)
  const int k = log2n / 2;
  for (int64_t chunk : {256, 4096}) {
    const int64_t threads = n / chunk;
    float ms2 = time_it([&] { hipLaunchKernelGGL((k_gather_roll<T, U>), dim3((unsigned)((threads + 255) / 256)),
                                                 dim3(256), 0, 0, tab, k, n, chunk, out); }, 3);
    printf("{\"test\":\"gather_roll\",\"name\":\"%s\",\"k\":%d,\"chunk\":%lld,\"unroll\":%d,\"Gaccess_per_s\":%.2f,\"ms\":%.3f}\n",
           name, k, (long long)chunk, U, n / (ms2 * 1e6), ms2);
  }
  fflush(stdout);
  CK(hipFree(tab));
  CK(hipFree(out));
}

int main() {
  const int64_t n = 1LL << 31;  // 2.1 G accesses
  run_gather<double, 8>("f64_k13", 26, n);
  run_gather<double, 16>("f64_k13", 26, n);
  run_gather<uint16_t, 8>("u16_k13", 26, n);
  run_gather<uint16_t, 16>("u16_k13", 26, n);
  run_gather<uint8_t, 16>("u8_k13", 26, n);
  run_gather<uint32_t, 16>("u32_k13", 26, n);
  run_gather<double, 16>("f64_k11", 22, n);
  run_gather<uint16_t, 16>("u16_k11", 22, n);
  run_gather<double, 16>("f64_k15", 30, n / 2);
  run_gather<uint16_t, 16>("u16_k15", 30, n / 2);
  for (int log2n : {14, 22, 26}) {
    uint32_t *tab;
    const size_t entries = (size_t)1 << log2n;
    CK(hipMalloc(&tab, entries * 4));
    CK(hipMemset(tab, 0, entries * 4));
    const int64_t na = 1LL << 30;
    float ms = time_it([&] { hipLaunchKernelGGL(k_atomic, dim3(256 * 16), dim3(256), 0, 0, tab,
                                                (uint32_t)(entries - 1), na); }, 2);
    printf("{\"test\":\"atomic_u32\",\"table_MiB\":%.2f,\"Gatomic_per_s\":%.2f,\"ms\":%.3f}\n",
           entries * 4 / 1048576.0, na / (ms * 1e6), ms);
    fflush(stdout);
    CK(hipFree(tab));
  }
  {
    const int64_t bytes = 3LL << 30;
    uint4 *a;
    CK(hipMalloc(&a, bytes));
    CK(hipMemset(a, 1, bytes));
    uint32_t *out;
    CK(hipMalloc(&out, 4));
    float ms = time_it([&] { hipLaunchKernelGGL(k_stream, dim3(256 * 8), dim3(256), 0, 0, a, bytes / 16, out); }, 5);
    printf("{\"test\":\"stream_read\",\"GB\":%.2f,\"GB_per_s\":%.1f,\"ms\":%.3f}\n", bytes / 1e9,
           bytes / (ms * 1e6), ms);
    CK(hipFree(a));
  }
  return 0;
}
