// gather_bench2.hip -- rates for the expanded (k+j)-mer table design:
// random gathers of 8/16/32-byte entries from 4-128 GiB tables, and the cost
// of the dependent uint16 -> FP64 LUT lookups (global memory vs LDS).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

template <typename T, int U>
__global__ void k_gw(const T *__restrict__ tab, uint64_t mask, int64_t n, double *out) {
  uint64_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; p < n; p += stride) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix(p + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += reinterpret_cast<const uint32_t *>(&v[u])[0];
  }
  if (acc == 12345) out[0] = (double)acc;
}

// u64 entry = 4 uint16 codes -> 4 FP64 LUT values
template <bool kLds, int U>
__global__ void __launch_bounds__(256) k_lut(const uint64_t *__restrict__ tab, uint64_t mask, const double *__restrict__ lut,
                                             int nlut, int64_t n, double *out) {
  extern __shared__ double slut[];
  if (kLds) {
    for (int i = threadIdx.x; i < nlut; i += blockDim.x) slut[i] = lut[i];
    __syncthreads();
  }
  double acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; p < n; p += stride) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix(p + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = (int)((v[u] >> (16 * t)) & 0xffff) % nlut;
        acc += kLds ? slut[c] : lut[c];
      }
  }
  if (acc == 12345.5) out[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <typename T, int U>
void gw(const char *name, int log2n, int64_t n, int grid) {
  const size_t entries = (size_t)1 << log2n;
  T *tab; CK(hipMalloc(&tab, entries * sizeof(T)));
  CK(hipMemset(tab, 1, entries * sizeof(T)));
  double *out; CK(hipMalloc(&out, 8));
  float ms = time_it([&] { hipLaunchKernelGGL((k_gw<T, U>), dim3(grid), dim3(256), 0, 0, tab, (uint64_t)(entries - 1), n, out); }, 3);
  printf("{\"test\":\"gather_wide\",\"name\":\"%s\",\"entry_B\":%zu,\"table_GiB\":%.2f,\"unroll\":%d,\"grid\":%d,\"Gaccess_per_s\":%.2f,\"GB_per_s_useful\":%.1f}\n",
         name, sizeof(T), entries * sizeof(T) / 1073741824.0, U, grid, n / (ms * 1e6), n * sizeof(T) / (ms * 1e6));
  fflush(stdout);
  CK(hipFree(tab)); CK(hipFree(out));
}

struct B16 { uint4 a; };
struct B32 { uint4 a, b; };

int main(int argc, char **argv) {
  const int64_t n = 1LL << 30;
  if (argc > 1 && argv[1][0] == 'b') {  // "big": 32 / 64 / 128 GiB tables of u64 entries
    gw<uint64_t, 8>("u64_4G_entries", 32, n, 4096);
    gw<uint64_t, 8>("u64_8G_entries", 33, n, 4096);
    gw<uint64_t, 8>("u64_16G_entries", 34, n, 4096);
    gw<uint64_t, 16>("u64_16G_entries", 34, n, 8192);
    return 0;
  }
  gw<uint64_t, 8>("u64_4G_entries", 32, n, 4096);   // 32 GiB
  gw<uint64_t, 16>("u64_4G_entries", 32, n, 4096);
  gw<uint64_t, 8>("u64_1G_entries", 30, n, 4096);   // 8 GiB
  gw<uint64_t, 8>("u64_4G_entries_g16k", 32, n, 16384);
  gw<B16, 8>("16B_1G_entries", 30, n, 4096);        // 16 GiB
  gw<B16, 8>("16B_256M_entries", 28, n, 4096);      // 4 GiB
  gw<B32, 4>("32B_1G_entries", 30, n, 4096);        // 32 GiB
  gw<B32, 8>("32B_256M_entries", 28, n, 4096);      // 8 GiB
  {
    const size_t entries = (size_t)1 << 32;
    uint64_t *tab; CK(hipMalloc(&tab, entries * 8));
    CK(hipMemset(tab, 0x35, entries * 8));
    double *lut; CK(hipMalloc(&lut, 65536 * 8)); CK(hipMemset(lut, 0, 65536 * 8));
    double *out; CK(hipMalloc(&out, 8));
    for (int nlut : {4096, 6752}) {
      float ms1 = time_it([&] { hipLaunchKernelGGL((k_lut<false, 8>), dim3(4096), dim3(256), 0, 0, tab, (uint64_t)(entries - 1), lut, nlut, n, out); }, 3);
      float ms2 = time_it([&] { hipLaunchKernelGGL((k_lut<true, 8>), dim3(4096), dim3(256), nlut * 8, 0, tab, (uint64_t)(entries - 1), lut, nlut, n, out); }, 3);
      printf("{\"test\":\"gather_u64_plus_4_lut\",\"nlut\":%d,\"global_lut_Gpos_per_s\":%.1f,\"lds_lut_Gpos_per_s\":%.1f}\n",
             nlut, 4 * n / (ms1 * 1e6), 4 * n / (ms2 * 1e6));
      fflush(stdout);
    }
  }
  return 0;
}
