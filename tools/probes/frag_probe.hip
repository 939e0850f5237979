// frag_probe.hip -- does the physical placement of the 128 GiB expanded
// table change the random-gather rate?  One allocation strategy per process:
//   fresh     hipMalloc of the table first
//   after     12 GiB of scratch allocated and written first, then the table
//   churn     scratch allocated, freed, then the table
//   contig    hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   vmm N     hipMemCreate chunks of N GiB mapped back to back
// Prints alloc ms and the rate of 16-byte random gathers (G gathers/s).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

__global__ void k_gather(const uint4 *__restrict__ tab, uint64_t mask, int64_t n, uint32_t *out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; p < n; p += stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = tab[mix(p + u) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u].x;
  }
  if (acc == 0x12345u) out[0] = acc;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "fresh";
  const size_t gib = (size_t)1 << 30;
  const size_t bytes = 128 * gib;
  void *scratch = nullptr;
  if (!strcmp(mode, "after") || !strcmp(mode, "churn")) {
    CK(hipMalloc(&scratch, 12 * gib));
    CK(hipMemset(scratch, 1, 12 * gib));
    CK(hipDeviceSynchronize());
    if (!strcmp(mode, "churn")) {
      CK(hipFree(scratch));
      scratch = nullptr;
    }
  }
  void *tab = nullptr;
  double t0 = now_ms();
  if (!strcmp(mode, "contig")) {
    CK(hipExtMallocWithFlags(&tab, bytes, hipDeviceMallocContiguous));
  } else if (!strcmp(mode, "vmm")) {
    const size_t chunk = (argc > 2 ? (size_t)atoi(argv[2]) : 1) * gib;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    printf("granularity %zu\n", gran);
    hipDeviceptr_t base;
    CK(hipMemAddressReserve((void **)&base, bytes, chunk, nullptr, 0));
    for (size_t off = 0; off < bytes; off += chunk) {
      hipMemGenericAllocationHandle_t h;
      CK(hipMemCreate(&h, chunk, &prop, 0));
      CK(hipMemMap((char *)base + off, chunk, 0, h, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess((char *)base, bytes, &acc, 1));
    tab = (void *)base;
  } else {
    CK(hipMalloc(&tab, bytes));
  }
  CK(hipDeviceSynchronize());
  const double t_alloc = now_ms() - t0;
  t0 = now_ms();
  CK(hipMemsetD32Async((hipDeviceptr_t)tab, 0x01010101, bytes / 4, nullptr));
  CK(hipDeviceSynchronize());
  const double t_fill = now_ms() - t0;
  uint32_t *out;
  CK(hipMalloc(&out, 64));
  const int64_t n = (int64_t)1 << 32;
  const uint64_t mask = bytes / 16 - 1;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int it = 0; it < 4; ++it) {
    CK(hipEventRecord(a, nullptr));
    hipLaunchKernelGGL(k_gather, dim3(256 * 32), dim3(256), 0, nullptr, (const uint4 *)tab, mask, n, out);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  printf("%-7s alloc %8.1f ms  fill %7.1f ms  gather %.2f G/s\n", mode, t_alloc, t_fill, n / (best * 1e-3) / 1e9);
  return 0;
}
