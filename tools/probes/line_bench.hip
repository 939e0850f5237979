// line_bench.hip -- random reads of whole 16/32/64/128/256-byte lines from a
// physically contiguous 128 GiB buffer (the expanded-table allocation): does
// a 64-B or 128-B line cost one random request at the ~50 G/s wall, or one per
// 64 B?  Decides the continuation-line table design.
//   lane  : one lane reads the whole line (L/16 consecutive 16-B loads)
//   group : L/16 lanes each read one 16-B piece of the same line (coalesced)
// Prints one JSON line per case: G lines/s and GB/s of line bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// kPer = 16-B pieces per line; U = lines in flight per lane
template <int kPer, int U>
__global__ void __launch_bounds__(256) k_lane(const uint4 *__restrict__ tab, uint64_t line_mask, int64_t nlines,
                                              uint32_t *out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; p < nlines; p += stride) {
    uint4 v[U][kPer];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 *l = tab + (mix(p + u) & line_mask) * kPer;
#pragma unroll
      for (int q = 0; q < kPer; ++q) v[u][q] = l[q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < kPer; ++q) acc += v[u][q].x ^ v[u][q].w;
  }
  if (acc == 0x12345u) out[0] = acc;
}

template <int kPer, int U>
__global__ void __launch_bounds__(256) k_group(const uint4 *__restrict__ tab, uint64_t line_mask, int64_t nlines,
                                               uint32_t *out) {
  uint32_t acc = 0;
  const int g = threadIdx.x % kPer;
  const int64_t lanes_groups = (int64_t)gridDim.x * (blockDim.x / kPer);
  const int64_t stride = lanes_groups * U;
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

template <typename F>
float best_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

static const uint4 *g_tab;
static size_t g_bytes;
static uint32_t *g_out;

template <int kPer, int U, bool kGroup>
void run(const char *mode, int grid) {
  const uint64_t lines = g_bytes / (16 * kPer);
  const int64_t n = (int64_t)1 << 31;  // lines read per launch
  float ms = best_ms([&] {
    if (kGroup)
      hipLaunchKernelGGL((k_group<kPer, U>), dim3(grid), dim3(256), 0, 0, g_tab, lines - 1, n, g_out);
    else
      hipLaunchKernelGGL((k_lane<kPer, U>), dim3(grid), dim3(256), 0, 0, g_tab, lines - 1, n, g_out);
  }, 3);
  printf("{\"mode\":\"%s\",\"line_B\":%d,\"in_flight\":%d,\"grid\":%d,\"table_GiB\":%.3f,\"G_lines_per_s\":%.2f,"
         "\"GB_per_s\":%.0f,\"G_64B_per_s\":%.2f}\n",
         mode, 16 * kPer, U, grid, g_bytes / 1073741824.0, n / (ms * 1e6), n * 16.0 * kPer / (ms * 1e6),
         n * 16.0 * kPer / 64.0 / (ms * 1e6));
  fflush(stdout);
}

// usage: line_bench [table MiB (131072)] [group]  -- "group": the coalesced
// group forms only (the PMC calibration of round 6 runs them under
// rocprofv3 --pmc FETCH_SIZE: HBM bytes counted per line read)
int main(int argc, char **argv) {
  const size_t mib = (size_t)1 << 20;
  g_bytes = (argc > 1 ? (size_t)atoll(argv[1]) : 131072) * mib;
  const bool only_group = argc > 2 && strcmp(argv[2], "group") == 0;
  void *tab = nullptr;
  if (hipExtMallocWithFlags(&tab, g_bytes, hipDeviceMallocContiguous) != hipSuccess) {
    (void)hipGetLastError();
    CK(hipMalloc(&tab, g_bytes));
    printf("# plain hipMalloc\n");
  }
  CK(hipMemsetD32Async((hipDeviceptr_t)tab, 0x01010101, g_bytes / 4, nullptr));
  CK(hipMalloc(&g_out, 64));
  CK(hipDeviceSynchronize());
  g_tab = (const uint4 *)tab;
  const int grid = 256 * 32;
  if (!only_group) {
    run<1, 4, false>("lane", grid);
    run<1, 8, false>("lane", grid);
    run<2, 4, false>("lane", grid);
    run<4, 2, false>("lane", grid);
    run<4, 4, false>("lane", grid);
    run<8, 2, false>("lane", grid);
  }
  run<2, 8, true>("group", grid);
  run<4, 4, true>("group", grid);
  run<4, 8, true>("group", grid);
  run<8, 4, true>("group", grid);
  run<8, 8, true>("group", grid);
  run<16, 4, true>("group", grid);
  run<16, 8, true>("group", grid);
  return 0;
}
