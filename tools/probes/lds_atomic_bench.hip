// lds_atomic_bench.hip -- LDS atomic rates on gfx950 with 2,048 random
// buckets (the count scatter's shape): no-return adds, returning adds whose
// value is consumed (a dependent 2-B stage store, as k_part_scatter_st), and
// returning adds issued 4 at a time before their uses.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1;} } while (0)
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}
template <int kMode>
__global__ void __launch_bounds__(1024) k_lds(int64_t n, uint32_t *out) {
  __shared__ uint32_t h[2048];
  __shared__ uint16_t stage[2048 * 16];
  for (int i = threadIdx.x; i < 2048; i += 1024) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) {
    const uint64_t x = mix(p);
    if (kMode == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(&h[(x >> (11 * j)) & 2047], 1u);
    } else if (kMode == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t b = (x >> (11 * j)) & 2047;
        const uint32_t s = atomicAdd(&h[b], 1u);
        stage[b * 16 + (s & 15)] = (uint16_t)j;
      }
    } else {
      uint32_t s[4], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) { b[j] = (x >> (11 * j)) & 2047; s[j] = atomicAdd(&h[b[j]], 1u); }
#pragma unroll
      for (int j = 0; j < 4; ++j) stage[b[j] * 16 + (s[j] & 15)] = (uint16_t)j;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 1024) acc += h[i] + stage[i];
  if (acc == 0x7fffffffu) out[1] = acc;
}
int main() {
  uint32_t *out; CK(hipMalloc(&out, 64));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int64_t n = (int64_t)1 << 30;
  for (int grid : {256, 512}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto go = [&] {
        if (mode == 0) hipLaunchKernelGGL(k_lds<0>, dim3(grid), dim3(1024), 0, 0, n, out);
        else if (mode == 1) hipLaunchKernelGGL(k_lds<1>, dim3(grid), dim3(1024), 0, 0, n, out);
        else hipLaunchKernelGGL(k_lds<2>, dim3(grid), dim3(1024), 0, 0, n, out);
      };
      go(); CK(hipDeviceSynchronize());
      CK(hipEventRecord(a)); go(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"grid\":%d,\"mode\":\"%s\",\"G_atomics_per_s\":%.1f}\n", grid,
             mode == 0 ? "noret" : mode == 1 ? "ret+store" : "ret4+stores", 4.0 * n / (ms * 1e6));
    }
  }
  return 0;
}
