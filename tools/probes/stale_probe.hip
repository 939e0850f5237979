// stale_probe: after hipFree + hipMalloc of the same size (the host entry
// points' workspace under memory policy 0, or a slot that grows), does a
// kernel read what the previous allocation held where a kernel of the new
// allocation has just written?
//
// Round-4 record (case 268): the stitch read a chunk's tail begin as 0 at
// words 8..23 of an array whose 128-B line, in the previous call's layout,
// held that call's binade array (7 words written, the rest never written:
// zero) -- the previous call's content of the line, not this call's.
//
// Each round: hipMalloc(big) (same size every round), then on one stream
//   K_pre   (optional) reads every word of the first `span` bytes from
//           blocks shifted by 5 (lines cached on other XCDs before the write),
//   K_write writes round-tagged words (block b: words [64b, 64b + 64)),
//   K_check reads every word from blocks shifted by 3 (another XCD than the
//           writer) and counts words that differ: equal to the previous
//           round's tag (stale), zero, or other,
// then hipFree.  A persistent counter buffer collects the counts.
//
// Build: hipcc -O2 --offload-arch=gfx950 tools/probes/stale_probe.hip -o tools/probes/stale_probe
// Run:   tools/probes/stale_probe [rounds] [big_mib] [span_kib] [pre 0/1] [sizes 0/1]
// sizes 1: alternate two allocation sizes (a slot that grows and shrinks);
// sizes 2: a host call's pattern -- 16 buffers a round, sizes drawn from
// 4 KiB .. big in a random order (addresses and pages shuffle between
// rounds), each written and checked as above, all freed at the round's end.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(2);                                                                            \
    }                                                                                     \
  } while (0)

__device__ __forceinline__ uint32_t tag(uint32_t round, uint32_t i) { return (round << 20) ^ (i * 2654435761u) ^ 1u; }

__global__ void k_pre(const uint32_t *p, int64_t n, unsigned long long *sink) {
  const int64_t nb = (n + 63) / 64;
  const int64_t b = (blockIdx.x + 5) % nb;
  const int64_t i = b * 64 + threadIdx.x;
  uint32_t v = i < n ? p[i] : 0;
  if (v == 0x12345678u) atomicAdd(sink, 1ull);  // (keeps the load)
}

__global__ void k_write(uint32_t *p, int64_t n, uint32_t round) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) p[i] = tag(round, (uint32_t)i);
}

__global__ void k_check(const uint32_t *p, int64_t n, uint32_t round, unsigned long long *cnt) {
  const int64_t nb = (n + 63) / 64;
  const int64_t b = (blockIdx.x + 3) % nb;
  const int64_t i = b * 64 + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = p[i];
  if (v != tag(round, (uint32_t)i)) {
    atomicAdd(&cnt[0], 1ull);
    if (round > 0 && v == tag(round - 1, (uint32_t)i)) atomicAdd(&cnt[1], 1ull);
    else if (v == 0) atomicAdd(&cnt[2], 1ull);
    else atomicAdd(&cnt[3], 1ull);
  }
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  const size_t big = (size_t)(argc > 2 ? atoi(argv[2]) : 256) << 20;
  const int64_t n = ((int64_t)(argc > 3 ? atoi(argv[3]) : 64) << 10) / 4;
  const bool pre = argc > 4 ? atoi(argv[4]) != 0 : true;
  const bool sizes = argc > 5 ? atoi(argv[5]) != 0 : false;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long *cnt = nullptr, *sink = nullptr;
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(cnt, 0, 64));
  CK(hipMemset(sink, 0, 8));
  const unsigned nb = (unsigned)((n + 63) / 64);
  void *prev = nullptr;
  long long same_va = 0;
  if (argc > 5 && atoi(argv[5]) == 2) {
    unsigned long long rng = 0x9E3779B97F4A7C15ull;
    auto next = [&]() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; };
    const size_t choices[6] = {(size_t)4 << 10, (size_t)64 << 10, (size_t)1 << 20, (size_t)16 << 20, big / 2, big};
    for (int r = 0; r < rounds; ++r) {
      void *bufs[16];
      for (int b = 0; b < 16; ++b) {
        const size_t sz = choices[next() % 6] + 4096 * (next() % 4);
        CK(hipMalloc(&bufs[b], sz));
        const int64_t nn = std::min<int64_t>(n, (int64_t)(sz / 4));
        const unsigned nbb = (unsigned)((nn + 63) / 64);
        uint32_t *p = static_cast<uint32_t *>(bufs[b]);
        if (pre) hipLaunchKernelGGL(k_pre, dim3(nbb), dim3(64), 0, st, p, nn, sink);
        hipLaunchKernelGGL(k_write, dim3(nbb), dim3(64), 0, st, p, nn, (uint32_t)(16 * r + b));
        hipLaunchKernelGGL(k_check, dim3(nbb), dim3(64), 0, st, p, nn, (uint32_t)(16 * r + b), cnt);
        CK(hipGetLastError());
      }
      CK(hipStreamSynchronize(st));
      for (int b = 0; b < 16; ++b) CK(hipFree(bufs[b]));
      if ((r + 1) % 100 == 0) {
        unsigned long long h[4];
        CK(hipMemcpy(h, cnt, 32, hipMemcpyDeviceToHost));
        printf("round %d: bad %llu (zero %llu, other %llu)\n", r + 1, h[0], h[2], h[1] + h[3]);
        fflush(stdout);
      }
    }
    unsigned long long h[4];
    CK(hipMemcpy(h, cnt, 32, hipMemcpyDeviceToHost));
    printf("RESULT rounds %d x 16 buffers up to %zu MiB span %lld KiB pre %d: bad %llu zero %llu other %llu\n", rounds,
           big >> 20, (long long)n * 4 / 1024, (int)pre, h[0], h[2], h[1] + h[3]);
    return 0;
  }
  for (int r = 0; r < rounds; ++r) {
    void *buf = nullptr;
    const size_t sz = sizes && (r & 1) ? big + ((size_t)64 << 20) : big;
    CK(hipMalloc(&buf, sz));
    same_va += buf == prev;
    uint32_t *p = static_cast<uint32_t *>(buf);
    if (pre) hipLaunchKernelGGL(k_pre, dim3(nb), dim3(64), 0, st, p, n, sink);
    hipLaunchKernelGGL(k_write, dim3(nb), dim3(64), 0, st, p, n, (uint32_t)r);
    hipLaunchKernelGGL(k_check, dim3(nb), dim3(64), 0, st, p, n, (uint32_t)r, cnt);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(st));
    CK(hipFree(buf));
    prev = buf;
    if ((r + 1) % 500 == 0) {
      unsigned long long h[4];
      CK(hipMemcpy(h, cnt, 32, hipMemcpyDeviceToHost));
      printf("round %d: bad %llu (previous round's tag %llu, zero %llu, other %llu), same VA %lld\n", r + 1, h[0], h[1],
             h[2], h[3], same_va);
      fflush(stdout);
    }
  }
  unsigned long long h[4];
  CK(hipMemcpy(h, cnt, 32, hipMemcpyDeviceToHost));
  printf("RESULT rounds %d big %zu MiB span %lld KiB pre %d sizes %d: bad %llu stale %llu zero %llu other %llu same_va %lld\n",
         rounds, big >> 20, (long long)n * 4 / 1024, (int)pre, (int)sizes, h[0], h[1], h[2], h[3], same_va);
  return 0;
}
