// Host <-> device transfer rates on the GPU box (what bounds the host entry
// points' staging): pinned and pageable H2D / D2H, multi-threaded host
// memcpy into pinned memory, and the same with the 4-bit base packing.
// Build: hipcc -O3 -std=c++17 -mssse3 tools/probes/pcie_bench.cpp -o tools/probes/pcie_bench
#include <hip/hip_runtime.h>
#include <tmmintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static void pack(uint8_t *dst, const char *src, size_t n) {
  const __m128i lc = _mm_set1_epi8(0x20), nn = _mm_set1_epi8('n'), three = _mm_set1_epi8(3),
                four = _mm_set1_epi8(4), mul = _mm_set1_epi16(0x1001);
  for (size_t i = 0; i + 32 <= n; i += 32) {
    __m128i p[2];
    for (int h = 0; h < 2; ++h) {
      const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16 * h));
      const __m128i isn = _mm_cmpeq_epi8(_mm_or_si128(x, lc), nn);
      const __m128i code = _mm_and_si128(_mm_srli_epi16(x, 1), three);
      p[h] = _mm_maddubs_epi16(_mm_or_si128(_mm_andnot_si128(isn, code), _mm_and_si128(isn, four)), mul);
    }
    _mm_storeu_si128(reinterpret_cast<__m128i *>(dst + i / 2), _mm_packus_epi16(p[0], p[1]));
  }
}

template <class F>
static double par(int nthr, size_t n, F f) {
  const double t0 = now_ms();
  std::vector<std::thread> th;
  const size_t per = (n / nthr + 63) & ~(size_t)63;
  for (int t = 0; t < nthr; ++t)
    th.emplace_back([=] {
      const size_t a = std::min(n, t * per), b = std::min(n, a + per);
      if (b > a) f(a, b);
    });
  for (auto &x : th) x.join();
  return now_ms() - t0;
}

int main(int argc, char **argv) {
  const size_t n = (argc > 1 ? atol(argv[1]) : 1536) << 20;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  void *d = nullptr, *hp = nullptr;
  CK(hipMalloc(&d, n));
  CK(hipHostMalloc(&hp, n, hipHostMallocDefault));
  std::vector<char> pg(n);
  for (size_t i = 0; i < n; ++i) pg[i] = "ACGT"[(i * 2654435761u >> 7) & 3];
  memset(hp, 1, n);
  auto rate = [&](const char *what, double ms, size_t bytes) {
    printf("{\"what\":\"%s\",\"MiB\":%zu,\"ms\":%.2f,\"GB_per_s\":%.2f}\n", what, bytes >> 20, ms, bytes / ms / 1e6);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now_ms();
    CK(hipMemcpyAsync(d, hp, n, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    rate("h2d_pinned", now_ms() - t0, n);
    t0 = now_ms();
    CK(hipMemcpyAsync(hp, d, n, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    rate("d2h_pinned", now_ms() - t0, n);
    t0 = now_ms();
    CK(hipMemcpyAsync(d, pg.data(), n / 3, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    rate("h2d_pageable", now_ms() - t0, n / 3);
    for (int nt : {1, 4, 8, 16}) {
      char name[64];
      snprintf(name, sizeof name, "memcpy_to_pinned_t%d", nt);
      rate(name, par(nt, n, [&](size_t a, size_t b) { memcpy((char *)hp + a, pg.data() + a, b - a); }), n);
      snprintf(name, sizeof name, "pack_to_pinned_t%d(input)", nt);
      rate(name, par(nt, n, [&](size_t a, size_t b) { pack((uint8_t *)hp + a / 2, pg.data() + a, b - a); }), n);
    }
    // two streams at once: n / 2 in 32 MiB pieces on st and n / 3 on st2
    {
      static hipStream_t st2 = nullptr;
      static void *d2 = nullptr, *hp2 = nullptr;
      if (!st2) {
        CK(hipStreamCreate(&st2));
        CK(hipMalloc(&d2, n / 3));
        CK(hipHostMalloc(&hp2, n / 3, hipHostMallocDefault));
        memset(hp2, 2, n / 3);
      }
      t0 = now_ms();
      size_t o1 = 0, o2 = 0;
      while (o1 < n / 2 || o2 < n / 3) {
        if (o1 < n / 2) {
          CK(hipMemcpyAsync((char *)d + o1, (char *)hp + o1, std::min<size_t>(32u << 20, n / 2 - o1),
                            hipMemcpyHostToDevice, st));
          o1 += 32u << 20;
        }
        if (o2 < n / 3) {
          CK(hipMemcpyAsync((char *)d2 + o2, (char *)hp2 + o2, std::min<size_t>(32u << 20, n / 3 - o2),
                            hipMemcpyHostToDevice, st2));
          o2 += 32u << 20;
        }
      }
      CK(hipStreamSynchronize(st));
      CK(hipStreamSynchronize(st2));
      rate("h2d_two_streams(total)", now_ms() - t0, n / 2 + n / 3);
      t0 = now_ms();
      for (size_t o = 0; o < n / 2; o += 32u << 20)
        CK(hipMemcpyAsync((char *)d + o, (char *)hp + o, std::min<size_t>(32u << 20, n / 2 - o),
                          hipMemcpyHostToDevice, st));
      for (size_t o = 0; o < n / 3; o += 32u << 20)
        CK(hipMemcpyAsync((char *)d2 + o, (char *)hp2 + o, std::min<size_t>(32u << 20, n / 3 - o),
                          hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      rate("h2d_one_stream_both(total)", now_ms() - t0, n / 2 + n / 3);
    }
    // pinned chunked H2D of the half-size packed stream, 32 MiB pieces
    t0 = now_ms();
    for (size_t off = 0; off < n / 2; off += (32u << 20))
      CK(hipMemcpyAsync((char *)d + off, (char *)hp + off, std::min<size_t>(32u << 20, n / 2 - off),
                        hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    rate("h2d_pinned_32MiB_chunks", now_ms() - t0, n / 2);
  }
  return 0;
}
