// Host <-> device staging for the host entry points (ks_abi.cpp): the
// sequences of a call cross PCIe in a compact form and are rewritten on the
// device as bytes of the same class; tables and results go through the
// ctx's pinned buffer with worker threads on the host side.
//
// What the scan, the count and the runs read of a base is its class: 'n'
// or 'N' (LC(c) == 'n', kmer_spans.c:265) or the 2-bit code (c >> 1) & 3
// (UPDATE_OFFSET, :34).  So a base is sent as its 2-bit code plus, per
// chunk, the list of its N runs (0.25 B per base on a genome whose Ns come
// in gaps), or, for a chunk with too many N runs, as a 4-bit class
// (0..3 = the code, 4 = N; 0.5 B per base).  The device writes 'A' 'C' 'T'
// 'G' 'N' for the classes; those bytes give every kernel the same k-mers,
// Ns and codes as the caller's bytes (raw-byte staging, KS_STAGE_BYTES=1,
// is kept for comparison).
#include <tmmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "ks_internal.h"

namespace ks {
namespace {

// Bases per chunk: the unit of host packing, H2D and device unpacking
// (16 Mi bases = 4 MiB as 2-bit codes; the first copy starts ~2 ms in).
constexpr size_t kStageChunk = (size_t)16 << 20;

inline uint8_t code2(uint8_t c) { return (c >> 1) & 3; }
inline uint8_t nib_class(uint8_t c) { return is_n(c) ? 4 : code2(c); }

__attribute__((target("ssse3"))) void pack_nib(uint8_t *dst, const char *src, size_t n) {
  // dst[j] = class(src[2j]) | class(src[2j + 1]) << 4; n even
  const __m128i lc = _mm_set1_epi8(0x20), nn = _mm_set1_epi8('n'), three = _mm_set1_epi8(3),
                four = _mm_set1_epi8(4), mul = _mm_set1_epi16(0x1001);
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    __m128i p[2];
    for (int h = 0; h < 2; ++h) {
      const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16 * h));
      const __m128i isn = _mm_cmpeq_epi8(_mm_or_si128(x, lc), nn);
      const __m128i code = _mm_and_si128(_mm_srli_epi16(x, 1), three);  // bits 1-2 of each byte
      const __m128i cls = _mm_or_si128(_mm_andnot_si128(isn, code), _mm_and_si128(isn, four));
      p[h] = _mm_maddubs_epi16(cls, mul);  // even + 16 x odd
    }
    _mm_storeu_si128(reinterpret_cast<__m128i *>(dst + i / 2), _mm_packus_epi16(p[0], p[1]));
  }
  for (; i < n; i += 2)
    dst[i / 2] = (uint8_t)(nib_class((uint8_t)src[i]) | nib_class((uint8_t)src[i + 1]) << 4);
}

// One chunk in 2-bit form: codes at pay (byte j = bases 4j..4j+3, low bits
// first) and N runs (chunk-relative start, length: uint32 pairs) after them.
struct TwoBit {
  uint8_t *pay;
  uint32_t *runs;
  size_t cap, nr = 0;
  bool over = false;
  void run(uint32_t p, uint32_t len) {
    if (nr && runs[2 * nr - 2] + runs[2 * nr - 1] == p) {
      runs[2 * nr - 1] += len;
    } else if (nr == cap) {
      over = true;
    } else {
      runs[2 * nr] = p;
      runs[2 * nr + 1] = len;
      ++nr;
    }
  }
  void put(uint32_t p, uint8_t c) {  // one base (read-modify-write of its byte)
    uint8_t &b = pay[p >> 2];
    const int s = 2 * (p & 3);
    b = (uint8_t)((b & ~(3u << s)) | (uint32_t)code2(c) << s);
    if (is_n(c)) run(p, 1);
  }
  // bases [p, p + n) of the chunk from src; p % 4 == 0 in the vector body
  __attribute__((target("ssse3"))) void span(uint32_t p, const char *src, size_t n) {
    size_t i = 0;
    for (; i < n && ((p + i) & 3); ++i) put(p + (uint32_t)i, (uint8_t)src[i]);
    const __m128i lc = _mm_set1_epi8(0x20), nn = _mm_set1_epi8('n'), three = _mm_set1_epi8(3),
                  m1 = _mm_set1_epi16(0x0401), m2 = _mm_set1_epi32(0x00100001);
    for (; i + 64 <= n && !over; i += 64) {
      __m128i v[4];
      uint64_t nm = 0;
      for (int h = 0; h < 4; ++h) {
        const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16 * h));
        nm |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_or_si128(x, lc), nn)) << (16 * h);
        const __m128i code = _mm_and_si128(_mm_srli_epi16(x, 1), three);
        v[h] = _mm_madd_epi16(_mm_maddubs_epi16(code, m1), m2);  // per 4 bases: c0 + 4c1 + 16c2 + 64c3
      }
      _mm_storeu_si128(reinterpret_cast<__m128i *>(pay + ((p + i) >> 2)),
                       _mm_packus_epi16(_mm_packs_epi32(v[0], v[1]), _mm_packs_epi32(v[2], v[3])));
      while (nm) {  // the block's N runs
        const int a = __builtin_ctzll(nm);
        const uint64_t rest = ~(nm >> a);
        const int len = rest ? __builtin_ctzll(rest) : 64 - a;
        run(p + (uint32_t)(i + a), (uint32_t)len);
        nm = (a + len >= 64) ? 0 : nm & (~0ull << (a + len));
      }
    }
    for (; i < n; ++i) put(p + (uint32_t)i, (uint8_t)src[i]);
  }
};

// 16 bases per thread: 8 nibble bytes in, 16 class bytes out
__global__ void k_unpack_nib(const uint2 *__restrict__ in, uint4 *__restrict__ out, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n16) return;
  const uint2 v = in[i];
  const uint32_t w[2] = {v.x, v.y};
  uint32_t o[4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      uint32_t r = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t nib = (w[h] >> (16 * b + 4 * j)) & 15u;
        r |= (uint32_t)((0x4E47544341ull >> (8 * nib)) & 0xff) << (8 * j);  // A C T G N
      }
      o[2 * h + b] = r;
    }
  out[i] = make_uint4(o[0], o[1], o[2], o[3]);
}

// 16 bases per thread: one dword of 2-bit codes in, 16 bytes out
__global__ void k_unpack_2bit(const uint32_t *__restrict__ in, uint4 *__restrict__ out, int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n16) return;
  const uint32_t v = in[i];
  uint32_t o[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) r |= ((0x47544341u >> (8 * ((v >> (8 * b + 2 * j)) & 3u))) & 0xffu) << (8 * j);
    o[b] = r;  // A C T G
  }
  out[i] = make_uint4(o[0], o[1], o[2], o[3]);
}

// 'N' over each run (chunk-relative), a block per run in turn
__global__ void k_fill_n(const uint32_t *__restrict__ runs, int64_t nruns, uint8_t *__restrict__ base) {
  for (int64_t r = blockIdx.x; r < nruns; r += gridDim.x) {
    const uint32_t a = runs[2 * r], len = runs[2 * r + 1];
    uint8_t *p = base + a;
    const uint32_t al = (16u - (uint32_t)((uintptr_t)p & 15u)) & 15u, head = al < len ? al : len;
    const uint32_t body = (len - head) & ~15u;
    for (uint32_t i = threadIdx.x; i < head; i += blockDim.x) p[i] = 'N';
    uint4 *q = reinterpret_cast<uint4 *>(p + head);
    const uint4 nv = make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu);
    for (uint32_t i = threadIdx.x; i < body / 16; i += blockDim.x) q[i] = nv;
    for (uint32_t i = head + body + threadIdx.x; i < len; i += blockDim.x) p[i] = 'N';
  }
}

}  // namespace

ks_status stage(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, Staged *st, bool compact,
                const std::function<ks_status(int64_t)> &on_bytes) {
  const double t_enter = now_ms();
  st->offs.assign((size_t)nseq + 1, 0);
  for (int32_t q = 0; q < nseq; ++q) st->offs[q + 1] = st->offs[q] + std::max<int64_t>(lens[q], 0);
  st->total = st->offs[nseq];
  const size_t total = (size_t)st->total;
  // format: 0 raw bytes, 1 nibbles, 2 two-bit codes + N runs (per chunk,
  // nibbles where the runs do not fit)
  int fmt = 0;
  if (compact && total >= ((size_t)1 << 20) && !getenv("KS_STAGE_BYTES")) fmt = getenv("KS_STAGE_NIB") ? 1 : 2;
  void *d_seq = nullptr, *d_offs = nullptr, *h = nullptr, *d_cmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_SEQ, total + 32, &d_seq));
  KS_TRY(ensure(ctx, SLOT_OFFS, ((size_t)nseq + 1) * 8, &d_offs));
  // compact forms: chunk c at c x S / 2 on both sides (the nibble size)
  if (fmt) KS_TRY(ensure(ctx, SLOT_STAGE_NIB, total / 2 + 64, &d_cmp));
  KS_TRY(ensure_pinned(ctx, (fmt ? total / 2 : total) + 64, &h));
  KS_HIP(hipMemcpyAsync(d_offs, st->offs.data(), ((size_t)nseq + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  st->dev.seq = static_cast<const uint8_t *>(d_seq);
  st->dev.offsets_dev = static_cast<const int64_t *>(d_offs);
  st->dev.offsets_host = st->offs.data();
  st->dev.nseq = nseq;
  char *hp = static_cast<char *>(h);
  uint8_t *hc = static_cast<uint8_t *>(h);
  const size_t nchunk = (total + kStageChunk - 1) / kStageChunk;
  std::vector<uint8_t> cfmt(nchunk, 0);   // per chunk: 1 nibbles, 2 two-bit
  std::vector<uint32_t> cruns(nchunk, 0);  // per two-bit chunk: its N runs
  auto chunk_of = [&](size_t c, int64_t *lo, int64_t *hi) {
    *lo = (int64_t)(c * kStageChunk);
    *hi = std::min<int64_t>(*lo + (int64_t)kStageChunk, (int64_t)total);
  };
  auto two_bit_pay = [](size_t n) { return ((n + 3) / 4 + 15) & ~(size_t)15; };
  // fill chunk c: the parts of the sequences overlapping it
  auto fill = [&](size_t c) {
    int64_t lo, hi;
    chunk_of(c, &lo, &hi);
    const int32_t q0 = (int32_t)(std::upper_bound(st->offs.begin(), st->offs.end(), lo) - st->offs.begin()) - 1;
    auto each = [&](auto &&f) {
      for (int32_t q = q0; q < nseq && st->offs[q] < hi; ++q) {
        const int64_t a = std::max(lo, st->offs[q]), b = std::min(hi, st->offs[q + 1]);
        if (b > a) f(a, b, seqs[q] + (a - st->offs[q]));
      }
    };
    if (fmt == 0) {
      each([&](int64_t a, int64_t b, const char *src) { memcpy(hp + a, src, (size_t)(b - a)); });
      return;
    }
    uint8_t *cb = hc + lo / 2;
    const size_t n = (size_t)(hi - lo);
    if (fmt == 2) {
      const size_t pay = two_bit_pay(n);
      // N-run slots after the codes, inside the chunk's nibble-sized share
      // (a short last chunk may have no room at all: it goes as nibbles)
      const size_t room = (n + 1) / 2 > pay ? ((n + 1) / 2 - pay) / 8 : 0;
      TwoBit tb{cb, reinterpret_cast<uint32_t *>(cb + pay), room};
      each([&](int64_t a, int64_t b, const char *src) {
        if (!tb.over) tb.span((uint32_t)(a - lo), src, (size_t)(b - a));
      });
      if (!tb.over) {
        cfmt[c] = 2;
        cruns[c] = (uint32_t)tb.nr;
        return;
      }
    }
    // nibbles: nibble p of byte p / 2 (low = even); a sequence may start or
    // end mid-byte (chunks start on even positions: a byte is one thread's)
    cfmt[c] = 1;
    each([&](int64_t a, int64_t b, const char *src) {
      if (a & 1) {
        hc[a / 2] = (uint8_t)((hc[a / 2] & 15u) | nib_class((uint8_t)*src) << 4);
        ++a;
        ++src;
      }
      const int64_t even = (b - a) & ~(int64_t)1;
      pack_nib(hc + a / 2, src, (size_t)even);
      if (a + even < b) hc[(a + even) / 2] = nib_class((uint8_t)src[even]);
    });
  };
  // queue chunk c: its H2D on ctx->stream; the rewrite into bytes on the
  // high-priority stream (the copy stream carries DMA only and never waits
  // behind kernels; the rewrites get CUs ahead of a caller's side-stream
  // work, e.g. counts of the pieces already staged)
  hipStream_t us = ctx->hi;
  auto queue = [&](size_t c) -> hipError_t {
    int64_t lo, hi;
    chunk_of(c, &lo, &hi);
    const size_t n = (size_t)(hi - lo);
    if (fmt == 0)
      return hipMemcpyAsync(static_cast<char *>(d_seq) + lo, hp + lo, n, hipMemcpyHostToDevice, ctx->stream);
    uint8_t *dc = static_cast<uint8_t *>(d_cmp) + lo / 2;
    const size_t pay = two_bit_pay(n);
    const size_t bytes = cfmt[c] == 2 ? pay + (size_t)cruns[c] * 8 : (n + 1) / 2;
    hipError_t e = hipMemcpyAsync(dc, hc + lo / 2, bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(ctx->ev[20], ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(us, ctx->ev[20], 0);
    if (e != hipSuccess) return e;
    const int64_t n16 = (int64_t)((n + 15) / 16);  // (the tail rounds up into the buffer's 32 B of slack)
    uint8_t *out = static_cast<uint8_t *>(d_seq) + lo;
    const unsigned g = (unsigned)((n16 + 255) / 256);
    if (cfmt[c] == 2) {
      hipLaunchKernelGGL(k_unpack_2bit, dim3(g), dim3(256), 0, us, reinterpret_cast<const uint32_t *>(dc),
                         reinterpret_cast<uint4 *>(out), n16);
      if (cruns[c])
        hipLaunchKernelGGL(k_fill_n, dim3(std::min<uint32_t>(cruns[c], 2048)), dim3(256), 0, us,
                           reinterpret_cast<const uint32_t *>(dc + pay), (int64_t)cruns[c], out);
    } else {
      hipLaunchKernelGGL(k_unpack_nib, dim3(g), dim3(256), 0, us, reinterpret_cast<const uint2 *>(dc),
                         reinterpret_cast<uint4 *>(out), n16);
    }
    return hipGetLastError();
  };
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t nthr = std::min<size_t>(std::min<size_t>(16, hw), nchunk);
  std::atomic<size_t> next{0};
  std::vector<std::atomic<uint8_t>> done(nchunk);
  for (auto &d : done) d.store(0, std::memory_order_relaxed);
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> pool;
  for (size_t t = 0; nthr > 1 && t < nthr; ++t)
    pool.emplace_back([&] {
      for (size_t c; (c = next.fetch_add(1)) < nchunk;) {
        fill(c);
        {
          std::lock_guard<std::mutex> g(mu);
          done[c].store(1, std::memory_order_release);
        }
        cv.notify_all();
      }
    });
  hipError_t err = hipSuccess;
  ks_status cb_rc = KS_OK;
  for (size_t c = 0; c < nchunk; ++c) {  // queue each chunk once it is full, in order
    if (nthr > 1) {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return done[c].load(std::memory_order_acquire) != 0; });
    } else {
      fill(c);
    }
    if (err == hipSuccess) err = queue(c);
    if (err == hipSuccess && on_bytes) {  // the side stream sees the bases so far
      err = hipEventRecord(ctx->ev[22], fmt ? us : ctx->stream);
      if (err == hipSuccess) err = hipStreamWaitEvent(ctx->side, ctx->ev[22], 0);
    }
    if (err == hipSuccess && cb_rc == KS_OK && on_bytes)
      cb_rc = on_bytes(std::min<int64_t>((int64_t)((c + 1) * kStageChunk), (int64_t)total));
  }
  if (err == hipSuccess && fmt) err = hipEventRecord(ctx->ev[21], us);  // the stream joins the rewrites
  if (err == hipSuccess && fmt) err = hipStreamWaitEvent(ctx->stream, ctx->ev[21], 0);
  const double t_q = now_ms();
  for (auto &th : pool) th.join();
  if (err != hipSuccess) return fail(KS_ERR_DEVICE, "sequence upload failed: %s", hipGetErrorString(err));
  if (cb_rc != KS_OK) return cb_rc;
  if (getenv("KS_DEBUG_HOST")) {
    size_t n2 = 0, nr = 0;
    for (size_t c = 0; c < nchunk; ++c) n2 += cfmt[c] == 2, nr += cruns[c];
    const double t_s0 = now_ms();
    KS_HIP(hipStreamSynchronize(ctx->stream));
    fprintf(stderr, "[stage] fmt %d: %zu chunks (%zu two-bit, %zu N runs), %zu threads: all queued %.2f, joined %.2f, "
            "synced %.2f ms\n", fmt, nchunk, n2, nr, nthr, t_q - t_enter, t_s0 - t_enter, now_ms() - t_enter);
  }
  KS_HIP(hipStreamSynchronize(ctx->stream));
  static const bool verify = getenv("KS_DEBUG_VERIFY") != nullptr;  // (diagnostics, ks_scan_chunked.hip)
  if (verify && total <= ((size_t)64 << 20)) {
    std::vector<uint8_t> back(total);
    std::vector<int64_t> ob((size_t)nseq + 1);
    KS_HIP(hipMemcpy(back.data(), d_seq, total, hipMemcpyDeviceToHost));
    KS_HIP(hipMemcpy(ob.data(), d_offs, ob.size() * 8, hipMemcpyDeviceToHost));
    long long bad = 0;
    for (int32_t q = 0; q < nseq; ++q) {
      if (ob[q] != st->offs[q]) fprintf(stderr, "[verify] staged offset %d = %lld, host %lld\n", q, (long long)ob[q],
                                        (long long)st->offs[q]);
      for (int64_t i = 0; i < lens[q]; ++i) {
        const uint8_t h = (uint8_t)seqs[q][i], d = back[st->offs[q] + i];
        const bool same = is_n(h) ? is_n(d) : (!is_n(d) && code2(h) == code2(d));
        if (!same && ++bad <= 8)
          fprintf(stderr, "[verify] staged base %d:%lld = %u, host %u\n", q, (long long)i, d, h);
      }
    }
    if (bad) fprintf(stderr, "[verify] %lld staged bases differ (format %d)\n", bad, fmt);
  }
  return KS_OK;
}

// Pageable host -> device through the ctx's pinned buffer: nthr threads
// fill 32 MiB pieces in order and each piece's H2D is queued once it is full
// (the runtime's own pageable path runs at 20-55 GB/s and serialises
// with the caller).  Synchronises ctx->stream.
ks_status h2d_pinned(ks_ctx *ctx, void *dst_dev, const void *src, size_t n, int nthr) {
  constexpr size_t kPiece = (size_t)32 << 20;
  void *h = nullptr;
  KS_TRY(ensure_pinned(ctx, n, &h));
  const size_t np = (n + kPiece - 1) / kPiece;
  std::atomic<size_t> next{0};
  std::vector<std::atomic<uint8_t>> done(np);
  for (auto &d : done) d.store(0, std::memory_order_relaxed);
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> pool;
  for (int t = 0; t < std::max(1, std::min<int>(nthr, (int)np)); ++t)
    pool.emplace_back([&] {
      for (size_t c; (c = next.fetch_add(1)) < np;) {
        const size_t a = c * kPiece, b = std::min(n, a + kPiece);
        memcpy(static_cast<char *>(h) + a, static_cast<const char *>(src) + a, b - a);
        {
          std::lock_guard<std::mutex> g(mu);
          done[c].store(1, std::memory_order_release);
        }
        cv.notify_all();
      }
    });
  hipError_t err = hipSuccess;
  for (size_t c = 0; c < np; ++c) {
    {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return done[c].load(std::memory_order_acquire) != 0; });
    }
    const size_t a = c * kPiece, b = std::min(n, a + kPiece);
    if (err == hipSuccess)
      err = hipMemcpyAsync(static_cast<char *>(dst_dev) + a, static_cast<char *>(h) + a, b - a,
                           hipMemcpyHostToDevice, ctx->stream);
  }
  for (auto &th : pool) th.join();
  if (err == hipSuccess) err = hipStreamSynchronize(ctx->stream);
  if (err != hipSuccess) return fail(KS_ERR_DEVICE, "host upload failed: %s", hipGetErrorString(err));
  return KS_OK;
}

// memcpy with up to 16 threads (host results out of the pinned buffer)
void par_memcpy(void *dst, const void *src, size_t n) {
  const size_t nthr = std::min<size_t>(std::min<size_t>(16, std::max(1u, std::thread::hardware_concurrency())),
                                       std::max<size_t>(1, n >> 24));
  if (nthr <= 1) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t per = (n + nthr - 1) / nthr;
  for (size_t t = 0; t < nthr; ++t)
    pool.emplace_back([=] {
      const size_t a = t * per, b = std::min(n, a + per);
      if (b > a) memcpy(static_cast<char *>(dst) + a, static_cast<const char *>(src) + a, b - a);
    });
  for (auto &th : pool) th.join();
}

ks_status copy_out(ks_ctx *ctx, void *dst, const void *src_dev, size_t n) {
  void *h = nullptr;
  KS_TRY(ensure_pinned(ctx, n, &h));
  KS_HIP(hipMemcpyAsync(h, src_dev, n, hipMemcpyDeviceToHost, ctx->stream));
  KS_HIP(hipStreamSynchronize(ctx->stream));
  par_memcpy(dst, h, n);
  return KS_OK;
}

int64_t stage_chunk_bases() { return (int64_t)kStageChunk; }

}  // namespace ks
