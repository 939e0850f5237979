// ks_count.hip -- K1: k-mer counting (sequence_kmer_count, kmer_spans.c:135-155).
//
// Position-parallel: every k-mer whose k bases lie in one N-free run of one
// sequence is counted once, at its last base.  Quirk Q1 (:142-144): the
// first window of a run is dropped when it ends exactly at the end of the
// string, i.e. a run of exactly k bases at the end of a sequence counts
// nothing.  Histograms wrap mod 2^32 like the reference's int counters.
//
// Layout: a persistent grid walks 4096-position tiles (256 threads x 16
// consecutive positions, two 16-byte loads per thread covering the 15-byte
// look-back).  k <= 7: the 4^k histogram is privatised in LDS (<= 64 KiB) and
// flushed once per block; k >= 8: global atomics into HBM.
#include <algorithm>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr int kTile = 4096;
constexpr int kPer = 16;
constexpr int kLook = 16;  // look-back bytes (k - 1 <= 14)

template <bool kLds>
__global__ void __launch_bounds__(256) k_count(const uint8_t *__restrict__ seq, int64_t total,
                                               const int64_t *__restrict__ offs, int32_t nseq, int k,
                                               uint32_t *__restrict__ counts,
                                               unsigned long long *__restrict__ n_words,
                                               int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[];
  __shared__ uint32_t bmask[(kTile + kLook + 32) / 32 + 1];
  __shared__ unsigned long long wsum[4];
  const uint32_t mask = (k >= 16) ? 0xffffffffu : ((1u << (2 * k)) - 1u);
  if (kLds) {
    const int nb = 1 << (2 * k);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) lds_hist[i] = 0;
  }
  unsigned long long my_words = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t t0 = tile * kTile;
    const int64_t base = t0 - kLook;  // bitmap bit r <-> position base + r
    __syncthreads();
    for (int i = threadIdx.x; i < (kTile + kLook + 32) / 32 + 1; i += blockDim.x) bmask[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      int lo = 0, hi = nseq + 1;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (offs[mid] < base) lo = mid + 1; else hi = mid;
      }
      for (int q = lo; q <= nseq && offs[q] <= t0 + kTile; ++q) {
        const int r = (int)(offs[q] - base);
        bmask[r >> 5] |= 1u << (r & 31);
      }
    }
    __syncthreads();
    const int64_t p0 = t0 + (int64_t)threadIdx.x * kPer;
    if (p0 >= total) continue;
    uint8_t b[kLook + kPer];
    if (p0 >= kLook && p0 + kPer <= total) {
      const uint4 v0 = *reinterpret_cast<const uint4 *>(seq + p0 - kLook);
      const uint4 v1 = *reinterpret_cast<const uint4 *>(seq + p0);
      const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int j = 0; j < kLook + kPer; ++j) b[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    } else {
#pragma unroll
      for (int j = 0; j < kLook + kPer; ++j) {
        const int64_t q = p0 - kLook + j;
        b[j] = (q >= 0 && q < total) ? seq[q] : (uint8_t)'N';
      }
    }
    uint32_t code = 0;
    int len = 0;
#pragma unroll
    for (int j = 1; j < kLook + kPer; ++j) {  // positions p0-15 .. p0+15
      const int64_t q = p0 - kLook + j;
      const int r = (int)(q - base);
      if ((bmask[r >> 5] >> (r & 31)) & 1u) len = 0;  // q starts a sequence
      if (!is_n(b[j])) {
        code = ((code << 2) | enc(b[j])) & mask;
        ++len;
      } else {
        len = 0;
      }
      if (j >= kLook && q < total && len >= k) {
        const int r1 = r + 1;
        const bool q1 = (len == k) && ((bmask[r1 >> 5] >> (r1 & 31)) & 1u);
        if (!q1) {
          ++my_words;
          if (kLds) atomicAdd(&lds_hist[code], 1u);
          else atomicAdd(&counts[code], 1u);
        }
      }
    }
  }
  // words: wave reduce then block reduce
  for (int d = 32; d >= 1; d >>= 1) my_words += __shfl_down(my_words, d, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = my_words;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += wsum[w];
    if (t) atomicAdd(n_words, t);
  }
  if (kLds) {
    const int nb = 1 << (2 * k);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
      const uint32_t v = lds_hist[i];
      if (v) atomicAdd(&counts[i], v);
    }
  }
}


// Batched counting (kmers.to.file counts several k over the
// same sequences, kmer_spans.R:149-151): one pass keeps the rolling code of
// the largest k and the N-free run length; every k of the batch takes the
// low 2k bits.  The k's whose 4^k histograms fit 64 KiB together are
// privatised in LDS; the rest use global atomics.
constexpr int kMaxBatch = 8;
struct KBatch {
  int32_t k[kMaxBatch];
  uint32_t *counts[kMaxBatch];
  int32_t lds_off[kMaxBatch];  // LDS word offset, -1: global
  int32_t nk, lds_words;
};

__global__ void __launch_bounds__(256) k_count_multi(const uint8_t *__restrict__ seq, int64_t total,
                                                     const int64_t *__restrict__ offs, int32_t nseq, KBatch kb,
                                                     unsigned long long *__restrict__ n_words, int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[];
  __shared__ uint32_t bmask[(kTile + kLook + 32) / 32 + 1];
  __shared__ unsigned long long wsum[4][kMaxBatch];
  for (int i = threadIdx.x; i < kb.lds_words; i += blockDim.x) lds_hist[i] = 0;
  int kmax = 1;
  for (int i = 0; i < kb.nk; ++i) kmax = kb.k[i] > kmax ? kb.k[i] : kmax;
  const uint32_t mask = (1u << (2 * kmax)) - 1u;
  unsigned long long my_words[kMaxBatch];
#pragma unroll
  for (int i = 0; i < kMaxBatch; ++i) my_words[i] = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t t0 = tile * kTile;
    const int64_t base = t0 - kLook;
    __syncthreads();
    for (int i = threadIdx.x; i < (kTile + kLook + 32) / 32 + 1; i += blockDim.x) bmask[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      int lo = 0, hi = nseq + 1;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (offs[mid] < base) lo = mid + 1; else hi = mid;
      }
      for (int q = lo; q <= nseq && offs[q] <= t0 + kTile; ++q) {
        const int r = (int)(offs[q] - base);
        bmask[r >> 5] |= 1u << (r & 31);
      }
    }
    __syncthreads();
    const int64_t p0 = t0 + (int64_t)threadIdx.x * kPer;
    if (p0 >= total) continue;
    uint8_t b[kLook + kPer];
    if (p0 >= kLook && p0 + kPer <= total) {
      const uint4 v0 = *reinterpret_cast<const uint4 *>(seq + p0 - kLook);
      const uint4 v1 = *reinterpret_cast<const uint4 *>(seq + p0);
      const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int j = 0; j < kLook + kPer; ++j) b[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    } else {
#pragma unroll
      for (int j = 0; j < kLook + kPer; ++j) {
        const int64_t q = p0 - kLook + j;
        b[j] = (q >= 0 && q < total) ? seq[q] : (uint8_t)'N';
      }
    }
    uint32_t code = 0;
    int len = 0;
#pragma unroll
    for (int j = 1; j < kLook + kPer; ++j) {
      const int64_t q = p0 - kLook + j;
      const int r = (int)(q - base);
      if ((bmask[r >> 5] >> (r & 31)) & 1u) len = 0;
      if (!is_n(b[j])) {
        code = ((code << 2) | enc(b[j])) & mask;
        ++len;
      } else {
        len = 0;
      }
      if (j >= kLook && q < total) {
        const int r1 = r + 1;
        const bool next_start = (bmask[r1 >> 5] >> (r1 & 31)) & 1u;
        for (int i = 0; i < kb.nk; ++i) {
          const int k = kb.k[i];
          if (len >= k && !(len == k && next_start)) {
            ++my_words[i];
            const uint32_t c = code & ((1u << (2 * k)) - 1u);
            if (kb.lds_off[i] >= 0) atomicAdd(&lds_hist[kb.lds_off[i] + c], 1u);
            else atomicAdd(&kb.counts[i][c], 1u);
          }
        }
      }
    }
  }
  for (int i = 0; i < kb.nk; ++i) {
    unsigned long long v = my_words[i];
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_down(v, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)kb.nk) {
    unsigned long long t = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += wsum[w][threadIdx.x];
    if (t) atomicAdd(&n_words[threadIdx.x], t);
  }
  for (int i = 0; i < kb.nk; ++i) {
    if (kb.lds_off[i] < 0) continue;
    const int nb = 1 << (2 * kb.k[i]);
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
      const uint32_t v = lds_hist[kb.lds_off[i] + j];
      if (v) atomicAdd(&kb.counts[i][j], v);
    }
  }
}

}  // namespace

ks_status launch_count(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const Runs &, int k,
                       int32_t *counts_dev, double *n_words) {
  hipStream_t st = ctx->stream;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_words = reinterpret_cast<unsigned long long *>(scal) + 1;
  KS_HIP(hipMemsetAsync(d_words, 0, 8, st));
  const int64_t ntiles = (total + kTile - 1) / kTile;
  if (ntiles > 0) {
    const bool lds = (k <= 7);
    int64_t grid = (int64_t)ctx->num_cus * (lds ? 2 : 8);
    if (grid > ntiles) grid = ntiles;
    if (lds) {
      hipLaunchKernelGGL(k_count<true>, dim3((unsigned)grid), dim3(256), (size_t)4 << (2 * k), st,
                         s->seq, total, s->offsets_dev, s->nseq, k, (uint32_t *)counts_dev, d_words,
                         ntiles);
    } else {
      hipLaunchKernelGGL(k_count<false>, dim3((unsigned)grid), dim3(256), 0, st, s->seq, total,
                         s->offsets_dev, s->nseq, k, (uint32_t *)counts_dev, d_words, ntiles);
    }
    KS_HIP(hipGetLastError());
  }
  unsigned long long w = 0;
  KS_HIP(hipMemcpyAsync(&w, d_words, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  *n_words = (double)w;
  return KS_OK;
}

ks_status launch_count_multi(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const int32_t *ks, int nk,
                             int32_t *const *counts_dev, double *n_words) {
  hipStream_t st = ctx->stream;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_words = reinterpret_cast<unsigned long long *>(scal) + 8;
  for (int b0 = 0; b0 < nk; b0 += kMaxBatch) {
    const int nb = std::min(kMaxBatch, nk - b0);
    KBatch kb{};
    kb.nk = nb;
    // LDS for the smallest k's first (64 KiB budget)
    std::vector<int> order(nb);
    for (int i = 0; i < nb; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int x, int y) { return ks[b0 + x] < ks[b0 + y]; });
    int words = 0;
    for (int i = 0; i < nb; ++i) {
      kb.k[i] = ks[b0 + i];
      kb.counts[i] = (uint32_t *)counts_dev[b0 + i];
      kb.lds_off[i] = -1;
    }
    for (int oi : order) {
      const int w = 1 << (2 * kb.k[oi]);
      if (kb.k[oi] <= 7 && words + w <= 16384) {
        kb.lds_off[oi] = words;
        words += w;
      }
    }
    kb.lds_words = words;
    KS_HIP(hipMemsetAsync(d_words, 0, 8 * kMaxBatch, st));
    const int64_t ntiles = (total + kTile - 1) / kTile;
    if (ntiles > 0) {
      int64_t grid = (int64_t)ctx->num_cus * (words ? 2 : 8);
      if (grid > ntiles) grid = ntiles;
      hipLaunchKernelGGL(k_count_multi, dim3((unsigned)grid), dim3(256), (size_t)words * 4, st, s->seq, total,
                         s->offsets_dev, s->nseq, kb, d_words, ntiles);
      KS_HIP(hipGetLastError());
    }
    unsigned long long w[kMaxBatch];
    KS_HIP(hipMemcpyAsync(w, d_words, 8 * kMaxBatch, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
    for (int i = 0; i < nb; ++i) n_words[b0 + i] = (double)w[i];
  }
  return KS_OK;
}

}  // namespace ks
