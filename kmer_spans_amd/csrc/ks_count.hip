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
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "ks_internal.h"
#include "ks_kmer_swar.h"

namespace ks {
namespace {

// Sequence starts in [base, lim] as bits (offs[q] - base) of the LDS bitmap,
// by the first wave: a 64-ary lower_bound over offs[0..nseq] (one dependent
// load per 64x narrowing instead of log2(nseq) single-lane loads: the tile
// loop's block waits on it), then the starts 64 at a time.
__device__ __forceinline__ void mark_seq_starts(const int64_t *__restrict__ offs, int32_t nseq, int64_t base,
                                                int64_t lim, uint32_t *bmask) {
  const int lane = threadIdx.x & 63;
  int64_t L = 0, R = (int64_t)nseq + 1;  // first i in [L, R) with offs[i] >= base, else R
  while (R - L > 64) {
    const int64_t step = (R - L + 63) / 64;
    const int64_t pv = L + lane * step;
    const bool lt = pv < R && offs[pv] < base;
    const int cnt = __popcll(__ballot(lt));
    if (cnt == 0) {
      R = L;
      break;
    }
    const int64_t last = L + (int64_t)(cnt - 1) * step;  // last pivot below base
    L = last + 1;
    R = min(R, last + step);
  }
  if (R > L) {
    const bool lt = L + lane < R && offs[L + lane] < base;
    L += __popcll(__ballot(lt));
  }
  for (int64_t q0 = L; q0 <= nseq; q0 += 64) {
    const int64_t q = q0 + lane;
    const bool in = q <= nseq && offs[q] <= lim;
    if (in) {
      const int r = (int)(offs[q] - base);
      atomicOr(&bmask[r >> 5], 1u << (r & 31));
    }
    if (__ballot(in) != __ballot(true)) break;  // offsets ascend: the rest lie past lim
  }
}

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
    if (threadIdx.x < 64) mark_seq_starts(offs, nseq, base, t0 + kTile, bmask);
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
    if (threadIdx.x < 64) mark_seq_starts(offs, nseq, base, t0 + kTile, bmask);
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

// ------------------------------------------------------------------------
// Partitioned counting for 4^k histograms far beyond L2 (k >= kPartMinK).
// Global atomics execute at the memory side (one 64-B request per 4-B add,
// MI355X_MICROARCH "Global float atomics"), so one random add per k-mer is
// bound at ~20 G adds/s.  Instead the 2k-bit code is split into a bucket
// (top T bits) and a bin (low L bits; 2^L counters fit LDS), and the k-mers
// are partitioned by bucket before each bucket is histogrammed in LDS.
// Each tile of 16K positions is counting-sorted by bucket in LDS before it
// is written, so a block appends runs (not single items) to at most 2048
// bucket tails.  One level up to k = 13 (2k - 15 <= 11 bucket bits), two
// levels beyond:
//   L1 k_part<1>   per block: LDS histogram of the top 11 bits -> mat[b][block]
//                  (exclusive sum over mat: each block's cursor per bucket)
//      k_part_scatter  same positions, same blocks: append the code's low
//                  2k - 11 bits (u32; u16 when single-level) to its bucket
//   L2 k_sub<1/2>  per level-1 bucket, C chunks: the same two passes on the
//                  next T - 11 bits, appending the bin (u16)
//   k_bins         one block per final bucket (or a share of one): LDS
//                  histogram of the bins, counts[bucket << L | bin] += h
// The k-mer test (runs, Q1) is the same code as k_count.
constexpr int kPartMinK = 11;
constexpr int kPT = 1024;            // threads per block
constexpr int kPTile = kPT * kPer;   // positions per tile
constexpr int kPBlocks = 512;        // persistent blocks, level 1
constexpr int kT1 = 11;              // level-1 bucket bits (2048 buckets: one level up to k = 13)
constexpr int kSubChunks = 8;        // level-2 blocks per level-1 bucket

struct PartGeo {
  int L, T, T1, T2;
};
inline PartGeo part_geo(int k) {
  const int B = 2 * k;
  const int L = B <= 15 ? B : 15;  // 2^15 u32 bins = 128 KiB of LDS per k_bins block
  const int T = B - L;
  const int T1 = T < kT1 ? T : kT1;
  return {L, T, T1, T - T1};
}

__global__ void k_part_sum_last(const unsigned long long *__restrict__ mat, const unsigned long long *__restrict__ ex,
                                size_t n, unsigned long long *__restrict__ last) {
  *last = ex[n - 1] + mat[n - 1];
}

// ---- lane windows of the partitioned counter.  A lane owns kPer
// consecutive positions and reads them with the kLook bytes before them (two
// 16-B loads), issued one tile ahead of use (the next tile's loads are in
// flight while this tile is processed).
struct LaneWin {
  uint4 a, b;
  bool fast;  // both loads in bounds (else the bytes are read one by one)
};

__device__ __forceinline__ void lane_load(const uint8_t *__restrict__ seq, int64_t total, int64_t p0, LaneWin &w) {
  w.fast = p0 >= kLook && p0 + kPer <= total;
  if (w.fast) {
    w.a = *reinterpret_cast<const uint4 *>(seq + p0 - kLook);
    w.b = *reinterpret_cast<const uint4 *>(seq + p0);
  }
}

// The same, always two loads (from the sequence's first bytes when the
// window is not in bounds): a loop that issues it has a fixed number of
// memory instructions per iteration.
__device__ __forceinline__ void lane_load_all(const uint8_t *__restrict__ seq, int64_t total, int64_t p0,
                                              LaneWin &w) {
  w.fast = p0 >= kLook && p0 + kPer <= total;
  const uint8_t *p = w.fast ? seq + p0 - kLook : seq;
  w.a = *reinterpret_cast<const uint4 *>(p);
  w.b = *reinterpret_cast<const uint4 *>(p + kLook);
}

// The lane's 32 bytes as 8 little-endian words (byte j = bits 8(j%4) of word j/4).
__device__ __forceinline__ void lane_bytes(const uint8_t *__restrict__ seq, int64_t total, int64_t p0,
                                           const LaneWin &w, uint32_t (&x)[8]) {
  if (w.fast) {
    x[0] = w.a.x, x[1] = w.a.y, x[2] = w.a.z, x[3] = w.a.w;
    x[4] = w.b.x, x[5] = w.b.y, x[6] = w.b.z, x[7] = w.b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = 0;
#pragma unroll
    for (int j = 0; j < kLook + kPer; ++j) {
      const int64_t q = p0 - kLook + j;
      const uint32_t c = (q >= 0 && q < total) ? seq[q] : (uint32_t)'N';
      x[j >> 2] |= c << (8 * (j & 3));
    }
  }
}

// The counted k-mers of a lane's positions: emit(i, code) for position
// p0 + i.  kStarts: some sequence starts inside the tile, marked in bmask
// (bit r = position base + r): a start resets the run, and the k-mer test
// drops a run of exactly k bases ending right before a start (Q1).  Without
// starts the tile needs neither.  Word-parallel (ks_kmer_swar.h).
static_assert(kLook == 16 && kPer == 16, "ks_kmer_swar.h: 16 look-back bytes, 16 positions per lane");
template <bool kStarts>
__device__ __forceinline__ SwarWin lane_window(const uint32_t (&x)[8], int64_t p0, int64_t total, int64_t base,
                                               const uint32_t *bmask, int k) {
  // byte j is position p0 - kLook + j: in the sequence while j < jend, bit r0 + j of bmask
  const int jend = p0 + kPer <= total ? kLook + kPer : (int)(total - (p0 - kLook));
  uint64_t sm = 0;
  if (kStarts) {
    const int r0 = (int)(p0 - kLook - base);  // (a multiple of 16: bits r0 .. r0 + 32 lie in two words)
    sm = ((((uint64_t)bmask[(r0 >> 5) + 1]) << 32) | bmask[r0 >> 5]) >> (r0 & 31);
  }
  return swar_window(x, sm, jend, k);
}

// Bucket of the lane's position i for the LDS bucket counters: positions that
// count nothing take a lane-private spare counter (index kT1 buckets + lane),
// so the counter updates need no per-position branch and never collide.
constexpr int kSpare = 64;
__device__ __forceinline__ uint32_t lane_bucket(const SwarWin &w, int i, uint32_t mask, int shift) {
  const bool on = (w.emit >> (kLook + i)) & 1u;
  return on ? swar_code(w, i, mask) >> shift : (uint32_t)((1 << kT1) + (threadIdx.x & 63));
}

// Per block, the sequence starts (offs[0..nseq], ascending) ahead of its
// tiles, which it visits in ascending order: *ci = the first index with
// offs >= base (the cursor only moves forward), *nx = that offset.
__device__ __forceinline__ void starts_seek(const int64_t *__restrict__ offs, int32_t nseq, int64_t base, int32_t *ci,
                                            int64_t *nx) {
  while (*nx < base) {
    ++*ci;
    *nx = *ci <= nseq ? offs[*ci] : INT64_MAX;
  }
}

__device__ __forceinline__ void starts_init(const int64_t *__restrict__ offs, int32_t nseq, int64_t base,
                                            int32_t *ci, int64_t *nx) {
  int32_t lo = 0, hi = nseq + 1;  // first index with offs >= base
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (offs[mid] < base) lo = mid + 1;
    else hi = mid;
  }
  *ci = lo;
  *nx = lo <= nseq ? offs[lo] : INT64_MAX;
}

// bmask for a tile holding starts (between barriers): bits of offs[ci..] <= lim.
template <int kWords>
__device__ __forceinline__ void starts_mark(const int64_t *__restrict__ offs, int32_t nseq, int32_t ci, int64_t base,
                                            int64_t lim, uint32_t *bmask) {
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) bmask[i] = 0;
  __syncthreads();
  for (int64_t q = ci + (int64_t)threadIdx.x; q <= nseq; q += blockDim.x) {
    const int64_t v = offs[q];
    if (v > lim) break;
    const int r = (int)(v - base);
    atomicOr(&bmask[r >> 5], 1u << (r & 31));
  }
  __syncthreads();
}

// Grouped region layout of the staged scatter: blocks in groups of gs, each
// group's regions bucket-major ([bucket][block of the group]).  A group spans
// under 2 GiB (a buffer-store window from its first region); a bucket is one
// contiguous segment per group.
__host__ __device__ __forceinline__ size_t grp_index(int blk, int b, int nb, int G, int gs) {
  const int g0 = blk / gs * gs, gsz = min(gs, G - g0);
  return (size_t)g0 * nb + (size_t)b * gsz + (blk - g0);
}

// Level 1 over the sequence: per block, the LDS histogram of the buckets
// (code >> shift, shift = 2k - T1) of the k-mers in its tiles, each count
// rounded up to a multiple of pad (the staged scatter writes whole pieces of
// pad items), into mat[bucket][block] (gs > 0: the grouped layout of
// grp_index); the unrounded total is added to *words.
__global__ void __launch_bounds__(kPT) k_part(const uint8_t *__restrict__ seq, int64_t total,
                                              const int64_t *__restrict__ offs, int32_t nseq, int k, int shift,
                                              unsigned long long *__restrict__ mat, int pad, int gs,
                                              unsigned long long *__restrict__ words, int64_t tile0, int64_t ntiles) {
  constexpr int kWords = (kPTile + kLook + 32) / 32 + 1;
  __shared__ uint32_t lds_b[(1 << kT1) + kSpare];
  __shared__ uint32_t bmask[kWords];
  __shared__ unsigned long long wsum[kPT / 64];
  const int nb = 1 << (2 * k - shift);
  const int G = gridDim.x;
  for (int i = threadIdx.x; i < nb; i += kPT) lds_b[i] = 0;
  if (threadIdx.x < kSpare) lds_b[(1 << kT1) + threadIdx.x] = 0;
  const uint32_t mask = (1u << (2 * k)) - 1u;
  int32_t ci = 0;
  int64_t nx = 0;
  int64_t tile = blockIdx.x;
  if (tile < ntiles) starts_init(offs, nseq, (tile0 + tile) * kPTile - kLook, &ci, &nx);
  LaneWin cur;
  if (tile < ntiles) lane_load(seq, total, (tile0 + tile) * kPTile + (int64_t)threadIdx.x * kPer, cur);
  __syncthreads();
  for (; tile < ntiles; tile += G) {
    const int64_t t0 = (tile0 + tile) * kPTile;
    const int64_t base = t0 - kLook, lim = t0 + kPTile;
    const int64_t p0 = t0 + (int64_t)threadIdx.x * kPer;
    LaneWin nxt;
    if (tile + G < ntiles) lane_load(seq, total, (tile0 + tile + G) * kPTile + (int64_t)threadIdx.x * kPer, nxt);
    starts_seek(offs, nseq, base, &ci, &nx);
    const bool st = nx <= lim;  // (uniform over the block)
    if (st) starts_mark<kWords>(offs, nseq, ci, base, lim, bmask);
    if (p0 < total) {
      uint32_t x[8];
      lane_bytes(seq, total, p0, cur, x);
      const SwarWin w = st ? lane_window<true>(x, p0, total, base, bmask, k)
                           : lane_window<false>(x, p0, total, base, bmask, k);
#pragma unroll
      for (int i = 0; i < kPer; ++i) atomicAdd(&lds_b[lane_bucket(w, i, mask, shift)], 1u);
    }
    if (st) __syncthreads();  // (bmask is rewritten by the next tile holding starts)
    cur = nxt;
  }
  __syncthreads();
  unsigned long long t = 0;
  for (int i = threadIdx.x; i < nb; i += kPT) {
    const uint32_t c = lds_b[i];
    t += c;
    mat[gs ? grp_index(blockIdx.x, i, nb, G, gs) : (size_t)i * G + blockIdx.x] =
        (c + (uint32_t)pad - 1u) / (uint32_t)pad * (uint32_t)pad;
  }
  for (int d = 32; d >= 1; d >>= 1) t += __shfl_down(t, d, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int w = 0; w < kPT / 64; ++w) s += wsum[w];
    if (s) atomicAdd(words, s);
  }
}

// Single-level scatter through a per-bucket LDS stage of kS items: every
// (block, bucket) region is a multiple of kS items (k_part with pad = kS,
// grouped: grp_index)
// starting 2*kS-byte aligned, and is written only in whole aligned pieces of
// kS items, so each HBM write request carries 2*kS bytes (round 6 at the
// metric genome's 6.2 GB of items: 16-B pieces 14.0 ms, 32-B 6.9 ms, 64-B
// no faster -- 2,048 x 32 items of stage fill 128 KiB of the 160 KiB LDS;
// the counting-sort scatter below writes ~4 items per bucket and sub-tile:
// 27.5 GB of partial writes).  The per-bucket fill counters are 16-bit halves
// of words (a sub-tile adds at most 16 K items).
// Per sub-tile: a k-mer takes slot = fill[bucket]++ (LDS atomic); slots < kS
// go to the stage, the rest stay in registers; buckets that reach kS flush
// the stage's piece (16-B stores), the registers' slots below the last whole
// piece go straight out (lanes of one wave hold consecutive slots of a hot
// bucket, so those stores coalesce) and the remainder moves into the stage.
// The bucket state (fill, cursor) is double-buffered: the flush writes the
// next sub-tile's state while the register phase still reads this one, two
// barriers per sub-tile.  The block's last remainders go out padded with
// kSentinel, which k_bins skips.
constexpr uint16_t kSentinel = 0xffffu;  // payloads are < 2^15 on the single level
__device__ __forceinline__ uint32_t fill_get(const uint32_t *f, uint32_t b) {
  return (f[b >> 1] >> ((b & 1u) << 4)) & 0xffffu;
}
template <int kS, int kT>
__global__ void __launch_bounds__(kT) k_part_scatter_st(const uint8_t *__restrict__ seq, int64_t total,
                                                         const int64_t *__restrict__ offs, int32_t nseq, int k,
                                                         int shift, const unsigned long long *__restrict__ ex,
                                                         int gs, uint16_t *__restrict__ part, int64_t tile0,
                                                         int64_t ntiles) {
  constexpr int kTile = kT * kPer;  // positions per sub-tile
  constexpr int kSub = kPTile / kTile;
  constexpr int kV = kS / 8;        // 16-B vectors per piece
  constexpr int kWords = (kTile + kLook + 32) / 32 + 1;
  constexpr int kFW = ((1 << kT1) + kSpare) / 2;  // fill words (two 16-bit counters each)
  constexpr uint32_t kDrop = 0x80000000u;         // a store offset past the window: the store is dropped
  static_assert(kPTile % kTile == 0 && kS % 8 == 0 && kTile + kS < 65536, "sub-tiles, pieces, 16-bit fills");
  static_assert(kT >= (1 << kT1) / 2, "one thread per fill word");
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  uint16_t *stage = reinterpret_cast<uint16_t *>(dyn);  // [nb][kS]
  __shared__ uint32_t fill[2][kFW], cur[2][1 << kT1];
  __shared__ uint32_t bmask[kWords];
  const int nb = 1 << (2 * k - shift);  // (even: k >= kPartMinK)
  const int G = gridDim.x;
  // the block's group's regions lie in one window of under 2 GiB from the
  // group's first region on; cursors are item offsets in the window
  const unsigned long long wbase = ex[(size_t)(blockIdx.x / gs * gs) * nb];
  const __amdgpu_buffer_rsrc_t win_rs = __builtin_amdgcn_make_buffer_rsrc(part + wbase, (short)0, 0x7fffffff, 0x00020000);
  for (int i = threadIdx.x; i < kFW; i += kT) fill[0][i] = fill[1][i] = 0;
  for (int i = threadIdx.x; i < nb; i += kT) cur[0][i] = (uint32_t)(ex[grp_index(blockIdx.x, i, nb, G, gs)] - wbase);
  const uint32_t mask = (1u << (2 * k)) - 1u;
  const uint32_t pmask = (1u << shift) - 1u;
  // the positions k_part's block counted: its kPTile-position tiles, each as
  // kSub sub-tiles in order; iteration it = (tile index - blockIdx.x) / G * kSub + sub
  const int64_t nit = blockIdx.x < ntiles ? ((ntiles - 1 - blockIdx.x) / G + 1) * kSub : 0;
  auto sub_t0 = [&](int64_t it) { return (tile0 + blockIdx.x + (it / kSub) * G) * kPTile + (it % kSub) * kTile; };
  int32_t ci = 0;
  int64_t nx = 0;
  LaneWin win;
  if (nit) {
    starts_init(offs, nseq, sub_t0(0) - kLook, &ci, &nx);
    lane_load_all(seq, total, sub_t0(0) + (int64_t)threadIdx.x * kPer, win);
    // (the first window waited for here: the loop's waits then need not
    // cover loads from before the loop, which would drain its stores)
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
  }
  // Every iteration issues the same memory instructions -- two window loads,
  // kV stores per fill-word half, kPer register-slot stores -- with the
  // stores that have nothing to write dropped by offset, not skipped by a
  // branch: the wait for the next window then counts past this iteration's
  // stores instead of draining them (gfx9 counts loads and stores on one
  // in-order counter).
  int ph = 0;
  for (int64_t it = 0; it < nit; ++it, ph ^= 1) {
    const int64_t t0 = sub_t0(it);
    const int64_t base = t0 - kLook, lim = t0 + kTile;
    const int64_t p0 = t0 + (int64_t)threadIdx.x * kPer;
    LaneWin nxt;
    lane_load_all(seq, total, sub_t0(it + 1 < nit ? it + 1 : it) + (int64_t)threadIdx.x * kPer, nxt);
    starts_seek(offs, nseq, base, &ci, &nx);
    const bool st = nx <= lim;  // (uniform over the block)
    __syncthreads();            // this phase's state is complete (init, or the last flush)
    if (st) starts_mark<kWords>(offs, nseq, ci, base, lim, bmask);
    uint32_t *fl = fill[ph], *cu = cur[ph];
    uint32_t br[kPer];    // bucket << 16 | slot of the items left in registers, or ~0u
    uint32_t pay[kPer / 2] = {};  // their payloads, two per word
#pragma unroll
    for (int j = 0; j < kPer; ++j) br[j] = ~0u;
    if (p0 < total) {
      uint32_t x[8];
      lane_bytes(seq, total, p0, win, x);
      const SwarWin w = st ? lane_window<true>(x, p0, total, base, bmask, k)
                           : lane_window<false>(x, p0, total, base, bmask, k);
      // the lane's 16 slot atomics back to back (one wait for all of them,
      // not one LDS round trip per position), then the stage stores
      uint32_t slot[kPer];
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const uint32_t b = lane_bucket(w, i, mask, shift), sh = (b & 1u) << 4;
        slot[i] = ((atomicAdd(&fl[b >> 1], 1u << sh)) >> sh) & 0xffffu;
      }
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        if (!((w.emit >> (kLook + i)) & 1u)) continue;
        const uint32_t code = swar_code(w, i, mask);
        const uint32_t bk = code >> shift, v = code & pmask;
        if (slot[i] < (uint32_t)kS) {
          stage[bk * kS + slot[i]] = (uint16_t)v;
        } else {
          br[i] = (bk << 16) | slot[i];
          pay[i >> 1] = (i & 1) ? ((pay[i >> 1] & 0xffffu) | (v << 16)) : ((pay[i >> 1] & 0xffff0000u) | v);
        }
      }
    }
    __syncthreads();
    // whole stage pieces out; the next sub-tile's state (a thread per fill
    // word: its two buckets)
    uint32_t *fl2 = fill[ph ^ 1], *cu2 = cur[ph ^ 1];
    {
      const int wd = threadIdx.x;
      const bool own = wd < nb / 2;
      const uint32_t fw = own ? fl[wd] : 0u;
      uint32_t nf = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = own ? 2 * wd + h : 0;
        const uint32_t f = (fw >> (16 * h)) & 0xffffu, c = cu[i];
        const uint32_t F = f / kS * kS;
        const uint4 *src = reinterpret_cast<const uint4 *>(stage + i * kS);
        const uint32_t off = f >= (uint32_t)kS ? c * 2u : kDrop;
#pragma unroll
        for (int v = 0; v < kV; ++v) {
          const uint4 y = src[v];
          const u32x4 yv = {y.x, y.y, y.z, y.w};
          __builtin_amdgcn_raw_buffer_store_b128(yv, win_rs, off + 16 * v, 0, 0);
        }
        nf |= (f - F) << (16 * h);
        if (own) cu2[i] = c + F;
      }
      if (own) fl2[wd] = nf;
    }
    if (threadIdx.x < kSpare / 2) fl2[(1 << kT1) / 2 + threadIdx.x] = 0;
    __syncthreads();
    // register slots: below the last whole piece straight out, the rest staged
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      uint32_t off = kDrop;
      const uint16_t v = (uint16_t)(pay[j >> 1] >> (16 * (j & 1)));
      if (br[j] != ~0u) {
        const uint32_t bk = br[j] >> 16, slot = br[j] & 0xffffu;
        const uint32_t F = fill_get(fl, bk) / kS * kS;
        if (slot < F) off = (cu[bk] + slot) * 2u;
        else stage[bk * kS + slot - F] = v;
      }
      __builtin_amdgcn_raw_buffer_store_b16(v, win_rs, off, 0, 0);
    }
    win = nxt;
  }
  __syncthreads();
  // the block's remainders, padded to a whole piece
  uint16_t *wpart = part + wbase;
  for (int i = threadIdx.x; i < nb; i += kT) {
    const uint32_t f = fill_get(fill[ph], i);
    if (f == 0) continue;
    uint4 *dst = reinterpret_cast<uint4 *>(wpart + cur[ph][i]);
    for (int v = 0; v < kV; ++v) {
      uint32_t w[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t e0 = v * 8 + 2 * h, e1 = e0 + 1;
        const uint32_t lo = e0 < f ? stage[i * kS + e0] : kSentinel;
        const uint32_t hi = e1 < f ? stage[i * kS + e1] : kSentinel;
        w[h] = lo | (hi << 16);
      }
      dst[v] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// Level-1 scatter.  Per 16K-position tile the block ranks its k-mers by
// bucket in LDS (counting sort), then writes each bucket's run of payloads
// contiguously at the block's cursor: consecutive lanes store consecutive
// addresses (a lane-per-k-mer scatter issues one memory request per k-mer
// and is request-bound at ~100 G/s).
template <typename Item, int kT>
__global__ void __launch_bounds__(kT) k_part_scatter(const uint8_t *__restrict__ seq, int64_t total,
                                                      const int64_t *__restrict__ offs, int32_t nseq, int k, int shift,
                                                      const unsigned long long *__restrict__ ex,
                                                      Item *__restrict__ part, int64_t tile0, int64_t ntiles) {
  constexpr int kTile = kT * kPer;  // positions per sub-tile
  static_assert(kPTile % kTile == 0, "sub-tiles");
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  Item *sorted = reinterpret_cast<Item *>(dyn);               // [kTile]
  uint16_t *bkt = reinterpret_cast<uint16_t *>(dyn + sizeof(Item) * kTile);  // [kTile]
  __shared__ unsigned long long cur[1 << kT1];
  __shared__ uint32_t cnt[1 << kT1], off[1 << kT1];
  __shared__ uint32_t wtot[kT / 64];
  __shared__ uint32_t bmask[(kTile + kLook + 32) / 32 + 1];
  const int nb = 1 << (2 * k - shift);
  const int G = gridDim.x;
  for (int i = threadIdx.x; i < nb; i += kT) cur[i] = ex[(size_t)i * G + blockIdx.x];
  const uint32_t mask = (1u << (2 * k)) - 1u;
  const uint32_t pmask = (1u << shift) - 1u;
  // the positions k_part<1>'s block counted: its kPTile-position tiles, each
  // as kPTile / kTile sub-tiles in order
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += G) {
    for (int sub = 0; sub < kPTile / kTile; ++sub) {
      const int64_t t0 = (tile0 + tile) * kPTile + (int64_t)sub * kTile;
      const int64_t base = t0 - kLook;
      __syncthreads();
      for (int i = threadIdx.x; i < (kTile + kLook + 32) / 32 + 1; i += kT) bmask[i] = 0;
      for (int i = threadIdx.x; i < nb; i += kT) cnt[i] = 0;
      __syncthreads();
      if (threadIdx.x < 64) mark_seq_starts(offs, nseq, base, t0 + kTile, bmask);
      __syncthreads();
      const int64_t p0 = t0 + (int64_t)threadIdx.x * kPer;
      uint32_t br[kPer];   // bucket << 16 | rank, or ~0u
      uint32_t pay[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) br[j] = ~0u;
      if (p0 < total) {
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
          if (j >= kLook && q < total && len >= k) {
            const int r1 = r + 1;
            const bool q1 = (len == k) && ((bmask[r1 >> 5] >> (r1 & 31)) & 1u);
            if (!q1) {
              const uint32_t bk = code >> shift;
              br[j - kLook] = (bk << 16) | atomicAdd(&cnt[bk], 1u);
              pay[j - kLook] = code & pmask;
            }
          }
        }
      }
      __syncthreads();
      {  // exclusive scan of the (<= 2048) bucket counts: two per thread, wave
         // scans, then the 16 wave totals
        constexpr int kPerT = (1 << kT1) / kT;
        static_assert(kPerT * kT == (1 << kT1), "buckets per thread");
        uint32_t v[kPerT], sum = 0;
#pragma unroll
        for (int i = 0; i < kPerT; ++i) {
          const int bi = threadIdx.x * kPerT + i;
          v[i] = bi < nb ? cnt[bi] : 0;
          sum += v[i];
        }
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        uint32_t inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t o = __shfl_up(inc, d, 64);
          if (lane >= d) inc += o;
        }
        if (lane == 63) wtot[wv] = inc;
        __syncthreads();
        if (threadIdx.x < 64) {
          uint32_t t = threadIdx.x < kT / 64 ? wtot[threadIdx.x] : 0, ti = t;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(ti, d, 64);
            if ((int)threadIdx.x >= d) ti += o;
          }
          if (threadIdx.x < kT / 64) wtot[threadIdx.x] = ti - t;  // exclusive
        }
        __syncthreads();
        uint32_t run = wtot[wv] + inc - sum;
#pragma unroll
        for (int i = 0; i < kPerT; ++i) {
          const int bi = threadIdx.x * kPerT + i;
          if (bi < nb) off[bi] = run;
          run += v[i];
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (br[j] != ~0u) {
          const uint32_t bk = br[j] >> 16, pos = off[bk] + (br[j] & 0xffffu);
          sorted[pos] = (Item)pay[j];
          bkt[pos] = (uint16_t)bk;
        }
      __syncthreads();
      const uint32_t n_items = off[nb - 1] + cnt[nb - 1];
      for (uint32_t i = threadIdx.x; i < n_items; i += kT) {
        const uint32_t bk = bkt[i];
        part[cur[bk] + (i - off[bk])] = sorted[i];
      }
      __syncthreads();
      for (int i = threadIdx.x; i < nb; i += kT) cur[i] += cnt[i];
    }
  }
}

// Level-2 scatter: the same tile-local counting sort on the items of one
// level-1 bucket chunk, by sub-bucket (<= 128), writing the u16 bins.
__global__ void __launch_bounds__(kPT) k_sub_scatter(const uint32_t *__restrict__ rem,
                                                     const unsigned long long *__restrict__ s1, int C, int L, int T2,
                                                     const unsigned long long *__restrict__ ex2,
                                                     uint16_t *__restrict__ out) {
  __shared__ uint16_t sorted[kPTile];
  __shared__ uint8_t bkt[kPTile];
  __shared__ unsigned long long cur[128];
  __shared__ uint32_t cnt[128], off[128];
  const int b1 = blockIdx.x / C, c = blockIdx.x % C;
  const int ns = 1 << T2;
  const unsigned long long a0 = s1[b1], n = s1[b1 + 1] - a0;
  const unsigned long long a = a0 + n * c / C, e = a0 + n * (c + 1) / C;
  for (int i = threadIdx.x; i < ns; i += kPT) cur[i] = ex2[((((size_t)b1 << T2) | i) * C) + c];
  const uint32_t lmask = (1u << L) - 1u;
  for (unsigned long long t0 = a; t0 < e; t0 += kPTile) {
    __syncthreads();
    for (int i = threadIdx.x; i < ns; i += kPT) cnt[i] = 0;
    __syncthreads();
    uint32_t br[kPer], pay[kPer];
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const unsigned long long i = t0 + (unsigned long long)j * kPT + threadIdx.x;
      br[j] = ~0u;
      if (i < e) {
        const uint32_t v = rem[i];
        const uint32_t sb = v >> L;
        br[j] = (sb << 16) | atomicAdd(&cnt[sb], 1u);
        pay[j] = v & lmask;
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      uint32_t v0 = threadIdx.x * 2 < (unsigned)ns ? cnt[threadIdx.x * 2] : 0;
      uint32_t v1 = threadIdx.x * 2 + 1 < (unsigned)ns ? cnt[threadIdx.x * 2 + 1] : 0;
      uint32_t inc = v0 + v1;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if ((int)threadIdx.x >= d) inc += o;
      }
      const uint32_t ex = inc - v0 - v1;
      if (threadIdx.x * 2 < (unsigned)ns) off[threadIdx.x * 2] = ex;
      if (threadIdx.x * 2 + 1 < (unsigned)ns) off[threadIdx.x * 2 + 1] = ex + v0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (br[j] != ~0u) {
        const uint32_t sb = br[j] >> 16, pos = off[sb] + (br[j] & 0xffffu);
        sorted[pos] = (uint16_t)pay[j];
        bkt[pos] = (uint8_t)sb;
      }
    __syncthreads();
    const uint32_t n_items = off[ns - 1] + cnt[ns - 1];
    for (uint32_t i = threadIdx.x; i < n_items; i += kPT) {
      const uint32_t sb = bkt[i];
      out[cur[sb] + (i - off[sb])] = sorted[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ns; i += kPT) cur[i] += cnt[i];
  }
}

// Level 2 inside level-1 bucket b1 = blockIdx.x / C, chunk c of C:
// sub-bucket = rem >> L (T2 bits), bin = rem & (2^L - 1).  mat2 index
// ((b1 << T2) | sub) * C + c, so its exclusive sum orders the final buckets.
template <int kPass>
__global__ void __launch_bounds__(kPT) k_sub(const uint32_t *__restrict__ rem,
                                             const unsigned long long *__restrict__ s1, int C, int L, int T2,
                                             unsigned long long *__restrict__ mat2,
                                             const unsigned long long *__restrict__ bstart2,
                                             uint16_t *__restrict__ out) {
  __shared__ uint32_t cur[128];
  const int b1 = blockIdx.x / C, c = blockIdx.x % C;
  const int ns = 1 << T2;
  const unsigned long long a0 = s1[b1], n = s1[b1 + 1] - a0;
  const unsigned long long a = a0 + n * c / C, e = a0 + n * (c + 1) / C;
  if (kPass == 1) {
    for (int i = threadIdx.x; i < ns; i += kPT) cur[i] = 0;
  } else {
    for (int i = threadIdx.x; i < ns; i += kPT) {
      const size_t fb = ((size_t)b1 << T2) | i;
      cur[i] = (uint32_t)(mat2[fb * C + c] - bstart2[fb]);
    }
  }
  __syncthreads();
  const uint32_t lmask = (1u << L) - 1u;
  for (unsigned long long i = a + threadIdx.x; i < e; i += kPT) {
    const uint32_t v = rem[i];
    const uint32_t sb = v >> L;
    if (kPass == 1) {
      atomicAdd(&cur[sb], 1u);
    } else {
      const uint32_t slot = atomicAdd(&cur[sb], 1u);
      out[bstart2[((size_t)b1 << T2) | sb] + slot] = (uint16_t)(v & lmask);
    }
  }
  if (kPass == 1) {
    __syncthreads();
    for (int i = threadIdx.x; i < ns; i += kPT) mat2[((((size_t)b1 << T2) | i) * C) + c] = cur[i];
  }
}

// bstart[i] = ex[i * stride] (exclusive sums of each bucket's first
// block); bstart[nb] = total.
__global__ void k_part_starts(const unsigned long long *__restrict__ ex, int stride, int nb,
                              unsigned long long *__restrict__ bstart, const unsigned long long *__restrict__ last) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb) bstart[i] = ex[(size_t)i * stride];
  if (i == nb) bstart[nb] = *last;
}

// Bucket sizes of the grouped layout (grp_index): the sum over groups of
// the bucket's segment, a thread per bucket.
__global__ void k_bucket_tot(const unsigned long long *__restrict__ mat, const unsigned long long *__restrict__ ex,
                             int G, int gs, int nb, unsigned long long *__restrict__ bsize) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  unsigned long long t = 0;
  for (int g0 = 0; g0 < G; g0 += gs) {
    const size_t i0 = grp_index(g0, b, nb, G, gs), i1 = i0 + min(gs, G - g0) - 1;
    t += ex[i1] + mat[i1] - ex[i0];
  }
  bsize[b] = t;
}

// Work list of k_bins (one block, nb <= 4096): the non-empty buckets in
// descending size (bitonic sort of (size, index) keys in LDS), each cut into
// shares = ceil(size / target) blocks of about target items, target = the
// mean share of 2048 blocks.  The largest buckets -- the all-A / all-T
// prefixes hold 6.5x the mean at the metric genome, mostly runs of one
// k-mer -- no longer end the kernel as one block each.  work[i] = bucket |
// share << 12 | shares << 22 for block i < *nwork.
constexpr int kWorkMax = 4096 + 2048;
// Bucket sizes from bstart (contiguous buckets) or, when bsize is given,
// from bsize with *btotal their sum (segmented buckets).
__global__ void __launch_bounds__(1024) k_bins_work(const unsigned long long *__restrict__ bstart,
                                                    const unsigned long long *__restrict__ bsize,
                                                    const unsigned long long *__restrict__ btotal, int nb,
                                                    uint32_t *__restrict__ work, uint32_t *__restrict__ nwork) {
  __shared__ unsigned long long key[4096];
  __shared__ uint32_t shs[4096];
  __shared__ uint32_t wsum[16];
  auto size_of = [&](int b) -> unsigned long long { return bsize ? bsize[b] : bstart[b + 1] - bstart[b]; };
  const unsigned long long tot = bsize ? *btotal : bstart[nb] - bstart[0];
  const unsigned long long target = tot / 2048 + 1;
  for (int i = threadIdx.x; i < 4096; i += 1024) {
    const unsigned long long sz = i < nb ? size_of(i) : 0;
    key[i] = ((0xffffffffull - (sz > 0xffffffffull ? 0xffffffffull : sz)) << 12) | (unsigned)(i & 4095);
  }
  __syncthreads();
  for (int kk = 2; kk <= 4096; kk <<= 1)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < 4096; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long x = key[i], y = key[l];
          const bool up = (i & kk) == 0;
          if ((x > y) == up) {
            key[i] = y;
            key[l] = x;
          }
        }
      }
      __syncthreads();
    }
  // shares of the r-th largest bucket, then an exclusive scan over r
  for (int r = threadIdx.x; r < 4096; r += 1024) {
    const int b = (int)(key[r] & 4095);
    const unsigned long long sz = b < nb ? size_of(b) : 0;
    shs[r] = sz ? (uint32_t)min<unsigned long long>((sz + target - 1) / target, 1023) : 0;
  }
  __syncthreads();
  // block scan of 4096 values: 4 per thread
  uint32_t v[4], t = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = shs[threadIdx.x * 4 + q];
    t += v[q];
  }
  uint32_t inc = t;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t base = 0;
  for (int w = 0; w < wv; ++w) base += wsum[w];
  uint32_t pos = base + inc - t;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = threadIdx.x * 4 + q;
    const uint32_t b = (uint32_t)(key[r] & 4095);
    for (uint32_t j = 0; j < v[q]; ++j) work[pos + j] = b | (j << 12) | (v[q] << 22);
    pos += v[q];
  }
  if (threadIdx.x == 1023) *nwork = pos;
}

// One block per work item (bucket, share of its items): the LDS histogram of
// the share's bins, added to counts[bucket << L | bin] (a bucket's only share
// owns those counters; shares of a cut bucket add with atomics).  Runs of
// equal items (the hot buckets' single-k-mer runs) are added once per run of
// a lane's 8 items.  kSentinel (the staged scatter's padding) is skipped.
// Grouped buckets (sex given: the staged scatter's grp_index layout; bstart
// is then the bucket sizes): bucket b is one contiguous segment per group of
// gs blocks, [sex[i0], sex[i1] + smat[i1]) for its first and last region of
// the group; share s of split takes [size s / split, size (s + 1) / split)
// of the segments' concatenation.
__global__ void __launch_bounds__(kPT) k_bins(const uint16_t *__restrict__ part,
                                              const unsigned long long *__restrict__ bstart, int L,
                                              uint32_t *__restrict__ counts, const uint32_t *__restrict__ work,
                                              const uint32_t *__restrict__ nwork,
                                              const unsigned long long *__restrict__ sex,
                                              const unsigned long long *__restrict__ smat, int G, int gs, int snb) {
  extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // [2^L]
  // (no work list: block = bucket, one share; the two-level counts' 2^13-2^15 buckets)
  if (work && blockIdx.x >= *nwork) return;
  const uint32_t wi = work ? work[blockIdx.x] : (1u << 22);
  const int bucket = work ? (int)(wi & 4095) : (int)blockIdx.x;
  const int s = (int)((wi >> 12) & 1023), split = (int)(wi >> 22);
  const int nbin = 1 << L;
  for (int i = threadIdx.x; i < nbin; i += kPT) h[i] = 0;
  __syncthreads();
  auto add8 = [&](const uint4 &x) {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
    uint32_t cur = w[0] & 0xffffu, run = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t y = (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
      if (y != cur) {
        if (cur != kSentinel) atomicAdd(&h[cur], run);
        cur = y;
        run = 0;
      }
      ++run;
    }
    if (cur != kSentinel) atomicAdd(&h[cur], run);
  };
  // the items [a, e) of part (head and tail one by one, the aligned body
  // 8 per 16-byte load)
  auto range = [&](unsigned long long a, unsigned long long e) {
    unsigned long long ah = (a + 7) & ~7ull;
    if (ah > e) ah = e;
    const unsigned long long eb = ah + ((e - ah) & ~7ull);
    for (unsigned long long i = a + threadIdx.x; i < ah; i += kPT)
      if (part[i] != kSentinel) atomicAdd(&h[part[i]], 1u);
    for (unsigned long long i = eb + threadIdx.x; i < e; i += kPT)
      if (part[i] != kSentinel) atomicAdd(&h[part[i]], 1u);
    const uint4 *v = reinterpret_cast<const uint4 *>(part + ah);
    const unsigned long long nv = (eb - ah) / 8;
    unsigned long long i = threadIdx.x;
    for (; i + 3 * kPT < nv; i += 4 * kPT) {  // four loads in flight per lane
      const uint4 x0 = v[i], x1 = v[i + kPT], x2 = v[i + 2 * kPT], x3 = v[i + 3 * kPT];
      add8(x0);
      add8(x1);
      add8(x2);
      add8(x3);
    }
    for (; i < nv; i += kPT) add8(v[i]);
  };
  if (sex) {
    const unsigned long long tot = bstart[bucket];
    const unsigned long long vs = tot * s / split, ve = tot * (s + 1) / split;
    unsigned long long vo = 0;
    for (int g0 = 0; g0 < G && vo < ve; g0 += gs) {
      const size_t i0 = grp_index(g0, bucket, snb, G, gs), i1 = i0 + min(gs, G - g0) - 1;
      const unsigned long long st = sex[i0], len = sex[i1] + smat[i1] - st;
      const unsigned long long lo = vs > vo ? vs : vo, hi = ve < vo + len ? ve : vo + len;
      if (lo < hi) range(st + lo - vo, st + hi - vo);
      vo += len;
    }
  } else {
    const unsigned long long a0 = bstart[bucket], n = bstart[bucket + 1] - a0;
    range(a0 + n * s / split, a0 + n * (s + 1) / split);
  }
  __syncthreads();
  uint32_t *out = counts + ((size_t)bucket << L);
  if (split == 1) {
    for (int i = threadIdx.x; i < nbin; i += kPT) {
      const uint32_t c = h[i];
      if (c) out[i] += c;
    }
  } else {
    for (int i = threadIdx.x; i < nbin; i += kPT) {
      const uint32_t c = h[i];
      if (c) atomicAdd(&out[i], c);
    }
  }
}

}  // namespace

// Partitioned count of one k into counts_dev (accumulated): the k-mers
// ending at positions [p_lo, total) (p_lo a multiple of kPTile; the bytes
// before p_lo are read as their left context), on stream st.  n_words null:
// no read-back of the k-mer total (and no synchronisation).
static ks_status count_partitioned(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, int32_t *counts_dev,
                                   double *n_words, int64_t p_lo = 0, hipStream_t st = nullptr) {
  if (!st) st = ctx->stream;
  const PartGeo g = part_geo(k);
  const int nb1 = 1 << g.T1, nbf = 1 << g.T;
  const int shift = 2 * k - g.T1;
  const int64_t tile0 = p_lo / kPTile;
  const int64_t ntiles = (total + kPTile - 1) / kPTile - tile0;
  const int G = (int)std::max<int64_t>(1, std::min<int64_t>(kPBlocks, ntiles));
  const int C = kSubChunks;
  const size_t m1 = (size_t)nb1 * G, m2 = g.T2 ? (size_t)nbf * C : 0;
  void *w = nullptr, *p1 = nullptr, *p2 = nullptr, *tmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_CHUNK_A, (m1 * 2 + m2 * 2 + nb1 + nbf + 8) * 8, &w));
  unsigned long long *mat1 = static_cast<unsigned long long *>(w);
  unsigned long long *ex1 = mat1 + m1;
  unsigned long long *mat2 = ex1 + m1;
  unsigned long long *ex2 = mat2 + m2;
  unsigned long long *s1 = ex2 + m2;            // [nb1 + 1]
  unsigned long long *sf = s1 + nb1 + 1;        // [nbf + 1]
  unsigned long long *last = sf + nbf + 1;      // [2]: level ends; [2]: the k-mer total
  // single level: the staged scatter, 16-item (32-B) pieces x 1024 lanes
  // (A/Bs in DESIGN.md: the counting-sort scatter below, 512-lane staging;
  // 8-item pieces 14.0 vs 9.9 ms, 32-item pieces 10.67 vs 10.51 ms per count,
  // profiles/r6/count/)
  const int stS = 16;
  const int64_t n_items = total - p_lo;
  // (groups of gs blocks, 8 groups at full size: group windows under 2 GiB,
  // the staged scatter's buffer-store offsets)
  const int gs = (G + 7) / 8;
  const int64_t grp_items = (((ntiles + G - 1) / G) * kPTile + (int64_t)nb1 * stS) * gs;
  const bool staged = !g.T2 && stS > 0 && n_items + (int64_t)m1 * stS < ((int64_t)1 << 32) &&
                      grp_items * 2 < ((int64_t)1 << 31) - 64 && total >= kLook + kPer;
  const int pad = staged ? stS : 1;
  const size_t item1 = g.T2 ? 4 : 2;
  KS_TRY(ensure(ctx, SLOT_CHUNK_B, (size_t)(n_items + (int64_t)m1 * (pad - 1)) * item1 + 64, &p1));
  if (g.T2) KS_TRY(ensure(ctx, SLOT_CHUNK_C, (size_t)n_items * 2 + 64, &p2));
  size_t tb = 0, tb2 = 0;
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, mat1, ex1, (int64_t)m1, st));
  if (m2) KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, mat2, ex2, (int64_t)m2, st));
  tb = std::max(tb, tb2);
  KS_TRY(ensure(ctx, SLOT_SORT_TMP, tb + 16, &tmp));
  // level 1
  KS_HIP(hipMemsetAsync(last + 2, 0, 8, st));
  hipLaunchKernelGGL(k_part, dim3(G), dim3(kPT), 0, st, s->seq, total, s->offsets_dev, s->nseq, k, shift, mat1, pad,
                     staged ? gs : 0, last + 2, tile0, ntiles);
  KS_HIP(hipGetLastError());
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, mat1, ex1, (int64_t)m1, st));
  hipLaunchKernelGGL(k_part_sum_last, dim3(1), dim3(1), 0, st, mat1, ex1, m1, last);
  if (staged) hipLaunchKernelGGL(k_bucket_tot, dim3((nb1 + 255) / 256), dim3(256), 0, st, mat1, ex1, G, gs, nb1, s1);
  else hipLaunchKernelGGL(k_part_starts, dim3((nb1 + 1 + 255) / 256), dim3(256), 0, st, ex1, G, nb1, s1, last);
  if (g.T2) {
    const size_t lds = (size_t)kPTile * (4 + 2);  // items + u16 bucket tags
    KS_HIP(hipFuncSetAttribute((const void *)k_part_scatter<uint32_t, kPT>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_part_scatter<uint32_t, kPT>), dim3(G), dim3(kPT), lds, st, s->seq, total, s->offsets_dev, s->nseq,
                       k, shift, ex1, static_cast<uint32_t *>(p1), tile0, ntiles);
  } else if (staged) {
    const size_t lds = (size_t)nb1 * stS * 2;
#define KS_ST(S, T)                                                                                          \
  do {                                                                                                       \
    KS_HIP(hipFuncSetAttribute((const void *)k_part_scatter_st<S, T>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                               (int)lds));                                                                   \
    hipLaunchKernelGGL((k_part_scatter_st<S, T>), dim3(G), dim3(T), lds, st, s->seq, total, s->offsets_dev, s->nseq, \
                       k, shift, ex1, gs, static_cast<uint16_t *>(p1), tile0, ntiles);                       \
  } while (0)
    KS_ST(16, kPT);
#undef KS_ST
  } else {
    // single level (k <= 13) past the staged scatter's index range: 512-lane
    // blocks on 8K-position sub-tiles, half the LDS, two blocks per CU
    const size_t lds = (size_t)(kPT / 2) * kPer * (2 + 2);
    KS_HIP(hipFuncSetAttribute((const void *)k_part_scatter<uint16_t, kPT / 2>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_part_scatter<uint16_t, kPT / 2>), dim3(G), dim3(kPT / 2), lds, st, s->seq, total,
                       s->offsets_dev, s->nseq, k, shift, ex1, static_cast<uint16_t *>(p1), tile0, ntiles);
  }
  KS_HIP(hipGetLastError());
  const uint16_t *bins = static_cast<const uint16_t *>(p1);
  unsigned long long *bstart = s1;
  if (g.T2) {
    // level 2
    hipLaunchKernelGGL(k_sub<1>, dim3(nb1 * C), dim3(kPT), 0, st, static_cast<const uint32_t *>(p1), s1, C, g.L,
                       g.T2, mat2, nullptr, nullptr);
    KS_HIP(hipGetLastError());
    KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, mat2, ex2, (int64_t)m2, st));
    hipLaunchKernelGGL(k_part_sum_last, dim3(1), dim3(1), 0, st, mat2, ex2, m2, last + 1);
    hipLaunchKernelGGL(k_part_starts, dim3((nbf + 1 + 255) / 256), dim3(256), 0, st, ex2, C, nbf, sf, last + 1);
    hipLaunchKernelGGL(k_sub_scatter, dim3(nb1 * C), dim3(kPT), 0, st, static_cast<const uint32_t *>(p1), s1, C, g.L,
                       g.T2, ex2, static_cast<uint16_t *>(p2));
    KS_HIP(hipGetLastError());
    bins = static_cast<const uint16_t *>(p2);
    bstart = sf;
  }
  // k_bins over a device work list (nbf <= 4096 buckets)
  const size_t lds_h = (size_t)4 << g.L;
  KS_HIP(hipFuncSetAttribute((const void *)k_bins, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_h));
  if (nbf > 4096) {  // two-level counts (k >= 14): a block per final bucket
    hipLaunchKernelGGL(k_bins, dim3((unsigned)nbf), dim3(kPT), lds_h, st, bins, bstart, g.L, (uint32_t *)counts_dev,
                       nullptr, nullptr, nullptr, nullptr, 0, 1, 0);
  } else {
    void *ob = nullptr;
    KS_TRY(ensure(ctx, SLOT_CHUNK_D, (size_t)(kWorkMax + 16) * 4, &ob));
    uint32_t *work = static_cast<uint32_t *>(ob), *nwork = work + kWorkMax;
    // (staged: s1 holds the bucket sizes, last[0] their sum, and each
    // bucket is a segment per group of the grouped regions)
    hipLaunchKernelGGL(k_bins_work, dim3(1), dim3(1024), 0, st, bstart, staged ? s1 : nullptr, last, nbf, work,
                       nwork);
    KS_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_bins, dim3((unsigned)(nbf + 2048)), dim3(kPT), lds_h, st, bins, bstart, g.L,
                       (uint32_t *)counts_dev, work, nwork, staged ? ex1 : nullptr, mat1, G, gs, nb1);
  }
  KS_HIP(hipGetLastError());
  if (!n_words) return KS_OK;
  unsigned long long words = 0;
  KS_HIP(hipMemcpyAsync(&words, last + 2, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  *n_words = (double)words;
  return KS_OK;
}

bool count_range_ok(int k, int64_t total) {
  return k >= kPartMinK && total > 0 && total < ((int64_t)1 << 32);
}

int64_t count_range_align() { return kPTile; }

namespace {
// Sum of a histogram's counts read as uint32 (wave sums, one atomic per wave).
__global__ void __launch_bounds__(256) k_sum_u32(const uint32_t *__restrict__ c, int64_t n,
                                                 unsigned long long *__restrict__ out) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += c[i];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(out, s);
}
}  // namespace

// The words counted into a histogram (sequence_kmer_count's return, summed as
// the callers do, kmer_spans.c:592-601) from the histogram itself: exact when
// no count can reach 2^32, i.e. for any total < 2^32 (count_range_ok).
ks_status count_words(ks_ctx *ctx, hipStream_t st, const int32_t *counts_dev, int k, double *n_words) {
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d = reinterpret_cast<unsigned long long *>(scal) + kScSumWords;
  KS_HIP(hipMemsetAsync(d, 0, 8, st));
  const int64_t n = (int64_t)1 << (2 * k);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cus * 8));
  hipLaunchKernelGGL(k_sum_u32, dim3(grid), dim3(256), 0, st, reinterpret_cast<const uint32_t *>(counts_dev), n, d);
  KS_HIP(hipGetLastError());
  unsigned long long w = 0;
  KS_HIP(hipMemcpyAsync(&w, d, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  *n_words = (double)w;
  return KS_OK;
}

ks_status launch_count_range(ks_ctx *ctx, hipStream_t st, const ks_dev_seqs *s, int64_t p_lo, int64_t p_hi, int k,
                             int32_t *counts_dev) {
  if (p_lo % kPTile != 0 || p_hi <= p_lo) return fail(KS_ERR_ARG, "launch_count_range: bad range");
  return count_partitioned(ctx, s, p_hi, k, counts_dev, nullptr, p_lo, st);
}

ks_status launch_count(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const Runs &, int k,
                       int32_t *counts_dev, double *n_words) {
  if (count_range_ok(k, total)) return count_partitioned(ctx, s, total, k, counts_dev, n_words);
  hipStream_t st = ctx->stream;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_words = reinterpret_cast<unsigned long long *>(scal) + kScWords;
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
  // k's whose histograms are far beyond L2 take the partitioned counter
  // one by one; the rest share passes of k_count_multi.
  const bool part_ok = total > 0 && total < ((int64_t)1 << 32);
  std::vector<int32_t> rest_k;
  std::vector<int32_t *> rest_c;
  std::vector<int> rest_i;
  for (int i = 0; i < nk; ++i) {
    if (part_ok && ks[i] >= kPartMinK) {
      KS_TRY(count_partitioned(ctx, s, total, ks[i], counts_dev[i], &n_words[i]));
    } else {
      rest_k.push_back(ks[i]);
      rest_c.push_back(counts_dev[i]);
      rest_i.push_back(i);
    }
  }
  if (rest_k.size() < (size_t)nk) {
    std::vector<double> w(rest_k.size());
    if (!rest_k.empty())
      KS_TRY(launch_count_multi(ctx, s, total, rest_k.data(), (int)rest_k.size(), rest_c.data(), w.data()));
    for (size_t j = 0; j < rest_i.size(); ++j) n_words[rest_i[j]] = w[j];
    return KS_OK;
  }
  hipStream_t st = ctx->stream;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_words = reinterpret_cast<unsigned long long *>(scal) + kScMultiWords;
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
