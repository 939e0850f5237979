// ks_table.hip -- device score tables.
//
// s[code] = w[code] - thr is formed on the device with the very FP64
// subtraction the reference performs per base (kmer_spans.c:268), once per
// table instead of once per base.  If the table has <= 65536 distinct values
// (bitwise), it is re-expressed exactly as a uint16 code table + FP64 LUT:
// log2(f/f_med) and +-1 tables depend only on the k-mer count, so at k=13 the
// 512 MiB FP64 table becomes a 128 MiB code table that stays resident in the
// 256 MiB Infinity Cache while the sequence streams past.
#include <hip/hip_fp16.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "ks_internal.h"

namespace ks {
namespace {

__global__ void k_sub_thr(const double *__restrict__ w, double thr, double *__restrict__ s,
                          unsigned long long *__restrict__ bits, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = w[i] - thr;
    s[i] = v;
    if (bits) bits[i] = (unsigned long long)__double_as_longlong(v);
  }
}

// max |s| over the finite values (as the bits of a non-negative double), a
// flag for NaN or +Inf (-Inf only ever clamps to 0) and a flag for any s
// that is not a finite integer of magnitude <= 2^20 (ks_table::int_exact).
__global__ void k_absmax(const double *__restrict__ s, int64_t n, unsigned long long *__restrict__ out) {
  unsigned long long m = 0, bad = 0, nonint = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = s[i];
    if (isfinite(v)) m = max(m, (unsigned long long)__double_as_longlong(fabs(v)));
    else if (!(v < 0)) bad = 1;  // NaN or +Inf
    if (!(isfinite(v) && v == rint(v) && fabs(v) <= 0x1p20)) nonint = 1;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    m = max(m, (unsigned long long)__shfl_down(m, d, 64));
    bad |= __shfl_down(bad, d, 64);
    nonint |= __shfl_down(nonint, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], m);
    if (bad) atomicOr(&out[1], 1ull);
    if (nonint) atomicOr(&out[2], 1ull);
  }
}

// OR of all counts (as uint32): its highest set bit bounds the key bits the
// count sort must order (a wrapped, negative count sets bit 31: all 32 bits)
__global__ void k_count_or(const int32_t *__restrict__ c, int64_t n, unsigned int *__restrict__ out) {
  unsigned int m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m |= (unsigned int)c[i];
  for (int d = 32; d >= 1; d >>= 1) m |= __shfl_down(m, d, 64);
  __shared__ unsigned int wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {  // (one atomic per block: a wave each serialised 16 K of them on one address, 0.2 ms)
    const unsigned int b = wm[0] | wm[1] | wm[2] | wm[3];
    if (b) atomicOr(out, b);
  }
}

// The distinct count values and their multiplicities without a sort (log2 /
// pm1 tables need only those, ascending): a dense histogram hist[R] of the
// values, R = max(2^end_bit, kValLds).  Per block an LDS histogram of the
// values below kValLds, written as the block's row of rows[G][kValLds] and
// summed over the rows by k_val_cols; values above it (repeat k-mers, rare)
// add to hist with global atomics.  Then the nonzero bins compacted in order
// (flags, exclusive sum, k_val_compact), and dense[v] = v's index among them
// for k_map_dense.
constexpr int kValLds = 8192;
constexpr int kValBlocks = 256;
__global__ void __launch_bounds__(1024) k_val_hist(const int32_t *__restrict__ c, int64_t n,
                                                   uint32_t *__restrict__ rows, uint32_t *__restrict__ hist) {
  __shared__ uint32_t h[kValLds];
  for (int i = threadIdx.x; i < kValLds; i += 1024) h[i] = 0;
  __syncthreads();
  const int4 *c4 = reinterpret_cast<const int4 *>(c);  // (n = 4^k: a multiple of 4)
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * 1024) {
    const int4 q = c4[i];
    const uint32_t v[4] = {(uint32_t)q.x, (uint32_t)q.y, (uint32_t)q.z, (uint32_t)q.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (v[j] < (uint32_t)kValLds) atomicAdd(&h[v[j]], 1u);
      else atomicAdd(&hist[v[j]], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kValLds; i += 1024) rows[(size_t)blockIdx.x * kValLds + i] = h[i];
}

__global__ void k_val_cols(const uint32_t *__restrict__ rows, int G, uint32_t *__restrict__ hist) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= kValLds) return;
  uint32_t t = 0;
  for (int g = 0; g < G; ++g) t += rows[(size_t)g * kValLds + v];
  hist[v] = t;
}

__global__ void k_val_flags(const uint32_t *__restrict__ hist, int64_t R, uint32_t *__restrict__ flags) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < R; v += (int64_t)gridDim.x * blockDim.x)
    flags[v] = hist[v] != 0;
}

__global__ void k_val_compact(const uint32_t *__restrict__ hist, const uint32_t *__restrict__ pos, int64_t R,
                              int32_t *__restrict__ uniq, int *__restrict__ mult, int *__restrict__ nu,
                              uint32_t *__restrict__ dense) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < R; v += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t m = hist[v], p = pos[v];
    if (m) {
      uniq[p] = (int32_t)v;
      mult[p] = (int)m;
      dense[v] = p;
    }
    if (v == R - 1) *nu = (int)(p + (m != 0));
  }
}

__global__ void k_assign_codes(const double *__restrict__ s, const unsigned long long *__restrict__ uniq,
                               int64_t nu, uint16_t *__restrict__ codes, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = (unsigned long long)__double_as_longlong(s[i]);
    int64_t lo = 0, hi = nu - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (uniq[mid] < key) lo = mid + 1; else hi = mid;
    }
    codes[i] = (uint16_t)lo;
  }
}

// Expanded table, uint16 codes: entry for the (k+J-1)-mer x packs the codes of
// its J k-mers (first k-mer in the low 16 bits).  Lane p builds the entry
// pair 2p, 2p+1: their first J-1 k-mers coincide ((2p + d) >> 2(J-1-t) does
// not depend on d for t < J-1), their last k-mers are two consecutive codes
// (one 4-B load).  Consecutive lanes write consecutive pairs, so one store
// instruction covers a contiguous span; the table is far larger than every
// cache, so the stores are nontemporal.  The code reads repeat across the
// wave and stay cached: the build is a write stream.
typedef unsigned long long ks_u64x2 __attribute__((ext_vector_type(2)));
// kU pairs per lane and trip, loads ahead of the stores (as k_build_ext_c12;
// A/B: KS_EXT_U1).
template <int J, typename E, int kU = 1>
__global__ void k_build_ext_u16(const uint16_t *__restrict__ codes, int k, uint64_t nent, E *__restrict__ ext) {
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  const uint64_t npair = nent >> 1;
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  auto pair = [&](uint64_t p) -> ks_u64x2 {
    const uint64_t e0 = p << 1;
    uint64_t v = 0;
#pragma unroll
    for (int t = 0; t < J - 1; ++t) v |= (uint64_t)codes[(e0 >> (2 * (J - 1 - t))) & mk] << (16 * t);
    const uint32_t w = *reinterpret_cast<const uint32_t *>(codes + (e0 & mk));
    ks_u64x2 o;
    o.x = v | ((uint64_t)(w & 0xffffu) << (16 * (J - 1)));
    o.y = v | ((uint64_t)(w >> 16) << (16 * (J - 1)));
    return o;
  };
  auto put = [&](uint64_t p, const ks_u64x2 &o) {
    if (sizeof(E) == 8)
      __builtin_nontemporal_store(o, reinterpret_cast<ks_u64x2 *>(ext) + p);
    else
      __builtin_nontemporal_store((uint64_t)(uint32_t)o.x | ((uint64_t)(uint32_t)o.y << 32),
                                  reinterpret_cast<uint64_t *>(ext) + p);
  };
  uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; p + (kU - 1) * S < npair; p += kU * S) {
    ks_u64x2 o[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) o[u] = pair(p + u * S);
#pragma unroll
    for (int u = 0; u < kU; ++u) put(p + u * S, o[u]);
  }
  for (; p < npair; p += S) put(p, pair(p));
}

// Position weight of every uint16 code in [lo, lo + kHistBins): number of
// k-mers with that code, or (with a frequency hint) the number of positions
// scoring them.  LDS-privatised 64-bit histogram (one 1024-lane block per CU:
// 128 KiB of bins), flushed with one global atomic per non-zero bin and
// block: the codes of log2/+-1 tables are heavily skewed (most k-mers have a
// count near the median), which serialised the former global atomics
// (77 ms at k = 13, profiles/r1_v24) on a few hot bins.
constexpr int kHistBins = 16384;
__global__ void __launch_bounds__(1024) k_code_hist(const uint16_t *__restrict__ codes,
                                                    const int32_t *__restrict__ freq, int64_t n, int lo,
                                                    unsigned long long *__restrict__ hist) {
  __shared__ unsigned long long h[kHistBins];
  for (int i = threadIdx.x; i < kHistBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n8 = n >> 3;  // 8 codes (16 B) and 8 weights (2 x 16 B) per lane and step
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += stride) {
    const uint4 c = reinterpret_cast<const uint4 *>(codes)[v];
    uint4 f0 = make_uint4(1, 1, 1, 1), f1 = f0;
    if (freq) {
      f0 = reinterpret_cast<const uint4 *>(freq)[2 * v];
      f1 = reinterpret_cast<const uint4 *>(freq)[2 * v + 1];
    }
    const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
    const uint32_t fw[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t b = ((cw[q >> 1] >> (16 * (q & 1))) & 0xffffu) - (uint32_t)lo;
      if (b < (uint32_t)kHistBins && fw[q]) atomicAdd(&h[b], (unsigned long long)fw[q]);
    }
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t b = (uint32_t)codes[i] - (uint32_t)lo;
    const unsigned long long w = freq ? (unsigned long long)(uint32_t)freq[i] : 1ull;
    if (b < (uint32_t)kHistBins && w) atomicAdd(&h[b], w);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHistBins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[lo + i], h[i]);
}

// codes[i] = perm[codes[i]]: the uint16 codes renumbered by position weight
// (perm staged in LDS, 128 KiB for 65536 codes).
__global__ void __launch_bounds__(1024) k_remap_codes(uint16_t *__restrict__ codes,
                                                      const uint16_t *__restrict__ perm, int nperm, int64_t n) {
  __shared__ uint16_t p[65536];
  for (int i = threadIdx.x; i < nperm; i += blockDim.x) p[i] = perm[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n8 = n >> 3;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n8; v += stride) {
    uint4 c = reinterpret_cast<uint4 *>(codes)[v];
    uint32_t *w = reinterpret_cast<uint32_t *>(&c);
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = (uint32_t)p[w[q] & 0xffffu] | ((uint32_t)p[w[q] >> 16] << 16);
    reinterpret_cast<uint4 *>(codes)[v] = c;
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    codes[i] = p[codes[i]];
}

// Expanded table, 12-bit codes: J = 5 codes per uint64 entry, first k-mer
// in the low 12 bits.  The uint16 codes are numbered by position weight
// (choose_code12), so a code below 4095 is its own 12-bit code and every
// other code escapes (0xFFF).  Same pair-per-lane layout and nontemporal
// stores as k_build_ext_u16 (was four entries per lane as two 16-B stores
// at a 32-B stride: 42-56 ms for the 128 GiB table at k = 13).
__device__ __forceinline__ uint64_t c12_of(uint32_t code) { return code < 0xFFFu ? code : 0xFFFu; }
// kU pairs per lane and trip (grid-strided), their code loads all issued
// before the first store: a trip costs one round trip to L2 / the Infinity
// Cache for kU x 16 B of stores (A/B: KS_EXT_U1 / KS_EXT_U4 / KS_EXT_U16 pairs per trip,
// KS_EXT_PLAIN for plain stores).
template <int kU, bool kNT = true>
__global__ void k_build_ext_c12(const uint16_t *__restrict__ codes, int k, uint64_t nent,
                                uint64_t *__restrict__ ext) {
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  const uint64_t npair = nent >> 1;
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  auto pair = [&](uint64_t p) -> ks_u64x2 {
    const uint64_t e0 = p << 1;
    uint64_t base = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) base |= c12_of(codes[(e0 >> (2 * (4 - t))) & mk]) << (12 * t);
    const uint32_t w = *reinterpret_cast<const uint32_t *>(codes + (e0 & mk));
    ks_u64x2 o;
    o.x = base | (c12_of(w & 0xffffu) << 48);
    o.y = base | (c12_of(w >> 16) << 48);
    return o;
  };
  uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; p + (kU - 1) * S < npair; p += kU * S) {
    ks_u64x2 o[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) o[u] = pair(p + u * S);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (kNT)
        __builtin_nontemporal_store(o[u], reinterpret_cast<ks_u64x2 *>(ext) + p + u * S);
      else
        reinterpret_cast<ks_u64x2 *>(ext)[p + u * S] = o[u];
    }
  }
  for (; p < npair; p += S) __builtin_nontemporal_store(pair(p), reinterpret_cast<ks_u64x2 *>(ext) + p);
}

// Expanded table, FP64 values: J values per entry (double2 / double4).  A
// lane per 16-B half entry, so that each store instruction covers whole
// lines across the wave (nontemporal: written once, read later at random);
// a lane per 32-B entry with two strided 16-B stores ran at 44.6 ms for
// 128 GiB on scattered VRAM and 78.8 ms on contiguous VRAM.
typedef double ks_f64x2 __attribute__((ext_vector_type(2)));
// kU slots per lane and trip (grid-strided), loads ahead of the stores as in
// k_build_ext_c12 (A/B: KS_EXT_U1).
template <int J, int kU = 1>
__global__ void k_build_ext_f64(const double *__restrict__ vals, int k, uint64_t nent, double *__restrict__ ext) {
  constexpr int H = (J <= 2) ? 1 : 2;  // 16-B halves per entry
  const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
  const uint64_t nslot = nent * H;
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  auto half = [&](uint64_t sl) -> ks_f64x2 {
    const uint64_t e = H == 2 ? sl >> 1 : sl;
    const int t0 = H == 2 ? 2 * (int)(sl & 1) : 0;  // first value of this half
    ks_f64x2 o;
    o.x = (t0 < J) ? vals[(e >> (2 * (J - 1 - t0))) & mk] : 0.0;
    o.y = (t0 + 1 < J) ? vals[(e >> (2 * (J - 2 - t0))) & mk] : 0.0;
    return o;
  };
  uint64_t sl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; sl + (kU - 1) * S < nslot; sl += kU * S) {
    ks_f64x2 o[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) o[u] = half(sl + u * S);
#pragma unroll
    for (int u = 0; u < kU; ++u) __builtin_nontemporal_store(o[u], reinterpret_cast<ks_f64x2 *>(ext) + sl + u * S);
  }
  for (; sl < nslot; sl += S) __builtin_nontemporal_store(half(sl), reinterpret_cast<ks_f64x2 *>(ext) + sl);
}

// Line tables (ks_table::line_kind): one 64-B line per m-mer x (m = k + own
// - 1), holding the values of the own k-mers inside x and of the k-mers one
// and two bases past it for every continuation:
//   uint16 codes: [own][L1: x.c for c in ACTG order][L2: x.c1.c2], own + 20 <= 32
//   FP64 values:  [own][L1], own + 4 <= 8
// (zeros pad the line).  own k-mer t is (x >> 2 (own - 1 - t)) & mask; L1 c
// is ((x << 2) | c) & mask, L2 c1 c2 is ((x << 4) | c1 c2) & mask: the L1 /
// L2 entries of consecutive lines are consecutive code-table entries.
typedef uint32_t ks_u32x4 __attribute__((ext_vector_type(4)));

// Line builds, lane per line: the lane reads its line's entries (own
// k-mers: three scattered reads; the L1 / L2 / L3 continuations: 4 / 16 / 64
// consecutive code-table entries from ((x << 2 lev) & mask)) and packs them
// with compile-time offsets.  The lines are walked as x = (hi << lb) | lo
// with lo (the low lb = 2k - 2 levmax bits, which alone decide the L-region
// reads) fixed per lane -- a block's 64 consecutive lo values, the same for
// its four waves -- and hi the loop (four values per trip, one per wave): a
// block re-reads the same 2-8 KiB of the code table on every trip (L1
// hits), and a wave's 64 lines are consecutive, so after a transpose through
// LDS each 16-B store instruction writes 1 KiB of whole lines.  Mode 0: uint16 64-B lines, 1: FP64 64-B
// lines, 2: wide 128-B lines (13-bit own / L1 / L2 codes at bits 13 j, the
// 64 L3 codes as 11-bit codes from bit 13 (own + 20), >= 2047 -> 2047).
// Mode 3: weighted-rank code lines, 128 B: the 32-bit rank codes (ks_table::
// d_rcodes) of own, L1 and L2 at dwords 0 .. own + 19 (k_pass1r).
template <int OWN, int kMode>
__global__ void __launch_bounds__(256) k_build_lines(const uint16_t *__restrict__ codes,
                                                     const double *__restrict__ vals,
                                                     const uint32_t *__restrict__ codes32, int k, int m,
                                                     ks_u32x4 *__restrict__ out) {
  constexpr int LB = kMode >= 2 ? 128 : 64;  // line bytes
  constexpr int NP = LB / 16;               // 16-B pieces per line
  constexpr int LEV = kMode == 0 || kMode == 3 ? 2 : (kMode == 1 ? 1 : 3);
  __shared__ ks_u32x4 s_t[4][64 * NP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t kmask = (uint32_t)(((uint64_t)1 << (2 * k)) - 1);
  const int lb = 2 * k - 2 * LEV;
  const uint64_t nhi = ((uint64_t)1 << (2 * m - lb)) / gridDim.y;  // hi range of this block row (>= 4)
  const uint64_t lo = (uint64_t)blockIdx.x * 64 + lane;
  for (uint64_t hi = blockIdx.y * nhi + wv; hi < (blockIdx.y + 1) * nhi; hi += 4) {
    const uint64_t x = (hi << lb) | lo;
    uint32_t w[LB / 4];
#pragma unroll
    for (int q = 0; q < LB / 4; ++q) w[q] = 0;
    if (kMode == 3) {  // 32-bit rank codes: [own][L1][L2]
#pragma unroll
      for (int t = 0; t < OWN; ++t) w[t] = codes32[(uint32_t)(x >> (2 * (OWN - 1 - t))) & kmask];
      const uint4 l1 = *reinterpret_cast<const uint4 *>(codes32 + (((uint32_t)(x << 2)) & kmask));
      w[OWN] = l1.x; w[OWN + 1] = l1.y; w[OWN + 2] = l1.z; w[OWN + 3] = l1.w;
      const uint4 *l2 = reinterpret_cast<const uint4 *>(codes32 + (((uint32_t)(x << 4)) & kmask));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = l2[q];
        w[OWN + 4 + 4 * q] = v.x; w[OWN + 5 + 4 * q] = v.y; w[OWN + 6 + 4 * q] = v.z; w[OWN + 7 + 4 * q] = v.w;
      }
    } else if (kMode == 1) {  // FP64: [own][L1]
      double d[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) d[t] = 0.0;
#pragma unroll
      for (int t = 0; t < OWN; ++t) d[t] = vals[(uint32_t)(x >> (2 * (OWN - 1 - t))) & kmask];
      const double2 *l1 = reinterpret_cast<const double2 *>(vals + (((uint32_t)(x << 2)) & kmask));
      const double2 a0 = l1[0], a1 = l1[1];
      d[OWN] = a0.x; d[OWN + 1] = a0.y; d[OWN + 2] = a1.x; d[OWN + 3] = a1.y;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        w[2 * t] = (uint32_t)__double_as_longlong(d[t]);
        w[2 * t + 1] = (uint32_t)((uint64_t)__double_as_longlong(d[t]) >> 32);
      }
    } else {
      uint32_t h[OWN + 20];
#pragma unroll
      for (int t = 0; t < OWN; ++t) h[t] = codes[(uint32_t)(x >> (2 * (OWN - 1 - t))) & kmask];
      const uint2 l1 = *reinterpret_cast<const uint2 *>(codes + (((uint32_t)(x << 2)) & kmask));
      h[OWN] = l1.x & 0xffffu; h[OWN + 1] = l1.x >> 16; h[OWN + 2] = l1.y & 0xffffu; h[OWN + 3] = l1.y >> 16;
      const uint4 *l2 = reinterpret_cast<const uint4 *>(codes + (((uint32_t)(x << 4)) & kmask));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint4 v = l2[q];
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[OWN + 4 + 8 * q + 2 * r] = vw[r] & 0xffffu;
          h[OWN + 4 + 8 * q + 2 * r + 1] = vw[r] >> 16;
        }
      }
      if (kMode == 0) {
#pragma unroll
        for (int j = 0; j < OWN + 20; ++j) w[j >> 1] |= h[j] << (16 * (j & 1));
      } else {
        auto put = [&](int b, uint32_t v) {  // compile-time b after unrolling
          w[b >> 5] |= v << (b & 31);
          if ((b & 31) != 0) w[(b >> 5) + 1] |= v >> (32 - (b & 31));
        };
#pragma unroll
        for (int j = 0; j < OWN + 20; ++j) put(13 * j, h[j] & 0x1fffu);
        const uint4 *l3 = reinterpret_cast<const uint4 *>(codes + (((uint32_t)(x << 6)) & kmask));
        constexpr int B3 = 13 * (OWN + 20);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint4 v = l3[q];
          const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const uint32_t cd = (vw[r >> 1] >> (16 * (r & 1))) & 0xffffu;
            put(B3 + 11 * (8 * q + r), cd < 2047u ? cd : 2047u);
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      ks_u32x4 v;
      v.x = w[4 * p]; v.y = w[4 * p + 1]; v.z = w[4 * p + 2]; v.w = w[4 * p + 3];
      s_t[wv][lane * NP + p] = v;
    }
    // (a wave's LDS accesses execute in order: no barrier for its own image)
    const uint64_t x0 = x - lane;  // the wave's first line
#pragma unroll
    for (int p = 0; p < NP; ++p) __builtin_nontemporal_store(s_t[wv][p * 64 + lane], out + x0 * NP + p * 64 + lane);
  }
}

// out[i] = lut[index of counts[i] in dv]: dv = the sorted distinct counts
// (every count occurs in it), staged in LDS with the LUT when they fit.
constexpr int kMapLds = 8192;
template <typename V>
__global__ void __launch_bounds__(1024) k_map_counts(const int32_t *__restrict__ counts, int64_t n,
                                                     const int32_t *__restrict__ dv, int64_t nu,
                                                     const V *__restrict__ lut, V *__restrict__ out) {
  __shared__ int32_t s_dv[kMapLds];
  __shared__ V s_lut[kMapLds];
  const bool lds = nu <= kMapLds;
  if (lds) {
    for (int i = threadIdx.x; i < nu; i += blockDim.x) {
      s_dv[i] = dv[i];
      s_lut[i] = lut[i];
    }
    __syncthreads();
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = counts[i];
    int64_t lo = 0, hi = nu - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((lds ? s_dv[mid] : dv[mid]) < c) lo = mid + 1; else hi = mid;
    }
    out[i] = lds ? s_lut[lo] : lut[lo];
  }
}

// out[i] = lut[dense[counts[i]]] (dense from k_val_compact: every count's
// index among the distinct values).
template <typename V>
__global__ void k_map_dense(const int32_t *__restrict__ counts, int64_t n, const uint32_t *__restrict__ dense,
                            const V *__restrict__ lut, V *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = lut[dense[counts[i]]];
}

// Weighted ranks from the closed-form prefix (RankPiece, ks_internal.h):
// sorted position j (stable (count, index) order, idx = the sorted indices)
// takes its piece's value; 16 consecutive positions per lane, one binary
// search per lane.
__global__ void k_rank_fill(const uint32_t *__restrict__ idx, int64_t n, const RankPiece *__restrict__ P, int64_t np,
                            double *__restrict__ ranks) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g * 16 < n; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j0 = g * 16;
    int64_t lo = 0, hi = np - 1;  // last piece starting at or before j0
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (P[mid].j0 <= j0) lo = mid; else hi = mid - 1;
    }
    const int64_t j1 = min(n, j0 + 16);
    for (int64_t j = j0; j < j1; ++j) {
      while (lo + 1 < np && P[lo + 1].j0 <= j) ++lo;
      ranks[idx[j]] = rank_piece_value(P[lo], j);
    }
  }
}

// Rank codes (ks_table::d_rcodes): sorted position j takes the code of its
// uniform piece (pieces sorted by start uj0; uh = the piece's index in
// weight order, the code's piece field).
__global__ void k_rank_codes(const uint32_t *__restrict__ idx, int64_t n, const int64_t *__restrict__ uj0,
                             const int32_t *__restrict__ uh, int64_t np, uint32_t *__restrict__ codes) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g * 16 < n; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j0 = g * 16;
    int64_t lo = 0, hi = np - 1;  // last piece starting at or before j0
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (uj0[mid] <= j0) lo = mid; else hi = mid - 1;
    }
    const int64_t j1 = min(n, j0 + 16);
    for (int64_t j = j0; j < j1; ++j) {
      while (lo + 1 < np && uj0[lo + 1] <= j) ++lo;
      codes[idx[j]] = ((uint32_t)uh[lo] << kRankOffBits) | (uint32_t)(j - uj0[lo]);
    }
  }
}

// Every code decodes to the rank the closed form filled, bit for bit
// (mismatches counted; the code lines are built only with none).
__global__ void k_rank_codes_check(const uint32_t *__restrict__ codes, const unsigned long long *__restrict__ pc,
                                   const double *__restrict__ ranks, int64_t n, int64_t np,
                                   unsigned long long *__restrict__ bad) {
  unsigned long long nb = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = codes[i];
    const uint32_t p = c >> kRankOffBits;
    if ((int64_t)p >= np) {
      ++nb;
      continue;
    }
    const unsigned long long bits = pc[2 * p] + (unsigned long long)(c & ((1u << kRankOffBits) - 1)) * pc[2 * p + 1];
    if (bits != (unsigned long long)__double_as_longlong(ranks[i])) ++nb;
  }
  if (nb) atomicAdd(bad, nb);
}

__global__ void k_iota(uint32_t *__restrict__ x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = (uint32_t)i;
}

// Approximate prefix table (the binade predictor of the chunked scan): for
// each kp-base prefix p, the mean of s over the 4^(k-kp) k-mers extending it,
// weighted by their position frequency (the counts hint; 1 without one).
// Non-finite values and zero weights are left out.  A wave per prefix when
// it has >= 64 k-mers (coalesced reads, one wave reduction; round 6:
// the lane-per-prefix walk took 1.6 ms at k = 13 -- 16 K lanes each reading
// 4,096 entries 8 KiB apart -- and sat in every table build), else a lane.
__device__ __forceinline__ void approx_acc(const uint16_t *__restrict__ codes, const double *__restrict__ lut,
                                           const double *__restrict__ vals, const int32_t *__restrict__ freq,
                                           int64_t i, double &num, double &den) {
  const double v = codes ? lut[codes[i]] : vals[i];
  const double wt = freq ? (double)(uint32_t)freq[i] : 1.0;
  if (wt > 0 && isfinite(v)) {
    num += wt * v;
    den += wt;
  }
}

__global__ void __launch_bounds__(256) k_build_approx(const uint16_t *__restrict__ codes, const double *__restrict__ lut,
                                                      const double *__restrict__ vals, const int32_t *__restrict__ freq,
                                                      int k, int kp, uint16_t *__restrict__ out) {
  const int64_t np = (int64_t)1 << (2 * kp);
  const int sub = 2 * (k - kp);
  if (sub >= 6) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); p < np; p += nw) {
      double num = 0.0, den = 0.0;
      const int64_t b = p << sub, e = (p + 1) << sub;
      for (int64_t i = b + lane; i < e; i += 64) approx_acc(codes, lut, vals, freq, i, num, den);
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        num += __shfl_xor(num, d, 64);
        den += __shfl_xor(den, d, 64);
      }
      if (lane == 0) out[p] = __half_as_ushort(__float2half(den > 0 ? (float)(num / den) : 0.0f));
    }
    return;
  }
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < np; p += (int64_t)gridDim.x * blockDim.x) {
    double num = 0.0, den = 0.0;
    const int64_t b = p << sub, e = (p + 1) << sub;
    for (int64_t i = b; i < e; ++i) approx_acc(codes, lut, vals, freq, i, num, den);
    out[p] = __half_as_ushort(__float2half(den > 0 ? (float)(num / den) : 0.0f));
  }
}

}  // namespace

// Process-wide pool of expanded-table buffers, per device ONE, or TWO whose
// sum stays within kPoolPairMax (two tables alive at once, e.g. genome g + 1's
// table built while genome g is scanned).  A fresh hipMalloc of 32-128 GiB
// takes 0.3 ms to 6 s on the box (the driver clears new VRAM;
// tools/probes/alloc_probe.py), while a buffer freed by this process is handed back
// at once; tables built per call (one table per genome) would pay that on
// every table.  A destroyed table's buffer is kept here and reused by the
// next expansion that fits in it; ks_release_cache() returns them to the
// driver (the host entry points do at the end of each call unless
// ks_set_host_cache(1)); KS_EXT_POOL=0 disables the pool.
namespace {
std::mutex g_pool_mu;
struct PoolBuf {
  void *p = nullptr;
  size_t bytes = 0;
};
// (two 64 GiB tables; a weighted-rank table's 128 GiB code lines and 64 GiB
// FP64 form, round 6 -- the pool then holds both between tables)
constexpr size_t kPoolPairMax = (size_t)200 << 30;
PoolBuf g_pool[64][2];
bool pool_on() {
  static const bool on = !(getenv("KS_EXT_POOL") && atoi(getenv("KS_EXT_POOL")) == 0);
  return on;
}
size_t pool_bytes(int dev) { return g_pool[dev][0].bytes + g_pool[dev][1].bytes; }  // (under g_pool_mu)
PoolBuf g_cpool[64];  // (cpool_take / cpool_give below)
void pool_free_all(int dev) {  // (under g_pool_mu)
  for (PoolBuf &b : g_pool[dev]) {
    if (b.p) (void)hipFree(b.p);
    b = PoolBuf();
  }
  if (g_cpool[dev].p) (void)hipFree(g_cpool[dev].p);
  g_cpool[dev] = PoolBuf();
}
void *pool_take(int dev, size_t bytes, size_t *cap) {
  if (!pool_on() || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_pool_mu);
  PoolBuf *best = nullptr;  // the smallest that fits
  for (PoolBuf &b : g_pool[dev])
    if (b.p && b.bytes >= bytes && (!best || b.bytes < best->bytes)) best = &b;
  if (!best) return nullptr;
  void *p = best->p;
  *cap = best->bytes;
  *best = PoolBuf();
  return p;
}
void pool_give(int dev, void *p, size_t bytes) {
  if (!p) return;
  if (pool_on() && dev >= 0 && dev < 64) {
    // the next table's build may run on another stream: every kernel that
    // reads this buffer must have finished before it is handed out again
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    if (cur >= 0) (void)hipSetDevice(cur);
    std::lock_guard<std::mutex> g(g_pool_mu);
    PoolBuf *s = g_pool[dev];
    PoolBuf *slot = nullptr;
    if (!s[0].p && !s[1].p) slot = &s[0];
    else if ((!s[0].p || !s[1].p) && pool_bytes(dev) + bytes <= kPoolPairMax) slot = s[0].p ? &s[1] : &s[0];
    if (slot) {
      slot->p = p;
      slot->bytes = bytes;
      p = nullptr;
    } else {  // the smaller kept buffer goes if this one is larger
      PoolBuf *small = !s[0].p ? &s[1] : !s[1].p ? &s[0] : (s[0].bytes <= s[1].bytes ? &s[0] : &s[1]);
      if (small->bytes < bytes) {
        std::swap(small->p, p);
        std::swap(small->bytes, bytes);
      }
    }
  }
  if (p) (void)hipFree(p);
}
// One kept uint16 code array per device (4^k x 2 B: 128 MiB at k = 13): a
// table built per genome (config 5) otherwise pays a fresh hipMalloc of it
// (~0.4 ms) on every build.  Given back by ks_table_destroy after the device
// synchronisation pool_give already does for the expanded table.
void *cpool_take(int dev, size_t bytes) {
  if (!pool_on() || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> g(g_pool_mu);
  PoolBuf &b = g_cpool[dev];
  if (!b.p || b.bytes != bytes) return nullptr;
  void *p = b.p;
  b = PoolBuf();
  return p;
}
void cpool_give(int dev, void *p, size_t bytes) {
  if (!p) return;
  if (pool_on() && dev >= 0 && dev < 64) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipDeviceSynchronize();
    if (cur >= 0) (void)hipSetDevice(cur);
    std::lock_guard<std::mutex> g(g_pool_mu);
    std::swap(g_cpool[dev].p, p);
    std::swap(g_cpool[dev].bytes, bytes);
  }
  if (p) (void)hipFree(p);
}
}  // namespace

// Expanded-table allocation: physically contiguous VRAM when the driver has
// it (hipDeviceMallocContiguous), else a plain hipMalloc.  Random 16-byte
// gathers over 128 GiB run at 49.3-50.6 G/s from a contiguous buffer and
// 47.5-48.7 G/s from a plain one on the same box (tools/probes/frag_probe.hip,
// profiles/r2/frag_probe.txt): fewer, larger translation fragments.
static hipError_t ext_malloc(void **p, size_t bytes) {
  static const bool dbg = getenv("KS_DEBUG_ALLOC") != nullptr;
  if (bytes >= ((size_t)1 << 30)) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) {
      if (dbg) fprintf(stderr, "[ext alloc] contiguous %zu bytes at %p\n", bytes, *p);
      return hipSuccess;
    }
    (void)hipGetLastError();
  }
  const hipError_t e = hipMalloc(p, bytes);
  if (dbg) fprintf(stderr, "[ext alloc] plain %zu bytes at %p (%d)\n", bytes, *p, (int)e);
  return e;
}

// Tables whose chunked scan predicts carry binades before pass 1: compressed
// tables scanned by the pipelined pass, FP64 line tables (weighted rank), and
// small k (k <= 7, the table staged in LDS by pass 1; there the prefix table
// holds the values themselves).
static bool k_approx_ok(const ks_table *t) { return t->k >= 1; }

// Entry bytes of an expanded table with J values per entry.
static size_t ext_entry_bytes(bool u16, int J) {
  if (u16) return J <= 2 ? 4 : 8;
  return J <= 2 ? 16 : 32;
}

// 12-bit code assignment for J = 5: the uint16 codes are renumbered by
// position weight (heaviest first, ties by code), the LUT permuted to match,
// so that the 4095 heaviest codes are their own 12-bit codes (0..4094) and
// every other code escapes.  Sets *use = false (and changes nothing) if the
// escape share is above max_escape.
static ks_status choose_code12(ks_ctx *ctx, ks_table *t, const int32_t *freq_dev, double max_escape, bool *use,
                               int64_t ndirect_max = 4095) {
  *use = false;
  hipStream_t st = ctx->stream;
  const int64_t n = (int64_t)1 << (2 * t->k);
  const int64_t nu = t->distinct;
  unsigned long long *d_hist = nullptr;
  KS_HIP(hipMalloc(&d_hist, 65536 * 8));
  KS_HIP(hipMemsetAsync(d_hist, 0, 65536 * 8, st));
  const unsigned grid = (unsigned)std::min<int64_t>((n / 8 + 1023) / 1024, (int64_t)ctx->num_cus);
  for (int64_t lo = 0; lo < nu; lo += kHistBins)
    hipLaunchKernelGGL(k_code_hist, dim3(std::max(grid, 1u)), dim3(1024), 0, st, t->d_codes, freq_dev, n, (int)lo,
                       d_hist);
  KS_HIP(hipGetLastError());
  std::vector<unsigned long long> h(65536);
  std::vector<double> lut(nu);
  KS_HIP(hipMemcpyAsync(h.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(lut.data(), t->d_lut, nu * 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  KS_HIP(hipFree(d_hist));
  std::vector<int32_t> order(nu);
  for (int64_t i = 0; i < nu; ++i) order[i] = (int32_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return h[a] > h[b]; });
  const int64_t ndirect = std::min<int64_t>(nu, ndirect_max);
  long double tot = 0, cov = 0;
  for (int64_t i = 0; i < nu; ++i) tot += h[order[i]];
  for (int64_t i = 0; i < ndirect; ++i) cov += h[order[i]];
  t->escape_frac = tot > 0 ? (double)(1.0L - cov / tot) : 0.0;
  if (t->escape_frac > max_escape) return KS_OK;
  std::vector<uint16_t> perm(nu), map12(4096, 0);
  std::vector<double> nlut(nu), lut12(4096, 0.0);
  for (int64_t i = 0; i < nu; ++i) {
    perm[order[i]] = (uint16_t)i;
    nlut[i] = lut[order[i]];
  }
  for (int64_t i = 0; i < 4096; ++i) {  // identity: a short code is the uint16 code
    map12[i] = (uint16_t)i;
    lut12[i] = i < nu ? nlut[i] : 0.0;
  }
  uint16_t *d_perm = nullptr;
  KS_HIP(hipMalloc(&d_perm, nu * 2));
  KS_HIP(hipMemcpyAsync(d_perm, perm.data(), nu * 2, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_remap_codes, dim3(std::max(grid, 1u)), dim3(1024), 0, st, t->d_codes, d_perm, (int)nu, n);
  KS_HIP(hipGetLastError());
  KS_HIP(hipMemcpyAsync(t->d_lut, nlut.data(), nu * 8, hipMemcpyHostToDevice, st));
  KS_HIP(hipMalloc(&t->d_map12, 4096 * 2));
  KS_HIP(hipMalloc(&t->d_lut12, 4096 * 8));
  KS_HIP(hipMemcpyAsync(t->d_map12, map12.data(), 4096 * 2, hipMemcpyHostToDevice, st));
  KS_HIP(hipMemcpyAsync(t->d_lut12, lut12.data(), 4096 * 8, hipMemcpyHostToDevice, st));
  KS_HIP(hipStreamSynchronize(st));
  KS_HIP(hipFree(d_perm));
  *use = true;
  return KS_OK;
}

// Allocation of an expanded / line table: a pooled buffer of a destroyed
// table when it fits, else contiguous VRAM (ext_malloc).  nullptr: no memory.
static void *ext_alloc(ks_ctx *ctx, size_t bytes, size_t *cap) {
  *cap = bytes;
  void *ext = pool_take(ctx->device, bytes, cap);
  if (ext) {
    debug_poison(ext, bytes);  // (KS_DEBUG_POISON: a pooled buffer taken again)
    return ext;
  }
  *cap = bytes;
  if (ext_malloc(&ext, bytes) == hipSuccess) {
    debug_poison(ext, bytes);
    return ext;
  }
  (void)hipGetLastError();
  {  // pooled buffers too small for this table may be what is in the way
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (ctx->device >= 0 && ctx->device < 64) pool_free_all(ctx->device);
  }
  if (ext_malloc(&ext, bytes) == hipSuccess) {
    debug_poison(ext, bytes);
    return ext;
  }
  (void)hipGetLastError();
  return nullptr;
}

// Distinct values of a wide line table (13-bit codes, LUT staged in LDS by
// k_pass1w: ks_scan_chunked.hip kLineLutMax).
constexpr int64_t kWideLut = 7168;

// Launch of k_build_lines: 2^lb lanes (lb = 2k - 2 levmax), the hi range
// split over grid rows until ~2^20 lanes run.
template <int OWN, int kMode>
static void launch_build_lines(hipStream_t st, const ks_table *t, int m, void *out) {
  const int lev = kMode == 0 || kMode == 3 ? 2 : (kMode == 1 ? 1 : 3);
  const int lb = 2 * t->k - 2 * lev;
  const int hb = 2 * m - lb;  // >= 4 (m >= k + 1, levmax >= 1)
  int ys = 0;
  while (lb + ys < 22 && ys + 2 < hb) ++ys;
  hipLaunchKernelGGL((k_build_lines<OWN, kMode>), dim3((unsigned)(((uint64_t)1 << lb) / 64), 1u << ys), dim3(256), 0,
                     st, t->d_codes, t->d_vals, t->d_rcodes, t->k, m, (ks_u32x4 *)out);
}

// Binade predictor of the pass-1 summaries (k_predict), built with the
// expanded / line table of a compressed table.
static ks_status build_approx(ks_ctx *ctx, ks_table *t, const int32_t *freq_dev) {
  if (!k_approx_ok(t)) return KS_OK;
  // prefix length of the binade predictor: 7 bases, 32 KiB of fp16 means --
  // four predictor blocks per CU, and the second half's predictor no longer
  // holds whole CUs beside the first half's pass 1: metric step 14.37 vs
  // 14.89-15.18 ms with 8 bases (128 KiB, one block per CU), the summary
  // fixes unchanged (profiles/r4/ab3/approx_k*.json)
  const int kp_max = 7;
  const int kp = std::min(t->k, kp_max);
  if (hipMalloc(&t->d_approx, ((size_t)2 << (2 * kp)) + 16) != hipSuccess) {
    (void)hipGetLastError();
    t->d_approx = nullptr;
    return KS_OK;
  }
  debug_poison(t->d_approx, ((size_t)2 << (2 * kp)) + 16);
  t->approx_k = kp;
  const int64_t np = (int64_t)1 << (2 * kp);
  const int64_t per_block = 2 * (t->k - kp) >= 6 ? 4 : 256;  // (a wave per prefix, else a lane)
  hipLaunchKernelGGL(k_build_approx, dim3((unsigned)std::min<int64_t>((np + per_block - 1) / per_block, 4096)),
                     dim3(256), 0, ctx->stream, t->d_codes, t->d_lut, t->d_vals, freq_dev, t->k, kp, t->d_approx);
  KS_HIP(hipGetLastError());
  return KS_OK;
}

// Line table of k in [8, 15] (k <= 7 scans with its table in LDS): wide
// 128-B lines where they apply (below), else the largest own count of 64-B
// lines (m = k + own - 1 <= 15, own <= 5 / 4, k <= 13) whose 4^m x 64 B fit
// the budget, own >= 2.  Sets *built.
static ks_status table_lines(ks_ctx *ctx, ks_table *t, size_t &budget, const int32_t *freq_dev, bool *built) {
  *built = false;
  const bool u16 = t->compressed;
  if (t->k < 8 || t->k > 15 || getenv("KS_NO_LINES")) return KS_OK;
  // wide 128-B lines (J = own + 3) where they beat the 64-B ones: k = 12 to 15
  // (m = 15: own = 16 - k, J = 6 at k = 13, 4 at k = 15 against 3 for the
  // 17-mer expanded table), at most kWideLut distinct values (13-bit codes),
  // and an L3 escape share (positions whose value is not among the 2047
  // heaviest) of at most 10 %.  KS_NO_WIDE_LINES: the 64-B forms (k <= 13)
  // or the expanded table.
  if (u16 && t->k >= 12 && t->distinct <= kWideLut && ((size_t)128 << 30) <= budget &&
      !getenv("KS_NO_WIDE_LINES")) {
    bool use = false;
    const double t0 = now_ms();
    KS_TRY(choose_code12(ctx, t, freq_dev, 0.10, &use, 2047));  // renumbers the codes by weight
    t->ms_codes12 = now_ms() - t0;
    if (t->d_map12) (void)hipFree(t->d_map12);
    if (t->d_lut12) (void)hipFree(t->d_lut12);
    t->d_map12 = nullptr;
    t->d_lut12 = nullptr;
    if (use) {
      const int own = 16 - t->k;
      const uint64_t nlines = (uint64_t)1 << 30;
      const size_t bytes = nlines * 128;
      const double ta = now_ms();
      size_t cap = 0;
      void *ext = ext_alloc(ctx, bytes, &cap);
      if (ext) {
        t->ms_ext_alloc = now_ms() - ta;
        t->ext_cap = cap;
        hipStream_t st = ctx->stream;
        hipEvent_t a, b;
        KS_HIP(hipEventCreate(&a));
        KS_HIP(hipEventCreate(&b));
        KS_HIP(hipEventRecord(a, st));
        if (own == 1) launch_build_lines<1, 2>(st, t, 15, ext);
        else if (own == 2) launch_build_lines<2, 2>(st, t, 15, ext);
        else if (own == 3) launch_build_lines<3, 2>(st, t, 15, ext);
        else launch_build_lines<4, 2>(st, t, 15, ext);
        KS_HIP(hipGetLastError());
        KS_HIP(hipEventRecord(b, st));
        KS_HIP(hipEventSynchronize(b));
        float ms = 0;
        KS_HIP(hipEventElapsedTime(&ms, a, b));
        KS_HIP(hipEventDestroy(a));
        KS_HIP(hipEventDestroy(b));
        KS_TRY(build_approx(ctx, t, freq_dev));
        t->d_ext = ext;
        t->line_kind = 3;
        t->line_own = own;
        t->ext_J = own + 3;
        t->ext_bits = 13;
        t->ext_bytes = bytes;
        t->ms_ext = ms;
        *built = true;
        return KS_OK;
      }
    }
  }
  // weighted-rank code lines for pass 1 (k = 13..15: one 128-B line per
  // 15-mer, own = 16 - k, J = own + 2 = 5 / 4 / 3 against 4 / 3 / 2 for the
  // FP64 forms; 128 GiB) when the FP64 form the later passes read (64-B lines
  // at k = 13, the expanded table above it: 64 GiB) fits beside them
  if (!u16 && t->d_rcodes && t->k >= 13 && t->k <= 15 && ((size_t)192 << 30) <= budget) {
    const double t0 = now_ms();
    const size_t bytes = ((size_t)1 << 30) * 128;
    size_t cap = 0;
    void *rl = ext_alloc(ctx, bytes, &cap);
    if (rl) {
      if (t->k == 13) launch_build_lines<3, 3>(ctx->stream, t, 15, rl);
      else if (t->k == 14) launch_build_lines<2, 3>(ctx->stream, t, 15, rl);
      else launch_build_lines<1, 3>(ctx->stream, t, 15, rl);
      KS_HIP(hipGetLastError());
      KS_HIP(hipStreamSynchronize(ctx->stream));
      t->d_rlines = rl;
      t->rlines_bytes = bytes;
      t->rlines_cap = cap;
      budget -= bytes;
    }
    t->ms_rlines += now_ms() - t0;
  }
  if (t->d_rcodes) {  // (only the lines read the codes)
    (void)hipFree(t->d_rcodes);
    t->d_rcodes = nullptr;
  }
  if (t->k > 13) return KS_OK;  // (64-B lines need own >= 2: m <= 15)
  int own = std::min(u16 ? 5 : 4, 16 - t->k);
  for (; own >= 2; --own)
    if (((size_t)64 << (2 * (t->k + own - 1))) <= budget) break;
  if (own < 2) return KS_OK;
  const int m = t->k + own - 1;
  const uint64_t nlines = (uint64_t)1 << (2 * m);
  const size_t bytes = nlines * 64;
  const double ta = now_ms();
  size_t cap = 0;
  void *ext = ext_alloc(ctx, bytes, &cap);
  if (!ext) return KS_OK;
  t->ms_ext_alloc = now_ms() - ta;
  t->ext_cap = cap;
  hipStream_t st = ctx->stream;
  hipEvent_t a, b;
  KS_HIP(hipEventCreate(&a));
  KS_HIP(hipEventCreate(&b));
  KS_HIP(hipEventRecord(a, st));
  if (u16) {
    if (own == 5) launch_build_lines<5, 0>(st, t, m, ext);
    else if (own == 4) launch_build_lines<4, 0>(st, t, m, ext);
    else if (own == 3) launch_build_lines<3, 0>(st, t, m, ext);
    else launch_build_lines<2, 0>(st, t, m, ext);
  } else {
    if (own == 4) launch_build_lines<4, 1>(st, t, m, ext);
    else if (own == 3) launch_build_lines<3, 1>(st, t, m, ext);
    else launch_build_lines<2, 1>(st, t, m, ext);
  }
  KS_HIP(hipGetLastError());
  KS_HIP(hipEventRecord(b, st));
  KS_HIP(hipEventSynchronize(b));
  float ms = 0;
  KS_HIP(hipEventElapsedTime(&ms, a, b));
  KS_HIP(hipEventDestroy(a));
  KS_HIP(hipEventDestroy(b));
  KS_TRY(build_approx(ctx, t, freq_dev));
  t->d_ext = ext;
  t->line_kind = u16 ? 1 : 2;
  t->line_own = own;
  t->ext_J = own + (u16 ? 2 : 1);
  t->ext_bits = u16 ? 16 : 64;
  t->ext_bytes = bytes;
  t->ms_ext = ms;
  *built = true;
  return KS_OK;
}

ks_status table_expand(ks_ctx *ctx, ks_table *t, size_t max_bytes, const int32_t *freq_dev) {
  if (t->d_ext || t->ext_J > 1) return KS_OK;
  const bool u16 = t->compressed;
  size_t free_b = 0, total_b = 0;
  KS_HIP(hipMemGetInfo(&free_b, &total_b));
  {  // the pooled buffer of a destroyed table is free memory for this purpose
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (ctx->device >= 0 && ctx->device < 64) free_b += pool_bytes(ctx->device);
  }
  // leave room for the sequences and the scan workspace
  // (total / 8: ~34 GiB on MI355X; the metric scan's workspace is ~4 GB)
  const size_t reserve = std::max<size_t>((size_t)32 << 30, total_b / 8);
  size_t budget = std::min(max_bytes, free_b > reserve ? free_b - reserve : (size_t)0);
  const char *jmax_env = getenv("KS_EXT_MAX_J");  // tests: cap J to exercise every table form
  if (!jmax_env) {  // line tables first (k_pass1l); KS_NO_LINES: the (k+J-1)-mer forms below
    bool built = false;
    KS_TRY(table_lines(ctx, t, budget, freq_dev, &built));
    // (complete on return, the predictor included: a table may be scanned
    // from another context's stream, e.g. genome g + 1's table built while
    // genome g is scanned)
    if (built) KS_HIP(hipStreamSynchronize(ctx->stream));
    if (built) return KS_OK;
  }
  // candidates, best first: (J, code bits); (k+J-1)-mer indices up to 34 bits
  struct Cand { int J, bits; };
  const Cand cands_u16[] = {{5, 12}, {4, 16}, {3, 16}, {2, 16}};
  const Cand cands_f64[] = {{4, 64}, {3, 64}, {2, 64}};
  const Cand *cands = u16 ? cands_u16 : cands_f64;
  const int ncand = u16 ? 4 : 3;
  const int jmax = jmax_env ? atoi(jmax_env) : 5;
  const char *esc_env = getenv("KS_EXT_ESCAPE_MAX");
  const double max_escape = esc_env ? atof(esc_env) : 0.01;
  int J = 0, bits = 16;
  for (int i = 0; i < ncand; ++i) {
    const Cand c = cands[i];
    if (c.J > jmax) continue;
    const int kx = t->k + c.J - 1;
    if (kx > 17) continue;
    if (!u16 && kx > 16) continue;
    const size_t bytes = ((size_t)1 << (2 * kx)) * ext_entry_bytes(u16, c.J);
    if (bytes > budget) continue;
    if (c.bits == 12) {
      bool use = false;
      const double t0 = now_ms();
      KS_TRY(choose_code12(ctx, t, freq_dev, max_escape, &use));
      t->ms_codes12 = now_ms() - t0;
      if (!use) continue;
    }
    J = c.J;
    bits = c.bits;
    break;
  }
  if (J == 0) return KS_OK;
  const int kx = t->k + J - 1;
  const uint64_t nent = (uint64_t)1 << (2 * kx);
  const size_t bytes = nent * ext_entry_bytes(u16, J);
  hipStream_t st = ctx->stream;
  const double ta = now_ms();
  size_t cap = 0;
  void *ext = ext_alloc(ctx, bytes, &cap);
  if (!ext) return KS_OK;
  t->ms_ext_alloc = now_ms() - ta;
  t->ext_cap = cap;
  hipEvent_t a, b;
  KS_HIP(hipEventCreate(&a));
  KS_HIP(hipEventCreate(&b));
  KS_HIP(hipEventRecord(a, st));
  const unsigned grid = (unsigned)std::min<uint64_t>((nent + 255) / 256, (uint64_t)ctx->num_cus * 32);
  // builds with several entries' code loads ahead of their (nontemporal)
  // stores per trip: 12-bit 8 pairs 27.06 vs 28.2 (4), 29.3 (1) ms, plain
  // stores 36.8; FP64 8 halves 28.9 vs 34.2 ms (profiles/r2/s3/ab_ext_build_*)
  if (u16 && bits == 12) {
    hipLaunchKernelGGL(k_build_ext_c12<8>, dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint64_t *)ext);
  } else if (u16) {
    if (J == 4)
      hipLaunchKernelGGL((k_build_ext_u16<4, uint64_t, 8>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent,
                         (uint64_t *)ext);
    else if (J == 3) hipLaunchKernelGGL((k_build_ext_u16<3, uint64_t>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint64_t *)ext);
    else hipLaunchKernelGGL((k_build_ext_u16<2, uint32_t>), dim3(grid), dim3(256), 0, st, t->d_codes, t->k, nent, (uint32_t *)ext);
  } else {
    if (J == 4)
      hipLaunchKernelGGL((k_build_ext_f64<4, 8>), dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
    else if (J == 3) hipLaunchKernelGGL(k_build_ext_f64<3>, dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
    else hipLaunchKernelGGL(k_build_ext_f64<2>, dim3(grid), dim3(256), 0, st, t->d_vals, t->k, nent, (double *)ext);
  }
  KS_HIP(hipGetLastError());
  KS_HIP(hipEventRecord(b, st));
  KS_HIP(hipEventSynchronize(b));
  float ms = 0;
  KS_HIP(hipEventElapsedTime(&ms, a, b));
  KS_HIP(hipEventDestroy(a));
  KS_HIP(hipEventDestroy(b));
  if (bits != 12) {  // a 12-bit assignment that was not used
    if (t->d_map12) (void)hipFree(t->d_map12);
    if (t->d_lut12) (void)hipFree(t->d_lut12);
    t->d_map12 = nullptr;
    t->d_lut12 = nullptr;
  }
  KS_TRY(build_approx(ctx, t, freq_dev));
  KS_HIP(hipStreamSynchronize(ctx->stream));  // (complete on return, as above)
  t->d_ext = ext;
  t->ext_J = J;
  t->ext_bits = bits;
  t->ext_bytes = bytes;
  t->ms_ext = ms;
  return KS_OK;
}

}  // namespace ks

using namespace ks;

extern "C" ks_status ks_table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                     int32_t flags, ks_table **out) {
  return ks_table_create_hint(ctx, w_host, k, thr, flags, nullptr, out);
}

extern "C" ks_status ks_table_create_hint(ks_ctx *ctx, const double *w_host, int32_t k, double thr,
                                          int32_t flags, const int32_t *freq_dev, ks_table **out) {
  return table_create(ctx, w_host, k, thr, flags, freq_dev, 0, out);
}

ks_status ks::table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr, int32_t flags,
                           const int32_t *freq_dev, int64_t max_ext_bytes, ks_table **out) {
  const int32_t allow_compress = flags & KS_TABLE_COMPRESS;
  if (!ctx || !w_host || !out) return fail(KS_ERR_ARG, "ks_table_create: null argument");
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  KS_ENTER(ctx);
  const double t_start = now_ms();
  const int64_t n = (int64_t)1 << (2 * k);
  hipStream_t st = ctx->stream;
  ks_table *t = new ks_table();
  t->ctx = ctx;
  t->device = ctx->device;
  t->k = k;
  t->thr = thr;
  double *d_w = nullptr;
  unsigned long long *d_bits = nullptr, *d_sorted = nullptr;
  void *d_tmp = nullptr;
  int64_t *d_nu = nullptr;
  auto cleanup = [&]() {
    if (d_w) (void)hipFree(d_w);
    if (d_bits) (void)hipFree(d_bits);
    if (d_sorted) (void)hipFree(d_sorted);
    if (d_tmp) (void)hipFree(d_tmp);
    if (d_nu) (void)hipFree(d_nu);
  };
#define KS_TBL_HIP(call)                                                               \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      cleanup();                                                                       \
      ks_table_destroy(t);                                                             \
      return fail(KS_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_));      \
    }                                                                                  \
  } while (0)
  KS_TBL_HIP(hipMalloc(&d_w, n * sizeof(double)));
  KS_TBL_HIP(hipMalloc(&t->d_vals, n * sizeof(double)));
  if (allow_compress) KS_TBL_HIP(hipMalloc(&d_bits, n * sizeof(unsigned long long)));
  debug_poison(d_w, n * sizeof(double));  // (KS_DEBUG_POISON)
  debug_poison(t->d_vals, n * sizeof(double));
  if (allow_compress) debug_poison(d_bits, n * sizeof(unsigned long long));
  if (n * sizeof(double) >= ((size_t)64 << 20)) {  // (one hipMemcpy from pageable memory: 20-55 GB/s)
    const ks_status rc = h2d_pinned(ctx, d_w, w_host, n * sizeof(double), 8);
    if (rc != KS_OK) {
      cleanup();
      ks_table_destroy(t);
      return rc;
    }
  } else {
    KS_TBL_HIP(hipMemcpyAsync(d_w, w_host, n * sizeof(double), hipMemcpyHostToDevice, st));
  }
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_sub_thr, dim3(grid), dim3(256), 0, st, d_w, thr, t->d_vals, d_bits, n);
  KS_TBL_HIP(hipGetLastError());
  {  // finiteness and magnitude (tr_lr decides between the chunked and the literal path)
    unsigned long long *d_am = nullptr, h_am[3] = {0, 0, 0};
    KS_TBL_HIP(hipMalloc(&d_am, 24));
    KS_TBL_HIP(hipMemsetAsync(d_am, 0, 24, st));
    hipLaunchKernelGGL(k_absmax, dim3(grid), dim3(256), 0, st, t->d_vals, n, d_am);
    KS_TBL_HIP(hipMemcpyAsync(h_am, d_am, 24, hipMemcpyDeviceToHost, st));
    KS_TBL_HIP(hipStreamSynchronize(st));
    KS_TBL_HIP(hipFree(d_am));
    t->no_nan_posinf = h_am[1] == 0;
    t->int_exact = h_am[2] == 0;
    double ma = 0;
    memcpy(&ma, &h_am[0], 8);
    t->max_abs = ma;
  }
  t->ms_upload = now_ms() - t_start;
  t->distinct = -1;
  if (allow_compress) {
    KS_TBL_HIP(hipMalloc(&d_sorted, n * sizeof(unsigned long long)));
    KS_TBL_HIP(hipMalloc(&d_nu, sizeof(int64_t)));
    size_t b1 = 0, b2 = 0;
    KS_TBL_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, d_bits, d_sorted, (int)n, 0, 64, st));
    KS_TBL_HIP(hipcub::DeviceSelect::Unique(nullptr, b2, d_sorted, d_bits, d_nu, (int)n, st));
    KS_TBL_HIP(hipMalloc(&d_tmp, std::max(b1, b2)));
    KS_TBL_HIP(hipcub::DeviceRadixSort::SortKeys(d_tmp, b1, d_bits, d_sorted, (int)n, 0, 64, st));
    KS_TBL_HIP(hipcub::DeviceSelect::Unique(d_tmp, b2, d_sorted, d_bits, d_nu, (int)n, st));
    int64_t nu = 0;
    KS_TBL_HIP(hipMemcpyAsync(&nu, d_nu, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    KS_TBL_HIP(hipStreamSynchronize(st));
    t->distinct = nu;
    if (nu >= 1 && nu <= 65536) {
      KS_TBL_HIP(hipMalloc(&t->d_codes, n * sizeof(uint16_t)));
      KS_TBL_HIP(hipMalloc(&t->d_lut, nu * sizeof(double)));
      debug_poison(t->d_codes, n * sizeof(uint16_t));
      debug_poison(t->d_lut, nu * sizeof(double));
      KS_TBL_HIP(hipMemcpyAsync(t->d_lut, d_bits, nu * sizeof(double), hipMemcpyDeviceToDevice, st));
      hipLaunchKernelGGL(k_assign_codes, dim3(grid), dim3(256), 0, st, t->d_vals, d_bits, nu,
                         t->d_codes, n);
      KS_TBL_HIP(hipGetLastError());
      KS_TBL_HIP(hipStreamSynchronize(st));
      t->compressed = true;
      (void)hipFree(t->d_vals);
      t->d_vals = nullptr;
    }
  }
  KS_TBL_HIP(hipStreamSynchronize(st));
#undef KS_TBL_HIP
  cleanup();
  t->ms_compress = now_ms() - t_start - t->ms_upload;
  if (flags & KS_TABLE_EXPAND) {
    const ks_status rc = table_expand(ctx, t, max_ext_bytes > 0 ? (size_t)max_ext_bytes : (size_t)200 << 30, freq_dev);
    if (rc != KS_OK) { ks_table_destroy(t); return rc; }
  }
  t->ms_total = now_ms() - t_start;
  *out = t;
  return KS_OK;
}


extern "C" ks_status ks_table_from_counts(ks_ctx *ctx, const int32_t *counts_dev, int32_t k, int32_t score,
                                          double total, double thr, int32_t flags, int64_t max_ext_bytes,
                                          double *w_dev, ks_table **out) {
  if (!ctx || !counts_dev || !out) return fail(KS_ERR_ARG, "ks_table_from_counts: null argument");
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  if (score != KS_SCORE_LOG2 && score != KS_SCORE_PM1 && score != KS_SCORE_RANK)
    return fail(KS_ERR_ARG, "ks_table_from_counts: unknown score %d", score);
  KS_ENTER(ctx);
  const double t_start = now_ms();
  const int64_t n = (int64_t)1 << (2 * k);
  hipStream_t st = ctx->stream;
  const bool rank = score == KS_SCORE_RANK;
  ks_table *t = new ks_table();
  t->ctx = ctx;
  t->device = ctx->device;
  t->k = k;
  t->thr = thr;
  std::vector<void *> tmp;
  auto cleanup = [&]() {
    for (void *p : tmp) (void)hipFree(p);
    tmp.clear();
  };
#define KS_TFC(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      cleanup();                                                                       \
      ks_table_destroy(t);                                                             \
      return fail(KS_ERR_DEVICE, "%s failed: %s", #call, hipGetErrorString(e_));      \
    }                                                                                  \
  } while (0)
  auto dalloc = [&](size_t bytes) -> void * {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    tmp.push_back(p);
    debug_poison(p, bytes);  // (KS_DEBUG_POISON)
    return p;
  };
  // 1. the counts in stable (count, index) order, their distinct values and
  // multiplicities; scratch in the ctx's grow-only table slot (no per-call
  // hipMalloc of 4^k-sized buffers)
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  size_t b1 = 0, b2 = 0;
  KS_TFC(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, counts_dev, (int32_t *)nullptr, (uint32_t *)nullptr,
                                            (uint32_t *)nullptr, (int)n, 0, 32, st));
  KS_TFC(hipcub::DeviceRunLengthEncode::Encode(nullptr, b2, (int32_t *)nullptr, (int32_t *)nullptr, (int *)nullptr,
                                               (int *)nullptr, (int)n, st));
  {
    size_t bk = 0, bs = 0;
    KS_TFC(hipcub::DeviceRadixSort::SortKeys(nullptr, bk, counts_dev, (int32_t *)nullptr, (int)n, 0, 32, st));
    KS_TFC(hipcub::DeviceScan::ExclusiveSum(nullptr, bs, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, st));
    b1 = std::max(b1, std::max(bk, bs));
  }
  const size_t sn = ((size_t)n * 4 + 255) & ~(size_t)255, tmpb = (std::max(b1, b2) + 255) & ~(size_t)255;
  void *ws = nullptr;
  {
    const ks_status rc = ensure(ctx, SLOT_TABLE_TMP, 5 * sn + 256 + tmpb, &ws);
    if (rc != KS_OK) {
      ks_table_destroy(t);
      return rc;
    }
  }
  char *W = static_cast<char *>(ws);
  int32_t *d_keys = reinterpret_cast<int32_t *>(W);
  uint32_t *d_idx_in = reinterpret_cast<uint32_t *>(W + sn);
  uint32_t *d_idx = reinterpret_cast<uint32_t *>(W + 2 * sn);
  int32_t *d_uniq = reinterpret_cast<int32_t *>(W + 3 * sn);
  int *d_mult = reinterpret_cast<int *>(W + 4 * sn);
  int *d_nu = reinterpret_cast<int *>(W + 5 * sn);
  void *d_tmp = W + 5 * sn + 256;
  if (rank) {
    hipLaunchKernelGGL(k_iota, dim3(grid), dim3(256), 0, st, d_idx_in, n);
    KS_TFC(hipGetLastError());
  }
  // the sort orders only the bits some count uses (metric genome: < 2^24, three
  // 8-bit passes instead of four); a negative (wrapped) count keeps all 32
  int end_bit = 32;
  {
    unsigned int *d_or = reinterpret_cast<unsigned int *>(d_nu) + 4, h_or = 0;
    KS_TFC(hipMemsetAsync(d_or, 0, 4, st));
    hipLaunchKernelGGL(k_count_or, dim3((unsigned)std::min<int64_t>((n + 4095) / 4096, 1024)), dim3(256), 0, st,
                       counts_dev, n, d_or);
    KS_TFC(hipGetLastError());
    KS_TFC(hipMemcpyAsync(&h_or, d_or, 4, hipMemcpyDeviceToHost, st));
    KS_TFC(hipStreamSynchronize(st));
    end_bit = 1;
    while (end_bit < 32 && (h_or >> end_bit) != 0) ++end_bit;
  }
  // log2 / pm1 with a value histogram that fits the scratch: no sort (the
  // metric genome: 1.3 ms of radix sort and run-length encoding per table)
  const int64_t R = std::max<int64_t>((int64_t)1 << end_bit, kValLds);
  const uint32_t *d_dense = nullptr;
  if (!rank && end_bit < 32 && (size_t)R * 4 <= sn && (size_t)kValBlocks * kValLds * 4 <= sn) {
    uint32_t *hist = reinterpret_cast<uint32_t *>(d_keys), *rows = d_idx_in, *flags = d_idx, *pos = d_idx_in;
    const int gv = (int)std::min<int64_t>((R + 255) / 256, 4096);
    KS_TFC(hipMemsetAsync(hist, 0, (size_t)R * 4, st));
    hipLaunchKernelGGL(k_val_hist, dim3(kValBlocks), dim3(1024), 0, st, counts_dev, n, rows, hist);
    hipLaunchKernelGGL(k_val_cols, dim3(kValLds / 256), dim3(256), 0, st, rows, kValBlocks, hist);
    hipLaunchKernelGGL(k_val_flags, dim3(gv), dim3(256), 0, st, hist, R, flags);
    KS_TFC(hipGetLastError());
    KS_TFC(hipcub::DeviceScan::ExclusiveSum(d_tmp, b1, flags, pos, (int)R, st));  // (rows are summed by now)
    hipLaunchKernelGGL(k_val_compact, dim3(gv), dim3(256), 0, st, hist, pos, R, d_uniq, d_mult, d_nu, flags);
    KS_TFC(hipGetLastError());
    d_dense = flags;
  } else {
    if (rank)
      KS_TFC(hipcub::DeviceRadixSort::SortPairs(d_tmp, b1, counts_dev, d_keys, d_idx_in, d_idx, (int)n, 0, end_bit, st));
    else
      KS_TFC(hipcub::DeviceRadixSort::SortKeys(d_tmp, b1, counts_dev, d_keys, (int)n, 0, end_bit, st));
    KS_TFC(hipcub::DeviceRunLengthEncode::Encode(d_tmp, b2, d_keys, d_uniq, d_mult, d_nu, (int)n, st));
  }
  int nu = 0;
  KS_TFC(hipMemcpyAsync(&nu, d_nu, sizeof(int), hipMemcpyDeviceToHost, st));
  KS_TFC(hipStreamSynchronize(st));
  std::vector<int32_t> dv(nu);
  std::vector<int> dm32(nu);
  KS_TFC(hipMemcpyAsync(dv.data(), d_uniq, (size_t)nu * 4, hipMemcpyDeviceToHost, st));
  KS_TFC(hipMemcpyAsync(dm32.data(), d_mult, (size_t)nu * 4, hipMemcpyDeviceToHost, st));
  KS_TFC(hipStreamSynchronize(st));
  std::vector<int64_t> dm(dm32.begin(), dm32.end());
  t->distinct = -1;
  if (rank) {
    // 2r. ranks: closed-form prefix pieces filled on the device, then s = w - thr
    double *d_w = w_dev ? w_dev : static_cast<double *>(dalloc(n * 8));
    if (!d_w) {
      cleanup();
      ks_table_destroy(t);
      return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed (ranks)");
    }
    const std::vector<RankPiece> P = rank_pieces(dv.data(), dm.data(), nu, total);
    if (!P.empty()) {
      RankPiece *d_p = static_cast<RankPiece *>(dalloc(P.size() * sizeof(RankPiece)));
      if (!d_p) {
        cleanup();
        ks_table_destroy(t);
        return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed (pieces)");
      }
      KS_TFC(hipMemcpyAsync(d_p, P.data(), P.size() * sizeof(RankPiece), hipMemcpyHostToDevice, st));
      const unsigned g = (unsigned)std::min<int64_t>(((n + 15) / 16 + 255) / 256, 8192);
      hipLaunchKernelGGL(k_rank_fill, dim3(g), dim3(256), 0, st, d_idx, n, d_p, (int64_t)P.size(), d_w);
      KS_TFC(hipGetLastError());
      // 2r'. the 32-bit rank codes of the code lines (k = 13, expanded tables)
      if (k >= 13 && k <= 15 && (flags & KS_TABLE_EXPAND) && !getenv("KS_NO_RANK_CODES")) {
        const double tr0 = now_ms();
        // uniform pieces: bits(R_j) = base + (j - j0) * inc over [j0, j0 + len),
        // len <= 2^kRankOffBits; a kind-1 piece's first position is a piece of
        // its own (rank_piece_value); weight = positions covered (count x len)
        std::vector<int64_t> cls(nu + 1, 0);
        for (int i = 0; i < nu; ++i) cls[i + 1] = cls[i] + dm[i];
        struct UP {
          int64_t j0;
          unsigned long long base, inc;
          double wt;
        };
        std::vector<UP> up;
        bool ok = true;
        const int64_t lim = (int64_t)1 << kRankOffBits;
        for (size_t i = 0; i < P.size() && ok; ++i) {
          const int64_t a = P[i].j0, b = i + 1 < P.size() ? P[i + 1].j0 : n;
          const int ci = (int)(std::upper_bound(cls.begin(), cls.end(), a) - cls.begin()) - 1;
          const double c = (double)std::max(0, dv[std::max(0, std::min(ci, nu - 1))]);
          unsigned long long r0b;
          memcpy(&r0b, &P[i].r0, 8);
          auto add = [&](int64_t j0, int64_t j1, unsigned long long base, unsigned long long inc) {
            for (int64_t s0 = j0; s0 < j1; s0 += lim)
              up.push_back(UP{s0, base + (unsigned long long)(s0 - j0) * inc, inc, c * (double)(std::min(j1, s0 + lim) - s0)});
          };
          if (P[i].kind == 0) {
            add(a, b, r0b, 0ull);
          } else {
            add(a, a + 1, r0b, 0ull);
            if (b > a + 1) {
              const unsigned long long m = (r0b & ((1ull << 52) - 1)) | (1ull << 52);
              const unsigned long long base = ((unsigned long long)(P[i].e + 1023) << 52) + (m + (unsigned long long)P[i].inc1 - (1ull << 52));
              add(a + 1, b, base, (unsigned long long)P[i].inc);
            }
          }
          ok = up.size() <= ((size_t)1 << (32 - kRankOffBits));
        }
        if (ok && !up.empty()) {
          const int64_t np = (int64_t)up.size();
          std::vector<int32_t> ord(np);
          for (int64_t i = 0; i < np; ++i) ord[i] = (int32_t)i;
          std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return up[x].wt > up[y].wt; });
          std::vector<int32_t> uh(np);
          std::vector<unsigned long long> pc(2 * np);
          double wall = 0, whot = 0;
          for (int64_t h = 0; h < np; ++h) {
            const UP &u = up[ord[h]];
            uh[ord[h]] = (int32_t)h;
            pc[2 * h] = u.base;
            pc[2 * h + 1] = u.inc;
            wall += u.wt;
            if (h < kRankPieceLds) whot += u.wt;
          }
          std::vector<int64_t> uj0(np);
          for (int64_t i = 0; i < np; ++i) uj0[i] = up[i].j0;
          int64_t *d_uj0 = static_cast<int64_t *>(dalloc((size_t)np * 8));
          int32_t *d_uh = static_cast<int32_t *>(dalloc((size_t)np * 4));
          unsigned long long *d_bad = static_cast<unsigned long long *>(dalloc(8));
          uint32_t *d_rc = nullptr;
          unsigned long long *d_pc = nullptr;
          if (d_uj0 && d_uh && d_bad && hipMalloc(&d_rc, (size_t)n * 4) == hipSuccess &&
              hipMalloc(&d_pc, (size_t)np * 16) == hipSuccess) {
            KS_TFC(hipMemcpyAsync(d_uj0, uj0.data(), (size_t)np * 8, hipMemcpyHostToDevice, st));
            KS_TFC(hipMemcpyAsync(d_uh, uh.data(), (size_t)np * 4, hipMemcpyHostToDevice, st));
            KS_TFC(hipMemcpyAsync(d_pc, pc.data(), (size_t)np * 16, hipMemcpyHostToDevice, st));
            KS_TFC(hipMemsetAsync(d_bad, 0, 8, st));
            hipLaunchKernelGGL(k_rank_codes, dim3(g), dim3(256), 0, st, d_idx, n, d_uj0, d_uh, np, d_rc);
            hipLaunchKernelGGL(k_rank_codes_check, dim3(grid), dim3(256), 0, st, d_rc, d_pc, d_w, n, np, d_bad);
            KS_TFC(hipGetLastError());
            unsigned long long bad = 0;
            KS_TFC(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, st));
            KS_TFC(hipStreamSynchronize(st));
            if (bad == 0) {
              t->d_rcodes = d_rc;
              t->d_rpieces = d_pc;
              t->n_rpieces = (int32_t)np;
              t->rpieces_cover = wall > 0 ? whot / wall : 1.0;
              d_rc = nullptr;
              d_pc = nullptr;
            } else {
              fprintf(stderr, "kmer_spans_amd: %llu rank codes do not decode to their ranks; no code lines\n", bad);
            }
          } else {
            (void)hipGetLastError();
          }
          if (d_rc) (void)hipFree(d_rc);
          if (d_pc) (void)hipFree(d_pc);
        }
        t->ms_rlines = now_ms() - tr0;
      }
    } else {  // wrapped (negative) counts: the host's sequential prefix
      std::vector<int32_t> hc(n);
      std::vector<double> hr(n);
      KS_TFC(hipMemcpyAsync(hc.data(), counts_dev, n * 4, hipMemcpyDeviceToHost, st));
      KS_TFC(hipStreamSynchronize(st));
      const ks_status rc = rank_table_host(hc.data(), k, total, hr.data());
      if (rc != KS_OK) {
        cleanup();
        ks_table_destroy(t);
        return rc;
      }
      KS_TFC(hipMemcpyAsync(d_w, hr.data(), n * 8, hipMemcpyHostToDevice, st));
      KS_TFC(hipStreamSynchronize(st));
    }
    KS_TFC(hipMalloc(&t->d_vals, n * sizeof(double)));
    debug_poison(t->d_vals, n * sizeof(double));  // (KS_DEBUG_POISON)
    hipLaunchKernelGGL(k_sub_thr, dim3(grid), dim3(256), 0, st, d_w, thr, t->d_vals, nullptr, n);
    KS_TFC(hipGetLastError());
    unsigned long long *d_am = static_cast<unsigned long long *>(dalloc(24)), h_am[3] = {0, 0, 0};
    if (!d_am) {
      cleanup();
      ks_table_destroy(t);
      return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed");
    }
    KS_TFC(hipMemsetAsync(d_am, 0, 24, st));
    hipLaunchKernelGGL(k_absmax, dim3(grid), dim3(256), 0, st, t->d_vals, n, d_am);
    KS_TFC(hipMemcpyAsync(h_am, d_am, 24, hipMemcpyDeviceToHost, st));
    KS_TFC(hipStreamSynchronize(st));
    t->no_nan_posinf = h_am[1] == 0;
    t->int_exact = h_am[2] == 0;
    memcpy(&t->max_abs, &h_am[0], 8);
    t->ms_upload = now_ms() - t_start;
  } else {
    // 2s. log2 / +-1 of each distinct count on the host (glibc log2, exactly as
    // ks_log2_table / ks_pm1_table), s = w - thr, distinct s values by bits
    std::vector<double> wv(nu), sv(nu);
    score_of_counts(score == KS_SCORE_LOG2 ? 1 : 2, dv.data(), dm.data(), nu, wv.data());
    std::vector<uint64_t> sb(nu);
    double ma = 0.0;
    bool bad = false, nonint = false;
    for (int i = 0; i < nu; ++i) {
      sv[i] = wv[i] - thr;
      memcpy(&sb[i], &sv[i], 8);
      if (std::isfinite(sv[i])) ma = std::max(ma, std::fabs(sv[i]));
      else if (!(sv[i] < 0)) bad = true;
      if (!(std::isfinite(sv[i]) && sv[i] == std::rint(sv[i]) && std::fabs(sv[i]) <= 0x1p20)) nonint = true;
    }
    t->no_nan_posinf = !bad;
    t->int_exact = !nonint;
    t->max_abs = ma;
    std::vector<uint64_t> ub(sb);
    std::sort(ub.begin(), ub.end());
    ub.erase(std::unique(ub.begin(), ub.end()), ub.end());
    const int64_t nv = (int64_t)ub.size();
    t->distinct = nv;
    t->ms_upload = now_ms() - t_start;
    const int gm = (int)std::min<int64_t>((n + 1023) / 1024, (int64_t)ctx->num_cus * 8);
    if ((flags & KS_TABLE_COMPRESS) && nv <= 65536) {
      std::vector<uint16_t> cmap(nu);
      for (int i = 0; i < nu; ++i) cmap[i] = (uint16_t)(std::lower_bound(ub.begin(), ub.end(), sb[i]) - ub.begin());
      uint16_t *d_cmap = static_cast<uint16_t *>(dalloc((size_t)nu * 2 + 16));
      if (!d_cmap) {
        cleanup();
        ks_table_destroy(t);
        return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed");
      }
      t->d_codes = static_cast<uint16_t *>(cpool_take(ctx->device, n * sizeof(uint16_t)));
      t->codes_pooled = true;
      if (!t->d_codes) KS_TFC(hipMalloc(&t->d_codes, n * sizeof(uint16_t)));
      KS_TFC(hipMalloc(&t->d_lut, nv * sizeof(double)));
      KS_TFC(hipMemcpyAsync(t->d_lut, ub.data(), nv * 8, hipMemcpyHostToDevice, st));
      KS_TFC(hipMemcpyAsync(d_cmap, cmap.data(), (size_t)nu * 2, hipMemcpyHostToDevice, st));
      if (d_dense)
        hipLaunchKernelGGL(k_map_dense<uint16_t>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_dense, d_cmap, t->d_codes);
      else
        hipLaunchKernelGGL(k_map_counts<uint16_t>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_uniq, (int64_t)nu,
                           d_cmap, t->d_codes);
      KS_TFC(hipGetLastError());
      t->compressed = true;
    } else {
      double *d_sv = static_cast<double *>(dalloc((size_t)nu * 8 + 16));
      if (!d_sv) {
        cleanup();
        ks_table_destroy(t);
        return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed");
      }
      KS_TFC(hipMalloc(&t->d_vals, n * sizeof(double)));
    debug_poison(t->d_vals, n * sizeof(double));  // (KS_DEBUG_POISON)
      KS_TFC(hipMemcpyAsync(d_sv, sv.data(), (size_t)nu * 8, hipMemcpyHostToDevice, st));
      if (d_dense)
        hipLaunchKernelGGL(k_map_dense<double>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_dense, d_sv, t->d_vals);
      else
        hipLaunchKernelGGL(k_map_counts<double>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_uniq, (int64_t)nu, d_sv,
                           t->d_vals);
      KS_TFC(hipGetLastError());
    }
    if (w_dev) {
      double *d_wv = static_cast<double *>(dalloc((size_t)nu * 8 + 16));
      if (!d_wv) {
        cleanup();
        ks_table_destroy(t);
        return fail(KS_ERR_NOMEM, "ks_table_from_counts: device allocation failed");
      }
      KS_TFC(hipMemcpyAsync(d_wv, wv.data(), (size_t)nu * 8, hipMemcpyHostToDevice, st));
      if (d_dense)
        hipLaunchKernelGGL(k_map_dense<double>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_dense, d_wv, w_dev);
      else
        hipLaunchKernelGGL(k_map_counts<double>, dim3(gm), dim3(1024), 0, st, counts_dev, n, d_uniq, (int64_t)nu, d_wv,
                           w_dev);
      KS_TFC(hipGetLastError());
    }
  }
  KS_TFC(hipStreamSynchronize(st));
#undef KS_TFC
  cleanup();
  if (ctx->slots[SLOT_TABLE_TMP].bytes > ((size_t)4 << 30)) {  // k >= 14: ~20 B x 4^k of sort scratch
    (void)hipFree(ctx->slots[SLOT_TABLE_TMP].ptr);                // is not kept on the context
    ctx->slots[SLOT_TABLE_TMP] = DevBuf();
  }
  t->ms_compress = now_ms() - t_start - t->ms_upload;
  if (flags & KS_TABLE_EXPAND) {
    const size_t cap = max_ext_bytes > 0 ? (size_t)max_ext_bytes : (size_t)200 << 30;
    const ks_status rc = table_expand(ctx, t, cap, counts_dev);
    if (rc != KS_OK) {
      ks_table_destroy(t);
      return rc;
    }
  }
  t->ms_total = now_ms() - t_start;
  *out = t;
  return KS_OK;
}

extern "C" void ks_table_destroy(ks_table *t) {
  if (!t) return;
  if (!hip_usable_here()) {  // inherited across fork(): leave the parent's device memory alone
    delete t;
    return;
  }
  if (t->d_vals) (void)hipFree(t->d_vals);
  if (t->d_codes && t->codes_pooled) cpool_give(t->device, t->d_codes, ((size_t)2) << (2 * t->k));
  else if (t->d_codes) (void)hipFree(t->d_codes);
  if (t->d_lut) (void)hipFree(t->d_lut);
  if (t->d_ext) pool_give(t->device, t->d_ext, t->ext_cap);
  if (t->d_map12) (void)hipFree(t->d_map12);
  if (t->d_lut12) (void)hipFree(t->d_lut12);
  if (t->d_approx) (void)hipFree(t->d_approx);
  if (t->d_rcodes) (void)hipFree(t->d_rcodes);
  if (t->d_rpieces) (void)hipFree(t->d_rpieces);
  if (t->d_rlines) pool_give(t->device, t->d_rlines, t->rlines_cap);
  delete t;
}

namespace ks {
// The pooled buffer of one device goes back to the driver (ks_ctx_destroy).
void pool_release_device(int dev) {
  if (dev < 0 || dev >= 64) return;
  std::lock_guard<std::mutex> g(g_pool_mu);
  pool_free_all(dev);
}
}  // namespace ks

extern "C" void ks_release_cache(void) {
  regions_cache_release();
  if (!hip_usable_here()) return;
  janitor_release_all();
  std::lock_guard<std::mutex> g(g_pool_mu);
  for (int d = 0; d < 64; ++d) pool_free_all(d);
}

extern "C" int32_t ks_table_is_compressed(const ks_table *t) { return t && t->compressed ? 1 : 0; }
extern "C" int64_t ks_table_distinct(const ks_table *t) { return t ? t->distinct : -1; }
extern "C" int32_t ks_table_positions_per_read(const ks_table *t) {
  return t ? (t->d_rlines ? 18 - t->k : t->ext_J) : 0;  // (rank code lines: own 16 - k + L1 + L2)
}
extern "C" int32_t ks_table_code_bits(const ks_table *t) {
  if (!t) return 0;
  if (t->ext_J > 1 && t->compressed) return t->ext_bits;
  return t->compressed ? 16 : 64;
}
extern "C" ks_status ks_table_get_info(const ks_table *t, ks_table_info *out) {
  if (!t || !out) return fail(KS_ERR_ARG, "null argument");
  memset(out, 0, sizeof(*out));
  out->k = t->k;
  out->compressed = t->compressed ? 1 : 0;
  out->positions_per_read = ks_table_positions_per_read(t);  // (pass 1's: the rank code lines, k_pass1r)
  out->code_bits = t->d_rlines ? 32 : ks_table_code_bits(t);
  out->distinct = t->distinct;
  out->ext_bytes = (int64_t)(t->ext_bytes + t->rlines_bytes);
  out->escape_fraction = ks_table_escape_fraction(t);
  out->ms_upload = t->ms_upload;
  out->ms_compress = t->ms_compress;
  out->ms_codes12 = t->ms_codes12;
  out->ms_ext_alloc = t->ms_ext_alloc;
  out->ms_ext_build = t->ms_ext + t->ms_rlines;
  out->ms_total = t->ms_total;
  out->line_kind = t->d_rlines ? 4 : t->line_kind;  // (4: rank code lines for pass 1, FP64 lines after it)
  out->line_own = t->line_own;
  return KS_OK;
}

extern "C" double ks_table_escape_fraction(const ks_table *t) {
  // 12-bit (k+4)-mer tables: share of scan indices that escape; wide lines
  // (13): share of the L3 indices (one per line) that escape
  return (t && (t->ext_bits == 12 || t->ext_bits == 13)) ? t->escape_frac : 0.0;
}
