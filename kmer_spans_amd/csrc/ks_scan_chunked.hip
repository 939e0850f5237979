// ks_scan_chunked.hip -- chunked carry scan (algo 1): the span scan with
// parallelism inside runs, bit-exact with the sequential reference.
//
// The sequential state machine of kmer_regions (kmer_spans.c:243-307) is
// decomposed (SURVEY 8(a) a5', verified by oracle/pyoracle.py):
//   T_i = max(fl(T_{i-1} + s_i), 0) over each run's scan indices [a+k, b-1];
//   excursions = maximal stretches with T > 0 (beg, first argmax, max, end);
//   an emitted excursion adds a region and a fresh rescan of (argmax, end].
// Every run is cut into chunks of CH = 256 scan indices, one lane each.
//
//  P1 (gather pass, the only random-access pass): codes -> table values;
//     clean-entry trajectory C_j (entry 0) of every chunk: exit value, the
//     open trailing excursion, closed emittable excursions ("candidates");
//     approximate aggregates (sum, min/max prefix); compressed tables also
//     store each index's uint16 table code so later passes stream 2 B/index.
//  P2 approximate max-plus scan of (sum, clean exit) per run -> predicted
//     entry x~_j; where x~_j puts the whole chunk inside one binade
//     [2^e, 2^(e+1)) far from 0, the chunk's binade-integer summary is built:
//     with S = m * 2^(e-52), fl(S + s) = S + RN(s / 2^(e-52)) exactly, ties to
//     even decided by the parity of m, so a chunk is an integer map
//     m -> m + D[parity(m)] with max/argmax/min per entry parity.
//  P3 exact carry per run (sequential over chunks, O(1) per chunk):
//     entry 0 -> exit C_j exactly;  summary valid for the exact entry ->
//     integer arithmetic;  x + minprefix < -margin -> the true trajectory
//     clamps in the chunk and then coincides with C_j (monotone rounding),
//     so the exit is C_j exactly;  otherwise exact replay of the chunk.
//  P4 heads: per chunk with positive exact entry, the part of the carried
//     excursion before its first clamp (replay, or the summary).
//  P5 stitch per run: excursions from heads, tails and candidates; emit
//     regions + rescan ranges; rescans run on the lane kernel.
#include <hip/hip_fp16.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "ks_scan_common.h"

namespace ks {

ks_status launch_scan_lane(ks_ctx *ctx, const uint8_t *seq, int64_t total, const int64_t *ra, const int64_t *rb,
                           const int32_t *rs, int64_t n, int k, const TableView &tv, uint64_t mw,
                           double min_score, uint32_t *visits, const RegionBuf &out,
                           const unsigned long long *d_cnt = nullptr, int64_t segcap = 0,
                           const ScanMode &mode = ScanMode(), int init_step = 1, const int64_t *offs = nullptr,
                           const uint32_t *packed = nullptr, hipStream_t strm = nullptr);

namespace {

constexpr int CH = 256;  // scan indices per chunk (one lane)
constexpr int NB = 16;   // indices per gather batch
constexpr int kModeClean = 0, kModeL = 1, kModeR = 2, kModeU = 3;

struct Chunks {
  int64_t *start;  // first scan index (global position)
  int32_t *n;      // indices in the chunk
  int32_t *run;    // run id
  int64_t nch;     // chunks [c0, nch) are this launch's (a half of the runs, see scan_chunked)
  const uint32_t *packed;  // 2-bit base codes (Runs::packed), nullptr: roll the bytes
  int64_t c0 = 0;
};

struct P1 {  // per-chunk results of the gather pass
  double *cexit, *asum, *pmin, *pmax, *sabs, *tmax;
  int32_t *tbeg, *targ;  // trailing open excursion (relative), tbeg = -1: none
  uint8_t *special;      // a non-finite value occurred
  int32_t *parg;         // first index of the prefix maximum pmax
  // epoch guard: pass 1 stamps every chunk it wrote with this call's epoch
  // (ks_ctx::scan_epoch); the stitch checks the stamp of every chunk whose
  // pass-1 results it reads (error bit 32: results of another call)
  uint32_t *ep = nullptr;
  uint32_t epoch = 0;
};

struct Summ {  // binade-integer summaries for the predicted binade (P2)
  int32_t *e;             // binade, INT32_MIN: none
  long long *D, *M, *N;   // [2 * nch] by entry parity
  int32_t *A;             // [2 * nch]
  // pass-1 summaries (p1summ): sel[c] < 2 = the chunk's summary is pass 1's
  // slot 2c + sel[c] of pD..pA for both entry parities (k_marks_select keeps
  // it in place instead of copying it into D..A); 2 = D..A.  sel null: D..A.
  uint8_t *sel = nullptr;
  const long long *pD = nullptr, *pM = nullptr, *pN = nullptr;
  const int32_t *pA = nullptr;
};

// Where chunk c's summary fields are: index i0 (entry parity 0) and i1
// (parity 1) into D / M / N / A.
struct SummAt {
  const long long *D, *M, *N;
  const int32_t *A;
  int64_t i0, i1;
};
__device__ __forceinline__ SummAt summ_at(const Summ &sm, int64_t c) {
  if (sm.sel) {
    const int s = sm.sel[c];
    if (s < 2) return SummAt{sm.pD, sm.pM, sm.pN, sm.pA, 2 * c + s, 2 * c + s};
  }
  return SummAt{sm.D, sm.M, sm.N, sm.A, 2 * c, 2 * c + 1};
}

struct SummP1 {  // binade summaries computed by pass 1 for the predicted binade (single trajectory)
  int32_t *e;             // [2 * nch] binade, INT32_MIN: none (no prediction, a tie, out of range)
  long long *D, *M, *N;   // [2 * nch] total, max, min (units 2^(e-52))
  int32_t *A;             // [2 * nch] first argmax
};

// A pass-1 summary of chunk c in binade e (slot t of the predicted binade and
// its neighbour): the binade-integer map of the chunk (D, M, N, A as
// chunk_summary_impl) from the steps r = (s + 1.5 * 2^e) - 1.5 * 2^e summed
// in FP64.  Valid if no step was a tie (bad), every |s| < 2^(e-1) (so the
// magic constant rounds s to the ulp 2^(e-52)) and every partial sum of the
// r inside (-2^e, 2^e) (so the sums are exact multiples of the ulp): then D,
// the maximum M and the minimum N are the integer trajectory's, exactly.
// (Until round 5 every partial sum of |s| had to stay below 2^(e-1) and N was
// a lower bound from the FP64 prefix minimum minus a 130-ulp margin; the
// exact form measured the same: metric step 14.59 vs 14.72 ms, weighted rank
// k = 15 61.9 vs 61.7 ms, profiles/r5/ab/ab_p1summ_exact*.txt)
__device__ __forceinline__ void summ_put(const SummP1 &sp, int64_t c, int t, int e, bool bad, double maxabs,
                                         double cur, double mx, double mn, int a) {
  const double lim = ldexp(1.0, e);
  // (a NaN step leaves cur NaN; fmin / fmax skip it in mn, mx, maxabs)
  const bool ok = e != INT32_MIN && !bad && cur == cur && maxabs < 0.5 * lim && mn <= mx && mx < lim && mn > -lim;
  sp.e[2 * c + t] = ok ? e : INT32_MIN;
  if (ok) {
    const double sc = ldexp(1.0, 52 - e);
    sp.D[2 * c + t] = (long long)(cur * sc);
    sp.M[2 * c + t] = (long long)(mx * sc);
    sp.N[2 * c + t] = (long long)(mn * sc);
    sp.A[2 * c + t] = a;
  }
}                        // slot 2c: the predicted binade, 2c + 1: its neighbour near an edge

struct Carry {  // P3/P4
  double *x;      // exact entry value
  uint8_t *mode;
  int32_t *hq;    // first clamp in the chunk (relative), -1 none
  double *hmax;   // max of the carried head (valid if the head is non-empty)
  int32_t *harg;
};

// Composites of the global 64-chunk tiles (chunks [64t, 64t + 64)) for the
// carry's tile batches: k_tile_comp writes, per tile whose chunks all have a
// summary in one binade e, the composed increment D_p of the tile and the
// interval [LO_p, HI_p] of entry mantissas (parity p) for which every
// chunk's trajectory stays inside the binade -- exactly the fast-tile test
// of carry_segment, reduced over the tile.  em / ee: the entry mantissa and
// binade of each tile the carry accepted in a batch (ee = INT32_MIN: not
// batched), expanded per chunk by k_tile_apply.
struct TileComp {
  int32_t *e;                // [tiles] binade, INT32_MIN: no composite
  long long *D, *LO, *HI;    // [2 * tiles] by entry parity
  long long *em;             // [tiles]
  int32_t *ee;               // [tiles]
};

// Values of the chunks the carry will likely replay (no summary, a predicted
// positive entry that does not clamp for certain), gathered ahead in
// parallel (k_summ_fixw): a replay then costs one coalesced 32-B load
// per lane instead of the dependent base / code / LUT loads of values4.
struct ReplayBuf {
  int32_t *slot;             // [nch] slot of chunk c, -1: none
  int64_t *chunk;            // [2 * cap] chunk of a slot
  double *v;                 // [2 * cap * 256] values, lane-major (4 per lane)
  unsigned long long *count; // [2] listed chunks per half (may exceed cap: those are not listed)
  int64_t cap;               // slots per half
};

struct Cand {  // closed emittable excursions of the clean trajectories (segmented append)
  long long *beg, *arg, *rst;
  double *best;
  unsigned long long *count;  // [kSegs]
  int64_t cap, segcap;
};

struct Rescan {
  int64_t *a, *b;  // virtual runs [a, b) for the lane kernel (segmented append)
  int32_t *seq;
  unsigned long long *count;  // [kSegs]
  int64_t cap, segcap;
};

// Emission rules of the scan (kmer_regions or tr_lr, see ScanMode).
struct EmitCfg {
  int trlr;
  uint64_t mw;          // kmer_regions: (size_t)min_width
  double min_score;     // kmer_regions
  int64_t min_len;      // tr_lr
  const double *ks;     // tr_lr: score of each run's first k-mer
  int k;
};

// tr_lr position of scan index j in a run whose first scan index is f: the
// first k-mer's step sits at f, the transition of the k-mer ending at p at
// index p + 1.  kmer_regions reports scan indices.
__device__ __forceinline__ int64_t pos_of(const EmitCfg &ec, int64_t j, int64_t f) {
  return (ec.trlr && j != f) ? j - 1 : j;
}

// What an excursion (beg, first argmax arg, max best, ending at scan index
// end; closed = it returned to 0 there, else open at the run end) produces:
// a region record and/or a rescan range (virtual run [res_a, res_b) for the
// lane kernel).  f = the run's first scan index.
struct Emission {
  bool reg, res;
  int64_t rbeg, rend;    // region record (positions)
  int64_t res_a, res_b;
};

__device__ __forceinline__ Emission decide(const EmitCfg &ec, int64_t f, int64_t beg, int64_t arg, double best,
                                           int64_t end, bool closed) {
  Emission e;
  if (!ec.trlr) {  // kmer_regions: emitted excursions rescan (arg, end], open ones included
    e.reg = (uint64_t)(arg - beg) >= ec.mw && best >= ec.min_score;
    e.res = e.reg && arg + 1 <= end;
    e.rbeg = beg;
    e.rend = arg;
    e.res_a = arg + 1 - ec.k;
    e.res_b = end + 1;
  } else {  // tr_lr: positions; every closed excursion rescans (pos(arg), pos(end)]
    const int64_t pb = pos_of(ec, beg, f), pa = pos_of(ec, arg, f), pe = pos_of(ec, end, f);
    e.reg = pa - pb >= ec.min_len;
    // ... but only a tail that can hold a region (>= min_len + 1 positions, and
    // >= 2: a one-position tail cannot even hold an excursion) changes the
    // output; the scan after the tail is the top-level one either way
    e.res = closed && pe - pa - 1 >= (ec.min_len > 1 ? ec.min_len : 1);
    e.rbeg = pb;
    e.rend = pa;
    e.res_a = pa + 1 - ec.k;  // lane kernel (tr_lr): positions [res_a + k, res_b)
    e.res_b = pe + 1;
  }
  (void)best;
  return e;
}

// Bits of a positive normal double in binade e: x = m * 2^(e-52), m in [2^52, 2^53).
__device__ __forceinline__ int binade_of(double x) {
  return (int)((__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
}
__device__ __forceinline__ long long mant_of(double x) {
  return (__double_as_longlong(x) & ((1LL << 52) - 1)) | (1LL << 52);
}
__device__ __forceinline__ double from_mant(long long m, int e) {
  return __longlong_as_double(((long long)(e + 1023) << 52) | (m - (1LL << 52)));
}

__device__ __forceinline__ uint32_t roll(uint32_t c, uint8_t b, uint32_t mask) {
  return ((c << 2) | enc(b)) & mask;
}

// 16 bytes at an arbitrary position (two aligned 16-byte loads).
__device__ __forceinline__ void load16(const uint8_t *__restrict__ seq, int64_t p, int64_t total,
                                       uint8_t out[16]) {
  const int64_t a0 = p & ~(int64_t)15;
  const int sh = (int)(p - a0);
  uint32_t w[8];
  uint4 v0 = make_uint4(0x4e4e4e4eu, 0x4e4e4e4eu, 0x4e4e4e4eu, 0x4e4e4e4eu), v1 = v0;
  if (a0 < total) v0 = *reinterpret_cast<const uint4 *>(seq + a0);
  if (a0 + 16 < total) v1 = *reinterpret_cast<const uint4 *>(seq + a0 + 16);
  w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w; w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int q = sh + j;
    out[j] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
  }
}

__device__ __forceinline__ size_t code_slot(int64_t c, int i) {
  // [tile = c/64][i/4][lane = c%64][i%4]: a wave's lanes store 8 B each, contiguous
  return ((((size_t)(c >> 6) * (CH / 4) + (size_t)(i >> 2)) * 64 + (size_t)(c & 63)) << 2) + (size_t)(i & 3);
}

// Three dwords at a 4-byte-aligned address (one global_load_dwordx3).
typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// The 16 codes of indices b0 .. b0+15 (b0 % 4 == 0) as 8 words of 2 codes.
__device__ __forceinline__ void load_codes16(const uint16_t *__restrict__ codes, int64_t c, int b0, uint32_t w[8]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const uint2 x = *reinterpret_cast<const uint2 *>(codes + code_slot(c, b0 + 4 * h));
    w[2 * h] = x.x;
    w[2 * h + 1] = x.y;
  }
}

// Values of NV consecutive scan indices from a line table (ks_table
// line_kind), OWN + 1 per line read: the line's own entries and the L1 entry
// chosen by the next base (its first 16-32 B; lane-wise reads, for the
// passes after pass 1).  x: 64 bits of packed bases from the first base of
// index b0's k-mer; indices past n read nothing and get 0.
template <int OWN, int NV>
__device__ __forceinline__ void line_values(const TableView &tv, uint64_t x, int k, int b0, int n, double v[NV],
                                            const double *s_lut) {
  constexpr int JL = OWN + 1;
  const int kx = k + OWN;  // the (m + 1)-mer: line index and the L1 base
  const uint64_t xmask = (1ull << (2 * kx)) - 1ull;
#pragma unroll
  for (int o = 0; o < NV; o += JL) {
    double lv[JL];
#pragma unroll
    for (int t = 0; t < JL; ++t) lv[t] = 0.0;
    if (b0 + o < n) line_entries<OWN>(tv, (x >> (64 - 2 * (o + kx))) & xmask, lv, s_lut);
#pragma unroll
    for (int t = 0; t < JL; ++t)
      if (o + t < NV) v[o + t] = (b0 + o + t < n) ? lv[t] : 0.0;
  }
}

template <int NV>
__device__ __forceinline__ void line_values_any(const TableView &tv, uint64_t x, int k, int b0, int n, double v[NV],
                                                const double *s_lut) {
  switch (tv.line_own) {
    case 1: line_values<1, NV>(tv, x, k, b0, n, v, s_lut); break;  // (wide lines at k = 15)
    case 2: line_values<2, NV>(tv, x, k, b0, n, v, s_lut); break;
    case 3: line_values<3, NV>(tv, x, k, b0, n, v, s_lut); break;
    case 4: line_values<4, NV>(tv, x, k, b0, n, v, s_lut); break;
    default: line_values<5, NV>(tv, x, k, b0, n, v, s_lut); break;
  }
}

// Values of scan indices b0 .. b0+15 of chunk c (0 past n) of a compressed
// table whose per-index codes were not stored (small-k pass 1): the 16
// k-mers from one 64-bit window of packed bases (bytes near the buffer end),
// each looked up in the base code table (L2-resident for small k) and the LUT.
template <int NV = 16>
__device__ __forceinline__ void values16_nostore(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total,
                                                 int k, const TableView &tv, int64_t c, int b0, int n, double v[NV],
                                                 const double *s_lut) {
  const int64_t p = g.start[c] + b0 - k;  // first base of index b0's k-mer
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  uint64_t x = 0;
  const bool pk = packed_bits(g.packed, total, p, x);
  if (pk && tv.line) {  // line table: OWN + 1 indices per read
    line_values_any<NV>(tv, x, k, b0, n, v, s_lut);
    return;
  }
  if (pk && tv.compressed && tv.ext && tv.ext_J >= 2 && k + tv.ext_J - 1 + 15 <= 32) {
    // one expanded-table read per J indices (the gathers of k_summ_fixw and
    // the heads: 4 random requests per 16 indices at J = 5 instead of 32;
    // uint16 / 12-bit code entries: FP64 tables take the base table below)
    const int J = tv.ext_J, kx = k + J - 1;
    const uint64_t xmask = (kx >= 32) ? ~0ull : ((1ull << (2 * kx)) - 1ull);
    const bool c12 = tv.ext_bits == 12;
    for (int o = 0; o < NV; o += J) {
      if (b0 + o >= n) {
        for (int t = o; t < NV; ++t) v[t] = 0.0;
        break;
      }
      const uint64_t gx = (x >> (64 - 2 * (o + kx))) & xmask;
      uint64_t e;
      if (J <= 2) e = reinterpret_cast<const uint32_t *>(tv.ext)[gx];
      else e = reinterpret_cast<const uint64_t *>(tv.ext)[gx];
      for (int t = 0; t < J && o + t < NV; ++t) {
        const int j = o + t;
        double val = 0.0;
        if (b0 + j < n) {
          uint32_t q;
          if (c12) {
            const uint32_t q12 = (uint32_t)(e >> (12 * t)) & 0xfffu;
            q = q12 != 0xfffu ? (uint32_t)tv.map12[q12]
                              : (uint32_t)tv.codes[(uint32_t)(x >> (64 - 2 * (j + k))) & kmask];
          } else {
            q = (uint32_t)(e >> (16 * t)) & 0xffffu;
          }
          val = s_lut ? s_lut[q] : tv.lut[q];
        }
        v[j] = val;
      }
    }
    return;
  }
  uint32_t code = pk ? 0u : prime_code(seq, p, k);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    if (pk) code = (uint32_t)(x >> (64 - 2 * (j + k))) & kmask;
    else if (j > 0 && b0 + j < n) code = ((code << 2) | enc(seq[p + k - 1 + j])) & kmask;
    if (!tv.compressed) {  // FP64 base table (small k with the table in LDS for pass 1)
      v[j] = b0 + j < n ? tv.vals[code] : 0.0;
      continue;
    }
    const uint32_t q = b0 + j < n ? tv.codes[code] : 0u;
    v[j] = b0 + j < n ? (s_lut ? s_lut[q] : tv.lut[q]) : 0.0;
  }
}

// Values of scan indices b0 .. b0+15 of a chunk starting at start (0 past
// n) from an FP64 table: the line table (OWN + 1 indices per read) where the
// packed bases cover the window, else the base table by rolling codes.
// code: the k-mer of index b0 on entry, of b0 + 16 on exit.
__device__ __forceinline__ void values16_f64(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                             const TableView &tv, int64_t start, int b0, int n, uint32_t &code,
                                             uint32_t mask, double v[NB]) {
  uint64_t xb = 0;
  if (tv.line && packed_bits(g.packed, total, start + b0 - k, xb)) {
    line_values_any<NB>(tv, xb, k, b0, n, v, nullptr);
    code = (uint32_t)(xb >> (64 - 2 * (NB + k))) & mask;
    return;
  }
  uint8_t by[16];
  load16(seq, start + b0, total, by);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    v[j] = (b0 + j < n) ? tv.vals[code] : 0.0;
    code = roll(code, by[j], mask);
  }
}

// The values4 of a replay from an FP64 64-B line table with own = 3 (weighted
// rank, k = 13: one line per lane, its three own entries and the L1 entry of
// the next base), fetched by the whole wave together: lanes 4m .. 4m + 3 load
// the four 16-B pieces of line 16 r + m (r = 0 .. 3), so each line costs one
// coalesced 64-B request instead of three divergent loads of one lane
// (round 6: half of the weighted-rank rescans' time was those loads,
// DESIGN.md section 10), by LDS-DMA into 4 KiB of LDS per wave.  Every lane of the
// wave calls it (uniform), each with its packed bases x of index i0's k-mer.
__device__ __forceinline__ void values4_coop_f64(const TableView &tv, uint64_t x, int k, int i0, int n,
                                                 double v[4], uint4 *__restrict__ s_piece,
                                                 unsigned long long *__restrict__ s_key) {
  const int lane = threadIdx.x & 63;
  const int kx = k + 3;
  const uint64_t key = (x >> (64 - 2 * kx)) & ((1ull << (2 * kx)) - 1ull);
  const bool valid = i0 < n;
  s_key[lane] = valid ? (unsigned long long)(key >> 2) : ~0ull;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // LDS-DMA (global_load_lds_dwordx4): lane l's piece lands at s_piece[64 r + l] = piece l & 3 of
  // line 16 r + (l >> 2), no VGPRs on the way (the FP64 carry holds 168); a lane without a line
  // reads line 0 into a slot nobody reads
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const unsigned long long ln = s_key[16 * r + (lane >> 2)];
    const uint8_t *src = tv.line + (ln != ~0ull ? (size_t)ln * 64 : (size_t)0) + 16 * (lane & 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)(s_piece + 64 * r), 16, 0, 0);
  }
  // the DMA writes must have landed before any lane reads them: an explicit
  // vmcnt(0) lgkmcnt(0) (hipcc placed its own wait only before the
  // conditional reads below, not before the hoisted L1 one)
  __builtin_amdgcn_s_waitcnt(0x0070);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const double *L = reinterpret_cast<const double *>(s_piece + 4 * lane);
  const double l1 = L[3 + (int)(key & 3u)];
  v[0] = valid ? L[0] : 0.0;
  v[1] = i0 + 1 < n ? L[1] : 0.0;
  v[2] = i0 + 2 < n ? L[2] : 0.0;
  v[3] = i0 + 3 < n ? l1 : 0.0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // (the next call's writes after these reads)
}

// Values of scan indices i0 .. i0+3 of chunk c (0 past n): one 8-byte code
// load (compressed) or one k-mer prime plus three rolls.  start: the chunk's
// first scan index (g.start[c]), loaded by the caller ahead of time; xin
// (have_x): the 64 packed bits from base start + i0 - k, prefetched.
__device__ __forceinline__ void values4(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                        const TableView &tv, const uint16_t *__restrict__ codes, int64_t c,
                                        int64_t start, int i0, int n, double v[4], bool have_x = false,
                                        uint64_t xin = 0) {
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = 0.0;
  if (i0 >= n) return;
  if (codes) {
    const uint2 w = *reinterpret_cast<const uint2 *>(codes + code_slot(c, i0));
    const uint32_t cw[2] = {w.x, w.y};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i0 + q < n) v[q] = tv.lut[(cw[q >> 1] >> (16 * (q & 1))) & 0xffffu];
    return;
  }
  const int64_t p = start + i0;
  if (tv.line) {  // line table: OWN + 1 indices per read
    uint64_t xp = xin;
    if (have_x || packed_bits(g.packed, total, p - k, xp)) {
      line_values_any<4>(tv, xp, k, i0, n, v, nullptr);
      return;
    }
  }
  if (!tv.compressed && tv.ext && tv.ext_J == 4) {  // FP64 expanded table: the 4 values in one 32-B entry
    uint64_t xp = xin;
    const uint64_t gcode = (have_x || packed_bits(g.packed, total, p - k, xp))
                               ? (xp >> (64 - 2 * (k + 3)))
                               : prime_code_guarded64(seq, p - k, k + 3, total);
    const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
    const double2 e0 = E[2 * gcode], e1 = E[2 * gcode + 1];
    const double ev[4] = {e0.x, e0.y, e1.x, e1.y};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i0 + q < n) v[q] = ev[q];
    return;
  }
  if (!tv.compressed && !tv.line) {
    // FP64 J = 2 / 3 expanded tables (weighted rank, k = 14, 15) and FP64
    // base tables: the k-mers from the packed bases (prefetched by the carry),
    // not from k + 3 bytes
    uint64_t xp = xin;
    if (have_x || packed_bits(g.packed, total, p - k, xp)) {
      const uint64_t G = xp >> (64 - 2 * (k + 3));  // the (k + 3)-mer of indices i0 .. i0 + 3
      const uint64_t mk = ((uint64_t)1 << (2 * k)) - 1;
      double ev[4];
      if (tv.ext && tv.ext_J == 2) {  // entries (v_j, v_j+1) of (k + 1)-mers, 16 B
        const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
        const uint64_t m1 = ((uint64_t)1 << (2 * (k + 1))) - 1;
        const double2 a = E[G >> 4], b = E[G & m1];
        ev[0] = a.x;
        ev[1] = a.y;
        ev[2] = b.x;
        ev[3] = b.y;
      } else if (tv.ext && tv.ext_J == 3) {  // entries (v_j .. v_j+2, 0) of (k + 2)-mers, 32 B
        const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
        const uint64_t e = G >> 2;
        const double2 a = E[2 * e], b = E[2 * e + 1];
        ev[0] = a.x;
        ev[1] = a.y;
        ev[2] = b.x;
        ev[3] = tv.vals[G & mk];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) ev[q] = tv.vals[(G >> (2 * (3 - q))) & mk];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (i0 + q < n) v[q] = ev[q];
      return;
    }
  }
  const uint32_t mask = (1u << (2 * k)) - 1u;
  uint32_t code = prime_code(seq, p - k, k);
  v[0] = tv_get(tv, code);
#pragma unroll
  for (int q = 1; q < 4; ++q) {
    if (i0 + q < n) {
      code = ((code << 2) | enc(seq[p + q - 1])) & mask;
      v[q] = tv_get(tv, code);
    }
  }
}

// Packed-code words staged in LDS per pass-1 lane: bases [q0, q0 + 320) of
// its chunk (q0 = start + J - 1), loaded once (5 x 16 B) instead of one 12-B
// load per batch, so the lane's two 128-B lines are fetched once even when
// the random table reads evict them from L2 between batches.
constexpr bool kP1Stage = true;
// Table reads per batch of the pipelined pass 1: 3 leaves registers for two
// binade summaries (G = 4 spilled: 17.10 vs 14.66 ms; G = 8 at 768-lane
// blocks: 17.7 vs 16.4 ms).  The buffer-end margins below are computed for
// kP1G = 4 (conservative for 3).
constexpr int kP1GSumm = 3;
constexpr int kP1G = 4;
constexpr int kP1Block = 1024;  // lanes per pass-1 block (512 / 256: 147 / 108 vs 163 Gbases/s)
// Pass-1 summaries start at predicted entries of 1024 (below, exact halves
// make most chunks' single-trajectory summaries void; k_summ_fixw does those).
constexpr double kP1SumMin = 1024.0;
// A predicted entry within this relative distance of a binade edge is
// summarised in the neighbouring binade too.
constexpr double kP1Margin = 0.125;
static_assert(kP1Block % 64 == 0 && kP1Block <= 1024, "pass-1 block is whole waves");
constexpr int kP1StageWords = 20;
// Bases past its chunk's first scan index a pass-1 lane may read: the
// pipelined kernel's windows reach two batches ahead (< 256 + 2 * 40 + 3 * 16)
// and the LDS staging reads kP1StageWords words from word (start + J - 1) / 16.
// Lanes closer than this to the buffer end are left to k_pass1 (tail_only),
// so every packed word they stage exists (the packed array has total / 16 + 1
// words, ks_runs.hip).
constexpr int kP1WinReach = 4 + 255 + 2 * 5 * kP1G + 16 * 3;  // J - 1 + last b0 + 2 PB + window
constexpr int kP1StageReach = 16 * kP1StageWords + 21;
constexpr int kP1TailMargin = kP1WinReach > kP1StageReach ? (kP1WinReach > 352 ? kP1WinReach : 352)
                                                          : (kP1StageReach > 352 ? kP1StageReach : 352);
static_assert(16 * kP1StageWords + 4 <= kP1TailMargin + 16 + 1, "staged packed words stay inside the buffer");
static_assert(kP1WinReach <= kP1TailMargin + 1, "pipelined windows stay inside the buffer");

// Wave-uniform broadcast of lane j's value (v_readlane: a VALU op, unlike a
// variable-lane __shfl which goes through ds_bpermute).
__device__ __forceinline__ int rl32(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ long long rl64(long long v, int j) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(v & 0xffffffff), j);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(v >> 32), j);
  return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double rld(double v, int j) { return __longlong_as_double(rl64(__double_as_longlong(v), j)); }

// Wave64 scans on DPP lane moves (GFX9 DPP, a VALU operand modifier: no LDS
// round trip, unlike the ds_bpermute behind a variable __shfl): lane i reads
// lane i - d of its 16-lane row (row_shr:d), lane 15 of the row before
// (row_bcast:15, rows 1 and 3), lane 31 (row_bcast:31, rows 2 and 3), or
// lane i - 1 across the wave (wave_shr:1).  Lanes without a source read 0,
// the identity of every scan below.  The whole wave must be active.
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, 0xf, true);
}
template <int CTRL, int RM>
__device__ __forceinline__ long long dpp_i64(long long v) {
  const int lo = dpp_i32<CTRL, RM>((int)(v & 0xffffffff)), hi = dpp_i32<CTRL, RM>((int)(v >> 32));
  return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64(double v) {
  return __longlong_as_double(dpp_i64<CTRL, RM>(__double_as_longlong(v)));
}
constexpr int kDppShr1 = 0x111, kDppShr2 = 0x112, kDppShr4 = 0x114, kDppShr8 = 0x118, kDppBc15 = 0x142,
              kDppBc31 = 0x143, kDppWaveShr1 = 0x138;
// Inclusive wave scan of an associative op(left, right) whose identity is
// all-zero bits, on a value type V moved by Mov<CTRL, RM>(V).
#define KS_DPP_SCAN(V, x, MOV, OP)                     \
  do {                                                 \
    x = OP(MOV<kDppShr1, 0xf>(x), x);                  \
    x = OP(MOV<kDppShr2, 0xf>(x), x);                  \
    x = OP(MOV<kDppShr4, 0xf>(x), x);                  \
    x = OP(MOV<kDppShr8, 0xf>(x), x);                  \
    x = OP(MOV<kDppBc15, 0xa>(x), x);                  \
    x = OP(MOV<kDppBc31, 0xc>(x), x);                  \
  } while (0)

__device__ __forceinline__ double wave_sum_incl(double x) {
  auto add = [](double a, double b) { return a + b; };
  KS_DPP_SCAN(double, x, dpp_f64, add);
  return x;
}
// previous lane's value (0 in lane 0)
__device__ __forceinline__ long long wave_prev_i64(long long v) { return dpp_i64<kDppWaveShr1, 0xf>(v); }
__device__ __forceinline__ int wave_prev_i32(int v) { return dpp_i32<kDppWaveShr1, 0xf>(v); }

// Parity-pair integer maps (d0, d1): entry parity p -> increment d_p;
// (a then b)_p = a_p + b_{(p + a_p) & 1}.  Identity (0, 0).
struct PPair {
  long long d0, d1;
};
__device__ __forceinline__ PPair pp_compose(const PPair &a, const PPair &b) {
  return PPair{a.d0 + ((a.d0 & 1) ? b.d1 : b.d0), a.d1 + (((1 + a.d1) & 1) ? b.d1 : b.d0)};
}
template <int CTRL, int RM>
__device__ __forceinline__ PPair dpp_pp(const PPair &v) {
  return PPair{dpp_i64<CTRL, RM>(v.d0), dpp_i64<CTRL, RM>(v.d1)};
}
__device__ __forceinline__ PPair pp_scan_incl(PPair x) {
  KS_DPP_SCAN(PPair, x, dpp_pp, pp_compose);
  return x;
}
__device__ __forceinline__ PPair pp_prev(const PPair &v) { return PPair{wave_prev_i64(v.d0), wave_prev_i64(v.d1)}; }

// segmented parity-pair scan element (f: a segment starts in this lane's part)
struct SegPP {
  PPair s;
  int f;
};
template <int CTRL, int RM>
__device__ __forceinline__ SegPP dpp_seg(const SegPP &v) {
  return SegPP{dpp_pp<CTRL, RM>(v.s), dpp_i32<CTRL, RM>(v.f)};
}
__device__ __forceinline__ SegPP seg_op(const SegPP &l, const SegPP &r) {
  return SegPP{r.f ? r.s : pp_compose(l.s, r.s), l.f | r.f};
}
// forward fill of a flagged value
struct FillM {
  long long m;
  int f;
};
template <int CTRL, int RM>
__device__ __forceinline__ FillM dpp_fill(const FillM &v) {
  return FillM{dpp_i64<CTRL, RM>(v.m), dpp_i32<CTRL, RM>(v.f)};
}
__device__ __forceinline__ FillM fill_op(const FillM &l, const FillM &r) { return FillM{r.f ? r.m : l.m, l.f | r.f}; }

// DPP moves whose lanes without a source keep `old` (bound_ctrl off): scans
// whose identity is not all-zero bits.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64_or(double v, double old) {
  const long long x = __double_as_longlong(v), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffff), (int)(x & 0xffffffff), CTRL, RM, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(x >> 32), CTRL, RM, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// The predictor's max-plus pairs: (a1, b1) then (a2, b2) = (a1 + a2,
// max(b1 + a2, b2)); identity (0, -inf).
struct APair {
  double a, b;
};
template <int CTRL, int RM>
__device__ __forceinline__ APair dpp_ap(const APair &v) {
  return APair{dpp_f64_or<CTRL, RM>(v.a, 0.0), dpp_f64_or<CTRL, RM>(v.b, -INFINITY)};
}
__device__ __forceinline__ APair ap_op(const APair &l, const APair &r) { return APair{l.a + r.a, fmax(l.b + r.a, r.b)}; }
__device__ __forceinline__ APair ap_prev(const APair &v) { return dpp_ap<kDppWaveShr1, 0xf>(v); }

// ------------------------------------------------------------------- P0

// Chunk start, length and run, a wave per stitch tile (64 chunks of one run),
// the run from the tile map of k_tile_runs (in-process A/B against a binary
// search per chunk: 17.91-18.00 vs 18.01-18.13 ms).
__global__ void k_make_chunks(const int64_t *__restrict__ ra, const int64_t *__restrict__ cbase,
                              const int64_t *__restrict__ tbase, const int32_t *__restrict__ trun, int64_t ntiles,
                              int k, const int64_t *__restrict__ rbnd, int extra, Chunks g) {
  const int64_t t = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (t >= ntiles) return;
  const int64_t lo = trun[t];
  const int64_t c = cbase[lo] + (t - tbase[lo]) * 64 + (threadIdx.x & 63);
  if (c >= cbase[lo + 1]) return;
  const int64_t first = ra[lo] + k + (c - cbase[lo]) * CH;
  const int64_t last = rbnd[lo] - 1 + extra;  // tr_lr: one more index (the first k-mer's own step)
  g.start[c] = first;
  g.n[c] = (int32_t)min((int64_t)CH, last - first + 1);
  g.run[c] = (int32_t)lo;
}

// P0 binade predictor (pass-1 summaries): the approximate sum and clean
// exit of every chunk from the fp16 prefix means of the table (ks_table::
// d_approx, <= 128 KiB in LDS, one block per CU), rolled from the packed
// bases; a max-plus scan of them (k_approx_scan) predicts each chunk's entry,
// i.e. the binade pass 1 summarises in.  Only a prediction: a wrong binade
// costs one gathered summary (k_summ_fixw), never a result.
// The chunk's 18 packed words (bases q0 .. q0 + 287, q0 = start - k) in
// registers: five aligned 16-B loads (a quarter of the requests of 18 word
// loads: the lanes of a wave read 64 different lines per instruction), then
// the 18 words at offset w0 - wa selected in registers.
struct PredWords {
  uint32_t a[21];  // a[20]: the third word of the last 16 indices at o = 3 (past the loads: 0)
  int o;
  __device__ __forceinline__ void load(const uint32_t *__restrict__ packed, int64_t total, int64_t q0) {
    const int64_t w0 = q0 >> 4, last = total >> 4;
    const int64_t wa = w0 & ~(int64_t)3;
    if (wa + 20 <= last + 1) {
      const uint4 *P4 = reinterpret_cast<const uint4 *>(packed + wa);
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const uint4 v = P4[t];
        a[4 * t] = v.x;
        a[4 * t + 1] = v.y;
        a[4 * t + 2] = v.z;
        a[4 * t + 3] = v.w;
      }
      a[20] = 0;
      o = (int)(w0 - wa);
    } else {
#pragma unroll
      for (int t = 0; t < 18; ++t) a[t] = packed[min(w0 + t, last)];
      o = 0;
    }
  }
  __device__ __forceinline__ uint32_t w(int t) const {
    return o == 0 ? a[t] : (o == 1 ? a[t + 1] : (o == 2 ? a[t + 2] : a[t + 3]));
  }
};

// P0 binade predictor (pass-1 summaries): the approximate sum and clean
// exit of every chunk from the fp16 prefix means of the table (ks_table::
// d_approx, <= 128 KiB in LDS, one block per CU), rolled from the packed
// bases; a max-plus scan of them (k_approx_scan) predicts each chunk's entry,
// i.e. the binade pass 1 summarises in.  Only a prediction: a wrong binade
// costs one gathered summary (k_summ_fixw), never a result.  (A
// software-pipelined loop -- the next chunk's words in flight while one is
// summed -- measured the same: profiles/r4/ab/ab_log2.txt.)
template <int PS>
__global__ void __launch_bounds__(1024) k_predict(Chunks g, int64_t total, int k, const uint16_t *__restrict__ approx, int kp,
                                                  double *__restrict__ pa, double *__restrict__ pb) {
  extern __shared__ __half s_ap[];  // 4^kp entries (dynamic: 32 KiB at kp = 7 lets 4 blocks share a CU)
  const int np = 1 << (2 * kp);
  for (int i = threadIdx.x; i < np; i += blockDim.x) s_ap[i] = __ushort_as_half(approx[i]);
  __syncthreads();
  const uint32_t pmask = (uint32_t)np - 1u;
  const uint32_t *__restrict__ packed = g.packed;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto sum_chunk = [&](const PredWords &W, int64_t q0, int n, int64_t c) {
    const uint32_t bp = 2u * (uint32_t)(q0 & 15);
    float tsum = 0.f, tex = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (16 * t < n) {
        const uint64_t x = ((((uint64_t)W.w(t) << 32) | W.w(t + 1)) << bp) | (((uint64_t)W.w(t + 2) << bp) >> 32);
        // every PS-th index, weighted PS (A/B: PS = 2 cut the predictor 1.11 -> 0.80 ms with the
        // same 16.2 K gathered summaries at the metric config; PS = 4 is the default since round 4)
        float a[16 / PS];
#pragma unroll
        for (int j = 0; j < 16; j += PS)
          a[j / PS] = __half2float(s_ap[(uint32_t)(x >> (64 - 2 * (j + kp))) & pmask]);
#pragma unroll
        for (int j = 0; j < 16; j += PS) {
          const float aj = (16 * t + j < n) ? a[j / PS] * (float)PS : 0.f;
          tsum += aj;
          tex = fmaxf(tex + aj, 0.f);
        }
      }
    }
    pa[c] = tsum;
    pb[c] = tex;
  };
  for (int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < g.nch; c += stride) {
    PredWords W;
    const int64_t q0 = g.start[c] - k;  // index i's k-mer prefix: bases [q0 + i, q0 + i + kp)
    W.load(packed, total, q0);
    sum_chunk(W, q0, g.n[c], c);
  }
}

// ------------------------------------------------------------------- P1

// A closed excursion of a chunk's clean trajectory (chunk-relative beg, arg,
// end) is kept as a candidate if it could emit a region or (tr_lr) needs a
// rescan; first = the chunk starts its run.
__device__ __forceinline__ bool cand_wanted(const EmitCfg &ec, bool first, int64_t start, int beg, int arg, int end,
                                            double best) {
  const int64_t f = first ? start : -1;
  const Emission e = decide(ec, f, start + beg, start + arg, best, start + end, true);
  return e.reg || e.res;
}


// J = scan indices served by one table read: 1 reads the base table
// (uint16 code or FP64 value per index); J >= 2 reads the expanded table
// entry of the (k+J-1)-mer that spans J consecutive indices.
// kLds: the compressed LUT is copied to LDS once per 1024-lane block
// (random LUT reads hit LDS banks instead of the L1/L2 path).
template <int J, bool kCompressed, bool kLds>
__global__ void __launch_bounds__(J == 1 ? 256 : 1024) k_pass1(Chunks g, const uint8_t *__restrict__ seq, int64_t total,
                                                int k, TableView tv, uint16_t *__restrict__ codes,
                                                EmitCfg ec, uint32_t *__restrict__ visits, P1 o, Cand cand,
                                                int64_t c0, int tail_only) {
  constexpr int G = (J == 1) ? 16 : (J >= 3 ? 4 : 8);  // table reads in flight per lane and batch
  constexpr int PB = G * J;             // scan indices per batch (16, 16, 12, 16, 20)
  constexpr bool k12 = (J == 5);        // 12-bit codes with escapes (kCompressed only)
  using GC = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;  // (k+J-1)-mer code
  __shared__ double s_lut[kLds ? kLdsLutMax : 1];
  __shared__ double s_lut12[k12 ? 4096 : 1];
  __shared__ uint16_t s_map12[k12 ? 4096 : 1];
  if (kLds) {
    for (int i = threadIdx.x; i < tv.nlut; i += blockDim.x) s_lut[i] = tv.lut[i];
  }
  if (k12) {
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
      s_lut12[i] = tv.lut12[i];
      s_map12[i] = tv.map12[i];
    }
  }
  if (kLds || k12) __syncthreads();
  const int64_t c = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.nch) return;
  // tail_only: the chunks k_pass1p leaves (reads past the buffer end)
  if (tail_only && g.start[c] + g.n[c] + kP1TailMargin <= total) return;
  const int kx = k + J - 1;
  const GC xmask = (2 * kx >= 8 * (int)sizeof(GC)) ? ~(GC)0 : (((GC)1 << (2 * kx)) - 1);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  const int64_t start = g.start[c];
  const int n = g.n[c];
  const bool first = c == 0 || g.run[c - 1] != g.run[c];  // the chunk starts its run
  GC gcode = (GC)prime_code_guarded64(seq, start - k, kx, total);  // (k+J-1)-mer of group 0
  // tr_lr: the run's first scan index scores the first k-mer's own score
  const double first_val = (ec.trlr && first) ? ec.ks[(uint32_t)(gcode >> (2 * (J - 1))) & kmask] : 0.0;
  double prev = 0.0, best = 0.0;
  int beg = -1, arg = 0;
  double asum = 0.0, pmin = INFINITY, pmax = -INFINITY, sabs = 0.0;
  int parg = 0;
  bool special = false;
  for (int b0 = 0; b0 < n; b0 += PB) {
    uint8_t by[32];  // bytes rolled in by groups 1..G: start + b0 + J - 1 + [0, PB)
    load16(seq, start + b0 + J - 1, total, by);
    if (PB > 16) load16(seq, start + b0 + J - 1 + 16, total, by + 16);
    GC gc[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      gc[gi] = gcode;
#pragma unroll
      for (int t = 0; t < J; ++t) gcode = ((gcode << 2) | enc(by[gi * J + t])) & xmask;
    }
    double v[PB];
    uint16_t q[PB];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const bool live = b0 + gi * J < n;
      if (J == 1) {
        if (kCompressed) q[gi] = live ? tv.codes[gc[gi]] : (uint16_t)0;
        else v[gi] = live ? tv.vals[gc[gi]] : 0.0;
      } else if (kCompressed && k12) {
        const uint64_t e = live ? reinterpret_cast<const uint64_t *>(tv.ext)[gc[gi]] : 0ull;
#pragma unroll
        for (int t = 0; t < J; ++t) {
          const uint32_t c12 = (uint32_t)(e >> (12 * t)) & 0xfffu;
          if (c12 != 0xfffu) {
            q[gi * J + t] = s_map12[c12];
            v[gi * J + t] = s_lut12[c12];
          } else {  // value outside the 12-bit set: base table
            const uint16_t qe = tv.codes[(uint32_t)(gc[gi] >> (2 * (J - 1 - t))) & kmask];
            q[gi * J + t] = qe;
            v[gi * J + t] = tv.lut[qe];
          }
        }
      } else if (kCompressed) {
        uint64_t e = 0;
        if (live) e = (J <= 2) ? (uint64_t)reinterpret_cast<const uint32_t *>(tv.ext)[gc[gi]]
                               : reinterpret_cast<const uint64_t *>(tv.ext)[gc[gi]];
#pragma unroll
        for (int t = 0; t < J; ++t) q[gi * J + t] = (uint16_t)(e >> (16 * t));
      } else {
        double2 e0 = make_double2(0.0, 0.0), e1 = e0;
        if (live) {
          const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
          if (J <= 2) {
            e0 = E[gc[gi]];
          } else {
            e0 = E[2 * (size_t)gc[gi]];
            e1 = E[2 * (size_t)gc[gi] + 1];
          }
        }
        const double ev[4] = {e0.x, e0.y, e1.x, e1.y};
#pragma unroll
        for (int t = 0; t < J; ++t) v[gi * J + t] = ev[t];
      }
    }
    if (kCompressed) {
#pragma unroll
      for (int j = 0; j < PB; ++j)
        if (!k12) v[j] = kLds ? s_lut[q[j]] : tv.lut[q[j]];
#pragma unroll
      for (int r4 = 0; r4 < PB / 4; ++r4) {
        if (codes && b0 + 4 * r4 < CH) {
          uint2 w;
          w.x = q[4 * r4 + 0] | ((uint32_t)q[4 * r4 + 1] << 16);
          w.y = q[4 * r4 + 2] | ((uint32_t)q[4 * r4 + 3] << 16);
          *reinterpret_cast<uint2 *>(codes + code_slot(c, b0 + 4 * r4)) = w;
        }
      }
    }
    if (ec.trlr && first && b0 == 0) v[0] = first_val;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int i = b0 + j;
      if (i < n) {
        if (visits) atomicAdd(&visits[(uint32_t)(gc[j / J] >> (2 * (J - 1 - j % J))) & kmask], 1u);
        const double s = v[j];
        asum += s;
        pmin = fmin(pmin, asum);
        parg = asum > pmax ? i : parg;
        pmax = fmax(pmax, asum);
        sabs += fabs(s);
        special |= !isfinite(s);
        const double t = prev + s;
        const double S = t > 0 ? t : 0.0;
        if (prev == 0 && S > 0) {
          beg = i; arg = i; best = S;
        } else if (prev > 0 && S == 0) {
          if (cand_wanted(ec, first, start, beg, arg, i, best)) {
            const int64_t slot = append_one(cand.count, cand.segcap);
            if (slot >= 0) {
              cand.beg[slot] = start + beg;
              cand.arg[slot] = start + arg;
              cand.rst[slot] = start + i;
              cand.best[slot] = best;
            }
          }
          beg = -1;
        } else if (S > best) {
          best = S; arg = i;
        }
        prev = S;
      }
    }
  }
  o.cexit[c] = prev;
  o.asum[c] = asum;
  o.pmin[c] = pmin;
  o.pmax[c] = pmax;
  o.parg[c] = parg;
  o.sabs[c] = sabs;
  o.special[c] = special ? 1 : 0;
  o.ep[c] = o.epoch;
  if (prev > 0) {
    o.tbeg[c] = beg; o.tmax[c] = best; o.targ[c] = arg;
  } else {
    o.tbeg[c] = -1; o.tmax[c] = 0.0; o.targ[c] = 0;
  }
}

// Software-pipelined gather pass for expanded compressed tables (J >= 2):
// the reads of batch b+1 (and the sequence bytes of batch b+2) are issued
// before batch b is consumed, so every wave keeps its next table reads in
// flight while it runs the trajectory.  Loads are in-order on vmcnt, so the
// loop body must never wait on a load issued after those reads: the escape
// codes of batch b (J = 5: the first two escaped slots of the batch) are
// issued before them, all loads are unconditional (dead groups read entry 0)
// so the wait counts stay static, and the rare paths that do load (a third
// escape in one batch, the candidate append) drain explicitly inside the
// branch.  Results are identical to k_pass1.
template <int J, bool kLds, bool kTrlr>
__global__ void __launch_bounds__(kP1Block) k_pass1p(Chunks g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                                 TableView tv, EmitCfg ec,
                                                 uint32_t *__restrict__ visits, P1 o, Cand cand,
                                                 const uint32_t *__restrict__ packed, const double *__restrict__ xh,
                                                 SummP1 sp) {
  constexpr int G = kP1GSumm;           // table reads per batch
  constexpr int BS = kP1Block;          // lanes per block (LDS staging stride)
  constexpr int PB = G * J;             // scan indices per batch (8, 12, 16, 20)
  constexpr bool k12 = (J == 5);        // 12-bit codes with escapes
  using GC = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;
  using EW = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;  // entry word
  // LDS: the value LUT (all distinct values, kLds), the 12-bit code maps
  // (J = 5; with kLds the 12-bit values are read through s_lut[s_map12[]] to
  // leave room for the staged packed bases) and the staged bases.
  constexpr bool kLut12 = k12 && !(kLds && kP1Stage);
  __shared__ double s_lut[kLds ? kLdsLutMax : 1];
  __shared__ double s_lut12[kLut12 ? 4096 : 1];
  __shared__ uint16_t s_map12[k12 ? 4096 : 1];
  __shared__ uint32_t s_pk[kP1Stage ? kP1StageWords * BS : 1];  // [word][lane]: conflict-free
  if (kLds)
    for (int i = threadIdx.x; i < tv.nlut; i += blockDim.x) s_lut[i] = tv.lut[i];
  if (k12)
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
      if (kLut12) s_lut12[i] = tv.lut12[i];
      s_map12[i] = tv.map12[i];
    }
  if (kLds || k12) __syncthreads();
  const int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.nch) return;
  const EW *__restrict__ ext = reinterpret_cast<const EW *>(tv.ext);
  const int kx = k + J - 1;
  const GC xmask = (2 * kx >= 8 * (int)sizeof(GC)) ? ~(GC)0 : (((GC)1 << (2 * kx)) - 1);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  const int64_t start = g.start[c];
  const int n = g.n[c];
  const bool first = c == 0 || g.run[c - 1] != g.run[c];  // the chunk starts its run
  GC gcode = (GC)prime_code_guarded64(seq, start - k, kx, total);  // (k+J-1)-mer of group 0
  // tr_lr: the run's first scan index scores the first k-mer's own score
  const double first_val = (kTrlr && first) ? ec.ks[(uint32_t)(gcode >> (2 * (J - 1))) & kmask] : 0.0;
  // tail lanes (reads could pass the end of the buffer) are left to k_pass1
  if (start + n + kP1TailMargin > total) {
    sp.e[2 * c] = sp.e[2 * c + 1] = INT32_MIN;  // no pass-1 summary (the workspace is reused)
    return;
  }
  // Batch m rolls the 2-bit codes of bases [q0 + m*PB, q0 + m*PB + PB) in:
  // three packed words from word (q0 + m*PB) >> 4 (one load, 96 bits >= the
  // 2*PB <= 40 bits at any offset), so a lane touches one or two 128-B lines
  // of packed codes over its whole chunk.
  const int64_t q0 = start + J - 1;
  const int64_t w0 = q0 >> 4;
  uint32_t *const pk = s_pk + threadIdx.x;
  if (kP1Stage) {  // (the tail margin keeps these 20 words inside the packed array)
#pragma unroll
    for (int i = 0; i < kP1StageWords / 4; ++i) {
      const u32x4a4 v4 = *reinterpret_cast<const u32x4a4 *>(packed + w0 + 4 * i);
      pk[(4 * i + 0) * BS] = v4.x;
      pk[(4 * i + 1) * BS] = v4.y;
      pk[(4 * i + 2) * BS] = v4.z;
      pk[(4 * i + 3) * BS] = v4.w;
    }
  }
  // window of 3 words at packed word wq (staged: clamped to the lane's slot;
  // only prefetches past the chunk's last batch are clamped, and unused)
  constexpr int WW = (2 * PB > 64) ? 5 : 3;  // window words: 2 x 64 bits of bases when PB > 32
  struct Win { uint32_t w[WW]; };
  auto window = [&](int64_t wq) -> Win {
    Win r;
    if (!kP1Stage) {
#pragma unroll
      for (int q = 0; q < WW; ++q) r.w[q] = packed[wq + q];
      return r;
    }
    const int i = min((int)(wq - w0), kP1StageWords - WW);
#pragma unroll
    for (int q = 0; q < WW; ++q) r.w[q] = pk[(i + q) * BS];
    return r;
  };
  // bases [qb, qb + 64) of window wn (qb & 15 = the offset in its first word)
  auto bits = [&](const Win &wn, int64_t qb, uint64_t &lo, uint64_t &hi) {
    const uint32_t bp = 2u * (uint32_t)(qb & 15);
    lo = ((((uint64_t)wn.w[0] << 32) | wn.w[1]) << bp) | (((uint64_t)wn.w[2] << bp) >> 32);
    hi = 0;
    if (WW == 5) hi = ((((uint64_t)wn.w[2] << 32) | wn.w[3]) << bp) | (((uint64_t)wn.w[4] << bp) >> 32);
  };
  // the 2J bits of group gi (bases gi*J .. gi*J + J - 1 of the batch)
  auto field = [&](uint64_t lo, uint64_t hi, int gi) -> uint64_t {
    const int e = 2 * J * (gi + 1);  // end bit of the group in the 128-bit lo:hi
    uint64_t f;
    if (e <= 64) f = lo >> (64 - e);
    else if (e - 2 * J >= 64) f = hi >> (128 - e);
    else f = (lo << (e - 64)) | (hi >> (128 - e));
    return f & ((1ull << (2 * J)) - 1ull);
  };
  Win win = window(q0 >> 4);
  GC gc[G];
  EW e[G];
  {
    uint64_t lo, hi;
    bits(win, q0, lo, hi);
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      gc[gi] = gcode;
      gcode = ((gcode << (2 * J)) | (GC)field(lo, hi, gi)) & xmask;
    }
  }
  // prologue: reads of batch 0, window of batch 1
  win = window((q0 + PB) >> 4);
#pragma unroll
  for (int gi = 0; gi < G; ++gi) e[gi] = ext[(gi * J < n) ? gc[gi] : (GC)0];
  double prev = 0.0, best = 0.0;
  int beg = -1, arg = 0;
  double asum = 0.0, pmin = INFINITY, pmax = -INFINITY, sabs = 0.0;
  int parg = 0;
  bool special = false;
  // The binade-integer summary of this chunk for the binade of its
  // predicted entry xh (k_predict), single trajectory: s rounded to the binade's
  // ulp u = 2^(e-52) as (s + C) - C with C = 1.5 * 2^e, exact partial sums while
  // they stay within (-2^e, 2^e); an exact half (tie: the increment would depend
  // on the parity of the entry) or |s| >= 2^(e-1) voids it (k_summ_fixw then
  // recomputes it).  Replaces the per-position code store and k_summaries.
  // (|s| < 2^(e-1) is checked once through sabs, and the minimum through the
  // FP64 prefix minimum: N is stored as a lower bound, which keeps the carry's
  // validity test conservative; both save registers in this 128-VGPR kernel.)
  int se = INT32_MIN, se2 = INT32_MIN;
  double sC = 0.0, sH = 0.0, scur = 0.0, smx = -INFINITY, smn = INFINITY;
  double sC2 = 0.0, sH2 = 0.0, scur2 = 0.0, smx2 = -INFINITY, smn2 = INFINITY;
  double smaxabs = 0.0;  // max |s| (the rounding of every step, both binades)
  int sarg = 0, sarg2 = 0;
  bool sbad = false, sbad2 = false;
  {
    const double x = xh ? xh[c] : 0.0;  // (no predictor: no summaries)
    if (x >= kP1SumMin && x < 1.0e15) {
      se = binade_of(x);
      sC = 1.5 * ldexp(1.0, se);
      sH = ldexp(1.0, se - 53);
      const double lo = ldexp(1.0, se);
      if (x < lo * (1.0 + kP1Margin)) se2 = se - 1;
      else if (x > 2.0 * lo * (1.0 - kP1Margin)) se2 = se + 1;
      if (se2 != INT32_MIN) {
        sC2 = 1.5 * ldexp(1.0, se2);
        sH2 = ldexp(1.0, se2 - 53);
      }
    }
  }
  for (int b0 = 0; b0 < n; b0 += PB) {
    // 1. escape reads of batch b first: the first two escaped slots of the
    //    batch (a third one, ~6e-5 of lane-batches, loads inline)
    int ja = PB, jb = PB;
    uint32_t qa = 0, qb = 0;
    if (k12) {
      uint64_t m = 0;
#pragma unroll
      for (int gi = 0; gi < G; ++gi)
#pragma unroll
        for (int t = 0; t < J; ++t)
          if (((uint32_t)(e[gi] >> (12 * t)) & 0xfffu) == 0xfffu) m |= 1ull << (gi * J + t);
      const uint64_t m2 = m & (m - 1ull);
      ja = m ? __builtin_ctzll(m) : PB;
      jb = m2 ? __builtin_ctzll(m2) : PB;
      // k-mer of slot jj (index 0 when absent): group jj / 5, offset jj % 5
      // k-mer of slot jj (index 0 when absent), selected among per-group
      // values (not array elements, so gc[] is never indexed dynamically)
      auto kmer_of = [&](int jj) -> uint32_t {
        uint32_t km = 0;
#pragma unroll
        for (int q = 0; q < G; ++q) {
          const uint32_t t = (uint32_t)(jj - q * J);  // < J iff slot jj is in group q
          const uint32_t kq = (uint32_t)(gc[q] >> (2 * (J - 1 - (t < J ? t : 0u)))) & kmask;
          km = t < (uint32_t)J ? kq : km;
        }
        return km;
      };
      qa = tv.codes[kmer_of(ja)];
      qb = tv.codes[kmer_of(jb)];
    }
    // 2. reads of batch b+1 (entry 0 where the group is past the chunk end)
    GC gn[G];
    EW en[G];
    {
      uint64_t lo, hi;
      bits(win, q0 + b0 + PB, lo, hi);
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        gn[gi] = gcode;
        gcode = ((gcode << (2 * J)) | (GC)field(lo, hi, gi)) & xmask;
      }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      en[gi] = ext[(b0 + PB + gi * J < n) ? gn[gi] : (GC)0];
    }
    // 3. window of batch b+2
    win = window((q0 + b0 + 2 * PB) >> 4);
    // 4. batch b group by group: values, trajectory
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
#pragma unroll
      for (int t = 0; t < J; ++t) {
        const int j = gi * J + t;
        uint32_t qq;
        double s;
        if (k12) {
          const uint32_t c12 = (uint32_t)(e[gi] >> (12 * t)) & 0xfffu;
          if (c12 != 0xfffu) {
            qq = s_map12[c12];
            s = kLut12 ? s_lut12[c12] : s_lut[qq];
          } else {
            qq = (j == ja) ? qa : qb;
            if (j != ja && j != jb) {  // third escape of the batch: load and drain here
              qq = tv.codes[(uint32_t)(gc[gi] >> (2 * (J - 1 - t))) & kmask];
              __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): never at the loop's shared waits
            }
            s = kLds ? s_lut[qq] : tv.lut[qq];
          }
        } else {
          qq = (uint32_t)(e[gi] >> (16 * t)) & 0xffffu;
          s = kLds ? s_lut[qq] : tv.lut[qq];
        }
        if (kTrlr && first && b0 == 0 && j == 0) s = first_val;
        const int i = b0 + j;
        if (i < n) {
          if (visits) atomicAdd(&visits[(uint32_t)(gc[gi] >> (2 * (J - 1 - t))) & kmask], 1u);
          // aggregates (selects give fmin/fmax's values: asum is never a
          // signalling NaN and a NaN asum never replaces the extreme)
          asum += s;
          pmin = asum < pmin ? asum : pmin;
          parg = asum > pmax ? i : parg;
          pmax = asum > pmax ? asum : pmax;
          sabs += fabs(s);
          special |= !isfinite(s);
          if (se != INT32_MIN) {
            const double r = (s + sC) - sC;
            sbad |= fabs(r - s) == sH;
            smaxabs = fmax(smaxabs, fabs(s));
            scur += r;
            const bool su = scur > smx;
            smx = su ? scur : smx;
            sarg = su ? i : sarg;
            smn = fmin(smn, scur);
            if (se2 != INT32_MIN) {
              const double r2 = (s + sC2) - sC2;
              sbad2 |= fabs(r2 - s) == sH2;
              scur2 += r2;
              const bool su2 = scur2 > smx2;
              smx2 = su2 ? scur2 : smx2;
              sarg2 = su2 ? i : sarg2;
              smn2 = fmin(smn2, scur2);
            }
          }
          // clean trajectory, branch-free except for the rare candidate:
          // open (0 -> S > 0) starts an excursion, close (> 0 -> 0) ends it,
          // the first strict maximum is kept (S > best is false at a close
          // and while S stays 0, since best > 0 inside and >= 0 outside)
          const double tt = prev + s;
          const double S = tt > 0 ? tt : 0.0;
          const bool open = (prev == 0) & (S > 0);
          const bool close = (prev > 0) & (S == 0);
          // kmer_regions: decide()'s region test on chunk-relative indices
          // tr_lr: decide()'s tests on chunk-relative positions (pos_of: the
          // run's first index keeps its position, later ones report j - 1)
          const int f0 = first ? 0 : -1;
          const long long ml = kTrlr ? ec.min_len : 0;
          const bool want =
              kTrlr ? (close & (((long long)((arg != f0 ? arg - 1 : arg) - (beg != f0 ? beg - 1 : beg)) >= ml) |
                                ((long long)((i != f0 ? i - 1 : i) - (arg != f0 ? arg - 1 : arg) - 1) >=
                                 (ml > 1 ? ml : 1LL))))
                    : (close & ((uint64_t)(int64_t)(arg - beg) >= ec.mw) & (best >= ec.min_score));
          if (want) {
            const int64_t slot = append_one(cand.count, cand.segcap);
            if (slot >= 0) {
              cand.beg[slot] = start + beg;
              cand.arg[slot] = start + arg;
              cand.rst[slot] = start + i;
              cand.best[slot] = best;
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);
          }
          const bool up = open | (S > best);
          best = up ? S : best;
          arg = up ? i : arg;
          beg = open ? i : (close ? -1 : beg);
          prev = S;
        }
      }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      gc[gi] = gn[gi];
      e[gi] = en[gi];
    }
  }
  summ_put(sp, c, 0, se, sbad, smaxabs, scur, smx, smn, sarg);
  summ_put(sp, c, 1, se2, sbad2, smaxabs, scur2, smx2, smn2, sarg2);
  o.cexit[c] = prev;
  o.asum[c] = asum;
  o.pmin[c] = pmin;
  o.pmax[c] = pmax;
  o.parg[c] = parg;
  o.sabs[c] = sabs;
  o.special[c] = special ? 1 : 0;
  o.ep[c] = o.epoch;
  if (prev > 0) {
    o.tbeg[c] = beg; o.tmax[c] = best; o.targ[c] = arg;
  } else {
    o.tbeg[c] = -1; o.tmax[c] = 0.0; o.targ[c] = 0;
  }
}

// ------------------------------------------------------------------- P1 (line tables)

// Pass 1 on a line table (ks_table line_kind; k_build_line_u16 / _f64 in
// ks_table.hip): a lane scans its chunk in steps of J = own + LV indices (LV
// = 2 continuation levels for uint16 codes, 1 for FP64 values).  Step s reads
// the line of the m-mer (m = k + own - 1) ending at base start - 1 + sJ +
// own - 1: its own entries are indices sJ .. sJ + own - 1, its continuation
// entries, selected by the next LV bases, the following LV indices.  So the
// step's key is the (k + J - 1)-mer ending at base start + sJ + J - 2, as
// for the expanded tables, and one random 64-B request serves J indices.
// Lines are fetched cooperatively: four lanes load the four 16-B pieces of
// one lane's line (global_load_lds_dwordx4: a wave instruction touches 16
// whole lines; random 64-B lines come at ~50 G/s from a 64-128 GiB table,
// against 25-38 G/s when each lane loads its own entry, tools/probes/line_bench*.hip,
// profiles/r3/line_bench*.txt), straight into a two-slot LDS ring per wave:
// the lines land in lane order (lane L's line at L x 64 B), and the next
// step's lines are in flight while a step is processed.  The loads are inline
// asm (the compiler would otherwise drain every LDS-DMA before each LDS
// read); the only ordinary memory accesses in the loop are the rare candidate
// appends, and the bases come from the packed 2-bit codes loaded into
// registers once per lane.  Same outputs as k_pass1p (kSumm: compressed
// tables also summarise in the predicted binades) / k_pass1pf (FP64).
constexpr int kLineLutMax = 7168;  // LDS LUT entries of the uint16 line pass (ring 96 KiB + 56 KiB)
constexpr int kLineWords = 20;     // packed words per lane: <= 15 + 17 + 255 + J bases

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// One global_load_lds_dwordx4: 16 B from each lane's gsrc to LDS address
// lds + 16 x lane (lds wave-uniform).
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// Per-lane state of a line pass over one chunk: the clean-entry trajectory,
// its aggregates, closed candidates and (kSumm) the binade-integer summaries
// in the predicted binade and its neighbour -- the per-index work of
// k_pass1p, shared by k_pass1l and k_pass1w.
template <bool kSumm, bool kTrlr>
struct P1Lane {
  int64_t start;
  int n, f0;
  double prev = 0.0, best = 0.0;
  int beg = -1, arg = 0;
  double asum = 0.0, pmin = INFINITY, pmax = -INFINITY, sabs = 0.0;
  int parg = 0;
  bool special = false;
  int se = INT32_MIN, se2 = INT32_MIN;
  double sC = 0.0, sH = 0.0, scur = 0.0, smx = -INFINITY, smn = INFINITY;
  double sC2 = 0.0, sH2 = 0.0, scur2 = 0.0, smx2 = -INFINITY, smn2 = INFINITY;
  double smaxabs = 0.0;
  int sarg = 0, sarg2 = 0;
  bool sbad = false, sbad2 = false;

  __device__ __forceinline__ void init(int64_t st, int nn, bool first, bool live, double xp) {
    start = st;
    n = nn;
    f0 = first ? 0 : -1;
    if (kSumm && live && xp >= kP1SumMin && xp < 1.0e15) {
      se = binade_of(xp);
      sC = 1.5 * ldexp(1.0, se);
      sH = ldexp(1.0, se - 53);
      const double lo = ldexp(1.0, se);
      if (xp < lo * (1.0 + kP1Margin)) se2 = se - 1;
      else if (xp > 2.0 * lo * (1.0 - kP1Margin)) se2 = se + 1;
      if (se2 != INT32_MIN) {
        sC2 = 1.5 * ldexp(1.0, se2);
        sH2 = ldexp(1.0, se2 - 53);
      }
    }
  }

  // scan index i (< n) with value s
  __device__ __forceinline__ void step(double s, int i, const EmitCfg &ec, const Cand &cand) {
    asum += s;
    pmin = asum < pmin ? asum : pmin;
    parg = asum > pmax ? i : parg;
    pmax = asum > pmax ? asum : pmax;
    sabs += fabs(s);
    special |= !isfinite(s);
    if (kSumm && se != INT32_MIN) {
      const double r = (s + sC) - sC;
      sbad |= fabs(r - s) == sH;
      smaxabs = fmax(smaxabs, fabs(s));
      scur += r;
      const bool su = scur > smx;
      smx = su ? scur : smx;
      sarg = su ? i : sarg;
      smn = fmin(smn, scur);
      if (se2 != INT32_MIN) {
        const double r2 = (s + sC2) - sC2;
        sbad2 |= fabs(r2 - s) == sH2;
        scur2 += r2;
        const bool su2 = scur2 > smx2;
        smx2 = su2 ? scur2 : smx2;
        sarg2 = su2 ? i : sarg2;
        smn2 = fmin(smn2, scur2);
      }
    }
    // clean trajectory (k_pass1p)
    const double tt = prev + s;
    const double S = tt > 0 ? tt : 0.0;
    const bool open = (prev == 0) & (S > 0);
    const bool close = (prev > 0) & (S == 0);
    const long long ml = kTrlr ? ec.min_len : 0;
    const bool want =
        kTrlr ? (close & (((long long)((arg != f0 ? arg - 1 : arg) - (beg != f0 ? beg - 1 : beg)) >= ml) |
                          ((long long)((i != f0 ? i - 1 : i) - (arg != f0 ? arg - 1 : arg) - 1) >=
                           (ml > 1 ? ml : 1LL))))
              : (close & ((uint64_t)(int64_t)(arg - beg) >= ec.mw) & (best >= ec.min_score));
    if (want) {
      const int64_t slot = append_one(cand.count, cand.segcap);
      if (slot >= 0) {
        cand.beg[slot] = start + beg;
        cand.arg[slot] = start + arg;
        cand.rst[slot] = start + i;
        cand.best[slot] = best;
      }
    }
    const bool up = open | (S > best);
    best = up ? S : best;
    arg = up ? i : arg;
    beg = open ? i : (close ? -1 : beg);
    prev = S;
  }

  __device__ __forceinline__ void finish(int64_t c, const P1 &o, const SummP1 &sp) {
    if (kSumm) {  // as in k_pass1p
      summ_put(sp, c, 0, se, sbad, smaxabs, scur, smx, smn, sarg);
      summ_put(sp, c, 1, se2, sbad2, smaxabs, scur2, smx2, smn2, sarg2);
    }
    o.cexit[c] = prev;
    o.asum[c] = asum;
    o.pmin[c] = pmin;
    o.pmax[c] = pmax;
    o.parg[c] = parg;
    o.sabs[c] = sabs;
    o.special[c] = special ? 1 : 0;
    o.ep[c] = o.epoch;
    if (prev > 0) {
      o.tbeg[c] = beg; o.tmax[c] = best; o.targ[c] = arg;
    } else {
      o.tbeg[c] = -1; o.tmax[c] = 0.0; o.targ[c] = 0;
    }
  }
};

// The lane's packed 2-bit bases from the word holding base p0 on, kLineWords
// words in registers (guarded at the end of the packed array), and a rolling
// supply: acc holds na bases in its top 2 na bits; refill() appends the next
// word when 16 or fewer are left and shifts the word array down.
struct LaneBases {
  uint32_t a[kLineWords];
  uint64_t acc = 0;
  int na = 0;

  __device__ __forceinline__ void load(const uint32_t *__restrict__ packed, int64_t total, int64_t p0) {
    const int64_t w0 = p0 >> 4, wlast = total >> 4;  // words 0 .. total >> 4 exist
    const int64_t wa = w0 & ~(int64_t)3;
    if (wa + 24 <= wlast + 1) {
      uint32_t v[24];
      const uint4 *P4 = reinterpret_cast<const uint4 *>(packed + wa);
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const uint4 q = P4[t];
        v[4 * t] = q.x;
        v[4 * t + 1] = q.y;
        v[4 * t + 2] = q.z;
        v[4 * t + 3] = q.w;
      }
      const int off = (int)(w0 - wa);
#pragma unroll
      for (int t = 0; t < kLineWords; ++t)
        a[t] = off == 0 ? v[t] : (off == 1 ? v[t + 1] : (off == 2 ? v[t + 2] : v[t + 3]));
    } else {
#pragma unroll
      for (int t = 0; t < kLineWords; ++t) a[t] = packed[min(w0 + t, wlast)];
    }
    refill();
    refill();
    const int sk = (int)(p0 & 15);
    acc <<= 2 * sk;
    na -= sk;
  }
  __device__ __forceinline__ void refill() {
    const bool r = na <= 16;
    acc |= r ? ((uint64_t)a[0] << (32 - 2 * na)) : 0ull;
    na += r ? 16 : 0;
#pragma unroll
    for (int t = 0; t < kLineWords - 1; ++t) a[t] = r ? a[t + 1] : a[t];
  }
  // nb <= 16 bases (after a refill), first base most significant
  __device__ __forceinline__ uint64_t take(int nb) {
    const uint64_t v = acc >> (64 - 2 * nb);
    acc <<= 2 * nb;
    na -= nb;
    return v;
  }
  // the (kx)-mer of the next kx bases (kx <= 32), then steps of J bases
  __device__ __forceinline__ uint64_t first_key(int kx) {
    uint64_t x = 0;
    for (int left = kx; left > 0;) {
      refill();
      const int nb = left < 16 ? left : 16;
      x = (x << (2 * nb)) | take(nb);
      left -= nb;
    }
    return x;
  }
  __device__ __forceinline__ uint64_t next_key(uint64_t xp, int J, uint64_t xmask) {
    refill();
    return ((xp << (2 * J)) | take(J)) & xmask;
  }
};

template <int OWN, bool kF64, bool kLdsLut, bool kTrlr>
__global__ void __launch_bounds__(kF64 ? 1024 : 768) k_pass1l(Chunks g, int64_t total, int k, TableView tv,
                                                              EmitCfg ec, uint32_t *__restrict__ visits, P1 o,
                                                              Cand cand, const double *__restrict__ xh, SummP1 sp) {
  constexpr int BS = kF64 ? 1024 : 768;  // 16 / 12 waves: ring 128 / 96 KiB (+ the LUT)
  constexpr int LV = kF64 ? 1 : 2;
  constexpr int J = OWN + LV;
  constexpr int NS = (CH + J - 1) / J;  // steps per chunk (the same for the whole wave)
  constexpr bool kSumm = true;  // (xh == nullptr: no predicted binades, no summaries)
  constexpr bool kLut = !kF64 && kLdsLut;
  static_assert(kF64 ? OWN + 4 <= 8 : OWN + 20 <= 32, "line layout");
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[(BS / 64) * 2 * 4096];
  __shared__ double s_lut[kLut ? kLineLutMax : 1];
  if (kLut) {
    for (int i = threadIdx.x; i < tv.nlut; i += BS) s_lut[i] = tv.lut[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = g.c0 + (int64_t)blockIdx.x * BS + threadIdx.x;
  if (c - lane >= g.nch) return;  // the whole wave is past the end (the other lanes still fetch for theirs)
  const bool live = c < g.nch;
  const int64_t start = live ? g.start[c] : (int64_t)k;
  const int n = live ? g.n[c] : 0;
  const bool first = live && (c == 0 || g.run[c - 1] != g.run[c]);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  P1Lane<kSumm, kTrlr> L;
  L.init(start, n, first, live, (kSumm && live && xh) ? xh[c] : 0.0);
  LaneBases B;
  B.load(g.packed, total, start - k);
  const int kx = k + J - 1;  // key length (<= 17)
  const uint64_t xmask = (1ull << (2 * kx)) - 1ull;
  uint64_t x = B.first_key(kx);  // key of step 0
  // tr_lr: the run's first scan index scores the first k-mer's own score
  const double first_val = (kTrlr && first) ? ec.ks[(uint32_t)(x >> (2 * (J - 1))) & kmask] : 0.0;

  // ---- the ring: lane L's line of slot q at ring + q x 4096 + L x 64
  uint8_t *const ring = s_ring + wv * 8192;
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint8_t *__restrict__ lines = tv.line;
  auto issue = [&](uint32_t idx, int slot) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t li = (uint32_t)__shfl((int)idx, 16 * q + (lane >> 2));
      glds16(lines + (size_t)li * 64 + (lane & 3) * 16, ring_lds + (uint32_t)(slot * 4096 + q * 1024));
    }
  };
  // keys of the step being processed and of the two in flight
  uint64_t x1 = 0, x2 = 0;
  issue((uint32_t)(x >> (2 * LV)), 0);
  x1 = B.next_key(x, J, xmask);
  issue((uint32_t)(x1 >> (2 * LV)), 1);
  for (int st = 0; st < NS; ++st) {
    const uint64_t xs = x;  // key of this step
    // this step's lines complete (the next step's four loads may stay in flight)
    if (st + 1 < NS) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint8_t *ln = ring + (st & 1) * 4096 + lane * 64;
    double v[J];
    if (!kF64) {
      uint32_t h[16];  // halfwords 0 .. 15 of the line (own + L1 <= 9 codes: 0 .. 8)
      const uint4 q0 = *reinterpret_cast<const uint4 *>(ln);
      h[0] = q0.x & 0xffffu; h[1] = q0.x >> 16; h[2] = q0.y & 0xffffu; h[3] = q0.y >> 16;
      h[4] = q0.z & 0xffffu; h[5] = q0.z >> 16; h[6] = q0.w & 0xffffu; h[7] = q0.w >> 16;
      if (OWN + 4 > 8) {
        const uint4 q1 = *reinterpret_cast<const uint4 *>(ln + 16);
        h[8] = q1.x & 0xffffu; h[9] = q1.x >> 16; h[10] = q1.y & 0xffffu; h[11] = q1.y >> 16;
        h[12] = q1.z & 0xffffu; h[13] = q1.z >> 16; h[14] = q1.w & 0xffffu; h[15] = q1.w >> 16;
      }
      const uint32_t c1 = (uint32_t)(xs >> 2) & 3u, c2 = (uint32_t)xs & 3u;
      uint32_t cs[J];
#pragma unroll
      for (int t = 0; t < OWN; ++t) cs[t] = h[t];
      cs[OWN] = c1 == 0 ? h[OWN] : (c1 == 1 ? h[OWN + 1] : (c1 == 2 ? h[OWN + 2] : h[OWN + 3]));
      cs[OWN + 1] = *reinterpret_cast<const uint16_t *>(ln + 2 * (OWN + 4 + 4 * c1 + c2));
#pragma unroll
      for (int t = 0; t < J; ++t) v[t] = kLut ? s_lut[cs[t]] : tv.lut[cs[t]];
    } else {
      const double *lv = reinterpret_cast<const double *>(ln);
#pragma unroll
      for (int t = 0; t < OWN; ++t) v[t] = lv[t];
      v[OWN] = lv[OWN + ((int)xs & 3)];
    }
    // the step after next into the slot just read: two steps in flight
    // while this one is processed
    x = x1;
    if (st + 2 < NS) {
      x2 = B.next_key(x1, J, xmask);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done before it is refilled
      issue((uint32_t)(x2 >> (2 * LV)), st & 1);
      x1 = x2;
    }
#pragma unroll
    for (int t = 0; t < J; ++t) {
      const int i = st * J + t;
      if (i < n) {
        double sv = v[t];
        if (kTrlr && first && i == 0) sv = first_val;
        if (visits) atomicAdd(&visits[(uint32_t)(xs >> (2 * (J - 1 - t))) & kmask], 1u);
        L.step(sv, i, ec, cand);
      }
    }
  }
  if (live) L.finish(c, o, sp);
}

// Pass 1 on a wide line table (line_kind 3, 128-B lines, k_build_line_wide):
// own / L1 / L2 entries as 13-bit codes (the uint16 codes of a table with at
// most kLineLutMax distinct values: never an escape), the 64 L3 entries (the
// three-base continuations) as 11-bit codes, 2047 escaping to the base code
// table.  J = own + 3 indices per random request (6 at k = 13: 0.51 G
// requests per 3.06 G indices instead of 0.61 G), at 128 B per request: the
// size at which random lines still come at ~50 G/s (6.4 TB/s,
// profiles/r3/line_bench.txt).  Eight lanes load a line.  A step's L3 escape
// (one at most) is loaded right after its line is decoded
// (global_load_lds_dword of the code pair; a lane without one reads the
// table's first pair), and the step is processed one step later, when it
// has landed: every step then needs one counted wait, whatever the escapes.
// A step needs at most 7 of a line's 32 dwords (own + L1: 0 .. 2; the L2
// and L3 codes: two dwords each), so eight lanes gather exactly those
// dwords of a line (global_load_lds_dword; one line request either way):
// 2 KiB of ring per wave and step instead of 8, which leaves room for 12
// waves per CU beside the LUT (the whole 128-B lines fit 6).
constexpr int kWideBlock = 768;  // 12 waves: ring 48 KiB + LUT 56 KiB + escape slots 6 KiB

// One global_load_lds_dword: 4 B from each lane's gsrc to LDS lds + 4 x lane.
__device__ __forceinline__ void glds4(const void *gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

template <int OWN, bool kTrlr>
__global__ void __launch_bounds__(kWideBlock) k_pass1w(Chunks g, int64_t total, int k, TableView tv, EmitCfg ec,
                                                       uint32_t *__restrict__ visits, P1 o, Cand cand,
                                                       const double *__restrict__ xh, SummP1 sp) {
  constexpr int BS = kWideBlock;
  constexpr int J = OWN + 3;
  constexpr int NS = (CH + J - 1) / J;
  constexpr int N13 = OWN + 20;
  constexpr uint32_t B3 = 13 * N13;  // first L3 bit
  constexpr int NO = (13 * (OWN + 4) + 31) / 32;  // dwords of own + L1 (3 or 4)
  static_assert(NO + 4 <= 8, "own + L1, L2, L3 dwords in 8 lanes");
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[(BS / 64) * 2 * 2048];
  __shared__ __attribute__((aligned(16))) uint32_t s_esc[(BS / 64) * 2 * 64];
  __shared__ double s_lut[kLineLutMax];
  for (int i = threadIdx.x; i < tv.nlut; i += BS) s_lut[i] = tv.lut[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = g.c0 + (int64_t)blockIdx.x * BS + threadIdx.x;
  if (c - lane >= g.nch) return;
  const bool live = c < g.nch;
  const int64_t start = live ? g.start[c] : (int64_t)k;
  const int n = live ? g.n[c] : 0;
  const bool first = live && (c == 0 || g.run[c - 1] != g.run[c]);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  P1Lane<true, kTrlr> L;
  L.init(start, n, first, live, (live && xh) ? xh[c] : 0.0);
  LaneBases B;
  B.load(g.packed, total, start - k);
  const int kx = k + J - 1;  // key length (<= 18)
  const uint64_t xmask = (1ull << (2 * kx)) - 1ull;
  uint64_t x = B.first_key(kx);
  const double first_val = (kTrlr && first) ? ec.ks[(uint32_t)(x >> (2 * (J - 1))) & kmask] : 0.0;

  uint8_t *const ring = s_ring + wv * 4096;
  uint32_t *const esc = s_esc + wv * 128;
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint32_t esc_lds = __builtin_amdgcn_readfirstlane(lds_addr(esc));
  const uint8_t *__restrict__ lines = tv.line;
  // the dwords a step reads from its line (key xk): 0 .. NO - 1, the L2
  // code's two, the L3 code's two (a spare lane reloads dword 0)
  auto dwords = [&](uint64_t xk) -> uint32_t {
    const uint32_t c1 = (uint32_t)(xk >> 4) & 3u, c2 = (uint32_t)(xk >> 2) & 3u, c3 = (uint32_t)xk & 3u;
    const uint32_t d2 = (13u * (OWN + 4 + 4 * c1 + c2)) >> 5, d3 = (B3 + 11u * (16 * c1 + 4 * c2 + c3)) >> 5;
    return d2 | (d3 << 8);
  };
  auto issue = [&](uint64_t xk, int slot) {
    const uint32_t idx = (uint32_t)(xk >> 6), dd = dwords(xk);
    const int j = lane & 7;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int ow = 8 * q + (lane >> 3);
      const uint32_t li = (uint32_t)__shfl((int)idx, ow);
      const uint32_t od = (uint32_t)__shfl((int)dd, ow);
      const uint32_t d2 = od & 0xffu, d3 = od >> 8;
      const uint32_t dw = j < NO ? (uint32_t)j
                                 : (j < NO + 2 ? d2 + (uint32_t)(j - NO)
                                               : (j < NO + 4 ? min(d3 + (uint32_t)(j - NO - 2), 31u) : 0u));
      glds4(lines + (size_t)li * 128 + dw * 4, ring_lds + (uint32_t)(slot * 2048 + q * 256));
    }
  };
  // the step processed one iteration late: its values, key, escape
  double vp[J];
  uint64_t xp = 0;
  bool ep = false;
  auto process = [&](int sp_, const double *vv, uint64_t xk, bool e) {
    double v5 = vv[J - 1];
    if (e) {  // the escaped L3 value: its code pair landed in the escape slot
      const uint32_t pr = esc[(sp_ & 1) * 64 + lane];
      const uint32_t km = (uint32_t)xk & kmask;
      v5 = s_lut[(km & 1u) ? (pr >> 16) : (pr & 0xffffu)];
    }
#pragma unroll
    for (int t = 0; t < J; ++t) {
      const int i = sp_ * J + t;
      if (i < n) {
        double sv = t == J - 1 ? v5 : vv[t];
        if (kTrlr && first && i == 0) sv = first_val;
        if (visits) atomicAdd(&visits[(uint32_t)(xk >> (2 * (J - 1 - t))) & kmask], 1u);
        L.step(sv, i, ec, cand);
      }
    }
  };
  uint64_t x1 = 0, x2 = 0;
  issue(x, 0);
  x1 = B.next_key(x, J, xmask);
  issue(x1, 1);
  for (int st = 0; st < NS; ++st) {
    const uint64_t xs = x;
    // this step's lines and the previous step's escape complete (the next
    // step's eight loads may stay in flight)
    if (st + 1 < NS) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint8_t *ln = ring + (st & 1) * 2048 + lane * 32;  // the step's 8 dwords (dwords())
    double v[J];
    bool e = false;
    {
      const uint4 q0 = *reinterpret_cast<const uint4 *>(ln);
      const uint4 q1 = *reinterpret_cast<const uint4 *>(ln + 16);
      const uint32_t D[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
      const uint64_t lo = (uint64_t)D[0] | ((uint64_t)D[1] << 32);
      const uint64_t hi = (uint64_t)D[2] | (NO > 3 ? ((uint64_t)D[3] << 32) : 0ull);
      auto f13 = [&](int b) -> uint32_t {  // static b < 128 - 13
        const uint64_t w = b < 64 ? ((lo >> b) | (b > 51 ? (hi << (64 - b)) : 0ull)) : (hi >> (b - 64));
        return (uint32_t)w & 0x1fffu;
      };
      const uint32_t c1 = (uint32_t)(xs >> 4) & 3u, c2 = (uint32_t)(xs >> 2) & 3u, c3 = (uint32_t)xs & 3u;
      uint32_t cs[J];
#pragma unroll
      for (int t = 0; t < OWN; ++t) cs[t] = f13(13 * t);
      const uint32_t l0 = f13(13 * OWN), l1 = f13(13 * (OWN + 1)), l2 = f13(13 * (OWN + 2)),
                     l3 = f13(13 * (OWN + 3));
      cs[OWN] = c1 == 0 ? l0 : (c1 == 1 ? l1 : (c1 == 2 ? l2 : l3));
      const uint32_t b2 = 13u * (OWN + 4 + 4 * c1 + c2), b3 = B3 + 11u * (16 * c1 + 4 * c2 + c3);
      cs[OWN + 1] = (uint32_t)(((uint64_t)D[NO] | ((uint64_t)D[NO + 1] << 32)) >> (b2 & 31)) & 0x1fffu;
      const uint32_t c11 = (uint32_t)(((uint64_t)D[NO + 2] | ((uint64_t)D[NO + 3] << 32)) >> (b3 & 31)) & 0x7ffu;
      e = c11 == 0x7ffu;
      cs[OWN + 2] = e ? 0u : c11;
#pragma unroll
      for (int t = 0; t < J; ++t) v[t] = s_lut[cs[t]];
    }
    // this step's escape (every lane: a lane without one reads the first pair)
    {
      const uint32_t km = (uint32_t)xs & kmask;
      const uint16_t *src = e ? tv.codes + (km & ~1u) : tv.codes;
      glds4(src, esc_lds + (uint32_t)((st & 1) * 256));
    }
    x = x1;
    if (st + 2 < NS) {
      x2 = B.next_key(x1, J, xmask);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done before it is refilled
      issue(x2, st & 1);
      x1 = x2;
    }
    if (st > 0) process(st - 1, vp, xp, ep);
#pragma unroll
    for (int t = 0; t < J; ++t) vp[t] = v[t];
    xp = xs;
    ep = e;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  process(NS - 1, vp, xp, ep);
  if (live) L.finish(c, o, sp);
}

// Pass 1 over weighted-rank code lines (ks_table::d_rlines, line kind 4):
// one 128-B line per 15-mer x holding the 32-bit rank codes of its OWN
// k-mers and of every one- and two-base continuation (L1: 4, L2: 16), so a
// line read serves J = OWN + 2 consecutive indices (5 at k = 13, against 4
// for the FP64 64-B lines of k_pass1l).  The 8 lanes that share a line fetch
// the 5 dwords a step needs with LDS-DMA (k_pass1w's ring and counted waits).
// A code is piece << kRankOffBits | offset, and the k-mer's weighted rank --
// R_j of the sorted position j, the closed-form prefix of rank_kmers_w
// (kmer_spans.c:196-200; RankPiece) -- is bits(R) = base + offset * inc of its
// piece; s = R - thr in FP64, as the FP64 table holds it (k_sub_thr).  The
// kRankPieceLds hottest pieces (weight order) are staged in LDS, the rest
// read from the L2-resident piece table.  Same outputs as k_pass1l<OWN, true>.
constexpr int kRankBlock = 768;

template <int OWN>
__global__ void __launch_bounds__(kRankBlock) k_pass1r(Chunks g, int64_t total, int k, TableView tv, EmitCfg ec,
                                                       uint32_t *__restrict__ visits, P1 o, Cand cand) {
  constexpr int BS = kRankBlock;
  constexpr int J = OWN + 2;
  constexpr int NS = (CH + J - 1) / J;
  static_assert(OWN + 2 <= 8, "own, L1, L2 dwords in 8 lanes");
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[(BS / 64) * 2 * 2048];
  __shared__ unsigned long long s_pc[2 * kRankPieceLds];
  const int nl = min(tv.nrpc, kRankPieceLds);
  for (int i = threadIdx.x; i < 2 * nl; i += BS) s_pc[i] = tv.rpc[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = g.c0 + (int64_t)blockIdx.x * BS + threadIdx.x;
  if (c - lane >= g.nch) return;
  const bool live = c < g.nch;
  const int64_t start = live ? g.start[c] : (int64_t)k;
  const int n = live ? g.n[c] : 0;
  const bool first = live && (c == 0 || g.run[c - 1] != g.run[c]);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  P1Lane<false, false> L;  // (FP64 tables take no chunk summaries)
  L.init(start, n, first, live, 0.0);
  LaneBases B;
  B.load(g.packed, total, start - k);
  const int kx = k + J - 1;  // key length: the 15-mer of the line and the two continuation bases
  const uint64_t xmask = (1ull << (2 * kx)) - 1ull;
  uint64_t x = B.first_key(kx);
  uint8_t *const ring = s_ring + wv * 4096;
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
  const uint8_t *__restrict__ lines = tv.rline;
  const unsigned long long *__restrict__ gpc = tv.rpc;
  const double thr = tv.rthr;
  // the dwords a step reads (key xk): own 0 .. OWN - 1, L1 OWN + c1, L2 OWN + 4 + 4 c1 + c2
  auto issue = [&](uint64_t xk, int slot) {
    const uint32_t idx = (uint32_t)(xk >> 4);
    const uint32_t c1 = (uint32_t)(xk >> 2) & 3u, c2 = (uint32_t)xk & 3u;
    const uint32_t dd = (OWN + c1) | ((OWN + 4 + 4 * c1 + c2) << 8);
    const int j = lane & 7;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int ow = 8 * q + (lane >> 3);
      const uint32_t li = (uint32_t)__shfl((int)idx, ow);
      const uint32_t od = (uint32_t)__shfl((int)dd, ow);
      const uint32_t dw = j < OWN ? (uint32_t)j : (j == OWN ? (od & 0xffu) : (j == OWN + 1 ? (od >> 8) : 0u));
      glds4(lines + (size_t)li * 128 + dw * 4, ring_lds + (uint32_t)(slot * 2048 + q * 256));
    }
  };
  auto decode = [&](uint32_t code) -> double {
    const uint32_t p = code >> kRankOffBits;
    const unsigned long long off = code & ((1u << kRankOffBits) - 1u);
    unsigned long long base, inc;
    if ((int)p < nl) {
      base = s_pc[2 * p];
      inc = s_pc[2 * p + 1];
    } else {  // a cold piece: the L2-resident table
      base = gpc[2 * p];
      inc = gpc[2 * p + 1];
    }
    return __longlong_as_double((long long)(base + off * inc)) - thr;
  };
  double vp[J];
  uint64_t xp = 0;
  auto process = [&](int sp_, const double *vv, uint64_t xk) {
#pragma unroll
    for (int t = 0; t < J; ++t) {
      const int i = sp_ * J + t;
      if (i < n) {
        if (visits) atomicAdd(&visits[(uint32_t)(xk >> (2 * (J - 1 - t))) & kmask], 1u);
        L.step(vv[t], i, ec, cand);
      }
    }
  };
  uint64_t x1 = 0, x2 = 0;
  issue(x, 0);
  x1 = B.next_key(x, J, xmask);
  issue(x1, 1);
  for (int st = 0; st < NS; ++st) {
    const uint64_t xs = x;
    // this step's lines complete (the next step's eight loads may stay in flight)
    if (st + 1 < NS) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint8_t *ln = ring + (st & 1) * 2048 + lane * 32;
    uint32_t cs[J];
    {
      const uint4 q0 = *reinterpret_cast<const uint4 *>(ln);
      const uint4 q1 = *reinterpret_cast<const uint4 *>(ln + 16);
      const uint32_t D[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int t = 0; t < J; ++t) cs[t] = D[t];
    }
    x = x1;
    if (st + 2 < NS) {
      x2 = B.next_key(x1, J, xmask);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done before it is refilled
      issue(x2, st & 1);
      x1 = x2;
    }
    if (st > 0) process(st - 1, vp, xp);
#pragma unroll
    for (int t = 0; t < J; ++t) vp[t] = decode(cs[t]);
    xp = xs;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  process(NS - 1, vp, xp);
  if (live) L.finish(c, o, SummP1{});
}

// Pass 1 for small k (north_star: "the frequency table LDS-staged for small
// k"): the 4^k FP64 values s[code] (k <= 7: <= 128 KiB) are staged in LDS
// once per persistent block, so every scanned index costs one LDS read and no
// random HBM request; bases are rolled from the packed 2-bit codes (one
// 4-B word per 16 bases).  No code store: later passes re-derive values from
// the packed bases and the base table (values16_nostore / values4).  Same
// outputs as k_pass1.
constexpr int kLdsTableK = 7;
// Pass 1 of small-k integer tables (k <= 7, ks_table::int_exact): the
// clean trajectory of a chunk starts at 0 and moves by at most 2^20 per
// index, so it and the chunk aggregates fit int32 (|S| <= 2^28) and equal the
// FP64 chain exactly; 32-bit integer compares and selects instead of FP64
// ones (half the VALU work of this ALU-bound pass), the table as int32 in
// LDS (64 KiB at k = 7: two blocks per CU).  Outputs as k_pass1_lds<false,
// true> (FP64 aggregates, no |s| sum, no non-finite flag).
__global__ void __launch_bounds__(1024) k_pass1_lds_int(Chunks g, int64_t total, int k, TableView tv, EmitCfg ec,
                                                        uint32_t *__restrict__ visits, P1 o, Cand cand) {
  __shared__ int32_t s_val[1 << (2 * kLdsTableK)];
  const int nk = 1 << (2 * k);
  for (int i = threadIdx.x; i < nk; i += blockDim.x) s_val[i] = (int32_t)tv_get(tv, (uint32_t)i);
  __syncthreads();
  const uint32_t kmask = (uint32_t)nk - 1u;
  const uint32_t *__restrict__ packed = g.packed;
  const int64_t last = total >> 4;
  for (int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < g.nch;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t start = g.start[c];
    const int n = g.n[c];
    const int64_t q0 = start - k;
    auto load3 = [&](int64_t q) {
      const int64_t w = q >> 4;
      return make_uint3(packed[min(w, last)], packed[min(w + 1, last)], packed[min(w + 2, last)]);
    };
    uint3 cur = load3(q0);
    int32_t prev = 0, best = 0, asum = 0, pmin = INT32_MAX, pmax = INT32_MIN;
    int beg = -1, arg = 0, parg = 0;
    for (int b0 = 0; b0 < n; b0 += 16) {
      const uint3 nxt = load3(q0 + b0 + 16);
      const uint32_t bp = 2u * (uint32_t)((q0 + b0) & 15);
      const uint64_t x = ((((uint64_t)cur.x << 32) | cur.y) << bp) | (((uint64_t)cur.z << bp) >> 32);
      for (int j = 0; j < 16; ++j) {
        const int i = b0 + j;
        if (i >= n) break;
        const uint32_t code = (uint32_t)(x >> (64 - 2 * (j + k))) & kmask;  // k-mer ending at start + i - 1
        const int32_t sv = s_val[code];
        if (visits) atomicAdd(&visits[code], 1u);
        asum += sv;
        pmin = asum < pmin ? asum : pmin;
        parg = asum > pmax ? i : parg;
        pmax = asum > pmax ? asum : pmax;
        const int32_t tt = prev + sv;
        const int32_t S = tt > 0 ? tt : 0;
        const bool open = (prev == 0) & (S > 0);
        const bool close = (prev > 0) & (S == 0);
        const bool want = close & ((uint64_t)(int64_t)(arg - beg) >= ec.mw) & ((double)best >= ec.min_score);
        if (want) {
          const int64_t slot = append_one(cand.count, cand.segcap);
          if (slot >= 0) {
            cand.beg[slot] = start + beg;
            cand.arg[slot] = start + arg;
            cand.rst[slot] = start + i;
            cand.best[slot] = (double)best;
          }
        }
        const bool up = open | (S > best);
        best = up ? S : best;
        arg = up ? i : arg;
        beg = open ? i : (close ? -1 : beg);
        prev = S;
      }
      cur = nxt;
    }
    o.cexit[c] = (double)prev;
    o.asum[c] = (double)asum;
    o.pmin[c] = n > 0 ? (double)pmin : INFINITY;
    o.pmax[c] = n > 0 ? (double)pmax : -INFINITY;
    o.parg[c] = parg;
    o.sabs[c] = 0.0;
    o.special[c] = 0;
    o.ep[c] = o.epoch;
    if (prev > 0) {
      o.tbeg[c] = beg; o.tmax[c] = (double)best; o.targ[c] = arg;
    } else {
      o.tbeg[c] = -1; o.tmax[c] = 0.0; o.targ[c] = 0;
    }
  }
}

// kExact (integer tables, k_carry_exact): no |s| sum and no non-finite flag
// (neither is read on that path; two of the ~30 VALU ops per index of this
// ALU-bound pass)
template <bool kTrlr, bool kExact = false>
__global__ void __launch_bounds__(1024) k_pass1_lds(Chunks g, int64_t total, int k, TableView tv, EmitCfg ec,
                                                    uint32_t *__restrict__ visits, P1 o, Cand cand,
                                                    const double *__restrict__ xh, SummP1 sp) {
  __shared__ double s_val[1 << (2 * kLdsTableK)];
  const int nk = 1 << (2 * k);
  for (int i = threadIdx.x; i < nk; i += blockDim.x) s_val[i] = tv_get(tv, (uint32_t)i);
  __syncthreads();
  const uint32_t kmask = (uint32_t)nk - 1u;
  const uint32_t *__restrict__ packed = g.packed;
  for (int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < g.nch;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t start = g.start[c];
    const int n = g.n[c];
    const bool first = c == 0 || g.run[c - 1] != g.run[c];
    if (xh) {  // pass-1 summaries in the predicted binades (as k_pass1l): the P1Lane form
      P1Lane<true, kTrlr> L;
      L.init(start, n, first, true, xh[c]);
      const int64_t q0 = start - k, last = total >> 4;
      auto load3 = [&](int64_t q) {
        const int64_t w = q >> 4;
        return make_uint3(packed[min(w, last)], packed[min(w + 1, last)], packed[min(w + 2, last)]);
      };
      uint3 cur = load3(q0);
      for (int b0 = 0; b0 < n; b0 += 16) {
        const uint3 nxt = load3(q0 + b0 + 16);
        const uint32_t bp = 2u * (uint32_t)((q0 + b0) & 15);
        const uint64_t x = ((((uint64_t)cur.x << 32) | cur.y) << bp) | (((uint64_t)cur.z << bp) >> 32);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int i = b0 + j;
          if (i < n) {
            const uint32_t code = (uint32_t)(x >> (64 - 2 * (j + k))) & kmask;  // k-mer ending at start + i - 1
            double s = s_val[code];
            if (kTrlr && first && i == 0) s = ec.ks[code];
            if (visits) atomicAdd(&visits[code], 1u);
            L.step(s, i, ec, cand);
          }
        }
        cur = nxt;
      }
      L.finish(c, o, sp);
      continue;
    }
    // 16 indices per batch: their k-mers from one 64-bit window of packed
    // bases (three words, loaded one batch ahead, uniform across the wave)
    const int64_t q0 = start - k, last = total >> 4;
    auto load3 = [&](int64_t q) {
      const int64_t w = q >> 4;
      return make_uint3(packed[min(w, last)], packed[min(w + 1, last)], packed[min(w + 2, last)]);
    };
    uint3 cur = load3(q0);
    double prev = 0.0, best = 0.0;
    int beg = -1, arg = 0;
    double asum = 0.0, pmin = INFINITY, pmax = -INFINITY, sabs = 0.0;
    int parg = 0;
    bool special = false;
    for (int b0 = 0; b0 < n; b0 += 16) {
      const uint3 nxt = load3(q0 + b0 + 16);
      const uint32_t bp = 2u * (uint32_t)((q0 + b0) & 15);
      const uint64_t x = ((((uint64_t)cur.x << 32) | cur.y) << bp) | (((uint64_t)cur.z << bp) >> 32);
      for (int j = 0; j < 16; ++j) {
        const int i = b0 + j;
        if (i >= n) break;
        const uint32_t code = (uint32_t)(x >> (64 - 2 * (j + k))) & kmask;  // k-mer ending at start + i - 1
        double s = s_val[code];
        if (kTrlr && first && i == 0) s = ec.ks[code];  // tr_lr: the run's first k-mer's own score
        if (visits) atomicAdd(&visits[code], 1u);
        asum += s;
        pmin = asum < pmin ? asum : pmin;
        parg = asum > pmax ? i : parg;
        pmax = asum > pmax ? asum : pmax;
        if (!kExact) {
          sabs += fabs(s);
          special |= !isfinite(s);
        }
        const double tt = prev + s;
        const double S = tt > 0 ? tt : 0.0;
        const bool open = (prev == 0) & (S > 0);
        const bool close = (prev > 0) & (S == 0);
        const int f0 = first ? 0 : -1;
        const long long ml = kTrlr ? ec.min_len : 0;
        const bool want =
            kTrlr ? (close & (((long long)((arg != f0 ? arg - 1 : arg) - (beg != f0 ? beg - 1 : beg)) >= ml) |
                              ((long long)((i != f0 ? i - 1 : i) - (arg != f0 ? arg - 1 : arg) - 1) >=
                               (ml > 1 ? ml : 1LL))))
                  : (close & ((uint64_t)(int64_t)(arg - beg) >= ec.mw) & (best >= ec.min_score));
        if (want) {
          const int64_t slot = append_one(cand.count, cand.segcap);
          if (slot >= 0) {
            cand.beg[slot] = start + beg;
            cand.arg[slot] = start + arg;
            cand.rst[slot] = start + i;
            cand.best[slot] = best;
          }
        }
        const bool up = open | (S > best);
        best = up ? S : best;
        arg = up ? i : arg;
        beg = open ? i : (close ? -1 : beg);
        prev = S;
      }
      cur = nxt;
    }
    o.cexit[c] = prev;
    o.asum[c] = asum;
    o.pmin[c] = pmin;
    o.pmax[c] = pmax;
    o.parg[c] = parg;
    o.sabs[c] = sabs;
    o.special[c] = special ? 1 : 0;
    o.ep[c] = o.epoch;
    if (prev > 0) {
      o.tbeg[c] = beg; o.tmax[c] = best; o.targ[c] = arg;
    } else {
      o.tbeg[c] = -1; o.tmax[c] = 0.0; o.targ[c] = 0;
    }
  }
}

// Software-pipelined gather pass for uncompressed FP64 expanded tables
// (weighted-rank tables: every k-mer has its own value, so no codes): one
// 16-B (J = 2) or 32-B (J = 3, 4) entry per J scan indices, the next batch's
// entries in flight while the current batch runs the clean trajectory, bases
// rolled from the packed codes.  Same outputs as k_pass1<J, false, false>
// (no code store: later passes re-read the table), plus (xh != nullptr) the
// binade-integer summaries in the predicted binades (P1Lane, as k_pass1l):
// at k = 15 a separate k_summaries pass re-read the 64 GiB table.
template <int J, bool kTrlr, int kBlock = 512>
__global__ void __launch_bounds__(kBlock) k_pass1pf(Chunks g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                                  TableView tv, EmitCfg ec, uint32_t *__restrict__ visits, P1 o,
                                                  Cand cand, const uint32_t *__restrict__ packed,
                                                  const double *__restrict__ xh, SummP1 sp) {
  constexpr int G = (J == 2) ? 8 : 4;  // table reads per batch
  constexpr int PB = G * J;            // scan indices per batch (16, 12, 16)
  using GC = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;
  const int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.nch) return;
  const double2 *__restrict__ E = reinterpret_cast<const double2 *>(tv.ext);
  const int kx = k + J - 1;
  const GC xmask = (2 * kx >= 8 * (int)sizeof(GC)) ? ~(GC)0 : (((GC)1 << (2 * kx)) - 1);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  const int64_t start = g.start[c];
  const int n = g.n[c];
  const bool first = c == 0 || g.run[c - 1] != g.run[c];
  // tail lanes (reads could pass the end of the buffer) are left to k_pass1
  if (start + n + kP1TailMargin > total) {
    sp.e[2 * c] = sp.e[2 * c + 1] = INT32_MIN;  // no pass-1 summary (the workspace is reused)
    return;
  }
  P1Lane<true, kTrlr> L;
  L.init(start, n, first, true, xh ? xh[c] : 0.0);
  GC gcode = (GC)prime_code_guarded64(seq, start - k, kx, total);
  const double first_val = (kTrlr && first) ? ec.ks[(uint32_t)(gcode >> (2 * (J - 1))) & kmask] : 0.0;
  const int64_t q0 = start + J - 1;
  constexpr uint64_t fmask = (1ull << (2 * J)) - 1ull;
  auto roll = [&](u32x3a4 w, int64_t qb, GC gout[G]) {
    const uint32_t bp = 2u * (uint32_t)(qb & 15);
    const uint64_t x = ((((uint64_t)w.x << 32) | w.y) << bp) | (((uint64_t)w.z << bp) >> 32);
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      gout[gi] = gcode;
      gcode = ((gcode << (2 * J)) | (GC)((x >> (64 - 2 * J * (gi + 1))) & fmask)) & xmask;
    }
  };
  auto fetch = [&](const GC gg[G], int b0, double2 e0[G], double2 e1[G]) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const size_t ix = (b0 + gi * J < n) ? (size_t)gg[gi] : 0;
      if (J <= 2) {
        e0[gi] = E[ix];
      } else {
        e0[gi] = E[2 * ix];
        e1[gi] = E[2 * ix + 1];
      }
    }
  };
  GC gc[G];
  double2 e0[G], e1[G];
  u32x3a4 win = *reinterpret_cast<const u32x3a4 *>(packed + (q0 >> 4));
  roll(win, q0, gc);
  fetch(gc, 0, e0, e1);
  win = *reinterpret_cast<const u32x3a4 *>(packed + ((q0 + PB) >> 4));
  for (int b0 = 0; b0 < n; b0 += PB) {
    GC gn[G];
    double2 n0[G], n1[G];
    roll(win, q0 + b0 + PB, gn);
    fetch(gn, b0 + PB, n0, n1);
    win = *reinterpret_cast<const u32x3a4 *>(packed + ((q0 + b0 + 2 * PB) >> 4));
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const double ev[4] = {e0[gi].x, e0[gi].y, J > 2 ? e1[gi].x : 0.0, J > 3 ? e1[gi].y : 0.0};
#pragma unroll
      for (int t = 0; t < J; ++t) {
        const int j = gi * J + t;
        double s = ev[t];
        if (kTrlr && first && b0 == 0 && j == 0) s = first_val;
        const int i = b0 + j;
        if (i < n) {
          if (visits) atomicAdd(&visits[(uint32_t)(gc[gi] >> (2 * (J - 1 - t))) & kmask], 1u);
          L.step(s, i, ec, cand);
        }
      }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      gc[gi] = gn[gi];
      e0[gi] = n0[gi];
      e1[gi] = n1[gi];
    }
  }
  L.finish(c, o, sp);
}

// ------------------------------------------------------------------- P3

// Binade-integer summary of chunk c for binade e: with S = m * 2^(e-52) and
// the whole trajectory inside [2^e, 2^(e+1)), fl(S + s) = S + RN(s * 2^(52-e))
// with ties to even decided by the parity of m.  For both entry parities t:
// total D, max M (first argmax A) and min N of the integer trajectory.
// Returns false if a value is not representable (overflow, NaN, Inf).
template <bool kCompressed, bool kDual>
__device__ int chunk_summary_impl(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                  const TableView &tv, const uint16_t *__restrict__ codes, int64_t c, int e,
                                  long long D[2], long long M[2], int A[2], long long N[2]) {
  // returns 1 ok, 0 not representable, -1 (single-trajectory mode only) a tie occurred
  const int n = g.n[c];
  const int64_t start = g.start[c];
  const uint32_t mask = (1u << (2 * k)) - 1u;
  const double scale = ldexp(1.0, 52 - e);
  uint32_t code = kCompressed ? 0u : prime_code(seq, start - k, k);
  long long cur[2] = {0, 0};
  M[0] = M[1] = LLONG_MIN;
  N[0] = N[1] = LLONG_MAX;
  A[0] = A[1] = 0;
  bool ok = true, tie_seen = false;
  for (int b0 = 0; b0 < n; b0 += NB) {
    double v[NB];
    if (kCompressed && !codes) {
      values16_nostore(g, seq, total, k, tv, c, b0, n, v, nullptr);
    } else if (kCompressed) {
      uint32_t w[8];
      load_codes16(codes, c, b0, w);
#pragma unroll
      for (int j = 0; j < NB; ++j) v[j] = tv.lut[(w[j >> 1] >> (16 * (j & 1))) & 0xffffu];
    } else {
      values16_f64(g, seq, total, k, tv, start, b0, n, code, mask, v);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int i = b0 + j;
      if (i < n) {
        const double y = v[j] * scale;  // exact: power-of-two scaling
        ok &= fabs(y) < 4.0e18;         // also false for NaN / Inf
        const double fq = floor(y);
        const double f = y - fq;        // exact fractional part
        const bool up = f > 0.5, tie = f == 0.5;
        if (kDual) {
          const long long q = ok ? (long long)fq : 0;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const long long par = (t + cur[t]) & 1;
            cur[t] += q + ((up || (tie && ((par + q) & 1))) ? 1 : 0);
            if (cur[t] > M[t]) { M[t] = cur[t]; A[t] = i; }
            N[t] = min(N[t], cur[t]);
          }
        } else {  // no tie: the increment does not depend on the parity
          tie_seen |= tie;
          const long long q = ok ? (long long)(up ? fq + 1.0 : fq) : 0;
          cur[0] += q;
          if (cur[0] > M[0]) { M[0] = cur[0]; A[0] = i; }
          N[0] = min(N[0], cur[0]);
        }
      }
    }
  }
  if (!ok) return 0;
  if (!kDual) {
    if (tie_seen) return -1;
    cur[1] = cur[0]; M[1] = M[0]; N[1] = N[0]; A[1] = A[0];
  }
  D[0] = cur[0];
  D[1] = cur[1];
  return 1;
}

// Binade-integer summary of chunk c for binade e: with S = m * 2^(e-52) and
// the whole trajectory inside [2^e, 2^(e+1)), fl(S + s) = S + RN(s * 2^(52-e))
// with ties to even decided by the parity of m.  For both entry parities t:
// total D, max M (first argmax A) and min N of the integer trajectory.  One
// trajectory is tracked unless an exact tie occurs (then both parities).
// Single-trajectory binade summary in FP64 integer arithmetic: with
// |y| < 2^51, (y + 1.5*2^52) - 1.5*2^52 is y rounded half-to-even, an exact
// integer; partial sums stay exact while |sum| < 2^53 (checked through the
// extremes).  Returns 1 ok, 0 not representable, -1 a tie occurred (the
// increment then depends on the parity: the dual-parity path is used).
template <bool kCompressed, bool kLds>
__device__ int chunk_summary_fast(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                  const TableView &tv, const uint16_t *__restrict__ codes, int64_t c, int e,
                                  long long D[2], long long M[2], int A[2], long long N[2],
                                  const double *s_lut) {
  const int n = g.n[c];
  const int64_t start = g.start[c];
  const uint32_t mask = (1u << (2 * k)) - 1u;
  const double scale = ldexp(1.0, 52 - e);
  constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
  uint64_t xp = 0;
  uint32_t code = kCompressed ? 0u
                  : packed_bits(g.packed, total, start - k, xp) ? (uint32_t)(xp >> (64 - 2 * k))
                                                                : prime_code(seq, start - k, k);
  double cur = 0.0, mx = -INFINITY, mn = INFINITY;
  int arg = 0;
  bool ok = true, tie_seen = false;
  for (int b0 = 0; b0 < n; b0 += NB) {
    double v[NB];
    if (kCompressed && !codes) {
      values16_nostore(g, seq, total, k, tv, c, b0, n, v, kLds ? s_lut : nullptr);
    } else if (kCompressed) {
      uint32_t w[8];
      load_codes16(codes, c, b0, w);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const uint32_t q = (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        v[j] = kLds ? s_lut[q] : tv.lut[q];
      }
    } else if (tv.ext && tv.ext_J == 4) {  // FP64 expanded table: 4 values per 32-B read
      uint8_t by[16];
      uint64_t xb = 0;
      if (packed_bits(g.packed, total, start + b0, xb)) {  // bytes with the same enc() as the packed codes
#pragma unroll
        for (int j = 0; j < 16; ++j) by[j] = (uint8_t)(((xb >> (62 - 2 * j)) & 3u) << 1);
      } else {
        load16(seq, start + b0, total, by);
      }
      const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
#pragma unroll
      for (int gq = 0; gq < NB / 4; ++gq) {
        // (k+3)-mer of indices b0+4gq .. +3: the k-mer of the first, then 3 bytes
        const uint64_t gx = ((uint64_t)code << 6) | ((uint64_t)enc(by[4 * gq]) << 4) |
                            ((uint64_t)enc(by[4 * gq + 1]) << 2) | (uint64_t)enc(by[4 * gq + 2]);
        double2 e0 = make_double2(0.0, 0.0), e1 = e0;
        if (b0 + 4 * gq < n) {
          e0 = E[2 * gx];
          e1 = E[2 * gx + 1];
        }
        v[4 * gq] = e0.x;
        v[4 * gq + 1] = e0.y;
        v[4 * gq + 2] = e1.x;
        v[4 * gq + 3] = e1.y;
#pragma unroll
        for (int t = 0; t < 4; ++t) code = roll(code, by[4 * gq + t], mask);
      }
    } else {
      values16_f64(g, seq, total, k, tv, start, b0, n, code, mask, v);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (b0 + j < n) {
        const double y = v[j] * scale;  // exact: power-of-two scaling
        ok &= fabs(y) < 2251799813685248.0;  // 2^51; false for NaN / Inf
        const double r = (y + kMagic) - kMagic;
        tie_seen |= fabs(r - y) == 0.5;
        cur += r;
        if (cur > mx) { mx = cur; arg = b0 + j; }
        mn = fmin(mn, cur);
      }
    }
  }
  ok &= mx < 4503599627370496.0 && mn > -4503599627370496.0;  // |partial sums| < 2^52: all exact
  if (!ok) return 0;
  if (tie_seen) return -1;
  D[0] = D[1] = (long long)cur;
  M[0] = M[1] = (long long)mx;
  N[0] = N[1] = (long long)mn;
  A[0] = A[1] = arg;
  return 1;
}

template <bool kCompressed, bool kLds>
__device__ bool chunk_summary(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                              const TableView &tv, const uint16_t *__restrict__ codes, int64_t c, int e,
                              long long D[2], long long M[2], int A[2], long long N[2], const double *s_lut) {
  const int rc = chunk_summary_fast<kCompressed, kLds>(g, seq, total, k, tv, codes, c, e, D, M, A, N, s_lut);
  if (rc >= 0) return rc == 1;
  return chunk_summary_impl<kCompressed, true>(g, seq, total, k, tv, codes, c, e, D, M, A, N) == 1;
}

// ------------------------------------------------------------------- P2

// Approximate max-plus scan, one wave per run: chunk j maps x -> max(x + a, b)
// (a = sum, b = clean exit); x~_j = composite of chunks < j applied to 0.  Only
// a prediction (which binade the exact carry will be in); never trusted.
__global__ void __launch_bounds__(64) k_approx_scan(const int64_t *__restrict__ cbase, int64_t nruns, P1 o,
                                                    double *__restrict__ xt, int64_t r_lo) {
  const int64_t r = r_lo + blockIdx.x;
  if (r >= nruns) return;
  const int lane = threadIdx.x;
  const int64_t c0 = cbase[r], c1 = cbase[r + 1];
  double carry = 0.0;
  for (int64_t cb = c0; cb < c1; cb += 64) {
    const int64_t c = cb + lane;
    APair p{0.0, -INFINITY};  // identity
    if (c < c1) {
      p.a = o.special[c] ? -INFINITY : o.asum[c];
      p.b = o.cexit[c];
    }
    KS_DPP_SCAN(APair, p, dpp_ap, ap_op);
    const APair ex = ap_prev(p);
    const double ea = ex.a, eb = ex.b;
    if (c < c1) xt[c] = fmax(carry + ea, eb);
    const double la = rld(p.a, 63), lb = rld(p.b, 63);
    carry = fmax(carry + la, lb);
    if (!(carry == carry)) carry = 0.0;
  }
}

// Per-tile run map: block r writes r for the stitch tiles of run r.
__global__ void k_tile_runs(const int64_t *__restrict__ tbase, int64_t nruns, int32_t *__restrict__ trun) {
  const int64_t r = blockIdx.x;
  if (r >= nruns) return;
  for (int64_t t = tbase[r] + threadIdx.x; t < tbase[r + 1]; t += blockDim.x) trun[t] = (int32_t)r;
}

// Run of stitch tile t from the per-tile run map (k_tile_runs): one load
// instead of a dependent binary search over the runs, which bounded the
// wave-per-tile kernels by its latency (12 loads at 2,790 runs).
__device__ __forceinline__ void tile_of(const int64_t *__restrict__ tbase, const int64_t *__restrict__ cbase,
                                        const int32_t *__restrict__ trun, int64_t t, int64_t &r, int64_t &c0,
                                        int64_t &c1, int64_t nruns) {
  int64_t lo;
  if (trun) {
    lo = trun[t];
  } else {  // (KS_TILE_SEARCH: the binary search, A/B)
    lo = 0;
    int64_t hi = nruns - 1;  // last run with tbase[r] <= t
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (tbase[mid] <= t) lo = mid; else hi = mid - 1;
    }
  }
  r = lo;
  c0 = cbase[lo] + (t - tbase[lo]) * 64;
  c1 = min(c0 + 64, cbase[lo + 1]);
}

// The same prediction as k_approx_scan in three parallel steps over the
// 64-chunk tiles of the runs (the stitch tiles): (A) every tile's composite
// map, (B) per run a wave scan of its tiles' maps (64 tiles per step instead
// of 64 chunks), (C) every tile applies its entry to its chunks.  The
// composition order differs from k_approx_scan, so the FP64 results may
// differ in the last bits: only a prediction, never a result.
__device__ __forceinline__ void ascan_pair(double &a, double &b, int lane) {
  APair p{a, b};  // (a1,b1) then (a2,b2) = (a1+a2, max(b1+a2, b2))
  KS_DPP_SCAN(APair, p, dpp_ap, ap_op);
  a = p.a;
  b = p.b;
  (void)lane;
}
// the exclusive pair (the previous lane's inclusive one; identity in lane 0)
__device__ __forceinline__ void ascan_prev(double a, double b, double &ea, double &eb) {
  const APair ex = ap_prev(APair{a, b});
  ea = ex.a;
  eb = ex.b;
}
__global__ void __launch_bounds__(256) k_ascan_tiles(const int64_t *__restrict__ tbase, const int64_t *__restrict__ cbase,
                                                    int64_t nruns, const int32_t *__restrict__ trun, P1 o, double2 *__restrict__ tagg, int64_t t_lo,
                                                    int64_t t_hi) {
  const int64_t t = t_lo + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // wave per tile
  if (t >= t_hi) return;
  const int lane = threadIdx.x & 63;
  int64_t r, c0, c1;
  tile_of(tbase, cbase, trun, t, r, c0, c1, nruns);
  const int64_t c = c0 + lane;
  double a = 0.0, b = -INFINITY;
  if (c < c1) {
    a = o.special[c] ? -INFINITY : o.asum[c];
    b = o.cexit[c];
  }
  ascan_pair(a, b, lane);
  if (lane == 63) tagg[t] = make_double2(a, b);
}
__global__ void __launch_bounds__(64) k_ascan_runs(const int64_t *__restrict__ tbase, int64_t nruns,
                                                   const double2 *__restrict__ tagg, double *__restrict__ tin,
                                                   int64_t r_lo) {
  const int64_t r = r_lo + blockIdx.x;
  if (r >= nruns) return;
  const int lane = threadIdx.x;
  const int64_t t0 = tbase[r], t1 = tbase[r + 1];
  double carry = 0.0;
  for (int64_t tb = t0; tb < t1; tb += 64) {
    const int64_t t = tb + lane;
    double a = 0.0, b = -INFINITY;
    if (t < t1) {
      const double2 v = tagg[t];
      a = v.x;
      b = v.y;
    }
    ascan_pair(a, b, lane);
    double ea, eb;
    ascan_prev(a, b, ea, eb);
    double xin = fmax(carry + ea, eb);
    if (!(xin == xin)) xin = 0.0;
    if (t < t1) tin[t] = xin;
    const double la = rld(a, 63), lb = rld(b, 63);
    carry = fmax(carry + la, lb);
    if (!(carry == carry)) carry = 0.0;
  }
}
__global__ void __launch_bounds__(256) k_ascan_apply(const int64_t *__restrict__ tbase, const int64_t *__restrict__ cbase,
                                                    int64_t nruns, const int32_t *__restrict__ trun, P1 o, const double *__restrict__ tin,
                                                    double *__restrict__ xt, int64_t t_lo, int64_t t_hi) {
  const int64_t t = t_lo + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // wave per tile
  if (t >= t_hi) return;
  const int lane = threadIdx.x & 63;
  int64_t r, c0, c1;
  tile_of(tbase, cbase, trun, t, r, c0, c1, nruns);
  const int64_t c = c0 + lane;
  double a = 0.0, b = -INFINITY;
  if (c < c1) {
    a = o.special[c] ? -INFINITY : o.asum[c];
    b = o.cexit[c];
  }
  ascan_pair(a, b, lane);
  double ea, eb;
  ascan_prev(a, b, ea, eb);
  if (c < c1) xt[c] = fmax(tin[t] + ea, eb);
}

// Largest value of the predicted trajectory that keeps a binade summary
// meaningful; below kLMin the trajectory crosses binades every few steps.
constexpr double kLMin = 64.0;

// Carried chunks without a usable summary are replayed wave-parallel
// (replay_par) when its speculation verifies, else serially.
#ifdef KS_NO_PAR_REPLAY
constexpr bool kParReplay = false;
#else
constexpr bool kParReplay = true;
#endif

// Summary of each chunk for the binade of its predicted trajectory (lane per
// chunk, full occupancy); chunks predicted to leave the binade or to approach
// 0 get none.
// kTab (small k, k_pass1_lds): the table staged in LDS too (dynamic, <= 128
// KiB): with a compressed table whose LUT is in LDS (kLds) its uint16 codes,
// else its 4^k FP64 values (lut[codes[i]] for a compressed one) read as an
// uncompressed base table (instantiated with kCompressed = false).  At k = 7
// (`profiles/r3/smallk/`): +-1 (2 values) codes 3.75 ms vs values 4.18;
// log2 (16 K values, LUT beyond LDS) values 6.4 ms vs codes 9.1.
// (KS_NO_SUMMARIES A/B: no chunk gets a summary; every carried chunk replays)
__global__ void __launch_bounds__(1024) k_summ_none(Chunks g, Summ sm) {
  const int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < g.nch) sm.e[c] = INT32_MIN;
}

template <bool kCompressed, bool kLds, bool kTab = false>
__global__ void __launch_bounds__(1024) k_summaries(Chunks g, const uint8_t *__restrict__ seq, int64_t total,
                                                    int k, TableView tv, const uint16_t *__restrict__ codes, P1 o,
                                                    const double *__restrict__ xt, Summ sm) {
  __shared__ double s_lut[kLds ? kLdsLutMax : 1];
  extern __shared__ __attribute__((aligned(16))) uint8_t s_tab[];
  if (kLds)
    for (int i = threadIdx.x; i < tv.nlut; i += blockDim.x) s_lut[i] = tv.lut[i];
  if (kTab) {
    const int nk = 1 << (2 * k);
    if (kCompressed) {
      uint16_t *sc = reinterpret_cast<uint16_t *>(s_tab);
      for (int i = threadIdx.x; i < nk; i += blockDim.x) sc[i] = tv.codes[i];
      tv.codes = sc;
    } else {
      double *sv = reinterpret_cast<double *>(s_tab);
      for (int i = threadIdx.x; i < nk; i += blockDim.x) sv[i] = tv.compressed ? tv.lut[tv.codes[i]] : tv.vals[i];
      tv.vals = sv;
      tv.compressed = 0;
      tv.codes = nullptr;
    }
    tv.ext = nullptr;  // (values from the staged base table)
    tv.line = nullptr;
  }
  if (kLds || kTab) __syncthreads();
  const int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (the part's chunks)
  if (c >= g.nch) return;
  sm.e[c] = INT32_MIN;
  if (o.special[c]) return;
  const double x = xt[c];
  if (!(x >= kLMin) || !(x < 1.0e18)) return;
  const int e = (int)((__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
  const double lo = fmin(x, x + o.pmin[c]), hi = fmax(x, x + o.pmax[c]);
  const double slack = ldexp(1.0, e - 24) + o.sabs[c] * 1e-9;
  if (!(lo - slack >= ldexp(1.0, e)) || !(hi + slack < ldexp(1.0, e + 1))) return;
  long long D[2], M[2], N[2];
  int A[2];
  if (!chunk_summary<kCompressed, kLds>(g, seq, total, k, tv, codes, c, e, D, M, A, N, s_lut)) return;
  sm.e[c] = e;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sm.D[2 * c + t] = D[t];
    sm.M[2 * c + t] = M[t];
    sm.N[2 * c + t] = N[t];
    sm.A[2 * c + t] = A[t];
  }
}

// Pass-1 summaries (kSumm): the summary of every chunk whose exact carry will
// want one (same test as k_summaries) is the pass-1 one when pass 1 predicted
// this binade; the others (no or another prediction, a tie, the tail chunks)
// are listed for k_summ_fixw.
// The per-chunk part of the selection: the selected summary (or none) of
// chunk c; want: list it for k_summ_fixw; rwant: list it for the replay
// prefetch.
__device__ __forceinline__ void select_one(const Chunks &g, const P1 &o, const double *__restrict__ xt,
                                           const SummP1 &sp, const Summ &sm, const double *__restrict__ xh,
                                           unsigned long long *__restrict__ why, const ReplayBuf &rp, int64_t c,
                                           bool &want, bool &rwant) {
  want = rwant = false;
  sm.e[c] = INT32_MIN;
  uint8_t sel = 2;
  const double x = xt[c];
  if (rp.slot) rp.slot[c] = -1;
  if (!o.special[c] && x >= kLMin && x < 1.0e18) {
    const int e = (int)((__double_as_longlong(x) >> 52) & 0x7ff) - 1023;
    const double lo = fmin(x, x + o.pmin[c]), hi = fmax(x, x + o.pmax[c]);
    const double slack = ldexp(1.0, e - 24) + o.sabs[c] * 1e-9;
    if (lo - slack >= ldexp(1.0, e) && hi + slack < ldexp(1.0, e + 1)) {
      const int t = sp.e[2 * c] == e ? 0 : (sp.e[2 * c + 1] == e ? 1 : -1);
      if (t >= 0) {
        sm.e[c] = e;
        if (sm.sel) {
          sel = (uint8_t)t;  // read in place (summ_at)
        } else {
          const long long D = sp.D[2 * c + t], M = sp.M[2 * c + t], N = sp.N[2 * c + t];
          const int A = sp.A[2 * c + t];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            sm.D[2 * c + q] = D;
            sm.M[2 * c + q] = M;
            sm.N[2 * c + q] = N;
            sm.A[2 * c + q] = A;
          }
        }
      } else {
        want = true;
        // diagnostics (KS_DEBUG_CARRY): no prediction / void summary / other binade
        if (why) atomicAdd(&why[sp.e[2 * c] != INT32_MIN ? 2 : (xh[c] >= kP1SumMin ? 1 : 0)], 1ull);
      }
    }
  }
  if (sm.sel) sm.sel[c] = sel;
  // no summary will serve it: a likely replay unless it enters at 0 or
  // clamps for certain (with a wide margin: a needless prefetch is cheap)
  rwant = rp.slot && !want && sel == 2 && sm.e[c] == INT32_MIN && !o.special[c] && x > 0.0 &&
          !(x + o.pmin[c] < -ldexp(fabs(x) + o.sabs[c], -8));
}

// Wave-aggregated appends of the wave's listed chunks (every lane calls it).
__device__ __forceinline__ void select_append(bool want, bool rwant, int64_t c, int64_t *__restrict__ fix,
                                              unsigned long long *__restrict__ nfix, const ReplayBuf &rp, int hi) {
  const int lane = threadIdx.x & 63;
  const unsigned long long b = __ballot(want);
  if (b) {
    const int leader = __ffsll((long long)b) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(nfix, (unsigned long long)__popcll(b));
    base = __shfl(base, leader, 64);
    if (want) fix[base + __popcll(b & ((1ull << lane) - 1ull))] = c;
  }
  const unsigned long long br = __ballot(rwant);
  if (br) {
    const int leader = __ffsll((long long)br) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(rp.count + hi, (unsigned long long)__popcll(br));
    base = __shfl(base, leader, 64);
    const unsigned long long q = base + __popcll(br & ((1ull << lane) - 1ull));
    if (rwant && (int64_t)q < rp.cap) {
      const int64_t sl = hi * rp.cap + (int64_t)q;
      rp.slot[c] = (int32_t)sl;
      rp.chunk[sl] = c;
    }
  }
}

__global__ void k_copy_u64(const unsigned long long *__restrict__ src, unsigned long long *__restrict__ dst, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// k_seg_marks and the summary selection in one pass (a wave per 64-chunk window from
// the one holding c0 - 1): the window's segment marks, then the summaries.
__global__ void __launch_bounds__(256) k_marks_select(Chunks g, P1 o, const double *__restrict__ xt,
                                                      uint8_t *__restrict__ flag, int64_t nw, SummP1 sp, Summ sm,
                                                      int64_t *__restrict__ fix, unsigned long long *__restrict__ nfix,
                                                      const double *__restrict__ xh,
                                                      unsigned long long *__restrict__ why, ReplayBuf rp, int hi) {
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wv >= nw) return;
  const int lane = threadIdx.x & 63;
  const int64_t e = ((g.c0 > 0 ? g.c0 - 1 : 0) / 64 + wv) * 64 + lane;
  bool elig = false, next_run = false;
  if (e + 1 < g.nch && e + 1 >= g.c0) {
    next_run = g.run[e + 1] != g.run[e];
    if (!next_run && e >= g.c0 && !o.special[e]) {
      const double x = xt[e];
      elig = x + o.pmin[e] < -ldexp(fabs(x) + o.sabs[e], -20);  // false for NaN
    }
  }
  const unsigned long long b = __ballot(elig);
  const int f = b ? __ffsll((long long)b) - 1 : 64;
  if (e + 1 < g.nch && e + 1 >= g.c0) flag[e + 1] = (next_run || lane == f) ? 1 : 0;
  if (e == 0 && g.c0 == 0) flag[0] = 1;
  bool want = false, rwant = false;
  if (e >= g.c0 && e < g.nch) select_one(g, o, xt, sp, sm, xh, why, rp, e, want, rwant);
  select_append(want, rwant, e, fix, nfix, rp, hi);
}

// Parity map of a run of steps: entry parity p -> the increment d_p of the
// integer trajectory (exact halves round to even, so a step's increment
// depends on the accumulator's parity).  Composition is associative.
struct PMap {
  long long d0, d1;
};
__device__ __forceinline__ PMap pm_compose(const PMap &a, const PMap &b) {  // a then b
  return PMap{a.d0 + ((a.d0 & 1) ? b.d1 : b.d0), a.d1 + (((1 + a.d1) & 1) ? b.d1 : b.d0)};
}

// Summaries of the listed chunks, one wave per listed chunk (4 indices per lane): the values
// through the expanded table in one or two round trips, the binade-integer
// increments as parity maps, a wave scan of the maps, and wave reductions
// for the total, first maximum and minimum of both entry parities -- the
// same summary chunk_summary_impl computes serially.
template <bool kLds>
__global__ void __launch_bounds__(256) k_summ_fixw(Chunks g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                                   TableView tv, const double *__restrict__ xt,
                                                   const int64_t *__restrict__ fix,
                                                   const unsigned long long *__restrict__ nfix, Summ sm,
                                                   ReplayBuf rp, int hi) {
  __shared__ double s_lut[kLds ? kLdsLutMax : 1];
  if (kLds) {
    for (int i = threadIdx.x; i < tv.nlut; i += blockDim.x) s_lut[i] = tv.lut[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nf = (int64_t)*nfix;
  // the waves past the fix list gather the listed likely replays
  const int64_t nr = rp.slot ? min((int64_t)rp.count[hi], rp.cap) : 0;
  for (int64_t f = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); f < nf + nr; f += nw) {
    if (f >= nf) {
      const int64_t sl = hi * rp.cap + (f - nf);
      const int64_t cr = rp.chunk[sl];
      double v[4];
      values16_nostore<4>(g, seq, total, k, tv, cr, 4 * lane, g.n[cr], v, kLds ? s_lut : nullptr);
      double2 *d = reinterpret_cast<double2 *>(rp.v + sl * 256 + 4 * lane);
      d[0] = make_double2(v[0], v[1]);
      d[1] = make_double2(v[2], v[3]);
      continue;
    }
    const int64_t c = fix[f];
    const int e = binade_of(xt[c]);
    const double scale = ldexp(1.0, 52 - e);
    const int n = g.n[c];
    double v[4];
    values16_nostore<4>(g, seq, total, k, tv, c, 4 * lane, n, v, kLds ? s_lut : nullptr);
    bool ok = true;
    PMap lm{0, 0}, pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (4 * lane + q < n) {
        const double y = v[q] * scale;  // exact: power-of-two scaling
        ok &= fabs(y) < 2251799813685248.0;  // 2^51; false for NaN / Inf
        const double fq = floor(y), fr = y - fq;
        const long long qi = ok ? (long long)fq : 0;
        const bool up = fr > 0.5, tie = fr == 0.5;
        const PMap el{qi + ((up || (tie && (qi & 1))) ? 1 : 0), qi + ((up || (tie && ((1 + qi) & 1))) ? 1 : 0)};
        lm = pm_compose(lm, el);
      }
      pre[q] = lm;
    }
    const PPair incp = pp_scan_incl(PPair{lm.d0, lm.d1});
    const PPair excp = pp_prev(incp);
    const PMap exc{excp.d0, excp.d1};
    const PMap tot{rl64(incp.d0, 63), rl64(incp.d1, 63)};
    ok = __all(ok);
    long long M[2], N[2];
    int A[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const long long et = t ? exc.d1 : exc.d0;
      const int pt = (int)((t + et) & 1);  // parity entering this lane's first step
      long long best = LLONG_MIN, mn = LLONG_MAX;
      int barg = 0x7fffffff;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (4 * lane + q < n) {
          const long long val = et + (pt ? pre[q].d1 : pre[q].d0);
          if (val > best) { best = val; barg = 4 * lane + q; }
          mn = min(mn, val);
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {  // max with the first index, min
        const long long ob = __shfl_xor(best, d, 64);
        const int oa = __shfl_xor(barg, d, 64);
        if (ob > best || (ob == best && oa < barg)) { best = ob; barg = oa; }
        mn = min(mn, (long long)__shfl_xor(mn, d, 64));
      }
      M[t] = best;
      N[t] = mn;
      A[t] = barg;
    }
    const long long lim = 4503599627370496LL;  // 2^52: partial sums exact and far from overflow
    ok = ok && M[0] < lim && M[1] < lim && N[0] > -lim && N[1] > -lim;
    if (lane == 0 && ok) {
      sm.e[c] = e;
      sm.D[2 * c] = tot.d0;
      sm.D[2 * c + 1] = tot.d1;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sm.M[2 * c + t] = M[t];
        sm.N[2 * c + t] = N[t];
        sm.A[2 * c + t] = A[t];
      }
    }
  }
}

// Segment starts: every run start, and after the first chunk of each
// 64-chunk window that is predicted to clamp by a wide margin (so that the
// exact entry, which differs from x~ by rounding only, clamps too).
__global__ void __launch_bounds__(256) k_seg_marks(Chunks g, P1 o, const double *__restrict__ xt,
                                                   uint8_t *__restrict__ flag, int64_t nw) {
  // windows of 64 chunks from the one holding c0 - 1 (a wave each, nw of
  // them); only this launch's chunks [c0, nch) are read and marked
  const int64_t wv = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wv >= nw) return;
  const int lane = threadIdx.x & 63;
  const int64_t e = ((g.c0 > 0 ? g.c0 - 1 : 0) / 64 + wv) * 64 + lane;
  bool elig = false, next_run = false;
  if (e + 1 < g.nch && e + 1 >= g.c0) {
    next_run = g.run[e + 1] != g.run[e];
    if (!next_run && e >= g.c0 && !o.special[e]) {
      const double x = xt[e];
      elig = x + o.pmin[e] < -ldexp(fabs(x) + o.sabs[e], -20);  // false for NaN
    }
  }
  const unsigned long long b = __ballot(elig);
  const int f = b ? __ffsll((long long)b) - 1 : 64;
  if (e + 1 < g.nch && e + 1 >= g.c0) flag[e + 1] = (next_run || lane == f) ? 1 : 0;
  if (e == 0 && g.c0 == 0) flag[0] = 1;
}


// Exact carry, one wave per run, walking 64-chunk tiles (lane j <-> chunk
// cb + j).  Per chunk, in order: entry 0 -> clean exit (CLEAN); a binade
// summary valid for the exact entry -> integer step (L; the summaries of the
// tile's lanes are computed wave-parallel, once per binade); a certain clamp
// (x + minprefix < -margin) -> clean exit (R); else exact replay (U).  The
// chain is wave-uniform; L chunks also get their head (max/argmax) here.

// Exact carry, one wave per run, walking 64-chunk tiles (lane j <-> chunk
// cb + j, its inputs in registers, broadcast with v_readlane).  Per chunk, in
// order: entry 0 -> clean exit (CLEAN); the chunk's precomputed binade summary
// is for the exact entry's binade and its integer trajectory stays inside ->
// integer step (L, also yields the head); a certain clamp (x + minprefix <
// -margin) -> clean exit (R); else exact replay (U): the wave loads the 256
// values into registers (4 per lane) and walks them with readlane.
//
// Segments: a run's chain is cut after chunks predicted (x~ from P2, with a
// wide margin) to clamp: the chunk after one starts a segment whose entry is
// assumed to be that chunk's clean exit, and the segments run in parallel.
// The wave of the preceding segment checks the assumption against its exact
// exit (bit 16 of err on mismatch; the host then redoes the carry per run).
// Wave-parallel exact replay of one chunk (U) from its exact entry x > 0, for
// a trajectory that stays positive (no clamp): speculate, then verify.
//  1. approximate prefix sums y_p (wave scan) give each position the binade
//     e_p its exact value S_p should have; every y_p must be farther than
//     the summation error bound from a binade edge and from 0;
//  2. inside a stretch of equal binades, fl(S + s) = S + RN(s / ulp) exactly
//     (lemma 2 of the summaries) once S and the result are known to share
//     binade e: integer increments d_p, an exact segmented prefix scan;
//  3. the first position of each stretch (a binade crossing) is the
//     reference's FP64 add on the exact previous value, walked in order
//     (a few per chunk);
//  4. every integer result is checked to lie strictly inside its binade
//     (m in [2^52 + 1, 2^53 - 2]), every crossing value to have the predicted
//     binade.  Half-ulp ties round to even, i.e. depend on the parity of m:
//     steps are parity pairs composed associatively (as in the summaries).
// Returns false (wave-uniform) if anything cannot be verified: the caller
// replays serially.  On success T = exit, hmax / harg = max and first argmax.
// Positions are lane-major: p = 4 * lane + q.
__device__ bool replay_par(const double v[4], int n, double x, double &T, double &hmax, int &harg) {
  const int lane = threadIdx.x & 63;
  bool live[4];
  double a[4];
  double loc = 0.0, labs = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    live[q] = 4 * lane + q < n;
    const double vq = live[q] ? v[q] : 0.0;
    loc += vq;
    labs += fabs(vq);
    a[q] = loc;
  }
  const double incl = wave_sum_incl(loc);
  const double sab = rld(wave_sum_incl(labs), 63);
  if (!(sab < 1.0e300)) return false;  // non-finite values: serial
  const double excl = incl - loc;
  const double err = ldexp(x + sab, -42);  // >> 2 * 256 * 2^-53 * (x + sum |s|)
  int e[4];
  bool ok = true;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double y = x + excl + a[q];
    const double lo = y - err, hi = y + err;
    e[q] = binade_of(y);
    if (live[q]) ok &= lo > 0x1p-1000 && hi < 1.0e300 && binade_of(lo) == binade_of(hi);
  }
  if (!__all(ok)) return false;
  // crossings and integer increments: a step inside binade e adds
  // RN(s / ulp) to the mantissa m; at an exact half the even result wins, so
  // the increment depends on the parity of m: each step is the pair
  // (d0, d1) = increment for an even / odd m, and pairs compose
  // associatively: (f then g)_b = f_b + g_{(b + f_b) & 1}.
  const int ex = binade_of(x);
  const int eprev_lane = wave_prev_i32(e[3]);
  bool cr[4];
  long long d0[4], d1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ep = q ? e[q - 1] : (lane ? eprev_lane : ex);
    cr[q] = live[q] && e[q] != ep;
    d0[q] = 0;
    d1[q] = 0;
    if (live[q] && !cr[q]) {
      const double yv = ldexp(v[q], 52 - e[q]);
      const double fl = floor(yv), fr = yv - fl;
      ok &= fabs(yv) < 0x1p60;
      const long long f = (long long)fl;
      if (fr == 0.5) {
        d0[q] = f + (f & 1);
        d1[q] = f + ((1 + f) & 1);
      } else {
        d0[q] = d1[q] = f + (fr > 0.5 ? 1 : 0);
      }
    }
  }
  if (!__all(ok)) return false;
  auto comp = [](long long f0, long long f1, long long g0, long long g1, long long &r0, long long &r1) {
    r0 = f0 + (((f0 & 1) == 0) ? g0 : g1);
    r1 = f1 + ((((1 + f1) & 1) == 0) ? g0 : g1);
  };
  // segmented inclusive scan: (Q0, Q1)[q] = composed increments since the
  // last crossing (a crossing position is a segment head with the identity)
  long long Q0[4], Q1[4];
  long long r0 = 0, r1 = 0;
  bool lflag = false;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (cr[q]) { r0 = 0; r1 = 0; lflag = true; }
    long long n0, n1;
    comp(r0, r1, d0[q], d1[q], n0, n1);
    r0 = n0; r1 = n1;
    Q0[q] = r0;
    Q1[q] = r1;
  }
  // segmented scan of the lane aggregates after their last crossing:
  // (L, R) -> R.f ? R : (L.s then R.s, L.f | R.f); identity ((0, 0), 0)
  SegPP sg{PPair{r0, r1}, lflag ? 1 : 0};
  KS_DPP_SCAN(SegPP, sg, dpp_seg, seg_op);
  const PPair cin = pp_prev(sg.s);  // exclusive carry-in (lane 0: identity)
  long long c0 = cin.d0, c1 = cin.d1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (cr[q]) break;
    long long n0, n1;
    comp(c0, c1, Q0[q], Q1[q], n0, n1);
    Q0[q] = n0;
    Q1[q] = n1;
  }
  // walk the crossings in order: S_c = fl(S_{c-1} + v_c) on the exact previous value
  long long Mc[4] = {0, 0, 0, 0};
  long long Mcur = mant_of(x);
  unsigned long long lm = __ballot(cr[0] || cr[1] || cr[2] || cr[3]);
  bool good = true;
  while (lm) {
    const int L = __ffsll((long long)lm) - 1;
    lm &= lm - 1;
    const int crm = __builtin_amdgcn_readlane((cr[0] ? 1 : 0) | (cr[1] ? 2 : 0) | (cr[2] ? 4 : 0) | (cr[3] ? 8 : 0), L);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!(crm & (1 << q))) continue;
      const int p = 4 * L + q;
      double sprev;
      if (p == 0) {
        sprev = x;
      } else {
        const int pl = (p - 1) >> 2, pq = (p - 1) & 3;
        const bool odd = Mcur & 1;
        const long long qsel = pq == 0 ? (odd ? Q1[0] : Q0[0]) : pq == 1 ? (odd ? Q1[1] : Q0[1])
                             : pq == 2 ? (odd ? Q1[2] : Q0[2]) : (odd ? Q1[3] : Q0[3]);
        const int esel = pq == 0 ? e[0] : pq == 1 ? e[1] : pq == 2 ? e[2] : e[3];
        const long long mp = Mcur + rl64(qsel, pl);
        const int ep = rl32(esel, pl);
        good &= mp >= (1LL << 52) + 1 && mp <= (1LL << 53) - 2;
        sprev = from_mant(mp, ep);
      }
      const double vc = rld(v[q], L);
      const double t = sprev + vc;  // the reference's add (kmer_spans.c:269)
      const int ec = rl32(e[q], L);
      good &= t > 0 && binade_of(t) == ec;
      Mcur = mant_of(t);
      if (lane == L) Mc[q] = Mcur;
    }
  }
  if (!good) return false;  // wave-uniform (built from broadcast values)
  // stretch-start mantissa per position (forward fill of the crossings) and
  // the exact values, verified strictly inside their binades
  long long lastm = 0;
  bool has = false;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (cr[q]) { lastm = Mc[q]; has = true; }
  // forward fill: (L, R) -> (R.f ? R.m : L.m, L.f | R.f); identity (0, 0)
  FillM fw{lastm, has ? 1 : 0};
  KS_DPP_SCAN(FillM, fw, dpp_fill, fill_op);
  long long start_m = wave_prev_i64(fw.m);
  const int start_f = wave_prev_i32(fw.f);
  if (lane == 0 || !start_f) start_m = mant_of(x);
  double S[4];
  bool inb = true;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (cr[q]) start_m = Mc[q];
    const long long m = cr[q] ? start_m : start_m + ((start_m & 1) ? Q1[q] : Q0[q]);
    if (live[q] && !cr[q]) inb &= m >= (1LL << 52) + 1 && m <= (1LL << 53) - 2;
    S[q] = from_mant(m, e[q]);
  }
  if (!__all(inb)) return false;
  // exit, max and first argmax
  const int pl = (n - 1) >> 2, pq = (n - 1) & 3;
  const double slast = pq == 0 ? S[0] : pq == 1 ? S[1] : pq == 2 ? S[2] : S[3];
  T = rld(slast, pl);
  double bm = -1.0;
  int bi = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (live[q] && S[q] > bm) { bm = S[q]; bi = 4 * lane + q; }
  // wave max (the DPP identity 0.0 is below no result: every S is >= 0)
  double wm = bm;
  auto dmax = [](double a, double b) { return fmax(a, b); };
  KS_DPP_SCAN(double, wm, dpp_f64, dmax);
  wm = rld(wm, 63);
  const unsigned long long bl = __ballot(bm == wm && bm >= 0.0);
  const int fl = __ffsll((long long)bl) - 1;
  hmax = wm;
  harg = __builtin_amdgcn_readlane(bi, fl);
  return true;
}

template <bool kCompressed>
__device__ __forceinline__ void carry_segment(const Chunks &g, int64_t c0, int64_t c1, const uint8_t *__restrict__ seq,
                                              int64_t total, int k, const TableView &tv,
                                              const uint16_t *__restrict__ codes, const P1 &o, const Summ &sm,
                                              const Carry &cr, const TileComp &tc, const ReplayBuf &rp,
                                              unsigned long long *__restrict__ nreplay,
                                              unsigned int *__restrict__ err, long long *__restrict__ dbg,
                                              int64_t r) {
  const int lane = threadIdx.x & 63;
  // (the cooperative FP64 line fetch of the replays, values4_coop_f64: a wave's slice)
  __shared__ uint4 s_coop[4][256];
  __shared__ unsigned long long s_ckey[4][64];
  double x = (c0 > 0 && g.run[c0] == g.run[c0 - 1]) ? o.cexit[c0 - 1] : 0.0;
  unsigned long long replays = 0;
  const long long t_start = dbg ? (long long)__builtin_amdgcn_s_memtime() : 0;
  long long n_l = 0, n_r = 0, n_par = 0;  // diagnostics: replays that clamp, replayed indices
  // per-lane inputs of one 64-chunk tile; the next tile's are loaded before
  // the current one is processed (all loads independent: hides their latency
  // behind the tile's scan)
  // (start: a replay's first memory round trip -- chunk start, then its
  // packed bases, then the table -- is taken here, with the tile's loads)
  struct TileIn {
    double exit, pmin, sabs;
    int64_t start;
    int spec, n, se, rs;
    long long D[2], M[2], N[2];
    int A[2];
  };
  auto load_tile = [&](int64_t cb, int64_t ce, TileIn &t) {
    const int64_t c = cb + lane;
    const bool live = c < ce;
    const int64_t cc = live ? c : c0;  // dead lanes read a valid chunk, values unused
    t.exit = o.cexit[cc];
    t.pmin = o.pmin[cc];
    t.sabs = o.sabs[cc];
    t.spec = live ? o.special[cc] : 1;
    t.n = live ? g.n[cc] : 0;
    t.start = g.start[cc];
    t.rs = (live && rp.slot) ? rp.slot[cc] : -1;
    const int se = sm.e[cc];
    t.se = live ? se : INT32_MIN;
    const SummAt r = summ_at(sm, cc);
    t.D[0] = r.D[r.i0];
    t.D[1] = r.D[r.i1];
    t.M[0] = r.M[r.i0];
    t.M[1] = r.M[r.i1];
    t.N[0] = r.N[r.i0];
    t.N[1] = r.N[r.i1];
    t.A[0] = r.A[r.i0];
    t.A[1] = r.A[r.i1];
  };
  // tiles are the global 64-chunk tiles (partial at the segment's ends)
  auto tile_end = [&](int64_t cb) { return min(c1, (cb & ~(int64_t)63) + 64); };
  TileIn cur;
  load_tile(c0, tile_end(c0), cur);
  long long t_fast = 0, t_rep = 0;  // diagnostics: cycles in fast tiles, in replays
  bool try_batch = true;
  // the packed bases of the chunk after a replayed one, loaded under that
  // replay's table reads (replays come in runs where the carry crosses
  // binades): pf_c = the chunk they belong to, pf_ok = packed_bits' result
  int64_t pf_c = -1;
  bool pf_ok = false;
  uint64_t pf_x = 0;
  for (int64_t cb = c0; cb < c1;) {
    const long long tt0 = dbg ? (long long)__builtin_amdgcn_s_memtime() : 0;
    // Tile batch: up to 64 whole tiles at once from their composites (the
    // serial fast path's test per tile, with the entries of all of them from
    // one wave scan of the composed increments); accepted tiles are expanded
    // per chunk by k_tile_apply.  The first rejected tile takes the per-tile
    // path below.
    if (tc.e && try_batch && (cb & 63) == 0 && x >= kLMin && x < 1.0e18) {
      const int e = binade_of(x);
      const int64_t ntl = min((int64_t)64, (c1 - cb) >> 6);
      if (e >= 6 && e <= 58 && ntl >= 2) {
        const int64_t t = (cb >> 6) + lane;
        const bool in = lane < ntl;
        const int te = in ? tc.e[t] : INT32_MIN;
        long long d0 = 0, d1 = 0, lo0 = 0, lo1 = 0, hi0 = -1, hi1 = -1;
        if (in) {
          d0 = tc.D[2 * t];
          d1 = tc.D[2 * t + 1];
          lo0 = tc.LO[2 * t];
          lo1 = tc.LO[2 * t + 1];
          hi0 = tc.HI[2 * t];
          hi1 = tc.HI[2 * t + 1];
        }
        if (!in || te != e) d0 = d1 = 0;  // identity beyond the first rejected tile (never used)
        const PPair ip = pp_scan_incl(PPair{d0, d1});  // inclusive composed increments
        const PPair xp = pp_prev(ip);
        const long long i0 = ip.d0, i1 = ip.d1, x0 = xp.d0, x1 = xp.d1;
        const long long m0 = mant_of(x);
        const long long mt = m0 + ((m0 & 1) ? x1 : x0);  // entry mantissa of tile t
        const int pt = (int)(mt & 1);
        const bool ok = in && te == e && mt >= (pt ? lo1 : lo0) && mt <= (pt ? hi1 : hi0);
        const unsigned long long bad = __ballot(!ok);
        const int f = bad ? __ffsll((long long)bad) - 1 : 64;
        if (f > 0) {
          if (lane < f) {
            tc.em[t] = mt;
            tc.ee[t] = e;
          }
          const long long mi = m0 + ((m0 & 1) ? i1 : i0);  // exit of tile t
          x = from_mant(rl64(mi, f - 1), e);
          n_l += 64 * f;
          cb += 64 * f;
          if (dbg) t_fast += (long long)__builtin_amdgcn_s_memtime() - tt0;
          if (cb >= c1) break;
          load_tile(cb, tile_end(cb), cur);
          try_batch = f == 64;  // a rejected tile goes through the per-tile path first
          continue;
        }
      }
    }
    try_batch = true;
    const int64_t ce = tile_end(cb);
    if (lane == 0 && tc.ee) tc.ee[cb >> 6] = INT32_MIN;  // not batched (the fallback pass reruns segments)
    TileIn nxt = cur;
    if (ce < c1) load_tile(ce, tile_end(ce), nxt);
    const int64_t c = cb + lane;
    const bool live = c < ce;
    const double l_exit = live ? cur.exit : 0.0;
    const double l_pmin = live ? cur.pmin : 0.0;
    const double l_sabs = live ? cur.sabs : 0.0;
    const int l_spec = cur.spec;
    const int l_n = cur.n;
    const int se = cur.se;
    long long D[2] = {0, 0}, M[2] = {0, 0}, N[2] = {0, 0};
    int A[2] = {0, 0};
    if (se != INT32_MIN) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        D[t] = cur.D[t];
        M[t] = cur.M[t];
        N[t] = cur.N[t];
        A[t] = cur.A[t];
      }
    }
    const int nb = (int)(ce - cb);
    double my_x = 0.0, my_hmax = -1.0;
    int my_mode = kModeClean, my_harg = 0, my_hq = -1;
    // Runs of summary chunks: from chunk j on, the chunks that have a summary
    // for the binade of the exact carry and stay inside it are taken at once:
    // their integer maps m -> m + D[m & 1] composed by a wave scan (chunks
    // before j and past the tile: identity), each checked at its exact entry.
    // The first other chunk takes the serial step.  (A fast tile is one run
    // from j = 0; a replay in mid-tile no longer walks the rest serially.)
    bool tile_done = true;  // diagnostics: no serial step in this tile
    for (int j = 0; j < nb; ++j) {
      if (x >= kLMin && x < 1.0e18 && rl32(se, j) == binade_of(x)) {
        const int e = binade_of(x);
        const bool in = live && lane >= j;
        const PPair ip = pp_scan_incl(PPair{in ? D[0] : 0, in ? D[1] : 0});  // inclusive composed map
        const PPair xp = pp_prev(ip);
        const long long x0 = xp.d0, x1 = xp.d1;
        const long long m0 = mant_of(x);
        const long long mj = m0 + ((m0 & 1) ? x1 : x0);  // exact entry of this lane's chunk
        const int pj = (int)(mj & 1);
        const bool ok = lane < j || (in && se == e && mj + (pj ? N[1] : N[0]) >= (1LL << 52) + 1 &&
                                     mj + (pj ? M[1] : M[0]) <= (1LL << 53) - 2);
        const unsigned long long bad = __ballot(!ok);
        const int f = bad ? __ffsll((long long)bad) - 1 : 64;  // <= nb
        if (f > j) {
          if (lane >= j && lane < f) {
            my_x = from_mant(mj, e);
            my_mode = kModeL;
            my_hmax = from_mant(mj + (pj ? M[1] : M[0]), e);
            my_harg = pj ? A[1] : A[0];
          }
          x = from_mant(rl64(mj + (pj ? D[1] : D[0]), f - 1), e);
          n_l += f - j;
          j = f - 1;
          continue;
        }
      }
      // Runs of clean and certain-clamp chunks at once: both leave the
      // chunk's clean exit, so from chunk j on, a chunk entered by its
      // predecessor's clean exit (x for chunk j) that enters at 0 or clamps
      // for certain -- and has no summary for its entry's binade, which the
      // serial order tries first -- takes its mode here; the first other
      // chunk takes the serial step.  (Weighted rank at config 3: 11 M of
      // 12 M chunks are clean or clamp; in-process k = 15 44.2 vs 44.9 ms,
      // k = 13 30.1 vs 30.6, metric unchanged: profiles/r5/ab/ab_bulk_clean_*.txt)
      {
        const double pe = __longlong_as_double(wave_prev_i64(__double_as_longlong(l_exit)));
        const double ent = lane == j ? x : pe;
        const bool in = live && lane >= j;
        const bool cl = ent == 0.0;
        const bool sm_ok = se != INT32_MIN && ent >= kLMin && ent < 1.0e18 && se == binade_of(ent);
        const bool rc = !cl && !sm_ok && !l_spec && ent + l_pmin < -ldexp(fabs(ent) + l_sabs, -40);
        const bool ok = lane < j || (in && (cl || rc));
        const unsigned long long bad = __ballot(!ok);
        const int f = bad ? __ffsll((long long)bad) - 1 : 64;
        if (f > j) {
          if (lane >= j && lane < f) {
            my_x = ent;
            my_mode = cl ? kModeClean : kModeR;
          }
          if (dbg) n_r += __popcll(__ballot(lane >= j && lane < f && rc));
          x = rld(l_exit, f - 1);
          j = f - 1;
          continue;
        }
      }
      tile_done = false;
      const double cj_exit = rld(l_exit, j);
      if (lane == j) my_x = x;
      int mode = kModeU;
      bool done = false;
      if (x == 0.0) {
        mode = kModeClean;
        x = cj_exit;
        done = true;
      } else if (x >= kLMin && x < 1.0e18 && rl32(se, j) == binade_of(x)) {
        const int e = binade_of(x);
        const long long m0 = mant_of(x);
        const int par = (int)(m0 & 1);
        const long long Nj = rl64(par ? N[1] : N[0], j), Mj = rl64(par ? M[1] : M[0], j);
        if (m0 + Nj >= (1LL << 52) + 1 && m0 + Mj <= (1LL << 53) - 2) {
          const long long Dj = rl64(par ? D[1] : D[0], j);
          mode = kModeL;
          if (lane == j) {
            my_hmax = from_mant(m0 + Mj, e);
            my_harg = par ? A[1] : A[0];
          }
          x = from_mant(m0 + Dj, e);
          done = true;
        }
      }
      if (!done && !rl32(l_spec, j) && x + rld(l_pmin, j) < -ldexp(fabs(x) + rld(l_sabs, j), -40)) {
        mode = kModeR;  // certain clamp -> coincides with the clean trajectory
        x = cj_exit;
        done = true;
      }
      const long long tr0 = dbg ? (long long)__builtin_amdgcn_s_memtime() : 0;
      if (!done) {  // exact replay of chunk cb + j from x; also yields its head
        mode = kModeU;
        ++replays;
        const int64_t cj = cb + j;
        const int n = rl32(l_n, j);
        double v[4];
        const int rsj = rl32(cur.rs, j);
        if (rsj >= 0) {  // gathered ahead (k_summ_fixw)
          const double2 *d = reinterpret_cast<const double2 *>(rp.v + (int64_t)rsj * 256 + 4 * lane);
          const double2 a = d[0], b = d[1];
          v[0] = a.x;
          v[1] = a.y;
          v[2] = b.x;
          v[3] = b.y;
        } else {
          const bool hx = !kCompressed && pf_c == cj && pf_ok;
          if (dbg && hx) n_par += 1LL << 32;  // (diagnostics: replays with their bases prefetched)
          uint64_t xq = pf_x;
          // (in-process at config 3: 24.63 vs 25.00 ms min, carry 4.83 vs 5.18 ms,
          // profiles/r6/rank/ab_carry_coop.txt)
          const bool coop = !kCompressed && tv.line && tv.line_kind == 2 && tv.line_own == 3 &&
                            __ballot(!(hx || packed_bits(g.packed, total, rl64(cur.start, j) + 4 * lane - k, xq))) == 0;
          if (coop) {
            values4_coop_f64(tv, xq, k, 4 * lane, n, v, s_coop[threadIdx.x >> 6], s_ckey[threadIdx.x >> 6]);
          } else {
            values4(g, seq, total, k, tv, kCompressed ? codes : nullptr, cj, rl64(cur.start, j), 4 * lane, n, v, hx,
                    pf_x);
          }
        }
        if (!kCompressed && cj + 1 < c1) {  // the next chunk's packed bases, under this replay's reads
          const int64_t stn = (j + 1 < nb) ? rl64(cur.start, j + 1) : rl64(nxt.start, 0);
          pf_ok = packed_bits(g.packed, total, stn + 4 * lane - k, pf_x);
          pf_c = cj + 1;
        }
        double T = x, hmax = -1.0;
        int hq = -1, harg = 0;
        const bool par = kParReplay && replay_par(v, n, x, T, hmax, harg);
        if (par) n_par += 1;
        for (int i = 0; i < 64 && hq < 0 && !par; ++i) {
          if (4 * i >= n) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int idx = 4 * i + q;
            if (idx < n && hq < 0) {
              const double t = T + rld(v[q], i);
              T = t > 0 ? t : 0.0;
              if (T == 0.0) hq = idx;
              else if (T > hmax) { hmax = T; harg = idx; }
            }
          }
        }
        if (lane == j) {
          my_hq = hq;
          my_hmax = hmax;
          my_harg = harg;
        }
        x = hq >= 0 ? cj_exit : T;
        if (dbg) t_rep += (long long)__builtin_amdgcn_s_memtime() - tr0;
      }
      if (lane == j) my_mode = mode;
      n_l += mode == kModeL;
      n_r += mode == kModeR;
    }
    if (live) {
      cr.x[c] = my_x;
      cr.mode[c] = (uint8_t)my_mode;
      if (my_mode == kModeL || my_mode == kModeU) {
        cr.hq[c] = my_hq;
        cr.hmax[c] = my_hmax;
        cr.harg[c] = my_harg;
      }
    }
    if (dbg && tile_done) t_fast += (long long)__builtin_amdgcn_s_memtime() - tt0;
    cur = nxt;
    cb = ce;
  }
  if (lane == 0 && replays) atomicAdd(nreplay, replays);
  if (lane == 0 && c1 < g.nch && g.run[c1] == g.run[c1 - 1] &&
      __double_as_longlong(x) != __double_as_longlong(o.cexit[c1 - 1]))
    atomicOr(err, 16u);  // the next segment assumed a different entry
  if (dbg && lane == 0) {  // accumulated per block (several segments per window)
    dbg[9 * r + 0] += (long long)__builtin_amdgcn_s_memtime() - t_start;
    dbg[9 * r + 1] += c1 - c0;
    dbg[9 * r + 2] += (long long)replays;
    dbg[9 * r + 3] += 1;
    dbg[9 * r + 4] += n_l;
    dbg[9 * r + 5] += n_r;
    dbg[9 * r + 6] += t_fast;
    dbg[9 * r + 7] += t_rep;
    dbg[9 * r + 8] += n_par;
  }
}

// Exact carry (tables of small integers, ks_table::int_exact): every partial
// sum is exact in FP64, so the max-plus prescan xt (k_ascan_*) is the exact
// entry of every chunk -- max(x + sum, clean exit) composes exactly -- and a
// chunk's carried head follows from its pass-1 aggregates: entered at 0, the
// clean trajectory; no clamp (x + prefix min > 0), the trajectory x + prefix
// with its maximum x + pmax first reached at parg (mode L); else mode R (the
// head up to the clamp: k_heads).  Replaces the predictor, the binade
// summaries and the replays.
__global__ void __launch_bounds__(256) k_carry_exact(Chunks g, P1 o, const double *__restrict__ xt, Carry cr) {
  const int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.nch) return;
  const double x = xt[c];
  cr.x[c] = x;
  if (x == 0.0) {
    cr.mode[c] = (uint8_t)kModeClean;
  } else if (x + o.pmin[c] > 0.0) {
    cr.mode[c] = (uint8_t)kModeL;
    cr.hq[c] = -1;
    cr.hmax[c] = x + o.pmax[c];
    cr.harg[c] = o.parg[c];
  } else {
    cr.mode[c] = (uint8_t)kModeR;
  }
}

// Tile composites (TileComp) of the global tiles of chunks [g.c0, g.nch):
// one wave per tile, from the final summaries (after k_summ_fixw).  Also
// clears the batch marks (ee) of the range.
__global__ void __launch_bounds__(256) k_tile_comp(Chunks g, Summ sm, TileComp tc) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (g.c0 >> 6) + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (g.nch <= g.c0 || t > ((g.nch - 1) >> 6)) return;  // whole waves
  const int64_t c = 64 * t + lane;
  const bool live = c >= g.c0 && c < g.nch;
  const int se = live ? sm.e[c] : INT32_MIN;
  const int e = __builtin_amdgcn_readfirstlane(se);
  if (lane == 0) tc.ee[t] = INT32_MIN;
  if (e == INT32_MIN || !__all(live && se == e)) {
    if (lane == 0) tc.e[t] = INT32_MIN;
    return;
  }
  const SummAt r = summ_at(sm, c);
  const long long D0 = r.D[r.i0], D1 = r.D[r.i1];
  const long long M0 = r.M[r.i0], M1 = r.M[r.i1];
  const long long N0 = r.N[r.i0], N1 = r.N[r.i1];
  const PPair ip = pp_scan_incl(PPair{D0, D1});
  const PPair xp = pp_prev(ip);
  const long long i0 = ip.d0, i1 = ip.d1, x0 = xp.d0, x1 = xp.d1;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    // entry mantissa m (parity p): chunk lane enters at m + inc with parity pj
    // and stays in the binade iff m + inc + N_pj >= 2^52 + 1 and
    // m + inc + M_pj <= 2^53 - 2 (carry_segment's fast-tile test)
    const long long inc = p ? x1 : x0;
    const int pj = (int)((p + inc) & 1);
    long long lo = (1LL << 52) + 1 - inc - (pj ? N1 : N0);
    long long hi = (1LL << 53) - 2 - inc - (pj ? M1 : M0);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      lo = max(lo, (long long)__shfl_xor(lo, d, 64));
      hi = min(hi, (long long)__shfl_xor(hi, d, 64));
    }
    const long long tot = __shfl(p ? i1 : i0, 63, 64);
    if (lane == 0) {
      tc.D[2 * t + p] = tot;
      tc.LO[2 * t + p] = lo;
      tc.HI[2 * t + p] = hi;
    }
  }
  if (lane == 0) tc.e[t] = e;
}

// Per-chunk carry of the tiles accepted in batches (ee != INT32_MIN): the
// fast-tile path of carry_segment from the tile's exact entry.  gated: only
// after a fallback (bit 16 of err), for the tiles k_carry_run batched.
__global__ void __launch_bounds__(256) k_tile_apply(Chunks g, Summ sm, TileComp tc, Carry cr,
                                                    const unsigned int *__restrict__ err, int gated) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (g.c0 >> 6) + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  if (g.nch <= g.c0 || t > ((g.nch - 1) >> 6)) return;
  if (gated && !(*(volatile const unsigned int *)err & 16u)) return;
  const int e = tc.ee[t];
  if (e == INT32_MIN) return;
  const long long m = tc.em[t];
  const int64_t c = 64 * t + lane;
  const bool live = c < g.nch;
  const int64_t cc = live ? c : 64 * t;
  const SummAt r = summ_at(sm, cc);
  const long long D0 = r.D[r.i0], D1 = r.D[r.i1];
  const PPair xp = pp_prev(pp_scan_incl(PPair{live ? D0 : 0, live ? D1 : 0}));
  const long long x0 = xp.d0, x1 = xp.d1;
  if (!live) return;
  const long long mj = m + ((m & 1) ? x1 : x0);
  const int pj = (int)(mj & 1);
  cr.x[c] = from_mant(mj, e);
  cr.mode[c] = (uint8_t)kModeL;
  cr.hq[c] = -1;
  cr.hmax[c] = from_mant(mj + r.M[pj ? r.i1 : r.i0], e);
  cr.harg[c] = r.A[pj ? r.i1 : r.i0];
}

// Carry by window: block w runs the segments that start in chunks
// [64w, 64w + 64) (segment starts flagged by k_seg_marks; a segment ends at
// the next flagged chunk, possibly windows later).
// kW: waves per SIMD the register allocation must allow (3: the FP64 form
// fits 168 VGPRs without spills instead of taking 170 at 2 waves; weighted
// rank in-process k = 13 30.4 vs 31.6 ms, k = 15 53.6 vs 55.1, metric
// unchanged: profiles/r5/ab/ab_carry_occ*.txt; 4 waves spill 64-87 VGPRs)
template <bool kCompressed, int kW = 3>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kW, 8))) k_carry_win(Chunks g, const uint8_t *__restrict__ flag,
                                                  const uint8_t *__restrict__ seq, int64_t total, int k, TableView tv,
                                                  const uint16_t *__restrict__ codes, P1 o, Summ sm, Carry cr,
                                                  TileComp tc, ReplayBuf rp, unsigned long long *__restrict__ nreplay,
                                                  unsigned int *__restrict__ err, long long *__restrict__ dbg) {
  // a wave per window: segment starts in [c0, nch); segments end by nch
  const int64_t w = g.c0 / 64 + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g.nch <= 0 || w > (g.nch - 1) / 64) return;
  const int lane = threadIdx.x & 63;
  const int64_t base = w * 64;
  unsigned long long m = __ballot(base + lane >= g.c0 && base + lane < g.nch && flag[base + lane]);
  while (m) {
    const int b = __ffsll((long long)m) - 1;
    m &= m - 1;
    const int64_t c0 = base + b;
    int64_t c1 = g.nch;
    if (m) {
      c1 = base + __ffsll((long long)m) - 1;
    } else {
      for (int64_t nb = base + 64; nb < g.nch; nb += 64) {
        const unsigned long long mm = __ballot(nb + lane < g.nch && flag[nb + lane]);
        if (mm) {
          c1 = nb + __ffsll((long long)mm) - 1;
          break;
        }
      }
    }
    carry_segment<kCompressed>(g, c0, c1, seq, total, k, tv, codes, o, sm, cr, tc, rp, nreplay, err, dbg, w);
  }
}

// Carry by run (the fallback when a segment assumption failed): gated on
// bit 16 of err, so it can be queued unconditionally.
template <bool kCompressed>
__global__ void __launch_bounds__(64) k_carry_run(Chunks g, const int64_t *__restrict__ cbase, int64_t nruns,
                                                  const uint8_t *__restrict__ seq, int64_t total, int k, TableView tv,
                                                  const uint16_t *__restrict__ codes, P1 o, Summ sm, Carry cr,
                                                  TileComp tc, ReplayBuf rp, unsigned long long *__restrict__ nreplay,
                                                  unsigned int *__restrict__ err, long long *__restrict__ dbg,
                                                  int64_t r_lo) {
  const int64_t r = r_lo + blockIdx.x;
  if (r >= nruns || !(*(volatile unsigned int *)err & 16u)) return;
  const int64_t c0 = cbase[r], c1 = cbase[r + 1];
  if (c0 < c1) carry_segment<kCompressed>(g, c0, c1, seq, total, k, tv, codes, o, sm, cr, tc, rp, nreplay, err, nullptr, r);
}

// Fallback preparation: after a failed segment check, the first heads pass
// may have flagged clamps against the wrong carry; clear everything but 16.
__global__ void k_fallback_prep(unsigned int *__restrict__ err, unsigned long long *__restrict__ nreplay,
                                int force) {
  if (force) *err |= 16u;
  if (*err & 16u) {
    *err = 16u;
    *nreplay = 0;
  }
}


// ------------------------------------------------------------------- P4

// Heads of the R chunks (the carried excursion up to its certain clamp):
// lane per chunk, from the exact entry.  Uncompressed tables read the
// expanded table (J indices per read) like P1.
template <int J, bool kCompressed, bool kWide = false>
__device__ __forceinline__ void head_walk(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                          const TableView &tv, const uint16_t *__restrict__ codes, const Carry &cr,
                                          unsigned int *__restrict__ err, int64_t c) {
  const uint32_t *__restrict__ packed = g.packed;
  const double x = cr.x[c];
  const int n = g.n[c];
  const int64_t start = g.start[c];
  double T = x, hmax = -1.0;
  int harg = 0, hq = -1;
  if (kCompressed) {
    for (int b0 = 0; b0 < n && hq < 0; b0 += NB) {
      double v[NB];
      if (!codes) {
        values16_nostore(g, seq, total, k, tv, c, b0, n, v, nullptr);
      } else {
        uint32_t w[8];
        load_codes16(codes, c, b0, w);
#pragma unroll
        for (int j = 0; j < NB; ++j) v[j] = tv.lut[(w[j >> 1] >> (16 * (j & 1))) & 0xffffu];
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int i = b0 + j;
        if (i < n && hq < 0) {
          const double t = T + v[j];
          T = t > 0 ? t : 0.0;
          if (T == 0.0) hq = i;
          else if (T > hmax) { hmax = T; harg = i; }
        }
      }
    }
  } else if (tv.line) {  // FP64 line table: OWN + 1 indices per read
    const uint32_t mask = (1u << (2 * k)) - 1u;
    uint64_t xp = 0;
    uint32_t code = packed_bits(packed, total, start - k, xp) ? (uint32_t)(xp >> (64 - 2 * k))
                                                              : prime_code_guarded(seq, start - k, k, total);
    // (kWide: two batches' reads in flight per round trip; FP64 line tables)
    constexpr int NW = kWide ? 2 * NB : NB;
    for (int b0 = 0; b0 < n && hq < 0; b0 += NW) {
      double v[NW];
      values16_f64(g, seq, total, k, tv, start, b0, n, code, mask, v);
      if (kWide) values16_f64(g, seq, total, k, tv, start, b0 + NB, n, code, mask, v + NB);
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const int i = b0 + j;
        if (i < n && hq < 0) {
          const double t = T + v[j];
          T = t > 0 ? t : 0.0;
          if (T == 0.0) hq = i;
          else if (T > hmax) { hmax = T; harg = i; }
        }
      }
    }
  } else {
    constexpr int G = (J == 1) ? 16 : (J == 4 ? 4 : 8);
    constexpr int PB = G * J;
    const int kx = k + J - 1;
    const uint32_t xmask = (kx >= 16) ? 0xffffffffu : ((1u << (2 * kx)) - 1u);
    // prime and the first batch's bases from the packed codes: one round trip
    uint64_t xp = 0;
    uint32_t gcode = packed_bits(packed, total, start - k, xp) ? (uint32_t)(xp >> (64 - 2 * kx))
                                                               : prime_code_guarded(seq, start - k, kx, total);
    for (int b0 = 0; b0 < n && hq < 0; b0 += PB) {
      uint32_t gc[G];
      uint64_t xb = 0;
      if (2 * PB <= 64 && packed_bits(packed, total, start + b0 + J - 1, xb)) {
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
          gc[gi] = gcode;
          gcode = ((gcode << (2 * J)) | (uint32_t)((xb >> (64 - 2 * J * (gi + 1))) & ((1u << (2 * J)) - 1u))) & xmask;
        }
      } else {
        uint8_t by[32];
        load16(seq, start + b0 + J - 1, total, by);
        if (PB > 16) load16(seq, start + b0 + J - 1 + 16, total, by + 16);
#pragma unroll
        for (int gi = 0; gi < G; ++gi) {
          gc[gi] = gcode;
#pragma unroll
          for (int t = 0; t < J; ++t) gcode = ((gcode << 2) | enc(by[gi * J + t])) & xmask;
        }
      }
      double v[PB];
#pragma unroll
      for (int gi = 0; gi < G; ++gi) {
        const bool live = b0 + gi * J < n;
        if (J == 1) {
          v[gi] = live ? tv.vals[gc[gi]] : 0.0;
        } else {
          double2 e0 = make_double2(0.0, 0.0), e1 = e0;
          if (live) {
            const double2 *E = reinterpret_cast<const double2 *>(tv.ext);
            if (J <= 2) {
              e0 = E[gc[gi]];
            } else {
              e0 = E[2 * (size_t)gc[gi]];
              e1 = E[2 * (size_t)gc[gi] + 1];
            }
          }
          const double ev[4] = {e0.x, e0.y, e1.x, e1.y};
#pragma unroll
          for (int t = 0; t < J; ++t) v[gi * J + t] = ev[t];
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int i = b0 + j;
        if (i < n && hq < 0) {
          const double t = T + v[j];
          T = t > 0 ? t : 0.0;
          if (T == 0.0) hq = i;
          else if (T > hmax) { hmax = T; harg = i; }
        }
      }
    }
  }
  if (hq < 0) atomicOr(err, 2u);  // predicted clamp did not happen
  cr.hq[c] = hq;
  cr.hmax[c] = hmax;
  cr.harg[c] = harg;
}

template <int J, bool kCompressed, bool kWide = false>
__device__ __forceinline__ void head_one(const Chunks &g, const uint8_t *__restrict__ seq, int64_t total, int k,
                                         const TableView &tv, const uint16_t *__restrict__ codes, const Carry &cr,
                                         unsigned int *__restrict__ err, int64_t c) {
  const int mode = cr.mode[c];
  if (mode == kModeL || mode == kModeU) return;  // head written by the carry (summary / replay)
  cr.hq[c] = -1;
  cr.hmax[c] = -1.0;
  cr.harg[c] = 0;
  if (mode == kModeClean) return;
  head_walk<J, kCompressed, kWide>(g, seq, total, k, tv, codes, cr, err, c);
}

// gated: the second pass, after a fallback only (bit 16 of err); queued
// unconditionally on a small grid (a grid-stride loop), so that the common
// case costs one short launch instead of a block per 256 chunks (80 us of
// empty blocks at the metric genome's second part)
template <int J, bool kCompressed, bool kWide = false>
__global__ void __launch_bounds__(256) k_heads(Chunks g, const uint8_t *__restrict__ seq, int64_t total,
                                               int k, TableView tv, const uint16_t *__restrict__ codes,
                                               Carry cr, unsigned int *__restrict__ err, int gated) {
  if (gated && !(*(volatile unsigned int *)err & 16u)) return;  // second pass only after a fallback
  for (int64_t c = g.c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < g.nch;
       c += (int64_t)gridDim.x * blockDim.x)
    head_one<J, kCompressed, kWide>(g, seq, total, k, tv, codes, cr, err, c);
}

// k_heads with the R chunks packed densely: a wave takes 256 chunks, lists
// its R chunks in LDS (ballot order) and walks them 64 at a time, so every
// lane of a walking wave has a head to walk (weighted rank: ~28% of the
// chunks are R, scattered; config 3 in-process 29.18 vs 29.90 ms, k = 15
// 43.7 vs 43.8: profiles/r5/ab/ab_heads_dense_lane_pf_*.txt, where the next
// rescan batch's bases loaded one batch ahead measured slower, 29.18 vs 28.51).
constexpr int kHeadSpan = 256;
template <int J, bool kCompressed, bool kWide = false>
__global__ void __launch_bounds__(256) k_heads_dense(Chunks g, const uint8_t *__restrict__ seq, int64_t total,
                                                     int k, TableView tv, const uint16_t *__restrict__ codes,
                                                     Carry cr, unsigned int *__restrict__ err, int gated) {
  if (gated && !(*(volatile unsigned int *)err & 16u)) return;
  __shared__ int32_t s_list[4][kHeadSpan];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t sp = g.c0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * kHeadSpan; sp < g.nch;
       sp += nw * kHeadSpan) {
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < kHeadSpan / 64; ++q) {
      const int64_t c = sp + q * 64 + lane;
      bool isr = false;
      if (c < g.nch) {
        const int mode = cr.mode[c];
        if (mode == kModeClean || mode == kModeR) {
          cr.hq[c] = -1;
          cr.hmax[c] = -1.0;
          cr.harg[c] = 0;
        }
        isr = mode == kModeR;
      }
      const unsigned long long b = __ballot(isr);
      if (isr) s_list[w][cnt + __popcll(b & ((1ull << lane) - 1ull))] = q * 64 + lane;
      cnt += __popcll(b);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = lane; t < cnt; t += 64)
      head_walk<J, kCompressed, kWide>(g, seq, total, k, tv, codes, cr, err, sp + s_list[w][t]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ------------------------------------------------------------------- P5

// One lane's emission (sporadic callers).
__device__ __forceinline__ void emit(const Emission &e, const RegionBuf &rb, const Rescan &rs, int32_t sid,
                                     double best) {
  if (e.reg) push_region(rb, sid, e.rbeg, e.rend, best);
  if (e.res) {
    const int64_t slot = append_one(rs.count, rs.segcap);
    if (slot >= 0) {
      rs.a[slot] = e.res_a;
      rs.b[slot] = e.res_b;
      rs.seq[slot] = sid;
    }
  }
}

// emit() for a whole wave (every lane calls it): one atomic per wave and
// buffer segment instead of one per record.
__device__ __forceinline__ void emit_wave(const Emission &e, const RegionBuf &rb, const Rescan &rs, int32_t sid,
                                          double best) {
  const unsigned long long m = __ballot(e.reg);
  const unsigned long long mr = __ballot(e.res);
  if ((m | mr) == 0) return;
  const int lane = (int)(threadIdx.x & 63);
  const int leader = __ffsll((long long)(m | mr)) - 1;
  const int sg = append_seg();
  unsigned long long base = 0, rbase = 0;
  if (lane == leader) {
    if (m) base = atomicAdd(&rb.count[sg], (unsigned long long)__popcll(m));
    if (mr) rbase = atomicAdd(&rs.count[sg], (unsigned long long)__popcll(mr));
  }
  base = __shfl(base, leader, 64);
  rbase = __shfl(rbase, leader, 64);
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (e.reg) {
    const unsigned long long i = base + (unsigned long long)__popcll(m & below);
    if ((int64_t)i < rb.segcap) {
      const int64_t slot = (int64_t)sg * rb.segcap + (int64_t)i;
      rb.seq[slot] = sid;
      rb.beg[slot] = e.rbeg;
      rb.end[slot] = e.rend;
      rb.score[slot] = best;
    }
  }
  if (e.res) {
    const unsigned long long i = rbase + (unsigned long long)__popcll(mr & below);
    if ((int64_t)i < rs.segcap) {
      const int64_t slot = (int64_t)sg * rs.segcap + (int64_t)i;
      rs.a[slot] = e.res_a;
      rs.b[slot] = e.res_b;
      rs.seq[slot] = sid;
    }
  }
}

// Stitch as a segmented scan, one wave per run.  Chunk c acts on the open
// excursion state by one of: RESET(tail or none) -- an excursion closes in the
// chunk and/or its clean tail opens a new one -- or EXTEND(head) -- the carried
// excursion takes the chunk's head maximum (first argmax: a later head wins
// only when strictly greater).  The operator is associative, so 64 chunks are
// combined per step with shuffles; the chunk that closes an excursion emits it.
struct XState {
  int reset;  // 1: RESET to (open, xb, xm, xa); 0: EXTEND by (xm, xa)
  int open;
  long long xb, xa;
  double xm;
};

__device__ __forceinline__ XState x_compose(const XState &f1, const XState &f2) {  // f1 then f2
  if (f2.reset) return f2;
  XState r = f1;
  if (f2.xm > f1.xm) { r.xm = f2.xm; r.xa = f2.xa; }
  return r;
}

__device__ __forceinline__ XState x_shfl(const XState &a, int l) {
  XState r;
  r.reset = __shfl(a.reset, l, 64);
  r.open = __shfl(a.open, l, 64);
  r.xb = __shfl(a.xb, l, 64);
  r.xa = __shfl(a.xa, l, 64);
  r.xm = __shfl(a.xm, l, 64);
  return r;
}

// First scan index at which a candidate or tail of the chunk is valid: after
// the carried head's clamp, or nowhere when the carried excursion spans it.
__device__ __forceinline__ int64_t valid_from(int mode, int hq, int64_t st, int64_t en) {
  if (mode == kModeClean) return st;
  return hq >= 0 ? st + hq + 1 : en;
}

// The operator of chunk c on the open-excursion state, plus what the chunk
// needs to emit a closing excursion.
struct ChunkOp {
  XState f;
  bool closes;
  int64_t close_pos;
  double hmax;
  int64_t harg;
  int mode;
};

__device__ __forceinline__ ChunkOp chunk_op(const Chunks &g, const P1 &o, const Carry &cr, int64_t c) {
  ChunkOp r;
  r.f = XState{0, 0, 0, 0, -INFINITY};  // identity
  r.closes = false;
  r.close_pos = 0;
  r.hmax = -INFINITY;
  r.harg = 0;
  const int64_t st = g.start[c];
  const int64_t en = st + g.n[c];
  const int mode = cr.mode[c];
  const int hq = cr.hq[c];
  const int tb = o.tbeg[c];
  r.mode = mode;
  const int64_t vf = valid_from(mode, hq, st, en);
  if (mode != kModeClean && hq != 0) { r.hmax = cr.hmax[c]; r.harg = st + cr.harg[c]; }
  r.closes = mode != kModeClean && hq >= 0;
  r.close_pos = st + hq;
  const bool opens = tb >= 0 && st + tb >= vf && !(mode != kModeClean && hq < 0);
  if (opens) {
    r.f = XState{1, 1, st + tb, st + o.targ[c], o.tmax[c]};
  } else if (r.closes) {
    r.f = XState{1, 0, 0, 0, -1.0};
  } else if (mode != kModeClean) {
    r.f = XState{0, 0, 0, r.harg, r.hmax};
  }
  return r;
}

// DPP move of a state; lanes without a source read the identity (EXTEND by
// nothing: xm = -inf)
template <int CTRL, int RM>
__device__ __forceinline__ XState dpp_x(const XState &a) {
  return XState{dpp_i32<CTRL, RM>(a.reset), dpp_i32<CTRL, RM>(a.open), dpp_i64<CTRL, RM>(a.xb),
                dpp_i64<CTRL, RM>(a.xa), dpp_f64_or<CTRL, RM>(a.xm, -INFINITY)};
}

__device__ __forceinline__ XState wave_inclusive(XState inc, int lane) {
  KS_DPP_SCAN(XState, inc, dpp_x, x_compose);
  (void)lane;
  return inc;
}

// Tile t (64 chunks of one run, aligned to the run's first chunk) -> run id
// and first chunk.

// Stitch as a three-phase segmented scan (tile aggregates in parallel, a
// short per-run scan of the aggregates, then every tile again with its
// carry-in).  Chunk c acts on the open excursion state by one of:
// RESET(tail or none) -- an excursion closes in the chunk and/or its clean
// tail opens a new one -- or EXTEND(head) -- the carried excursion takes the
// chunk's head maximum (first argmax: a later head wins only when strictly
// greater).  The operator is associative; the chunk that closes an excursion
// emits it.
struct XTiles {
  int32_t *reset, *open;
  long long *xb, *xa;
  double *xm;
};

__device__ __forceinline__ void xt_store(const XTiles &a, int64_t t, const XState &v) {
  a.reset[t] = v.reset; a.open[t] = v.open; a.xb[t] = v.xb; a.xa[t] = v.xa; a.xm[t] = v.xm;
}
__device__ __forceinline__ XState xt_load(const XTiles &a, int64_t t) {
  return XState{a.reset[t], a.open[t], a.xb[t], a.xa[t], a.xm[t]};
}

__global__ void __launch_bounds__(256) k_stitch_tiles(Chunks g, const int64_t *__restrict__ tbase,
                                                     const int64_t *__restrict__ cbase, int64_t nruns, const int32_t *__restrict__ trun, P1 o,
                                                     Carry cr, XTiles agg, int64_t t_lo, int64_t t_hi) {
  const int64_t t = t_lo + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // wave per tile
  if (t >= t_hi) return;
  const int lane = threadIdx.x & 63;
  int64_t r, c0, c1;
  tile_of(tbase, cbase, trun, t, r, c0, c1, nruns);
  const int64_t c = c0 + lane;
  XState f{0, 0, 0, 0, -INFINITY};
  if (c < c1) f = chunk_op(g, o, cr, c).f;
  const XState inc = wave_inclusive(f, lane);
  if (lane == 63) xt_store(agg, t, inc);
}

// Per run: exclusive scan of its tile aggregates (64 tiles per step) -> the
// state entering each tile; the excursion still open at the run end is
// emitted here.
__global__ void __launch_bounds__(64) k_stitch_runs(const int64_t *__restrict__ tbase, int64_t nruns,
                                                    const int64_t *__restrict__ ra, const int64_t *__restrict__ rb_end,
                                                    const int32_t *__restrict__ rseq, EmitCfg ec, XTiles agg,
                                                    XTiles tin, RegionBuf out, Rescan rs, int64_t r_lo) {
  const int64_t r = r_lo + blockIdx.x;  // runs [r_lo, nruns)
  if (r >= nruns) return;
  const int lane = threadIdx.x;
  const int64_t t0 = tbase[r], t1 = tbase[r + 1];
  if (t0 == t1) return;
  XState carry{1, 0, 0, 0, -1.0};  // closed
  for (int64_t tb = t0; tb < t1; tb += 64) {
    const int64_t t = tb + lane;
    XState f{0, 0, 0, 0, -INFINITY};
    if (t < t1) f = xt_load(agg, t);
    const XState inc = wave_inclusive(f, lane);
    const XState exc = dpp_x<kDppWaveShr1, 0xf>(inc);  // (lane 0: the identity)
    if (t < t1) xt_store(tin, t, x_compose(carry, exc));
    carry = x_compose(carry, x_shfl(inc, 63));
  }
  if (lane == 0 && carry.open) {  // excursion open at the run end
    const int64_t last = rb_end[r] - 1 + ec.trlr;  // last scan index of the run
    emit(decide(ec, ra[r] + ec.k, carry.xb, carry.xa, carry.xm, last, false), out, rs, rseq[r], carry.xm);
  }
}

__global__ void __launch_bounds__(256) k_stitch_emit(Chunks g, const int64_t *__restrict__ tbase,
                                                    const int64_t *__restrict__ cbase, int64_t nruns, const int32_t *__restrict__ trun,
                                                    const int64_t *__restrict__ ra, const int32_t *__restrict__ rseq,
                                                    P1 o, Carry cr, EmitCfg ec, XTiles tin, RegionBuf out,
                                                    Rescan rs, unsigned int *__restrict__ err, int64_t t_lo,
                                                    int64_t t_hi) {
  const int64_t t = t_lo + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // wave per tile
  if (t >= t_hi) return;
  const int lane = threadIdx.x & 63;
  int64_t r, c0, c1;
  tile_of(tbase, cbase, trun, t, r, c0, c1, nruns);
  const int64_t c = c0 + lane;
  const bool live = c < c1;
  ChunkOp op;
  op.f = XState{0, 0, 0, 0, -INFINITY};
  op.closes = false;
  if (live) {
    op = chunk_op(g, o, cr, c);
    if (o.ep[c] != o.epoch) atomicOr(err, 32u);  // pass-1 results of another call
  }
  const XState inc = wave_inclusive(op.f, lane);
  const XState exc = dpp_x<kDppWaveShr1, 0xf>(inc);  // (lane 0: the identity)
  const XState in = x_compose(xt_load(tin, t), exc);  // state entering chunk c
  double xm = in.xm;
  long long xa = in.xa;
  Emission e{false, false, 0, 0, 0, 0};
  if (live && op.closes) {
    if (!in.open) {
      atomicOr(err, 4u);
    } else {
      if (op.hmax > xm) { xm = op.hmax; xa = op.harg; }
      e = decide(ec, ra[r] + ec.k, in.xb, xa, xm, op.close_pos, true);
    }
  }
  emit_wave(e, out, rs, rseq[r], xm);
  if (live && !op.closes && op.f.reset == 0 && op.mode != kModeClean && !in.open) atomicOr(err, 8u);
}

// Candidates (closed emittable excursions of the clean trajectories) are
// valid when they begin at or after their chunk's valid_from.
__global__ void k_candidates(Chunks g, const int64_t *__restrict__ ra, const int64_t *__restrict__ cbase,
                             int64_t nruns, const int32_t *__restrict__ rseq, EmitCfg ec, Cand cand,
                             Carry cr, RegionBuf out, Rescan rs) {
  const int k = ec.k;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool want = false;
  int64_t b = 0, arg = 0, rst = 0, f = 0;
  double best = 0.0;
  int32_t sid = 0;
  if (i < cand.cap && (i % cand.segcap) < (int64_t)cand.count[i / cand.segcap]) {
    b = cand.beg[i];
    int64_t lo = 0, hi = nruns - 1;  // last run with ra <= b
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (ra[mid] <= b) lo = mid; else hi = mid - 1;
    }
    const int64_t c = cbase[lo] + (b - (ra[lo] + k)) / CH;
    const int64_t st = g.start[c];
    want = b >= valid_from(cr.mode[c], cr.hq[c], st, st + g.n[c]);
    sid = rseq[lo];
    arg = cand.arg[i];
    best = cand.best[i];
    rst = cand.rst[i];
    f = ra[lo] + k;
  }
  Emission e{false, false, 0, 0, 0, 0};
  if (want) e = decide(ec, f, b, arg, best, rst, true);
  emit_wave(e, out, rs, sid, best);
}

}  // namespace

// KS_DEBUG_VERIFY=1 (diagnostics): after a chunked scan of a small input
// (<= 64 Mi bases, k <= 11, kmer_regions mode), the device's packed codes,
// chunk layout, pass-1 results and carry modes are copied back and checked
// against a host recomputation from the sequence bytes and the base table;
// every mismatch goes to stderr with its chunk and both values.  Reads the
// buffers after the call's last kernel, so a value that is right here but was
// wrong when a kernel read it points at an ordering edge, one that is wrong
// here at the kernel that wrote it.
static void debug_verify(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, const TableView &tv,
                         const Chunks &g, const P1 &p1, const Carry &cr, bool exact, int trlr) {
  const int64_t nch = g.nch;
  if (trlr || k > 11 || total > ((int64_t)64 << 20) || nch <= 0) return;
  (void)hipDeviceSynchronize();
  auto get = [&](auto *dst, const void *src, size_t n) {
    if (n) (void)hipMemcpy(dst, src, n * sizeof(*dst), hipMemcpyDeviceToHost);
  };
  std::vector<uint8_t> seq((size_t)total);
  get(seq.data(), s->seq, (size_t)total);
  const int64_t nk = (int64_t)1 << (2 * k);
  std::vector<double> val((size_t)nk);
  if (tv.compressed) {
    std::vector<uint16_t> codes((size_t)nk);
    get(codes.data(), tv.codes, (size_t)nk);
    std::vector<double> lut((size_t)std::max(tv.nlut, 1));
    get(lut.data(), tv.lut, (size_t)tv.nlut);
    for (int64_t i = 0; i < nk; ++i) val[i] = lut[codes[i]];
  } else {
    get(val.data(), tv.vals, (size_t)nk);
  }
  long long bad = 0;
  auto report = [&](const char *what, int64_t c, double got, double want) {
    if (++bad <= 12)
      fprintf(stderr, "[verify] chunk %lld of %lld: %s = %.17g, host %.17g\n", (long long)c, (long long)nch, what, got,
              want);
  };
  std::vector<int64_t> start((size_t)nch);
  std::vector<int32_t> n((size_t)nch), run((size_t)nch), tbeg((size_t)nch), targ((size_t)nch);
  std::vector<double> cexit((size_t)nch), tmax((size_t)nch), cx((size_t)nch);
  std::vector<uint8_t> mode((size_t)nch);
  get(start.data(), g.start, (size_t)nch);
  get(n.data(), g.n, (size_t)nch);
  if (g.packed) {  // the words the chunks read (a part's run pass packs its own range only)
    const int64_t nw = total / 16 + 1;
    std::vector<uint32_t> pk((size_t)nw);
    std::vector<uint8_t> used((size_t)nw, 0);
    for (int64_t c = 0; c < nch; ++c)
      for (int64_t w = std::max<int64_t>(0, (start[c] - k) / 16); w <= (start[c] + n[c]) / 16 && w < nw; ++w) used[w] = 1;
    get(pk.data(), g.packed, (size_t)nw);
    for (int64_t w = 0; w < nw; ++w) {
      uint32_t want = 0;
      for (int q = 0; q < 16; ++q) want |= enc(16 * w + q < total ? seq[16 * w + q] : (uint8_t)'N') << (30 - 2 * q);
      if (used[w] && pk[w] != want && 16 * w + 16 <= total) report("packed word", w, (double)pk[w], (double)want);
    }
  }
  get(run.data(), g.run, (size_t)nch);
  get(tbeg.data(), p1.tbeg, (size_t)nch);
  get(targ.data(), p1.targ, (size_t)nch);
  get(cexit.data(), p1.cexit, (size_t)nch);
  get(tmax.data(), p1.tmax, (size_t)nch);
  get(cx.data(), cr.x, (size_t)nch);
  get(mode.data(), cr.mode, (size_t)nch);
  const uint64_t kmask = (uint64_t)nk - 1;
  for (int64_t c = 0; c < nch; ++c) {
    // clean trajectory from 0 over indices start .. start + n - 1 (k-mer
    // ending at index - 1), as P1Lane::step
    double prev = 0.0, best = 0.0;
    int beg = -1, arg = 0;
    for (int i = 0; i < n[c]; ++i) {
      const int64_t p = start[c] + i;
      uint64_t code = 0;
      for (int64_t q = p - k; q < p; ++q) code = ((code << 2) | enc(seq[q])) & kmask;
      const double sv = val[code];
      const double tt = prev + sv;
      const double S = tt > 0 ? tt : 0.0;
      const bool open = (prev == 0) & (S > 0), close = (prev > 0) & (S == 0);
      const bool up = open | (S > best);
      best = up ? S : best;
      arg = up ? i : arg;
      beg = open ? i : (close ? -1 : beg);
      prev = S;
    }
    auto ne = [](double a, double b) { return memcmp(&a, &b, 8) != 0; };
    if (ne(cexit[c], prev)) report("clean exit", c, cexit[c], prev);
    if (prev > 0) {
      if (tbeg[c] != beg) report("tail begin", c, tbeg[c], beg);
      if (targ[c] != arg) report("tail argmax", c, targ[c], arg);
      if (ne(tmax[c], best)) report("tail max", c, tmax[c], best);
    } else if (tbeg[c] != -1) {
      report("tail begin (none)", c, tbeg[c], -1);
    }
    const bool first = c == 0 || run[c - 1] != run[c];
    if (first && (mode[c] != kModeClean || cx[c] != 0.0)) report("run-first chunk carry mode", c, mode[c], kModeClean);
  }
  (void)exact;
  if (bad) fprintf(stderr, "[verify] %lld mismatches in %lld chunks (k %d, %lld bases)\n", bad, (long long)nch, k,
                   (long long)total);
}

ks_status scan_chunked(ks_ctx *ctx, const ks_dev_seqs *s, const Runs &runs, const RunLayout &lay, int k,
                       const TableView &tv, uint64_t mw, double min_score, uint32_t *visits,
                       uint32_t *visits_rescan, const RegionBuf &rb, ks_scan_stats *stats, const ScanMode &mode) {
  const EmitCfg ec{mode.trlr, mw, min_score, mode.min_len, mode.ks, k};
  hipStream_t st = ctx->stream;
  const int64_t total = s->offsets_host[s->nseq];
  const int64_t nruns = runs.n;
  const int64_t nch = lay.nch, ntiles = lay.ntiles;
  ctx->chunked_events = false;
  if (nruns == 0 || nch == 0) return KS_OK;
  const int64_t *d_cbase = lay.cbase, *d_tbase = lay.tbase;
  const bool comp = tv.compressed != 0;

  // ---- workspace
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const int64_t nwin = (nch + 63) / 64;
  size_t off = 0;
  const size_t o_start = off; off += al(nch * 8);
  const size_t o_n = off; off += al(nch * 4);
  const size_t o_run = off; off += al(nch * 4);
  const size_t o_p1d = off; off += al(nch * 8 * 6);
  const size_t o_p1i = off; off += al(nch * 4 * 3);
  const size_t o_spec = off; off += al(nch);
  const size_t o_ep = off; off += al(nch * 4);
  const size_t o_xt = off; off += al(nch * 8);
  const size_t o_se = off; off += al(nch * 4);
  const size_t o_sD = off; off += al(nch * 8 * 6);
  const size_t o_sA = off; off += al(nch * 4 * 2);
  const size_t o_x = off; off += al(nch * 8);
  const size_t o_mode = off; off += al(nch);
  const size_t o_hq = off; off += al(nch * 4 * 2);
  const size_t o_hmax = off; off += al(nch * 8);
  const size_t o_cnt = off; off += al(8 * (5 * kSegs + 8));  // + the region counters' copy, half 1's lists
  const size_t o_flag = off; off += al(nch + 64);
  const size_t o_xagg = off; off += al(ntiles * 32) * 2;
  // pass-1 summaries: predictor sums / exits / zero flags, predicted entries,
  // the summaries, the fix list
  const size_t o_pa = off; off += al(nch * 8);
  const size_t o_pb = off; off += al(nch * 8);
  const size_t o_pz = off; off += al(nch);
  const size_t o_xh = off; off += al(nch * 8);
  const size_t o_spe = off; off += al(nch * 4 * 2);
  const size_t o_spd = off; off += al(nch * 8 * 6);
  const size_t o_spa = off; off += al(nch * 4 * 2);
  const size_t o_fix = off; off += al(nch * 8 + 16);
  const size_t o_ssel = off; off += al(nch);  // Summ::sel
  const size_t o_tagg = off; off += al(ntiles * 16);  // parallel approximate scan: tile maps, tile entries
  const size_t o_tin = off; off += al(ntiles * 8);
  const size_t o_trun = off; off += al(ntiles * 4 + 4);  // stitch tile -> run (k_tile_runs)
  const int64_t ngt = nch / 64 + 2;  // global 64-chunk tiles (carry tile batches)
  const size_t o_gte = off; off += al(ngt * 4);
  const size_t o_gtd = off; off += al(ngt * 8 * 6);
  const size_t o_gtm = off; off += al(ngt * 8);
  const size_t o_gtee = off; off += al(ngt * 4);
  // likely-replay prefetch (k_marks_select lists, k_summ_fixw fills)
  const int64_t rcap_h = std::max<int64_t>(65536, nch / 128);  // slots per half
  const size_t o_rslot = off; off += al(nch * 4);
  const size_t o_rchunk = off; off += al(2 * rcap_h * 8);
  const size_t o_rcnt = off; off += al(64);
  const size_t o_rval = off; off += al(2 * rcap_h * 256 * 8);
  void *wsp = nullptr;
  KS_TRY(ensure(ctx, SLOT_CHUNK_A, off, &wsp));
  char *W = static_cast<char *>(wsp);
  Chunks g{reinterpret_cast<int64_t *>(W + o_start), reinterpret_cast<int32_t *>(W + o_n),
           reinterpret_cast<int32_t *>(W + o_run), nch, runs.packed};
  double *p1d = reinterpret_cast<double *>(W + o_p1d);
  int32_t *p1i = reinterpret_cast<int32_t *>(W + o_p1i);
  P1 p1{p1d, p1d + nch, p1d + 2 * nch, p1d + 3 * nch, p1d + 4 * nch, p1d + 5 * nch, p1i, p1i + nch,
        reinterpret_cast<uint8_t *>(W + o_spec), p1i + 2 * nch};
  p1.ep = reinterpret_cast<uint32_t *>(W + o_ep);
  p1.epoch = ++ctx->scan_epoch;
  double *xt = reinterpret_cast<double *>(W + o_xt);
  long long *sD = reinterpret_cast<long long *>(W + o_sD);
  Summ sm{reinterpret_cast<int32_t *>(W + o_se), sD, sD + 2 * nch, sD + 4 * nch,
          reinterpret_cast<int32_t *>(W + o_sA)};
  int32_t *hqp = reinterpret_cast<int32_t *>(W + o_hq);
  Carry cr{reinterpret_cast<double *>(W + o_x), reinterpret_cast<uint8_t *>(W + o_mode), hqp,
           reinterpret_cast<double *>(W + o_hmax), hqp + nch};
  unsigned long long *cnts = reinterpret_cast<unsigned long long *>(W + o_cnt);
  uint8_t *d_flag = reinterpret_cast<uint8_t *>(W + o_flag);
  auto xtiles = [&](char *p) {
    return XTiles{reinterpret_cast<int32_t *>(p), reinterpret_cast<int32_t *>(p) + ntiles,
                  reinterpret_cast<long long *>(p + ntiles * 8), reinterpret_cast<long long *>(p + ntiles * 16),
                  reinterpret_cast<double *>(p + ntiles * 24)};
  };
  const XTiles xagg = xtiles(W + o_xagg), xtin = xtiles(W + o_xagg + al(ntiles * 32));
  double2 *d_tagg = reinterpret_cast<double2 *>(W + o_tagg);
  int32_t *d_trun_map = reinterpret_cast<int32_t *>(W + o_trun);
  int32_t *d_trun = d_trun_map;
  long long *gtd = reinterpret_cast<long long *>(W + o_gtd);
  const TileComp tcomp{reinterpret_cast<int32_t *>(W + o_gte), gtd, gtd + 2 * ngt, gtd + 4 * ngt,
                       reinterpret_cast<long long *>(W + o_gtm), reinterpret_cast<int32_t *>(W + o_gtee)};
  ReplayBuf rpb{reinterpret_cast<int32_t *>(W + o_rslot), reinterpret_cast<int64_t *>(W + o_rchunk),
                reinterpret_cast<double *>(W + o_rval), reinterpret_cast<unsigned long long *>(W + o_rcnt), rcap_h};
  double *d_tin = reinterpret_cast<double *>(W + o_tin);
  // approximate max-plus scan of (sum, clean exit) over runs [r0, r1) (tiles
  // [t0, t1)): three parallel kernels (the one-wave-per-run k_approx_scan when
  // the range has no tile)
  // waves per block of the wave-per-tile / wave-per-window kernels (A/B: 2 of 1-4)
  constexpr int wpb = 2;
  auto ascan = [&](const P1 &o, double *out, int64_t r0, int64_t r1, int64_t t0, int64_t t1,
                   hipStream_t strm) -> ks_status {
    if (r1 <= r0) return KS_OK;
    if (t1 <= t0) {
      hipLaunchKernelGGL(k_approx_scan, dim3((unsigned)(r1 - r0)), dim3(64), 0, strm, d_cbase, r1, o, out, r0);
      KS_HIP(hipGetLastError());
      return KS_OK;
    }
    const unsigned g4 = (unsigned)((t1 - t0 + wpb - 1) / wpb);  // a wave per tile, wpb per block
    hipLaunchKernelGGL(k_ascan_tiles, dim3(g4), dim3(64 * wpb), 0, strm, d_tbase, d_cbase, nruns, d_trun, o, d_tagg, t0,
                       t1);
    hipLaunchKernelGGL(k_ascan_runs, dim3((unsigned)(r1 - r0)), dim3(64), 0, strm, d_tbase, r1, d_tagg, d_tin, r0);
    hipLaunchKernelGGL(k_ascan_apply, dim3(g4), dim3(64 * wpb), 0, strm, d_tbase, d_cbase, nruns, d_trun, o, d_tin, out,
                       t0, t1);
    KS_HIP(hipGetLastError());
    return KS_OK;
  };
  double *d_xh = reinterpret_cast<double *>(W + o_xh);
  long long *spd = reinterpret_cast<long long *>(W + o_spd);
  const SummP1 sp1{reinterpret_cast<int32_t *>(W + o_spe), spd, spd + 2 * nch, spd + 4 * nch,
                   reinterpret_cast<int32_t *>(W + o_spa)};
  unsigned long long *d_nfix = reinterpret_cast<unsigned long long *>(W + o_fix);  // [2]: one per half
  int64_t *d_fix = reinterpret_cast<int64_t *>(W + o_fix + 16);
  // cnts: [0, kSegs) candidate counters, [kSegs, 2 kSegs) rescan counters,
  // [2 kSegs + 2h] replays, [2 kSegs + 2h + 1] error bits (u32) of half h,
  // [2 kSegs + 8, 3 kSegs + 8) the region counters' copy, [3 kSegs + 8,
  // 5 kSegs + 8) the second half's candidate and rescan counters
  KS_HIP(hipMemsetAsync(cnts, 0, 8 * (2 * kSegs + 8), st));
  KS_HIP(hipMemsetAsync(cnts + 3 * kSegs + 8, 0, 8 * (2 * kSegs), st));
  unsigned long long *d_replays = cnts + 2 * kSegs;

  // Candidates and rescans in one list per half: the first half's are
  // emitted and rescanned while the second half is post-processed (a list
  // cannot be read while the other half's pass 1 still appends to it).
  int64_t ccap = std::max<int64_t>(1 << 16, nch / 4);  // per list
  const size_t cand_bytes = ctx->slots[SLOT_CHUNK_C].bytes;  // use what the grow-only slot holds
  if (cand_bytes > 2048 && (cand_bytes - 2048) / 80 > (size_t)ccap) ccap = (int64_t)((cand_bytes - 2048) / 80);
  const int64_t csegcap = ccap / kSegs;
  ccap = csegcap * kSegs;
  void *cbuf = nullptr;
  KS_TRY(ensure(ctx, SLOT_CHUNK_C, (size_t)ccap * 80 + 2048, &cbuf));
  auto cand_list = [&](int h) {
    long long *b = reinterpret_cast<long long *>(cbuf) + (size_t)h * 5 * ccap;
    return Cand{b, b + ccap, b + 2 * ccap, reinterpret_cast<double *>(b + 3 * ccap),
                h ? cnts + 3 * kSegs + 8 : cnts, ccap, csegcap};
  };
  const Cand cands[2] = {cand_list(0), cand_list(1)};
  Cand cand = cands[0];  // (the list the pass-1 launches below append to: the second half's switches it)
  // kmer_regions: a rescan accompanies a region in the same segment; tr_lr
  // rescans every closed excursion, so its capacity grows on its own
  const int64_t rsegcap = std::max<int64_t>(rb.segcap, ctx->rescan_segcap);
  const int64_t rcap = rsegcap * kSegs;  // per list
  void *rsb = nullptr;
  KS_TRY(ensure(ctx, SLOT_WORK_A, (size_t)rcap * 40 + 2048, &rsb));
  auto rescan_list = [&](int h) {
    int64_t *b = reinterpret_cast<int64_t *>(static_cast<char *>(rsb) + (size_t)h * ((size_t)rcap * 20 + 256));
    return Rescan{b, b + rcap, reinterpret_cast<int32_t *>(b + 2 * rcap), h ? cnts + 4 * kSegs + 8 : cnts + kSegs,
                  rcap, rsegcap};
  };
  const Rescan rss[2] = {rescan_list(0), rescan_list(1)};
  const Rescan &rs = rss[0];
  // KS_DEBUG_CARRY=1: per-window carry statistics to stderr (diagnostics only)
  static const bool dbg_on = getenv("KS_DEBUG_CARRY") != nullptr;
  long long *dbg = nullptr;
  if (dbg_on) {
    KS_HIP(hipMalloc(&dbg, (nwin * 9 + 4) * sizeof(long long)));
    KS_HIP(hipMemsetAsync(dbg, 0, (nwin * 9 + 4) * sizeof(long long), st));
  }

  // ---- P0 chunks, P1 gather pass
  KS_HIP(hipEventRecord(ctx->ev[7], st));
  if (nruns > 0) {
    hipLaunchKernelGGL(k_tile_runs, dim3((unsigned)nruns), dim3(256), 0, st, d_tbase, nruns, d_trun_map);
    KS_HIP(hipGetLastError());
  }
  if (ntiles > 0)
    hipLaunchKernelGGL(k_make_chunks, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, st, runs.a, d_cbase, d_tbase,
                       d_trun_map, ntiles, k, runs.b, mode.trlr, g);
  KS_HIP(hipGetLastError());
  const unsigned gch = (unsigned)((nch + 255) / 256);
  const unsigned gch1k = (unsigned)((nch + 1023) / 1024);
  const int Jt = (tv.ext != nullptr) ? tv.ext_J : 1;
  const bool lds_table = k <= kLdsTableK && runs.packed != nullptr && getenv("KS_NO_LDS_TABLE") == nullptr;
  // pass-1 summaries (no per-position code store): compressed expanded
  // tables on the pipelined pass with a binade predictor (a table without
  // one, a failed allocation of the predictor, is scanned unexpanded)
  const bool line = tv.line != nullptr && !lds_table && runs.packed != nullptr;  // line table: k_pass1l
  // (FP64 tables: no summaries by default -- see no_summ below; at k = 15
  // 50.6 vs 53.7 ms with k_pass1pf's pass-1 summaries and 59.4 with
  // k_summaries, at k = 13 29.8 vs 30.2 with k_summaries,
  // profiles/r5/ab/ab_nosumm_*.txt.  KS_F64_P1SUMM=1: pass-1 summaries (FP64
  // lines, expanded J 2..4, k_pass1pf); KS_F64_P1SUMM=0: k_summaries)
  const char *f64e = getenv("KS_F64_P1SUMM");
  const bool f64_summ = !comp && !lds_table && f64e && atoi(f64e) != 0 && (line || (Jt >= 2 && Jt <= 4));
  // (small k, the table in LDS: pass-1 summaries from the LDS-staged table;
  // the k_summaries path after the prescan took 13.3 vs 8.8 ms at k = 7 log2)
  const bool lds_summ = lds_table;
  // integer tables: the exact carry (k_carry_exact) needs no predictor and
  // no summaries (KS_NO_EXACT: the general path, for A/B runs and tests)
  // (on the table forms of the pipelined passes -- LDS, line, expanded; an
  // unexpanded table of another size takes the code-store pass and k_summaries)
  // (exact while every partial sum of a run is: |s| <= 2^20 over fewer than
  // 2^32 indices stays below 2^52; KS_TEST_SEG_FALLBACK, which forces the
  // general carry's per-run fallback, takes the general path)
  const int force_fb = getenv("KS_TEST_SEG_FALLBACK") != nullptr ? 1 : 0;  // tests: force the fallback path
  const bool exact = tv.exact && !mode.trlr && runs.packed != nullptr && (lds_table || line || Jt >= 2) &&
                     lay.longest < ((int64_t)1 << 32) && !force_fb && getenv("KS_NO_EXACT") == nullptr;
  // FP64 tables without KS_F64_P1SUMM: no chunk summaries at all (a summary
  // serves a chunk only while its carry-in stays >= 64 in one binade; weighted
  // rank values in [-0.5, 0.5] keep the carry far below that: 5,598 of 11.96 M
  // chunks at config 3 were summary-served, 1.0 M replayed)
  const bool no_summ = getenv("KS_NO_SUMMARIES") != nullptr || (!comp && !lds_table && !f64e);
  const bool p1summ = !exact && (lds_table ? lds_summ : (comp ? (Jt >= 2 || line) : f64_summ)) &&
                      runs.packed != nullptr && tv.approx != nullptr;
  // (the carry reads no replay slots unless k_marks_select wrote them)
  if (!p1summ) rpb.slot = nullptr;
  // pass-1 summaries are read where pass 1 wrote them (summ_at): the selection
  // writes a byte per chunk instead of copying 56 (metric step 14.47 vs 14.61 ms
  // median in-process, profiles/r4/ab4/ab_copy_log2.txt)
  if (p1summ) {
    sm.sel = reinterpret_cast<uint8_t *>(W + o_ssel);
    sm.pD = sp1.D;
    sm.pM = sp1.M;
    sm.pN = sp1.N;
    sm.pA = sp1.A;
  }
  // per-index code store (uint16 per scan index, 2 B x 256 per chunk):
  // written by the compressed unexpanded pass 1 (k_pass1<1, ...>) for the
  // binade summaries (k_summaries)
  uint16_t *codes = nullptr;
  if (comp && !p1summ && !exact && !lds_table) {
    void *cp = nullptr;
    const int64_t ctiles = (nch + 63) / 64;  // code store tiles (global chunk index / 64)
    KS_TRY(ensure(ctx, SLOT_CHUNK_B, (size_t)ctiles * 64 * CH * 2, &cp));
    codes = static_cast<uint16_t *>(cp);
  }
  // Two halves of the runs (pass-1-summary path): the second half's pass 1
  // (side stream) runs while the first half's latency-bound later passes
  // (carry, stitch) run on the main stream; halves split at a run boundary,
  // so no carry or stitch crosses it.
  struct Half {
    int64_t c0, c1, r0, r1, t0, t1;
  };
  const int64_t ctail_all = nch > 1024 ? nch - 1024 : 0;
  // FP64 line tables (weighted rank) without pass-1 summaries: one part.
  // Their two pass-1 launches ran side by side and ended together (15.2 ms
  // each, profiles/r5/rank/step_timeline_rank_k13_twopart.txt), so the first part's
  // post-processing never ran under the second's pass 1: 27.75 vs 28.56 ms
  // in one part (profiles/r5/ab/ab_nosplit_k13.txt).  (Round 3, with
  // k_summaries after pass 1: two parts 31.5 vs 32.7, profiles/r3/rank/.)
  // (the exact carry's post-processing is short: one part -- two measured the
  // same at lower run-to-run spread, 6.44 vs 6.55 ms median at k = 7,
  // profiles/r4/ab3/ab_k7pm1_exact_split.txt)
  // (below ~2 M chunks, ~500 Mbp, one part: at the 8-way shard, 1.5 M chunks,
  // 2.38 vs 2.42 ms in-process; 4-way, 3 M chunks, two parts 4.24 vs 4.37;
  // profiles/r5/ab/ab_one_part_*.txt.  KS_SPLIT_MIN_CHUNKS: the threshold --
  // tests set 0 to run the two-part path on small genomes)
  const char *smin = getenv("KS_SPLIT_MIN_CHUNKS");
  const int64_t split_min = smin ? atoll(smin) : ((int64_t)2 << 20);
  // (FP64 expanded tables without summaries stay in one part: two measured
  // 52.1 vs 51.6 ms at k = 15, 46.0 vs 44.8 at k = 14,
  // profiles/r5/ab/ab_nosumm_split_k15.txt, ab_nosumm_k14.txt)
  const bool split = p1summ &&
                     nch > split_min && lay.split_r > 0 && lay.split_r < nruns &&
                     lay.split_c >= 1024 && lay.split_c + 1024 <= ctail_all;
  Half halves[2];
  int nhalf = 1;
  halves[0] = Half{0, nch, 0, nruns, 0, ntiles};
  if (split) {
    nhalf = 2;
    halves[0] = Half{0, lay.split_c, 0, lay.split_r, 0, lay.split_t};
    halves[1] = Half{lay.split_c, nch, lay.split_r, nruns, lay.split_t, ntiles};
  }
  auto view = [&](const Half &h) {
    Chunks v = g;
    v.c0 = h.c0;
    v.nch = h.c1;
    return v;
  };
  bool side_forked = false;  // the side stream already waits for the chunks (P0 overlap)
  if (p1summ) {  // P0: predicted entries of each half (the second half's on the side stream, under
                 // the first half's predictor and pass 1)
    P1 pp = p1;
    pp.asum = reinterpret_cast<double *>(W + o_pa);
    pp.cexit = reinterpret_cast<double *>(W + o_pb);
    pp.special = reinterpret_cast<uint8_t *>(W + o_pz);
    auto predict = [&](const Half &h, hipStream_t strm) -> ks_status {
      KS_HIP(hipMemsetAsync(W + o_pz + h.c0, 0, (size_t)(h.c1 - h.c0), strm));
      const size_t lds = (size_t)2 << (2 * tv.approx_k);  // the fp16 prefix table
      const int per_cu = lds <= ((size_t)32 << 10) ? 4 : 1;
      const unsigned gl = (unsigned)std::max<int64_t>(
          1, std::min<int64_t>((h.c1 - h.c0 + 1023) / 1024, (int64_t)ctx->num_cus * per_cu));
      // every fourth index sampled, weighted 4 (at four 32-KiB blocks per CU:
      // metric step 14.48 vs 14.62 ms median with every second, predictor 0.56 vs
      // 0.64 ms; every eighth: predictor 0.21 ms but more mispredicted binades,
      // carry + stitch 1.18 vs 0.85 ms; profiles/r4/ab4/ab_pred_log2.txt).
      KS_HIP(hipFuncSetAttribute((const void *)k_predict<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(k_predict<4>, dim3(gl), dim3(1024), lds, strm, view(h), total, k, tv.approx, tv.approx_k,
                         pp.asum, pp.cexit);
      KS_HIP(hipGetLastError());
      return ascan(pp, d_xh, h.r0, h.r1, h.t0, h.t1, strm);
    };
    // the first half's predictor and prescan first (they gate its pass 1;
    // the predictor holds whole CUs: 128 KiB of LDS per block), then the
    // second half's on the side stream, under the first half's pass 1 (also
    // at shard sizes: both first on the main stream measured 2.48 vs 2.38 ms
    // at the 8-way shard, profiles/r4/ab/ab_shard8.txt)
    KS_TRY(predict(halves[0], st));
    if (split) {
      side_forked = true;
      KS_HIP(hipEventRecord(ctx->ev[16], st));
      KS_HIP(hipStreamWaitEvent(ctx->side, ctx->ev[16], 0));
      KS_TRY(predict(halves[1], ctx->side));
    }
  }
  KS_HIP(hipEventRecord(ctx->ev[8], st));
  const bool lds_lut = comp && tv.nlut <= kLdsLutMax;
#define KS_P1(J, C, L)                                                                                       \
  hipLaunchKernelGGL((k_pass1<J, C, L>), dim3(J == 1 ? gch : gch1k), dim3(J == 1 ? 256 : 1024), 0, st, g, s->seq, \
                     total, k, tv, codes, ec, visits, p1, cand, (int64_t)0, 0)
  // k_pass1p leaves the chunks whose reads could pass the end of the buffer
  // (chunk starts increase with the chunk index, so they are among the last
  // kP1TailMargin + CH chunks) to k_pass1
  const int64_t ctail = nch > 1024 ? nch - 1024 : 0;
#define KS_P1T(J, L) KS_P1TC(J, true, L)
#define KS_P1TC(J, C, L)                                                                                       \
  hipLaunchKernelGGL((k_pass1<J, C, L>), dim3((unsigned)((nch - ctail + 1023) / 1024)), dim3(1024), 0, side, g, \
                     s->seq, total, k, tv, p1summ ? nullptr : codes, ec, visits, p1, cand, ctail, 1)
  // compressed tables are scanned expanded only on the summarising pass
  const int J = (tv.ext != nullptr && (p1summ || exact || !comp)) ? tv.ext_J : 1;
  const bool pipelined = runs.packed != nullptr;
#define KS_P1P(J, L, GV, GRID, STRM)                                                                           \
  do {                                                                                                       \
    if (ec.trlr)                                                                                             \
      hipLaunchKernelGGL((k_pass1p<J, L, true>), dim3(GRID), dim3(kP1Block), 0, STRM, GV, s->seq, total, k, tv, \
                         ec, visits, p1, cand, runs.packed, p1summ ? d_xh : nullptr, sp1);                   \
    else                                                                                                     \
      hipLaunchKernelGGL((k_pass1p<J, L, false>), dim3(GRID), dim3(kP1Block), 0, STRM, GV, s->seq, total, k, tv, \
                         ec, visits, p1, cand, runs.packed, p1summ ? d_xh : nullptr, sp1);                   \
  } while (0)
  if (lds_table) {
    // small k: the whole table in LDS, persistent blocks (one per CU), no
    // code store; with pass-1 summaries the halves as for line tables
    // integer small-k tables: the int32 pass (4.72 vs 5.57 ms at k = 7,
    // profiles/r4/ab3/ab_k7pm1_int.txt; KS_NO_EXACT: the FP64 pass)
    const bool lds_int = true;
    auto p1lds = [&](const Half &h, hipStream_t strm) {
      const Chunks gv = view(h);
      const unsigned gl = (unsigned)std::max<int64_t>(1, std::min<int64_t>((h.c1 - h.c0 + 1023) / 1024, ctx->num_cus));
      const double *xh = p1summ ? d_xh : nullptr;
      if (ec.trlr)
        hipLaunchKernelGGL(k_pass1_lds<true>, dim3(gl), dim3(1024), 0, strm, gv, total, k, tv, ec, visits, p1, cand, xh,
                           sp1);
      else if (exact && lds_int)  // (two blocks per CU)
        hipLaunchKernelGGL(k_pass1_lds_int, dim3((unsigned)std::max<int64_t>(
                                                 1, std::min<int64_t>((h.c1 - h.c0 + 1023) / 1024, 2 * ctx->num_cus))),
                           dim3(1024), 0, strm, gv, total, k, tv, ec, visits, p1, cand);
      else if (exact)
        hipLaunchKernelGGL((k_pass1_lds<false, true>), dim3(gl), dim3(1024), 0, strm, gv, total, k, tv, ec, visits, p1,
                           cand, xh, sp1);
      else
        hipLaunchKernelGGL(k_pass1_lds<false>, dim3(gl), dim3(1024), 0, strm, gv, total, k, tv, ec, visits, p1, cand, xh,
                           sp1);
    };
    if (split) {
      KS_HIP(hipEventRecord(ctx->ev[17], st));
      KS_HIP(hipStreamWaitEvent(ctx->hi, ctx->ev[17], 0));
      if (!side_forked) KS_HIP(hipStreamWaitEvent(ctx->side, ctx->ev[17], 0));
      p1lds(halves[0], ctx->hi);
      KS_HIP(hipGetLastError());
      KS_HIP(hipEventRecord(ctx->ev[12], ctx->hi));
      KS_HIP(hipStreamWaitEvent(st, ctx->ev[12], 0));
      cand = cands[1];
      p1lds(halves[1], ctx->side);
    } else {
      p1lds(halves[0], st);
    }
    codes = nullptr;
  } else if (line && (p1summ || exact || !comp)) {
    // line tables: every chunk (no tail: a lane's bases come from guarded loads)
    const bool lut = tv.nlut <= kLineLutMax;
#define KS_P1L(O, F, L, GV, GRID, STRM)                                                                        \
  do {                                                                                                       \
    if (ec.trlr)                                                                                             \
      hipLaunchKernelGGL((k_pass1l<O, F, L, true>), dim3(GRID), dim3(F ? 1024 : 768), 0, STRM, GV, total, k, tv, ec, \
                         visits, p1, cand, p1summ ? d_xh : nullptr, sp1);                                    \
    else                                                                                                     \
      hipLaunchKernelGGL((k_pass1l<O, F, L, false>), dim3(GRID), dim3(F ? 1024 : 768), 0, STRM, GV, total, k, tv, \
                         ec, visits, p1, cand, p1summ ? d_xh : nullptr, sp1);                                \
  } while (0)
    auto p1l = [&](const Half &h, hipStream_t strm) {
      const Chunks gv = view(h);
      const int own = tv.line_own;
      if (tv.rline && !ec.trlr && !p1summ && own == 3) {  // weighted-rank code lines (k = 13)
        hipLaunchKernelGGL(k_pass1r<3>, dim3((unsigned)((h.c1 - h.c0 + kRankBlock - 1) / kRankBlock)),
                           dim3(kRankBlock), 0, strm, gv, total, k, tv, ec, visits, p1, cand);
        return;
      }
      if (tv.line_kind == 3) {  // wide lines
        const unsigned grid = (unsigned)((h.c1 - h.c0 + kWideBlock - 1) / kWideBlock);
#define KS_P1W(O)                                                                                             \
  do {                                                                                                      \
    if (ec.trlr)                                                                                            \
      hipLaunchKernelGGL((k_pass1w<O, true>), dim3(grid), dim3(kWideBlock), 0, strm, gv, total, k, tv, ec, visits, \
                         p1, cand, p1summ ? d_xh : nullptr, sp1);                                           \
    else                                                                                                    \
      hipLaunchKernelGGL((k_pass1w<O, false>), dim3(grid), dim3(kWideBlock), 0, strm, gv, total, k, tv, ec, visits, \
                         p1, cand, p1summ ? d_xh : nullptr, sp1);                                           \
  } while (0)
        if (own == 1) KS_P1W(1);  // k = 15 (J = 4)
        else if (own == 2) KS_P1W(2);  // k = 14 (J = 5)
        else if (own == 3) KS_P1W(3);  // k = 13 (J = 6)
        else KS_P1W(4);  // k = 12 (J = 7)
#undef KS_P1W
        return;
      }
      const int bs = comp ? 768 : 1024;
      const unsigned grid = (unsigned)((h.c1 - h.c0 + bs - 1) / bs);
      if (!comp) {
        if (own == 4) KS_P1L(4, true, false, gv, grid, strm);
        else if (own == 3) KS_P1L(3, true, false, gv, grid, strm);
        else KS_P1L(2, true, false, gv, grid, strm);
      } else if (lut) {
        if (own == 5) KS_P1L(5, false, true, gv, grid, strm);
        else if (own == 4) KS_P1L(4, false, true, gv, grid, strm);
        else if (own == 3) KS_P1L(3, false, true, gv, grid, strm);
        else KS_P1L(2, false, true, gv, grid, strm);
      } else {
        if (own == 5) KS_P1L(5, false, false, gv, grid, strm);
        else if (own == 4) KS_P1L(4, false, false, gv, grid, strm);
        else if (own == 3) KS_P1L(3, false, false, gv, grid, strm);
        else KS_P1L(2, false, false, gv, grid, strm);
      }
    };
#undef KS_P1L
    if (split) {  // the halves at once, as the expanded-table pass below
      KS_HIP(hipEventRecord(ctx->ev[17], st));
      KS_HIP(hipStreamWaitEvent(ctx->hi, ctx->ev[17], 0));
      if (!side_forked) KS_HIP(hipStreamWaitEvent(ctx->side, ctx->ev[17], 0));
      p1l(halves[0], ctx->hi);
      KS_HIP(hipGetLastError());
      KS_HIP(hipEventRecord(ctx->ev[12], ctx->hi));
      KS_HIP(hipStreamWaitEvent(st, ctx->ev[12], 0));
      cand = cands[1];
      p1l(halves[1], ctx->side);
    } else {
      p1l(halves[0], st);
    }
    KS_HIP(hipGetLastError());
  } else if (!comp && J >= 2 && J <= 4 && pipelined) {  // FP64 expanded table (weighted rank)
    hipStream_t side = ctx->side;
    const bool tail = nch > ctail;
    const double *xh = p1summ ? d_xh : nullptr;
#define KS_P1PF(J, GV, STRM, B)                                                                                \
    do {                                                                                                       \
      const unsigned grid_ = (unsigned)((h.c1 - h.c0 + (B) - 1) / (B));                                        \
      if (ec.trlr) hipLaunchKernelGGL((k_pass1pf<J, true, B>), dim3(grid_), dim3(B), 0, STRM, GV, s->seq, total, k, \
                                      tv, ec, visits, p1, cand, runs.packed, xh, sp1);                         \
      else hipLaunchKernelGGL((k_pass1pf<J, false, B>), dim3(grid_), dim3(B), 0, STRM, GV, s->seq, total, k, tv, \
                              ec, visits, p1, cand, runs.packed, xh, sp1);                                     \
    } while (0)
    // 512-lane blocks: up to 256 VGPRs, 152 used, no spills, 3 waves per SIMD
    // (1024-lane blocks capped it at 128 with 17-29 VGPRs spilled to scratch:
    // weighted rank k = 15 in-process 55.3 vs 61.4 ms, profiles/r5/ab/ab_p1pf_block.txt)
    auto p1f = [&](const Half &h, hipStream_t strm) {
      const Chunks gv = view(h);
      if (J == 4) KS_P1PF(4, gv, strm, 512); else if (J == 3) KS_P1PF(3, gv, strm, 512); else KS_P1PF(2, gv, strm, 512);
    };
    if (tv.rline && !ec.trlr && !p1summ && !split && (k == 14 || k == 15)) {
      // weighted-rank code lines (k = 14 / 15: J = 4 / 3 per 128-B line read
      // against 3 / 2 per FP64 expanded entry); every chunk (guarded base loads)
      const unsigned grid = (unsigned)((nch + kRankBlock - 1) / kRankBlock);
      if (k == 15)
        hipLaunchKernelGGL(k_pass1r<1>, dim3(grid), dim3(kRankBlock), 0, st, view(halves[0]), total, k, tv, ec, visits,
                           p1, cand);
      else
        hipLaunchKernelGGL(k_pass1r<2>, dim3(grid), dim3(kRankBlock), 0, st, view(halves[0]), total, k, tv, ec, visits,
                           p1, cand);
      KS_HIP(hipGetLastError());
    } else {
#undef KS_P1PF
    auto p1tail = [&]() {
      if (J == 4) KS_P1TC(4, false, false); else if (J == 3) KS_P1TC(3, false, false); else KS_P1TC(2, false, false);
    };
    if (split) {  // the halves at once, as the compressed pass below
      KS_HIP(hipEventRecord(ctx->ev[17], st));
      KS_HIP(hipStreamWaitEvent(ctx->hi, ctx->ev[17], 0));
      if (!side_forked) KS_HIP(hipStreamWaitEvent(side, ctx->ev[17], 0));
      p1f(halves[0], ctx->hi);
      KS_HIP(hipGetLastError());
      KS_HIP(hipEventRecord(ctx->ev[12], ctx->hi));
      KS_HIP(hipStreamWaitEvent(st, ctx->ev[12], 0));
      cand = cands[1];  // (the tail chunks are the second half's)
      if (tail) {
        p1tail();
        KS_HIP(hipGetLastError());
      }
      p1f(halves[1], side);
    } else {
      if (tail) {
        KS_HIP(hipEventRecord(ctx->ev[12], st));
        KS_HIP(hipStreamWaitEvent(side, ctx->ev[12], 0));
        p1tail();
        KS_HIP(hipGetLastError());
        KS_HIP(hipEventRecord(ctx->ev[13], side));
      }
      p1f(halves[0], st);
      KS_HIP(hipGetLastError());
      if (tail) KS_HIP(hipStreamWaitEvent(st, ctx->ev[13], 0));
    }
    }
    KS_HIP(hipGetLastError());
  } else if (p1summ || exact) {
    // the tail chunks (a latency-bound serial walk each) run on the side
    // stream, overlapped with the pipelined pass (of the last half)
    hipStream_t side = ctx->side;
    const bool tail = nch > ctail;
    auto p1p = [&](const Half &h, hipStream_t strm) {
      const Chunks gv = view(h);
      const unsigned grid = (unsigned)((h.c1 - h.c0 + kP1Block - 1) / kP1Block);
      if (lds_lut) {
        if (J == 5) KS_P1P(5, true, gv, grid, strm); else if (J == 4) KS_P1P(4, true, gv, grid, strm);
        else if (J == 3) KS_P1P(3, true, gv, grid, strm); else KS_P1P(2, true, gv, grid, strm);
      } else {
        if (J == 5) KS_P1P(5, false, gv, grid, strm); else if (J == 4) KS_P1P(4, false, gv, grid, strm);
        else if (J == 3) KS_P1P(3, false, gv, grid, strm); else KS_P1P(2, false, gv, grid, strm);
      }
    };
    if (split) {
      // first half on the highest-priority stream, the tail chunks and the
      // second half on the (lowest-priority) side stream at once: the second
      // half's blocks fill the CUs the first half leaves, its drain included,
      // and the first half ends first (its carry and stitch then run under
      // the rest of the second half; serial halves cost 0.6 ms in-process).
      KS_HIP(hipEventRecord(ctx->ev[17], st));
      KS_HIP(hipStreamWaitEvent(ctx->hi, ctx->ev[17], 0));
      if (!side_forked) KS_HIP(hipStreamWaitEvent(side, ctx->ev[17], 0));
      p1p(halves[0], ctx->hi);
      KS_HIP(hipGetLastError());
      KS_HIP(hipEventRecord(ctx->ev[12], ctx->hi));
      KS_HIP(hipStreamWaitEvent(st, ctx->ev[12], 0));
      cand = cands[1];  // (the tail chunks are the second half's)
      if (tail) {
        if (J == 5) KS_P1T(5, false);
        else if (lds_lut) { if (J == 4) KS_P1T(4, true); else if (J == 3) KS_P1T(3, true); else KS_P1T(2, true); }
        else { if (J == 4) KS_P1T(4, false); else if (J == 3) KS_P1T(3, false); else KS_P1T(2, false); }
        KS_HIP(hipGetLastError());
      }
      p1p(halves[1], side);
      KS_HIP(hipGetLastError());
    } else {
      if (tail) {
        KS_HIP(hipEventRecord(ctx->ev[12], st));
        KS_HIP(hipStreamWaitEvent(side, ctx->ev[12], 0));
        if (J == 5) KS_P1T(5, false);
        else if (lds_lut) { if (J == 4) KS_P1T(4, true); else if (J == 3) KS_P1T(3, true); else KS_P1T(2, true); }
        else { if (J == 4) KS_P1T(4, false); else if (J == 3) KS_P1T(3, false); else KS_P1T(2, false); }
        KS_HIP(hipGetLastError());
        KS_HIP(hipEventRecord(ctx->ev[13], side));
      }
      p1p(halves[0], st);
      KS_HIP(hipGetLastError());
      if (tail) KS_HIP(hipStreamWaitEvent(st, ctx->ev[13], 0));
    }
  } else if (comp) {
    KS_P1(1, true, false);  // unexpanded compressed table (with the code store)
  } else {
    KS_P1(1, false, false);  // (expanded FP64 tables take k_pass1pf above)
  }
#undef KS_P1
#undef KS_P1T
#undef KS_P1TC
#undef KS_P1P
  KS_HIP(hipGetLastError());
  // (the first half's post-processing on the high-priority stream, ahead of
  // the second half's pass-1 blocks, measured the same: 14.15 vs 14.15 ms,
  // profiles/r5/ab/ab_post0.txt)
  if (split) {
    // end of pass 1 = the later of the halves: the hi stream (idle now) joins the side stream's
    KS_HIP(hipEventRecord(ctx->ev[18], ctx->side));
    KS_HIP(hipStreamWaitEvent(ctx->hi, ctx->ev[18], 0));
    KS_HIP(hipEventRecord(ctx->ev[9], ctx->hi));
  } else {
    KS_HIP(hipEventRecord(ctx->ev[9], split ? ctx->side : st));  // end of pass 1 (the last half's stream)
  }
  // KS_TEST_EPOCH_STALE (tests): the post-processing expects another epoch
  // than pass 1 stamped -- what it would see reading an earlier call's
  // pass-1 results -- so the epoch guard must fail the call
  if (getenv("KS_TEST_EPOCH_STALE")) ++p1.epoch;

  // P2-P5 (without the candidates) of one half on stream strm, with its own
  // replay counter, error bits and fix list; ev[14] / ev[15] mark the last
  // half's phases
  auto post = [&](int hi, const Half &h, hipStream_t strm) -> ks_status {
    const bool last = hi == nhalf - 1;
    const Chunks gv = view(h);
    const int64_t nh = h.c1 - h.c0, nr = h.r1 - h.r0, nt = h.t1 - h.t0;
    if (nh <= 0) return KS_OK;
    unsigned long long *rep_h = d_replays + 2 * hi;
    unsigned int *err_h = reinterpret_cast<unsigned int *>(d_replays + 2 * hi + 1);
    const unsigned gch_h = (unsigned)((nh + 255) / 256);
    const unsigned gsum_h = (unsigned)((nh + 1023) / 1024);
    // ---- P2 prediction, segment starts, summaries
    KS_TRY(ascan(p1, xt, h.r0, h.r1, h.t0, h.t1, strm));
    const int64_t wl = (h.c0 > 0 ? h.c0 - 1 : 0) / 64;
    const int64_t nwm = (h.c1 + 63) / 64 - wl;
    // segment marks and summary selection in one pass over the chunks
    if (!p1summ && !exact) {
      hipLaunchKernelGGL(k_seg_marks, dim3((unsigned)((nwm + wpb - 1) / wpb)), dim3(64 * wpb), 0, strm, gv, p1, xt,
                         d_flag, nwm);
      KS_HIP(hipGetLastError());
    }
    if (exact) {  // the prescan is the carry (k_carry_exact)
      hipLaunchKernelGGL(k_carry_exact, dim3(gch_h), dim3(256), 0, strm, gv, p1, xt, cr);
    } else if (p1summ) {
      KS_HIP(hipMemsetAsync(d_nfix + hi, 0, 8, strm));
      KS_HIP(hipMemsetAsync(rpb.count + hi, 0, 8, strm));
      hipLaunchKernelGGL(k_marks_select, dim3((unsigned)((nwm + 3) / 4)), dim3(256), 0, strm, gv, p1, xt, d_flag, nwm,
                         sp1, sm, d_fix + h.c0, d_nfix + hi, d_xh,
                         dbg ? reinterpret_cast<unsigned long long *>(dbg + nwin * 9) : nullptr, rpb, hi);
      KS_HIP(hipGetLastError());
      // summaries of the listed chunks, a wave each; the LUT read through L2,
      // not staged in LDS: a 54 KB LDS copy per block (2048 blocks, most
      // without a listed chunk) cost more than the ~4 M lookups of the ~16 K
      // listed chunks
      const unsigned gw = (unsigned)std::max<int64_t>(1, (int64_t)ctx->num_cus * 8);
      hipLaunchKernelGGL(k_summ_fixw<false>, dim3(gw), dim3(256), 0, strm, g, s->seq, total, k, tv, xt,
                         d_fix + h.c0, d_nfix + hi, sm, rpb, hi);
    } else if (no_summ) {
      hipLaunchKernelGGL(k_summ_none, dim3(gsum_h), dim3(1024), 0, strm, gv, sm);
    } else if (lds_table) {
      // small k: the table staged in LDS as for k_pass1_lds (from HBM / L2: 12.8 / 18.7 vs 3.8 / 6.4 ms)
      if (comp && lds_lut) {
        const size_t tb = (size_t)2 << (2 * k);
        KS_HIP(hipFuncSetAttribute((const void *)k_summaries<true, true, true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)tb));
        hipLaunchKernelGGL((k_summaries<true, true, true>), dim3(gsum_h), dim3(1024), tb, strm, gv, s->seq, total, k,
                           tv, nullptr, p1, xt, sm);
      } else {
        const size_t tb = (size_t)8 << (2 * k);
        KS_HIP(hipFuncSetAttribute((const void *)k_summaries<false, false, true>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)tb));
        hipLaunchKernelGGL((k_summaries<false, false, true>), dim3(gsum_h), dim3(1024), tb, strm, gv, s->seq, total,
                           k, tv, nullptr, p1, xt, sm);
      }
    } else if (lds_lut)
      hipLaunchKernelGGL((k_summaries<true, true>), dim3(gsum_h), dim3(1024), 0, strm, gv, s->seq, total, k, tv, codes,
                         p1, xt, sm);
    else if (comp)
      hipLaunchKernelGGL((k_summaries<true, false>), dim3(gsum_h), dim3(1024), 0, strm, gv, s->seq, total, k, tv, codes,
                         p1, xt, sm);
    else
      hipLaunchKernelGGL((k_summaries<false, false>), dim3(gsum_h), dim3(1024), 0, strm, gv, s->seq, total, k, tv,
                         codes, p1, xt, sm);
    KS_HIP(hipGetLastError());
    if (last) KS_HIP(hipEventRecord(ctx->ev[14], strm));

    // ---- P3 carry by segments + P4 heads; then the gated per-run fallback
    const int64_t wc = h.c0 / 64;
    const unsigned nwc = (unsigned)((h.c1 - 1) / 64 - wc + 1);
    const TileComp tch = tcomp;
    const unsigned gtc = (unsigned)(((h.c1 - 1) / 64 - wc + 1 + 3) / 4);  // 4 tiles per block
    if (!exact) {
      hipLaunchKernelGGL(k_tile_comp, dim3(gtc), dim3(256), 0, strm, gv, sm, tch);
      KS_HIP(hipGetLastError());
    }
    if (exact) {
    } else if (comp)
      hipLaunchKernelGGL(k_carry_win<true>, dim3((nwc + wpb - 1) / wpb), dim3(64 * wpb), 0, strm, gv, d_flag, s->seq, total, k, tv, codes, p1,
                         sm, cr, tch, rpb, rep_h, err_h, dbg);
    else
      hipLaunchKernelGGL(k_carry_win<false>, dim3((nwc + wpb - 1) / wpb), dim3(64 * wpb), 0, strm, gv, d_flag, s->seq, total, k, tv, codes,
                         p1, sm, cr, tch, rpb, rep_h, err_h, dbg);
    KS_HIP(hipGetLastError());
    if (!exact) {
      hipLaunchKernelGGL(k_tile_apply, dim3(gtc), dim3(256), 0, strm, gv, sm, tch, cr, err_h, 0);
      KS_HIP(hipGetLastError());
    }
    // FP64 tables: the R chunks' heads packed densely (k_heads_dense; lane per
    // chunk, k_heads, measured slower at config 3: 29.9 vs 29.2 ms,
    // profiles/r5/ab/ab_heads_dense_lane_pf_*.txt); compressed tables: k_heads
    const bool dense_heads = !comp;
    auto heads = [&](int gated) {
      // (gated: a small grid-stride grid; it exits at once unless the carry fell back)
      const unsigned gd = (unsigned)((nh + 4 * kHeadSpan - 1) / (4 * kHeadSpan));
      const unsigned gh = gated ? std::min<unsigned>(dense_heads ? gd : gch_h, (unsigned)ctx->num_cus * 2)
                                : (dense_heads ? gd : gch_h);
#define KS_HEADS_D(J, W)                                                                                          \
  hipLaunchKernelGGL((k_heads_dense<J, false, W>), dim3(gh), dim3(256), 0, strm, gv, s->seq, total, k, tv, codes, \
                     cr, err_h, gated)
      if (comp) {
        hipLaunchKernelGGL((k_heads<1, true>), dim3(gh), dim3(256), 0, strm, gv, s->seq, total, k, tv, codes, cr,
                           err_h, gated);
      } else if (J == 4 && tv.line) KS_HEADS_D(4, true);
      else if (J == 4) KS_HEADS_D(4, false);
      else if (J == 3) KS_HEADS_D(3, false);
      else if (J == 2) KS_HEADS_D(2, false);
      else KS_HEADS_D(1, false);
#undef KS_HEADS_D
    };
    heads(0);
    KS_HIP(hipGetLastError());
    if (!exact) hipLaunchKernelGGL(k_fallback_prep, dim3(1), dim3(1), 0, strm, err_h, rep_h, force_fb);
    if (nr > 0 && !exact) {
      if (comp)
        hipLaunchKernelGGL(k_carry_run<true>, dim3((unsigned)nr), dim3(64), 0, strm, gv, d_cbase, h.r1, s->seq, total,
                           k, tv, codes, p1, sm, cr, tch, rpb, rep_h, err_h, nullptr, h.r0);
      else
        hipLaunchKernelGGL(k_carry_run<false>, dim3((unsigned)nr), dim3(64), 0, strm, gv, d_cbase, h.r1, s->seq,
                           total, k, tv, codes, p1, sm, cr, tch, rpb, rep_h, err_h, nullptr, h.r0);
      hipLaunchKernelGGL(k_tile_apply, dim3(gtc), dim3(256), 0, strm, gv, sm, tch, cr, err_h, 1);
    }
    if (!exact) heads(1);
    KS_HIP(hipGetLastError());
    if (last) KS_HIP(hipEventRecord(ctx->ev[15], strm));

    // ---- P5 stitch
    if (nt > 0) {
      hipLaunchKernelGGL(k_stitch_tiles, dim3((unsigned)((nt + wpb - 1) / wpb)), dim3(64 * wpb), 0, strm, g, d_tbase, d_cbase,
                         nruns, d_trun, p1, cr, xagg, h.t0, h.t1);
      KS_HIP(hipGetLastError());
    }
    if (nr > 0) {
      hipLaunchKernelGGL(k_stitch_runs, dim3((unsigned)nr), dim3(64), 0, strm, d_tbase, h.r1, runs.a, runs.b, runs.seq,
                         ec, xagg, xtin, rb, rss[hi], h.r0);
      KS_HIP(hipGetLastError());
    }
    if (nt > 0) {
      hipLaunchKernelGGL(k_stitch_emit, dim3((unsigned)((nt + wpb - 1) / wpb)), dim3(64 * wpb), 0, strm, g, d_tbase, d_cbase,
                         nruns, d_trun, runs.a, runs.seq, p1, cr, ec, xtin, rb, rss[hi], err_h, h.t0, h.t1);
      KS_HIP(hipGetLastError());
    }
    return KS_OK;
  };
  // ---- candidates (count read on the device), rescans: of each half's
  // list on the stream of its post-processing (the first half's under the
  // second half's, weighted rank: ~3.8 ms of lane walks), on st
  // (the rescan slots in list order: sorted longest first they took 5.23 vs
  // 3.56 ms at config 3, profiles/r4/ab2/ab_rank.txt)
  auto emit_rescan = [&](int h, hipStream_t rst) -> ks_status {
    hipLaunchKernelGGL(k_candidates, dim3((unsigned)((ccap + 255) / 256)), dim3(256), 0, rst, g, runs.a, d_cbase,
                       nruns, runs.seq, ec, cands[h], cr, rb, rss[h]);
    KS_HIP(hipGetLastError());
    if (h == nhalf - 1) KS_HIP(hipEventRecord(ctx->ev[10], rst));
    KS_TRY(launch_scan_lane(ctx, s->seq, total, rss[h].a, rss[h].b, rss[h].seq, rcap, k, tv, mw, min_score,
                            visits_rescan, rb, rss[h].count, rss[h].segcap, mode, 0, nullptr, runs.packed, rst));
    return KS_OK;
  };
  if (split) {
    // (the first half's rescans under the second half's post-processing: config 3
    // 32.1 vs 32.9 ms with both after the join, profiles/r4/ab3/)
    // (the second half's rescans on the side stream, beside the first half's
    // instead of after the join: 28.53 vs 28.46 ms at config 3, metric 14.71
    // vs 14.65, profiles/r5/ab/ab_rescan_side_*.txt)
    KS_TRY(post(0, halves[0], st));         // under the second half's pass 1
    KS_TRY(emit_rescan(0, st));             // under the second half's post-processing
    KS_TRY(post(1, halves[1], ctx->side));
    KS_HIP(hipEventRecord(ctx->ev[13], ctx->side));
    KS_HIP(hipStreamWaitEvent(st, ctx->ev[13], 0));
    KS_TRY(emit_rescan(1, st));
  } else {
    KS_TRY(post(0, halves[0], st));
    KS_TRY(emit_rescan(0, st));
  }
  KS_HIP(hipEventRecord(ctx->ev[11], st));
  // the region counters too (final: the rescans above append the last
  // regions), copied next to the scan's counters: one readback for both, and
  // scan_impl needs no round trip of its own
  hipLaunchKernelGGL(k_copy_u64, dim3(1), dim3(64), 0, st, rb.count, cnts + 2 * kSegs + 8, kSegs);
  KS_HIP(hipGetLastError());
  std::vector<unsigned long long> hcv(5 * kSegs + 8);
  KS_HIP(hipMemcpyAsync(hcv.data(), cnts, 8 * (5 * kSegs + 8), hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  std::copy(hcv.begin() + 2 * kSegs + 8, hcv.begin() + 3 * kSegs + 8, ctx->hreg);
  ctx->hreg_ok = true;
  static const bool verify = getenv("KS_DEBUG_VERIFY") != nullptr;
  if (verify) debug_verify(ctx, s, total, k, tv, g, p1, cr, exact, mode.trlr);
  unsigned long long cand_max = 0, res_max = 0, res_tot = 0;
  for (int q = 0; q < kSegs; ++q) {
    const unsigned long long c0 = hcv[q], c1 = hcv[3 * kSegs + 8 + q];
    const unsigned long long r0 = hcv[kSegs + q], r1 = hcv[4 * kSegs + 8 + q];
    cand_max = std::max(cand_max, std::max(c0, c1));
    res_max = std::max(res_max, std::max(r0, r1));
    res_tot += std::min<unsigned long long>(r0, (unsigned long long)rs.segcap) +
               std::min<unsigned long long>(r1, (unsigned long long)rs.segcap);
  }
  // hc: [0] largest candidate segment, [1] rescans, [2] replays, [3] error bits
  const unsigned long long hc[4] = {cand_max, res_tot, hcv[2 * kSegs] + hcv[2 * kSegs + 2],
                                     (hcv[2 * kSegs + 1] | hcv[2 * kSegs + 3]) & 0xffffffffull};

  const unsigned int errbits = (unsigned int)(hc[3] & 0xffffffffu);
  if ((errbits & 16u) && !force_fb)
    fprintf(stderr, "kmer_spans_amd: carry segment check failed; the carry was redone per run\n");
  if (dbg_on && p1summ) {
    unsigned long long nf = 0;
    unsigned long long nf2[2] = {0, 0};
    KS_HIP(hipMemcpy(nf2, d_nfix, 16, hipMemcpyDeviceToHost));
    nf = nf2[0] + nf2[1];
    unsigned long long why[3] = {0, 0, 0};
    KS_HIP(hipMemcpy(why, dbg + nwin * 9, 24, hipMemcpyDeviceToHost));
    fprintf(stderr, "[p1summ] chunks %lld gathered summaries %llu (no prediction %llu, void %llu, other binade %llu)\n",
            (long long)nch, nf, why[0], why[1], why[2]);
    if (rpb.slot) {
      unsigned long long rc[2] = {0, 0};
      KS_HIP(hipMemcpy(rc, rpb.count, 16, hipMemcpyDeviceToHost));
      fprintf(stderr, "[replay prefetch] listed %llu + %llu chunks (cap %lld per half)\n", rc[0], rc[1],
              (long long)rpb.cap);
    }
  }
  if (dbg) {
    std::vector<long long> h(nwin * 9);
    KS_HIP(hipMemcpy(h.data(), dbg, nwin * 9 * sizeof(long long), hipMemcpyDeviceToHost));
    KS_HIP(hipFree(dbg));
    std::vector<int64_t> idx(nwin);
    for (int64_t i = 0; i < nwin; ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return h[9 * a] > h[9 * b]; });
    long long tot[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = 0; i < nwin; ++i)
      for (int q = 0; q < 9; ++q) tot[q] += h[9 * i + q];
    fprintf(stderr, "[carry] windows %lld (runs %lld) chunks %lld replays %lld (wave-parallel %lld, bases prefetched "
            "%lld; cycles %lld, in fast tiles %lld, in replays %lld) segments %lld L %lld R %lld\n", (long long)nwin,
            (long long)nruns, tot[1], tot[2], tot[8] & 0xffffffffLL, tot[8] >> 32, tot[0], tot[6], tot[7], tot[3],
            tot[4], tot[5]);
    for (int64_t i = 0; i < std::min<int64_t>(nwin, 8); ++i) {
      const long long *d = &h[9 * idx[i]];
      fprintf(stderr, "[carry] window %lld cycles %lld (fast tiles %lld, replays %lld) chunks %lld replays %lld "
              "segments %lld L %lld R %lld\n", (long long)idx[i], d[0], d[6], d[7], d[1], d[2], d[3], d[4], d[5]);
    }
  }
  if (errbits & 32u)
    return fail(KS_ERR_DEVICE, "chunked scan epoch check failed: the stitch read pass-1 results not written by this "
                                 "call (epoch %u)", p1.epoch);
  if (errbits & ~16u) return fail(KS_ERR_INTERNAL, "chunked scan consistency check failed (bits %u)", errbits);
  if ((int64_t)cand_max > csegcap) {  // grow the candidate buffers and rerun the pass
    void *grown = nullptr;
    const size_t seg = (size_t)(cand_max + cand_max / 4 + 64);
    KS_TRY(ensure(ctx, SLOT_CHUNK_C, seg * kSegs * 80 + 2048, &grown));
    return KS_INTERNAL_RETRY;
  }
  if ((int64_t)res_max > rs.segcap) {  // grow the rescan buffer (regions may have overflowed too) and rerun
    ctx->rescan_segcap = (int64_t)(res_max + res_max / 4 + 64);
    return KS_INTERNAL_RETRY;
  }
  const int64_t nres = (int64_t)hc[1];
  if (dbg_on && nres > 0) {  // rescan length histogram (log2 buckets)
    std::vector<int64_t> a(rcap), b(rcap);
    KS_HIP(hipMemcpy(a.data(), rs.a, rcap * 8, hipMemcpyDeviceToHost));
    KS_HIP(hipMemcpy(b.data(), rs.b, rcap * 8, hipMemcpyDeviceToHost));
    long long hist[40] = {0}, tot = 0, mx = 0;
    for (int64_t i = 0; i < rcap; ++i) {
      if ((i % rs.segcap) >= (int64_t)hcv[kSegs + i / rs.segcap]) continue;
      const long long L = b[i] - a[i] - k;
      tot += L;
      mx = std::max(mx, L);
      int e = 0;
      while (e < 39 && (1LL << (e + 1)) <= L) ++e;
      ++hist[L > 0 ? e : 0];
    }
    fprintf(stderr, "[rescan] n %lld indices %lld max %lld |", (long long)nres, tot, mx);
    for (int e = 0; e < 40; ++e)
      if (hist[e]) fprintf(stderr, " 2^%d:%lld", e, hist[e]);
    fprintf(stderr, "\n");
  }
  if (stats) {  // (phase times: chunked_phase_times, after the call's last sync)
    stats->n_rescan = nres;
    stats->n_replay = (int64_t)hc[2];
  }
  ctx->chunked_events = true;
  return KS_OK;
}

// Phase times of the last chunked scan on ctx (its events are complete once
// the caller has synchronised after the region readback).
ks_status chunked_phase_times(ks_ctx *ctx, ks_scan_stats *stats) {
  if (!ctx->chunked_events) {  // nothing to scan (no run longer than k): no phase was recorded
    stats->ms_layout = stats->ms_scan = stats->ms_predict = stats->ms_carry = stats->ms_stitch = stats->ms_rescan = 0;
    return KS_OK;
  }
  float ms_lay = 0, ms_p1 = 0, ms_p2 = 0, ms_p34 = 0, ms_p5 = 0, ms_res = 0;
  KS_HIP(hipEventElapsedTime(&ms_lay, ctx->ev[7], ctx->ev[8]));
  KS_HIP(hipEventElapsedTime(&ms_p1, ctx->ev[8], ctx->ev[9]));
  KS_HIP(hipEventElapsedTime(&ms_p2, ctx->ev[9], ctx->ev[14]));
  KS_HIP(hipEventElapsedTime(&ms_p34, ctx->ev[14], ctx->ev[15]));
  KS_HIP(hipEventElapsedTime(&ms_p5, ctx->ev[15], ctx->ev[10]));
  KS_HIP(hipEventElapsedTime(&ms_res, ctx->ev[10], ctx->ev[11]));
  // (the second part's P2-P5 events can precede the end of the union of the
  // pass-1 launches when it finished first: such a phase counts 0)
  stats->ms_layout = ms_lay;
  stats->ms_scan = ms_p1;
  stats->ms_predict = std::max(0.0f, ms_p2);
  stats->ms_carry = std::max(0.0f, ms_p34);
  stats->ms_stitch = std::max(0.0f, ms_p5);
  stats->ms_rescan = ms_res;
  return KS_OK;
}

}  // namespace ks
