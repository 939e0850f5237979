// ks_runs.hip -- N-free run segmentation of device-resident sequences.
//
// The reference discovers runs on the fly (skip_n + init_kmer,
// kmer_spans.c:111-132).  Here runs are materialised once per call so that
// counting and scanning can parallelise over them: a run is a maximal
// [a, b) of non-N bytes inside one sequence.  Boundaries are sparse (N gaps,
// sequence ends), so one streaming pass (16 bytes per lane-step, SWAR N test)
// emits (position, START/END) events with a wave-aggregated atomic append,
// a second tiny kernel splits runs at sequence boundaries, and a radix sort
// restores position order;
// END sorts before START at the same position (sequence boundary between two
// non-N bytes), so the sorted events alternate START, END, START, ...
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ks_internal.h"

namespace ks {
namespace {

// Byte mask (bit i <-> byte i) of the N/n bytes of a 32-bit word: exact
// per-byte zero test of (w | 0x20) ^ 'n'.
__device__ __forceinline__ uint32_t n_mask4(uint32_t w) {
  const uint32_t x = (w | 0x20202020u) ^ 0x6e6e6e6eu;
  const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;  // 0x80 in zero bytes
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

// enc() (kmer_spans.c:34-35: (c >> 1) & 3) of the 4 bytes of w as one byte,
// first (lowest-addressed) byte in the top two bits.
__device__ __forceinline__ uint32_t enc_pack4(uint32_t w) {
  const uint32_t t = (w >> 1) & 0x03030303u;
  return ((t & 3u) << 6) | (((t >> 8) & 3u) << 4) | (((t >> 16) & 3u) << 2) | ((t >> 24) & 3u);
}
// The same with one multiply: byte i of t (i = 0..3, values 0..3) lands at
// bit 30 - 2i; every cross term stays below bit 24 without carries.
__device__ __forceinline__ uint32_t enc_pack4m(uint32_t w) {
  return (((w >> 1) & 0x03030303u) * 0x40100401u) >> 24;
}
// 0x80 in each N / n byte of w
__device__ __forceinline__ uint32_t n_flags4(uint32_t w) {
  const uint32_t x = (w | 0x20202020u) ^ 0x6e6e6e6eu;
  return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// Appends the events of `cnt` set bits of starts/ends (bit i <-> p0 + i).
__device__ __forceinline__ void append_events(uint32_t starts, uint32_t ends, int64_t p0,
                                              unsigned long long *__restrict__ ev,
                                              unsigned long long *__restrict__ ev_count, int64_t cap) {
  const int cnt = __popc(starts) + __popc(ends);
  if (__ballot(cnt > 0) == 0) return;
  const int lane = threadIdx.x & 63;
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  unsigned long long base = 0;
  if (lane == 63) base = atomicAdd(ev_count, (unsigned long long)incl);
  base = __shfl(base, 63, 64);
  unsigned long long slot = base + (unsigned long long)(incl - cnt);
  while (ends | starts) {
    const int je = ends ? __ffs(ends) - 1 : 99, js = starts ? __ffs(starts) - 1 : 99;
    if (je <= js) {  // END sorts before START at the same position anyway
      if ((int64_t)slot < cap) ev[slot] = ((unsigned long long)(p0 + je) << 1);
      ends &= ends - 1;
    } else {
      if ((int64_t)slot < cap) ev[slot] = ((unsigned long long)(p0 + js) << 1) | 1ull;
      starts &= starts - 1;
    }
    ++slot;
  }
}

// N-transition events of the whole buffer read as one string with N before
// position 0 and at position total: START at p (first non-N byte after an N),
// END at p (first N after a non-N byte).  16 bytes per step, persistent grid.
// packed (optional): the same pass stores the 2-bit codes of the 16 bytes as
// one word (bytes past total encode as 'N'), which the gather pass of the
// chunked scan reads instead of the bytes (a quarter of the lines).
// Range [p_lo, p_hi) (a part of the buffer cut at sequence boundaries, see
// scan_impl): bytes outside it read as N, so its runs and no others come
// out; units [u0, u1) are visited (the range plus a margin, whose packed
// words -- pure functions of the bytes -- the part's later passes may read).
// kPre: lane 0's byte before its unit is loaded with the unit loads (one
// memory round trip per step) instead of after them (A/B: KS_NEV_LATE_PREV=1).
// Four units per lane and step (eight, and nontemporal byte loads, measured
// the same: 0.89-0.95 ms, profiles/r4/ab/ab_nev.txt).
// Lane - 1's last byte comes by a DPP wave_shr:1 move (a VALU operand, no
// LDS round trip; 0.849 vs 0.875 ms with __shfl_up, profiles/r4/ab3/ab_log2.txt).
template <bool kMul, bool kPre>  // multiply-based byte packing, lane 0's preceding byte loaded early (both A/B winners)
__global__ void __launch_bounds__(256) k_n_events(const uint8_t *__restrict__ seq, int64_t total,
                                                  unsigned long long *__restrict__ ev,
                                                  unsigned long long *__restrict__ ev_count, int64_t cap,
                                                  uint32_t *__restrict__ packed, int64_t p_lo, int64_t p_hi,
                                                  int64_t u0, int64_t u1) {
  constexpr int U = 4;  // units per lane and step (U loads in flight)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  const int lane = threadIdx.x & 63;
  for (int64_t ub = u0 + (int64_t)blockIdx.x * blockDim.x * U; ub < u1; ub += stride) {
    uint4 v[U];
    uint32_t pb[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int64_t p0 = (ub + j * blockDim.x + threadIdx.x) * 16;
      v[j] = make_uint4(0, 0, 0, 0);
      if (p0 + 16 <= total) v[j] = *reinterpret_cast<const uint4 *>(seq + p0);
      pb[j] = 'N';
      if (kPre && lane == 0 && p0 > 0 && p0 - 1 < total) pb[j] = seq[p0 - 1];
    }
    // a step whose units all lie inside the range, before total, with a byte
    // before them (block-uniform, nearly every step): no range or end tests
    const int64_t step_end = ub + (int64_t)U * blockDim.x;  // one past its last unit
    const bool inner = ub * 16 > p_lo && step_end * 16 <= (p_hi < total ? p_hi : total) && step_end <= u1;
    auto units = [&](auto inner_tag) {
      constexpr bool kIn = decltype(inner_tag)::value;
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int64_t u = ub + j * blockDim.x + threadIdx.x;
        const int64_t p0 = u * 16;
        uint32_t starts = 0, ends = 0;
        // the byte before the unit: lane - 1's last byte (the same step's
        // previous unit), loaded by lane 0
        uint32_t prev_b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(v[j].w >> 24), 0x138, 0xf, 0xf, true);
        if (kPre && lane == 0)
          prev_b = pb[j];
        else if (lane == 0 || (!kIn && p0 + 16 > total))
          prev_b = p0 == 0 ? (uint32_t)'N' : (p0 - 1 < total ? seq[p0 - 1] : 'N');
        if (kIn || u < u1) {
          uint32_t nm = 0xffffu;
          if (kIn || p0 + 16 <= total) {
            if (kMul) {
              // byte flags first; the bit gather only for a unit holding an N
              // (most units hold none)
              const uint32_t f0 = n_flags4(v[j].x), f1 = n_flags4(v[j].y), f2 = n_flags4(v[j].z),
                             f3 = n_flags4(v[j].w);
              nm = 0;
              if (f0 | f1 | f2 | f3)
                nm = (((f0 >> 7) * 0x10204080u) >> 28) | ((((f1 >> 7) * 0x10204080u) >> 28) << 4) |
                     ((((f2 >> 7) * 0x10204080u) >> 28) << 8) | ((((f3 >> 7) * 0x10204080u) >> 28) << 12);
              if (packed)
                packed[u] = (enc_pack4m(v[j].x) << 24) | (enc_pack4m(v[j].y) << 16) | (enc_pack4m(v[j].z) << 8) |
                            enc_pack4m(v[j].w);
            } else {
              nm = n_mask4(v[j].x) | (n_mask4(v[j].y) << 4) | (n_mask4(v[j].z) << 8) | (n_mask4(v[j].w) << 12);
              if (packed)
                packed[u] = (enc_pack4(v[j].x) << 24) | (enc_pack4(v[j].y) << 16) | (enc_pack4(v[j].z) << 8) |
                            enc_pack4(v[j].w);
            }
          } else {
            uint32_t pw = 0;
            for (int q = 0; q < 16; ++q) {
              const uint8_t c = p0 + q < total ? seq[p0 + q] : (uint8_t)'N';
              if (p0 + q < total && !is_n(c)) nm &= ~(1u << q);
              pw |= enc(c) << (30 - 2 * q);
            }
            if (packed) packed[u] = pw;
          }
          if (!kIn && (p0 < p_lo || p0 + 16 > p_hi)) {  // a unit at an end of the range: outside reads as N
            for (int q = 0; q < 16; ++q)
              if (p0 + q < p_lo || p0 + q >= p_hi) nm |= 1u << q;
          }
          const uint32_t prev_n =
              (is_n((uint8_t)prev_b) || (!kIn && (p0 <= p_lo || p0 - 1 >= p_hi))) ? 1u : 0u;
          const uint32_t non = ~nm & 0xffffu;
          starts = non & ((nm << 1) | prev_n);
          ends = nm & ((non << 1) | (prev_n ^ 1u)) & 0xffffu;
          if (!kIn && p0 + 16 > p_hi) {  // no events past position p_hi
            const int keep = (int)(p_hi - p0) + 1;
            const uint32_t km = keep <= 0 ? 0u : keep >= 16 ? 0xffffu : ((1u << keep) - 1u);
            starts &= km;
            ends &= km;
          }
        }
        append_events(starts, ends, p0, ev, ev_count, cap);
      }
    };
    if (inner)
      units(std::integral_constant<bool, true>());
    else
      units(std::integral_constant<bool, false>());
  }
}

// Interior sequence boundaries between two non-N bytes split a run: END and
// START at the boundary (emitted once per distinct offset).
__global__ void k_seq_events(const uint8_t *__restrict__ seq, int64_t total, const int64_t *__restrict__ offs,
                             int32_t nseq, unsigned long long *__restrict__ ev,
                             unsigned long long *__restrict__ ev_count, int64_t cap, int64_t p_lo, int64_t p_hi) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < 1 || q >= nseq) return;
  const int64_t p = offs[q];
  if (offs[q - 1] == p || p <= p_lo || p >= p_hi || p >= total) return;
  if (is_n(seq[p - 1]) || is_n(seq[p])) return;
  const unsigned long long slot = atomicAdd(ev_count, 2ull);
  if ((int64_t)slot + 1 < cap) {
    ev[slot] = ((unsigned long long)p << 1);
    ev[slot + 1] = ((unsigned long long)p << 1) | 1ull;
  }
}

// Pair sorted events into runs and attach the sequence id.
__global__ void k_pair_runs(const unsigned long long *__restrict__ ev, int64_t nruns,
                            const int64_t *__restrict__ offs, int32_t nseq, int64_t *__restrict__ ra,
                            int64_t *__restrict__ rb, int32_t *__restrict__ rs) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  const int64_t a = (int64_t)(ev[2 * r] >> 1);
  const int64_t b = (int64_t)(ev[2 * r + 1] >> 1);
  int lo = 0, hi = nseq;  // last q with offs[q] <= a
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (offs[mid] <= a) lo = mid; else hi = mid - 1;
  }
  ra[r] = a;
  rb[r] = b;
  rs[r] = lo;
}

// Chunks and stitch tiles of every run, plus (wave-aggregated) totals.
__global__ void k_run_counts(const int64_t *__restrict__ ra, const int64_t *__restrict__ rb,
                             const int32_t *__restrict__ rs, const int64_t *__restrict__ offs, int64_t n, int k,
                             int trlr, int64_t *__restrict__ cnt_c, int64_t *__restrict__ cnt_t,
                             unsigned long long *__restrict__ agg) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long sc = 0, ns = 0, lo = 0;
  if (r < n) {
    const int64_t L = rb[r] - ra[r];
    int64_t P = L - k;
    if (trlr) P = (L >= k && ra[r] + k + 1 < offs[rs[r] + 1]) ? P + 1 : 0;
    const int64_t ch = P > 0 ? (P + kChunk - 1) / kChunk : 0;
    cnt_c[r] = ch;
    cnt_t[r] = (ch + kTileChunks - 1) / kTileChunks;
    if (P > 0) { sc = (unsigned long long)P; ns = 1; lo = (unsigned long long)L; }
  } else if (r == n) {
    cnt_c[r] = 0;
    cnt_t[r] = 0;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    sc += __shfl_down(sc, d, 64);
    ns += __shfl_down(ns, d, 64);
    const unsigned long long o = __shfl_down(lo, d, 64);
    lo = o > lo ? o : lo;
  }
  if ((threadIdx.x & 63) == 0 && (sc | ns | lo)) {
    atomicAdd(&agg[0], sc);
    atomicAdd(&agg[1], ns);
    atomicMax(&agg[2], lo);
  }
}

// The run where the first part of the chunks ends: first r with
// cbase[r] >= frac * cbase[n] (out: r, cbase[r], tbase[r]).
__global__ void k_split(const int64_t *__restrict__ cbase, const int64_t *__restrict__ tbase, int64_t n,
                        double frac, unsigned long long *__restrict__ out) {
  // frac < 0: by size -- 0.65 for a genome (a shorter predictor before the
  // first part's pass 1; in process on two boxes: 0.6 13.91-14.00 vs 0.7
  // 14.09-14.22 ms, then 0.65 14.07-14.11 vs 0.6 14.19-14.29 vs 0.7
  // 14.24-14.29 ms, rank and k = 15 unchanged: profiles/r4/ab4/ab_frac_*.txt;
  // 0.7 until round 4), 0.8 at
  // shard sizes (<= 2 M chunks, ~500 Mbp), where the post-processing is short
  // and the second part's own tail dominates (in-process A/B at the 8-way
  // shard: 2.47 vs 2.58 ms; 4-way equal)
  if (frac < 0) frac = cbase[n] <= (2ll << 20) ? 0.8 : 0.65;
  const int64_t half = (int64_t)((double)cbase[n] * frac);
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cbase[mid] < half) lo = mid + 1; else hi = mid;
  }
  out[0] = (unsigned long long)lo;
  out[1] = (unsigned long long)cbase[lo];
  out[2] = (unsigned long long)tbase[lo];
  out[3] = (unsigned long long)cbase[n];  // totals: one readback with the aggregates
  out[4] = (unsigned long long)tbase[n];
}

}  // namespace

ks_status run_layout(ks_ctx *ctx, const Runs &runs, int k, RunLayout *lay, int trlr, const int64_t *offs_dev) {
  hipStream_t st = ctx->stream;
  const int64_t n = runs.n;
  *lay = RunLayout{};
  void *buf = nullptr;
  KS_TRY(ensure(ctx, SLOT_LAYOUT, (size_t)(n + 1) * 8 * 4 + 256, &buf));
  int64_t *cnt_c = static_cast<int64_t *>(buf);
  int64_t *cnt_t = cnt_c + (n + 1);
  lay->cbase = cnt_t + (n + 1);
  lay->tbase = lay->cbase + (n + 1);
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *agg = reinterpret_cast<unsigned long long *>(scal) + kScLayout;
  KS_HIP(hipMemsetAsync(agg, 0, 24, st));
  if (trlr && !offs_dev) return fail(KS_ERR_INTERNAL, "run_layout: tr_lr needs sequence offsets");
  hipLaunchKernelGGL(k_run_counts, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, runs.a, runs.b,
                     runs.seq, offs_dev, n, k, trlr, cnt_c, cnt_t, agg);
  KS_HIP(hipGetLastError());
  size_t tb = 0;
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt_c, lay->cbase, (int)(n + 1), st));
  void *tmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_SORT_TMP, tb, &tmp));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt_c, lay->cbase, (int)(n + 1), st));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt_t, lay->tbase, (int)(n + 1), st));
  // the first half (highest priority) ends first; its carry and stitch run
  // under the rest of the second half (the first part's share by size, k_split)
  const double frac = -1.0;
  hipLaunchKernelGGL(k_split, dim3(1), dim3(1), 0, st, lay->cbase, lay->tbase, n, frac, agg + 3);
  KS_HIP(hipGetLastError());
  unsigned long long ha[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  KS_HIP(hipMemcpyAsync(ha, agg, 64, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  lay->nch = (int64_t)ha[6];
  lay->ntiles = (int64_t)ha[7];
  lay->scored = (int64_t)ha[0];
  lay->nscan = (int64_t)ha[1];
  lay->longest = (int64_t)ha[2];
  lay->split_r = (int64_t)ha[3];
  lay->split_c = (int64_t)ha[4];
  lay->split_t = (int64_t)ha[5];
  return KS_OK;
}

ks_status find_runs(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, Runs *runs, float *ms, bool want_packed,
                    int64_t p_lo, int64_t p_hi) {
  if (p_hi < 0) p_hi = total;
  hipStream_t st = ctx->stream;
  KS_HIP(hipEventRecord(ctx->ev[0], st));
  uint32_t *packed = nullptr;
  if (want_packed) {
    void *pp = nullptr;
    KS_TRY(ensure(ctx, SLOT_PACKED, (size_t)(total / 16 + 1) * 4, &pp));
    packed = static_cast<uint32_t *>(pp);
  }
  runs->packed = nullptr;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_count = reinterpret_cast<unsigned long long *>(scal) + kScEvents;
  int64_t cap = 1 << 20;
  if (ctx->slots[SLOT_EVENTS].bytes / 8 > (size_t)cap) cap = ctx->slots[SLOT_EVENTS].bytes / 8;
  unsigned long long n_ev = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    void *evp = nullptr;
    KS_TRY(ensure(ctx, SLOT_EVENTS, (size_t)cap * 8, &evp));
    KS_HIP(hipMemsetAsync(d_count, 0, 8, st));
    const int64_t nunits = total / 16 + 1;  // covers position total
    constexpr int64_t kMargin = 64;          // packed words past the range's ends (pass-1 staging reach)
    const int64_t u0 = std::max<int64_t>(0, p_lo / 16 - kMargin);
    const int64_t u1 = std::min<int64_t>(nunits, p_hi / 16 + 1 + kMargin);
    const unsigned grid = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((u1 - u0 + 1023) / 1024, (int64_t)ctx->num_cus * 16));
    // (the next step's loads issued before this step's units, software
    // pipelined: 14.387 vs 14.379 ms min in-process, profiles/r6/ab/ab_nev_pf.txt)
    hipLaunchKernelGGL((k_n_events<true, true>), dim3(grid), dim3(256), 0, st, s->seq, total,
                       (unsigned long long *)evp, d_count, cap, packed, p_lo, p_hi, u0, u1);
    KS_HIP(hipGetLastError());
    if (s->nseq > 1) {
      hipLaunchKernelGGL(k_seq_events, dim3((unsigned)((s->nseq + 255) / 256)), dim3(256), 0, st, s->seq, total,
                         s->offsets_dev, s->nseq, (unsigned long long *)evp, d_count, cap, p_lo, p_hi);
      KS_HIP(hipGetLastError());
    }
    KS_HIP(hipMemcpyAsync(&n_ev, d_count, 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
    if ((int64_t)n_ev <= cap) break;
    cap = (int64_t)n_ev;
  }
  if (n_ev & 1ull) return fail(KS_ERR_INTERNAL, "run segmentation produced an odd event count");
  const int64_t nruns = (int64_t)(n_ev / 2);
  runs->n = nruns;
  runs->packed = packed;
  if (nruns == 0) {
    KS_HIP(hipEventRecord(ctx->ev[1], st));
    KS_HIP(hipEventSynchronize(ctx->ev[1]));
    if (ms) KS_HIP(hipEventElapsedTime(ms, ctx->ev[0], ctx->ev[1]));
    return KS_OK;
  }
  // sort events by key
  void *evp = ctx->slots[SLOT_EVENTS].ptr, *evt = nullptr;
  KS_TRY(ensure(ctx, SLOT_EVENTS_TMP, (size_t)n_ev * 8, &evt));
  int end_bit = 2;
  while (end_bit < 64 && ((unsigned long long)(total) << 1 | 1ull) >> end_bit) ++end_bit;
  size_t tmp_bytes = 0;
  KS_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, (unsigned long long *)evp,
                                           (unsigned long long *)evt, (int)n_ev, 0, end_bit, st));
  void *tmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_SORT_TMP, tmp_bytes, &tmp));
  KS_HIP(hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, (unsigned long long *)evp,
                                           (unsigned long long *)evt, (int)n_ev, 0, end_bit, st));
  void *rbuf = nullptr;
  KS_TRY(ensure(ctx, SLOT_RUNS, (size_t)nruns * 20 + 64, &rbuf));
  runs->a = reinterpret_cast<int64_t *>(rbuf);
  runs->b = runs->a + nruns;
  runs->seq = reinterpret_cast<int32_t *>(runs->b + nruns);
  hipLaunchKernelGGL(k_pair_runs, dim3((unsigned)((nruns + 255) / 256)), dim3(256), 0, st,
                     (const unsigned long long *)evt, nruns, s->offsets_dev, s->nseq, runs->a,
                     runs->b, runs->seq);
  KS_HIP(hipGetLastError());
  KS_HIP(hipEventRecord(ctx->ev[1], st));
  if (ms) {
    KS_HIP(hipEventSynchronize(ctx->ev[1]));
    KS_HIP(hipEventElapsedTime(ms, ctx->ev[0], ctx->ev[1]));
  }
  return KS_OK;
}

}  // namespace ks
