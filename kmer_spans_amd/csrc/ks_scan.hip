// ks_scan.hip -- span scan driver and the lane-per-run kernel (algo 0).
//
// kmer_regions (kmer_spans.c:243-307) is a per-run state machine: scanning
// index i scores the k-mer ending at i-1 with s = w - thr, S = max(S + s, 0)
// (NaN -> 0), opens an excursion where S turns positive, keeps the first
// strict maximum, and at a reset (S back to 0) or at the run's end emits the
// excursion if (size_t)(max_pos - beg) >= min_width && max >= min_score, then
// restarts with fresh state at max_pos + 1.  Restarts never leave the run, so
// runs are independent.  k_scan_lane executes that state machine literally,
// one lane per run; it is the correctness baseline and the path for short
// runs.  The chunked carry scan (ks_scan_chunked.hip) parallelises inside
// long runs.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <condition_variable>
#include <type_traits>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <cstdlib>

#include "ks_scan_common.h"

namespace ks {

ks_status scan_chunked(ks_ctx *ctx, const ks_dev_seqs *s, const Runs &runs, const RunLayout &lay, int k,
                       const TableView &tv, uint64_t mw, double min_score, uint32_t *visits,
                       uint32_t *visits_rescan, const RegionBuf &rb, ks_scan_stats *stats, const ScanMode &mode);
ks_status chunked_phase_times(ks_ctx *ctx, ks_scan_stats *stats);
ks_status launch_scan_lane(ks_ctx *ctx, const uint8_t *seq, int64_t total, const int64_t *ra, const int64_t *rb,
                           const int32_t *rs, int64_t n, int k, const TableView &tv, uint64_t mw,
                           double min_score, uint32_t *visits, const RegionBuf &out,
                           const unsigned long long *d_cnt = nullptr, int64_t segcap = 0,
                           const ScanMode &mode = ScanMode(), int init_step = 1, const int64_t *offs = nullptr,
                           const uint32_t *packed = nullptr, hipStream_t strm = nullptr);

namespace {

// Values of a batch of consecutive scan indices are gathered before the
// sequential state machine consumes them, so a lane keeps several random
// table reads in flight instead of one (the gathers do not depend on S).
// With an expanded table one read serves J consecutive indices (the
// (k+J-1)-mer spanning them), as in the chunked gather pass.  (Issuing the
// next batch's reads before a batch is consumed measured no faster on the
// weighted-rank rescans: 3.94 vs 3.64 ms, profiles/r4/ab/ab_rank.txt.)
template <int J, bool kCompressed, int GW = 0>
__global__ void __launch_bounds__(64) k_scan_lane(const uint8_t *__restrict__ seq, int64_t total,
                                                  const int64_t *__restrict__ ra,
                                                  const int64_t *__restrict__ rbnd,
                                                  const int32_t *__restrict__ rseq, int64_t nruns,
                                                  int k, TableView tv, uint64_t mw, double min_score,
                                                  uint32_t *__restrict__ visits, RegionBuf out,
                                                  const unsigned long long *__restrict__ d_cnt, int64_t segcap,
                                                  const uint32_t *__restrict__ packed) {
  // reads per batch (GW: a wider batch -- FP64 line tables, 8 line reads = 32 indices per round trip:
  // weighted-rank rescans 3.76 -> 3.61 ms in-process, profiles/r3/rank/lane_ab.txt)
  constexpr int G = GW ? GW : ((J == 1) ? 16 : (J >= 4 ? 4 : (J == 3 ? 6 : 8)));
  constexpr int PB = G * J;                                           // indices per batch (16, 16, 18, 16, 20)
  using GC = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;  // (k+J-1)-mer code
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  if (d_cnt && (r % segcap) >= (int64_t)d_cnt[r / segcap]) return;  // segmented list: unused slot
  const int64_t a = ra[r], b = rbnd[r];
  if (b - a <= k) return;
  const int32_t sid = rseq[r];
  const int kx = k + J - 1;
  const GC xmask = (2 * kx >= 8 * (int)sizeof(GC)) ? ~(GC)0 : (((GC)1 << (2 * kx)) - 1);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  GC gcode = 0;
  // values and group keys of the batch at p0 (gcode rolls on to the next batch)
  auto gather = [&](int64_t p0, double vv[PB], GC gg[G]) {
    const int n = (int)((b - p0) < PB ? (b - p0) : PB);
    uint64_t xb = 0;  // the batch's PB <= 20 rolled-in bases from the packed codes (2 * PB <= 64 bits)
    const bool pk = packed_bits(packed, total, p0 + J - 1, xb);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      gg[g] = gcode;
      if (g * J < n) {
        gather_group<J, kCompressed>(tv, gcode, kmask, vv + g * J);
        if (pk) {
          gcode = ((gcode << (2 * J)) | (GC)((xb >> (64 - 2 * J * (g + 1))) & ((1ull << (2 * J)) - 1))) & xmask;
        } else {
#pragma unroll
          for (int t = 0; t < J; ++t) {
            const int64_t q = p0 + g * J + J - 1 + t;
            gcode = ((gcode << 2) | enc(q < total ? seq[q] : (uint8_t)'N')) & xmask;
          }
        }
      }
    }
  };
  int64_t i = a;  // priming point
  for (;;) {
    // (k+J-1)-mer of the group starting at scan index i + k
    gcode = (GC)prime_code_guarded64(seq, i, kx, total);
    double S = 0.0, prev = 0.0, best = 0.0;
    int64_t beg = 0, arg = 0;
    bool restart = false;
    double v[PB];
    GC gc[G];
    for (int64_t p0 = i + k; p0 < b && !restart; p0 += PB) {
      const int n = (int)((b - p0) < PB ? (b - p0) : PB);
      gather(p0, v, gc);
#pragma unroll
      for (int j = 0; j < PB; ++j) {  // fully unrolled: v[]/gc[] stay in registers
        if (j < n && !restart) {
          const int64_t p = p0 + j;
          if (visits) atomicAdd(&visits[(uint32_t)(gc[j / J] >> (2 * (J - 1 - j % J))) & kmask], 1u);
          const double t = prev + v[j];
          S = t > 0 ? t : 0.0;
          if (prev == 0 && S > 0) { beg = p; arg = p; best = S; }
          if (S == 0 && prev > 0) {
            if ((uint64_t)(arg - beg) >= mw && best >= min_score) {
              push_region(out, sid, beg, arg, best);
              i = arg + 1 - k;
              restart = true;
            } else {
              best = 0.0;
              arg = p;
            }
          }
          if (!restart) {
            if (S > best) { best = S; arg = p; }
            prev = S;
          }
        }
      }
    }
    if (restart) continue;
    if (S > 0 && (uint64_t)(arg - beg) >= mw && best >= min_score) {
      push_region(out, sid, beg, arg, best);
      i = arg + 1 - k;
      continue;
    }
    break;
  }
}

// find_kmer_tr_lr_regions (kmer_spans.c:329-395), literally, one lane per run
// (init_step = 1: real N-free runs, with the first k-mer's own step and the
// :341 skip) or per rescan range (init_step = 0: positions [a + k, b),
// transitions only, fresh state).  Position p adds the transition score of the
// k-mer ending at p; the maximum is tested before the clamp
// `s < 0 ? 0 : s` (NaN kept, as in the reference); every return to 0 restarts
// at max_pos + 1; an open region at the end is pushed without a restart.
// Positions are global; the caller converts them to 1-based local ones.
template <int J, bool kCompressed>
__global__ void __launch_bounds__(64) k_scan_lane_trlr(const uint8_t *__restrict__ seq, int64_t total,
                                                       const int64_t *__restrict__ ra,
                                                       const int64_t *__restrict__ rbnd,
                                                       const int32_t *__restrict__ rseq, int64_t nruns, int k,
                                                       TableView tv, const double *__restrict__ ks,
                                                       int64_t min_len, RegionBuf out,
                                                       const unsigned long long *__restrict__ d_cnt,
                                                       int64_t segcap, int init_step,
                                                       const int64_t *__restrict__ offs) {
  constexpr int G = (J == 1) ? 16 : (J >= 4 ? 4 : (J == 3 ? 6 : 8));  // reads per batch
  constexpr int PB = G * J;
  using GC = typename std::conditional<(J >= 3), uint64_t, uint32_t>::type;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  if (d_cnt && (r % segcap) >= (int64_t)d_cnt[r / segcap]) return;  // segmented list: unused slot
  const int64_t a = ra[r], b = rbnd[r];
  if (b - a < k) return;
  const int32_t sid = rseq[r];
  const int kx = k + J - 1;
  const GC xmask = (2 * kx >= 8 * (int)sizeof(GC)) ? ~(GC)0 : (((GC)1 << (2 * kx)) - 1);
  const uint32_t kmask = (1u << (2 * k)) - 1u;
  double last = 0.0, best = 0.0;
  int64_t beg = 0, arg = 0;
  if (init_step) {
    if (a + k + 1 >= offs[sid + 1]) return;  // the string ends within a base of the first k-mer (:341)
    double sc = ks[prime_code(seq, a, k)];
    sc = sc < 0 ? 0 : sc;
    if (sc > 0) { best = sc; arg = a + k; beg = a + k; }
    last = sc;
  }
  int64_t ps = a + k;  // first transition position
  const int64_t pe = b;
  for (;;) {
    // position p reads the k-mer ending at p: the (k+J-1)-mer of group 0 starts at ps + 1 - k
    GC gcode = (GC)prime_code_guarded64(seq, ps + 1 - k, kx, total);
    bool restart = false;
    for (int64_t p0 = ps; p0 < pe && !restart; p0 += PB) {
      const int n = (int)((pe - p0) < PB ? (pe - p0) : PB);
      double v[PB];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (g * J < n) {
          gather_group<J, kCompressed>(tv, gcode, kmask, v + g * J);
#pragma unroll
          for (int t = 0; t < J; ++t) {
            const int64_t q = p0 + 1 + g * J + J - 1 + t;
            gcode = ((gcode << 2) | enc(q < total ? seq[q] : (uint8_t)'N')) & xmask;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        if (j < n && !restart) {
          const int64_t p = p0 + j;
          double sc = last + v[j];
          if (sc > best) { best = sc; arg = p; }
          sc = sc < 0 ? 0 : sc;
          if (last == 0 && sc > 0) { best = sc; arg = p; beg = p; }
          if (sc == 0 && last > 0) {
            if (arg - beg >= min_len) push_region(out, sid, beg, arg, best);
            // rescans (init_step 0) skip a restart whose tail (arg, p] cannot
            // hold a region: the scan after p is the same either way (the
            // restarted trajectory is back at 0 at p); whole runs stay literal
            if (init_step || p - arg - 1 >= (min_len > 1 ? min_len : 1)) {
              ps = arg + 1;
              restart = true;
            }
            beg = arg;
            last = best = 0.0;
          } else {
            last = sc;
          }
        }
      }
    }
    if (!restart) break;
  }
  if (best > 0 && arg - beg >= min_len) push_region(out, sid, beg, arg, best);
}

// Compacted index j -> slot of the segmented region buffer.
struct SegPrefix {
  int64_t p[kSegs + 1];
  int64_t segcap;
};

__global__ void k_region_keys(const int64_t *__restrict__ beg, int64_t n, SegPrefix pre,
                              unsigned long long *__restrict__ keys, int32_t *__restrict__ idx) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  int lo = 0, hi = kSegs - 1;  // segment with p[s] <= j < p[s + 1]
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre.p[mid] <= j) lo = mid; else hi = mid - 1;
  }
  const int64_t slot = (int64_t)lo * pre.segcap + (j - pre.p[lo]);
  keys[j] = (unsigned long long)beg[slot];
  idx[j] = (int32_t)slot;
}

// Regions in (seq_id, beg) order == global begin order; local coordinates.
// one = 1: tr_lr's 1-based sequence ids and positions (kmer_spans.c:378,:699).
__global__ void k_region_gather(RegionBuf rb, const int32_t *__restrict__ perm, int64_t n,
                                const int64_t *__restrict__ offs, int one, int32_t *__restrict__ o_seq,
                                int32_t *__restrict__ o_beg, int32_t *__restrict__ o_end,
                                double *__restrict__ o_score) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t i = perm[j];
  const int32_t q = rb.seq[i];
  const int64_t base = offs[q];
  o_seq[j] = q + one;
  o_beg[j] = (int32_t)(rb.beg[i] - base + one);
  o_end[j] = (int32_t)(rb.end[i] - base + one);
  o_score[j] = rb.score[i];
}

// Top-level visits from the k-mer counts (kmer_spans.c:266-267): a run's
// top-level scan scores every k-mer of the run except its last one (quirk Q5),
// so visits = sequence_kmer_count's counts minus the last k-mer of every
// counted run: runs of length >= k, except a run of exactly k bases at the
// end of its sequence, which the count already skips (quirk Q1, :142-144).
__global__ void k_visit_correct(const int64_t *__restrict__ ra, const int64_t *__restrict__ rb,
                                const int32_t *__restrict__ rs, int64_t n, const int64_t *__restrict__ offs,
                                const uint8_t *__restrict__ seq, int k, uint32_t *__restrict__ vis) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int64_t a = ra[r], b = rb[r];
  if (b - a < k || (b - a == k && b == offs[rs[r] + 1])) return;
  atomicSub(&vis[prime_code(seq, b - k, k)], 1u);
}

__global__ void k_add_hist(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

}  // namespace

ks_status launch_scan_lane(ks_ctx *ctx, const uint8_t *seq, int64_t total, const int64_t *ra, const int64_t *rb,
                           const int32_t *rs, int64_t n, int k, const TableView &tv, uint64_t mw,
                           double min_score, uint32_t *visits, const RegionBuf &out,
                           const unsigned long long *d_cnt, int64_t segcap, const ScanMode &mode, int init_step,
                           const int64_t *offs, const uint32_t *packed, hipStream_t strm) {
  hipStream_t sq = strm ? strm : ctx->stream;
  if (n <= 0) return KS_OK;
  // line tables: own + 1 indices per read (gather_group's line form)
  const int J = tv.line ? tv.line_own + 1 : (tv.ext ? tv.ext_J : 1);
  if (mode.trlr) {
#define KS_LANE_T(J, C)                                                                                   \
  hipLaunchKernelGGL((k_scan_lane_trlr<J, C>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, sq, seq, \
                     total, ra, rb, rs, n, k, tv, mode.ks, mode.min_len, out, d_cnt, segcap, init_step, offs)
    if (tv.compressed) {
      if (J == 6) KS_LANE_T(6, true); else if (J == 5) KS_LANE_T(5, true); else if (J == 4) KS_LANE_T(4, true); else if (J == 3) KS_LANE_T(3, true); else if (J == 2) KS_LANE_T(2, true); else KS_LANE_T(1, true);
    } else {
      if (J == 5) KS_LANE_T(5, false); else if (J == 4) KS_LANE_T(4, false); else if (J == 3) KS_LANE_T(3, false); else if (J == 2) KS_LANE_T(2, false); else KS_LANE_T(1, false);
    }
#undef KS_LANE_T
    KS_HIP(hipGetLastError());
    return KS_OK;
  }
#define KS_LANE(J, C)                                                                                   \
  hipLaunchKernelGGL((k_scan_lane<J, C>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, sq, seq, total, \
                     ra, rb, rs, n, k, tv, mw, min_score, visits, out, d_cnt, segcap, packed)
  if (tv.compressed) {
    if (J == 6) KS_LANE(6, true); else if (J == 5) KS_LANE(5, true); else if (J == 4) KS_LANE(4, true); else if (J == 3) KS_LANE(3, true); else if (J == 2) KS_LANE(2, true); else KS_LANE(1, true);
  } else if (J >= 2 && J <= 4) {
    // FP64 line and expanded tables (weighted rank): wider batches, 24 / 30 /
    // 32 indices per round trip (k = 15 rescans 5.17 -> 3.19 ms in-process,
    // 16 reads 3.44; profiles/r5/ab/ab_lane_gw.txt)
#define KS_LANE_W(J, W)                                                                                           \
  hipLaunchKernelGGL((k_scan_lane<J, false, W>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, sq, seq, \
                     total, ra, rb, rs, n, k, tv, mw, min_score, visits, out, d_cnt, segcap, packed)
    if (J == 2) KS_LANE_W(2, 12);
    else if (J == 3) KS_LANE_W(3, 10);
    else KS_LANE_W(4, 8);
#undef KS_LANE_W
  } else {
    if (J == 5) KS_LANE(5, false); else if (J == 4) KS_LANE(4, false); else if (J == 3) KS_LANE(3, false); else if (J == 2) KS_LANE(2, false); else KS_LANE(1, false);
  }
#undef KS_LANE
  KS_HIP(hipGetLastError());
  return KS_OK;
}

static ks_status scan_core(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, const ks_table *t,
                           int32_t min_width, double min_score, int32_t *visits_dev, ks_regions *out,
                           ks_scan_stats *stats, const ScanMode &mode) {
  hipStream_t st = ctx->stream;
  ks_scan_stats local{};
  ks_scan_stats *S = stats ? stats : &local;
  *S = ks_scan_stats{};
  KS_HIP(hipEventRecord(ctx->ev[2], st));
  Runs runs;
  // (no timing sync here: the run phase's events are read after the call's last sync)
  KS_TRY(find_runs(ctx, s, total, &runs, nullptr, /*want_packed=*/true));
  // chunk layout, statistics and algorithm choice (device-side, one sync)
  RunLayout lay;
  if (runs.n) KS_TRY(run_layout(ctx, runs, k, &lay, mode.trlr, s->offsets_dev));
  const int64_t longest = lay.longest, scored = lay.scored;
  S->n_scored = scored;
  S->n_runs = lay.nscan;
  for (int32_t q = 0; q < s->nseq; ++q) {
    const int64_t L = s->offsets_host[q + 1] - s->offsets_host[q];
    if (L >= k) S->n_bases += L;
  }

  // a line table serves pass 1 only (k_pass1l); the other gathers read the
  // base table (ext = nullptr, J = 1)
  const bool line = t->line_kind != 0;
  TableView tv{t->d_vals,  t->d_codes,   t->d_lut,     t->compressed ? 1 : 0, line ? nullptr : t->d_ext,
               line ? 1 : t->ext_J, (int)t->distinct, t->ext_bits, t->d_lut12, t->d_map12, t->d_approx, t->approx_k,
               line ? static_cast<const uint8_t *>(t->d_ext) : nullptr, t->line_kind, t->line_own,
               t->int_exact ? 1 : 0};
  if (t->d_rlines) {  // (weighted-rank code lines: pass 1 only, k_pass1r)
    tv.rline = static_cast<const uint8_t *>(t->d_rlines);
    tv.rpc = t->d_rpieces;
    tv.nrpc = t->n_rpieces;
    tv.rthr = t->thr;
  }
  const uint64_t mw = (uint64_t)(int64_t)min_width;
  int algo = ctx->scan_algo;
  if (algo < 0) algo = (longest > (1 << 15)) ? 1 : 0;
  if (mode.trlr && !(mode.finite && mode.maxabs * (double)(longest + 2) < 1e300)) algo = 0;  // literal NaN rules
  S->scan_algo = algo;

  // region capacity: what the (grow-only) slot already holds, so that the
  // slot is not reallocated on every call; kSegs segments of segcap slots
  const size_t reg_bytes = ctx->slots[SLOT_REGIONS].bytes;
  int64_t segcap = std::max<int64_t>(std::max<int64_t>(65536, scored / 2048),
                                     reg_bytes > 64 ? (int64_t)((reg_bytes - 64) / 28) : 0) / kSegs;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_rcount = reinterpret_cast<unsigned long long *>(scal) + kScRegions;  // [kSegs]
  std::vector<unsigned long long> hcnt(kSegs, 0);
  auto read_counts = [&]() -> ks_status {  // -> hcnt (sync), or the copy the chunked scan made
    if (ctx->hreg_ok) {
      ctx->hreg_ok = false;
      std::copy(ctx->hreg, ctx->hreg + kSegs, hcnt.begin());
      return KS_OK;
    }
    KS_HIP(hipMemcpyAsync(hcnt.data(), d_rcount, 8 * kSegs, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
    return KS_OK;
  };
  auto max_count = [&]() {
    unsigned long long m = 0;
    for (auto c : hcnt) m = std::max(m, c);
    return (int64_t)m;
  };
  RegionBuf rb{};
  uint32_t *vis = reinterpret_cast<uint32_t *>(visits_dev);
  bool complete = false;
  for (int attempt = 0; attempt < 4 && !complete; ++attempt) {
    const int64_t cap = segcap * kSegs;
    void *rp = nullptr;
    KS_TRY(ensure(ctx, SLOT_REGIONS, (size_t)cap * 28 + 64, &rp));
    rb.beg = reinterpret_cast<int64_t *>(rp);
    rb.end = rb.beg + cap;
    rb.score = reinterpret_cast<double *>(rb.end + cap);
    rb.seq = reinterpret_cast<int32_t *>(rb.score + cap);
    rb.count = d_rcount;
    rb.cap = cap;
    rb.segcap = segcap;
    KS_HIP(hipMemsetAsync(d_rcount, 0, 8 * kSegs, st));
    ctx->hreg_ok = false;
    KS_HIP(hipEventRecord(ctx->ev[3], st));
    if (algo == 1) {
      // visits of the chunked path go to a scratch histogram first, so that a
      // fallback to the lane kernel cannot count them twice
      uint32_t *vscr = nullptr;
      const size_t nb = (size_t)4 << (2 * k);
      if (vis) {
        void *vp = nullptr;
        KS_TRY(ensure(ctx, SLOT_TABLE_TMP, nb, &vp));
        vscr = static_cast<uint32_t *>(vp);
        KS_HIP(hipMemsetAsync(vscr, 0, nb, st));
      }
      // top-level visits: from the k-mer counts (one partitioned count pass)
      // unless KS_VISITS_ATOMIC is set (one random atomic per scanned index in
      // pass 1, the former path, kept for A/B runs and tests)
      const bool vis_atomic = getenv("KS_VISITS_ATOMIC") != nullptr;
      ks_status rc = scan_chunked(ctx, s, runs, lay, k, tv, mw, min_score, vis_atomic ? vscr : nullptr, vscr, rb, S,
                                  mode);
      if (rc == KS_INTERNAL_RETRY) {  // a buffer did not fit: grow, rerun, visits untouched
        KS_TRY(read_counts());
        const int64_t m = max_count();
        if (m > segcap) segcap = m + m / 4 + 64;
        continue;
      }
      if (rc == KS_OK) {
        if (vis) {
          const int64_t n = (int64_t)1 << (2 * k);
          if (!vis_atomic) {
            double words = 0;
            if (mode.visits_counted) {
              // (the caller's count is already in visits_dev)
            } else if (ctx->vis_count_ext) {  // scan_impl adds the count (uint32 wrap-around makes the order free)
              ctx->vis_count_ext_used = true;
            } else {
              KS_TRY(launch_count(ctx, s, total, runs, k, visits_dev, &words));
            }
            if (runs.n > 0) {
              hipLaunchKernelGGL(k_visit_correct, dim3((unsigned)((runs.n + 255) / 256)), dim3(256), 0, st, runs.a,
                                 runs.b, runs.seq, runs.n, s->offsets_dev, s->seq, k, vis);
              KS_HIP(hipGetLastError());
            }
          }
          else if (mode.visits_counted)  // the atomic route counts the top level itself
            KS_HIP(hipMemsetAsync(vis, 0, (size_t)n * 4, st));
          hipLaunchKernelGGL(k_add_hist, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, st,
                             vis, vscr, n);
          KS_HIP(hipGetLastError());
        }
      } else if (rc == KS_ERR_INTERNAL) {
        fprintf(stderr, "kmer_spans_amd: chunked scan fell back to the lane kernel: %s\n", ks_last_error());
        ctx->hreg_ok = false;  // the lane kernel recounts the regions
        algo = 0;
        S->scan_algo = 0;
        KS_HIP(hipMemsetAsync(d_rcount, 0, 8 * kSegs, st));
      } else {
        return rc;
      }
    }
    if (algo == 0) {
      if (vis && mode.visits_counted)  // the lane kernel counts every visit itself
        KS_HIP(hipMemsetAsync(vis, 0, (size_t)4 << (2 * k), st));
      if (runs.n)
        KS_TRY(launch_scan_lane(ctx, s->seq, total, runs.a, runs.b, runs.seq, runs.n, k, tv, mw, min_score, vis, rb,
                                nullptr, 0, mode, 1, s->offsets_dev, runs.packed));
    }
    KS_HIP(hipEventRecord(ctx->ev[4], st));
    KS_TRY(read_counts());
    if (algo == 0) {  // (the chunked scan times itself; its counters came without a sync here)
      float ms = 0;
      KS_HIP(hipEventSynchronize(ctx->ev[4]));
      KS_HIP(hipEventElapsedTime(&ms, ctx->ev[3], ctx->ev[4]));
      S->ms_scan = ms;
    }
    const int64_t m = max_count();
    if (m <= segcap) {
      complete = true;
      break;
    }
    segcap = m + m / 4 + 64;
    vis = nullptr;  // visits were complete on the first pass
  }
  if (!complete) return fail(KS_ERR_INTERNAL, "region buffer overflow");

  // Order regions by global begin == (seq_id, beg) on the device (radix sort),
  // convert to sequence-local coordinates, copy out.
  KS_HIP(hipEventRecord(ctx->ev[5], st));
  SegPrefix pre;
  pre.p[0] = 0;
  for (int q = 0; q < kSegs; ++q) pre.p[q + 1] = pre.p[q] + (int64_t)hcnt[q];
  pre.segcap = segcap;
  const int64_t n = pre.p[kSegs];
  out->n = n;
  // one block (ks_regions_free frees seq_id): [seq_id | beg | end] int32 (a
  // 3 x n matrix, the layout of the reference's `pos`), then [score | 0.0]
  // doubles (2 x n, `score`'s layout with the reference's second row, :280)
  // (allocated while the device orders the regions)
  auto alloc_out = [&]() -> ks_status { return regions_alloc(out, n); };
  if (n > 0) {
    void *tmpb = nullptr;
    const size_t nn = (size_t)n;
    KS_TRY(ensure(ctx, SLOT_REG_TMP, nn * (8 + 8 + 4 + 4) + nn * 20 + 1024, &tmpb));
    unsigned long long *k_in = static_cast<unsigned long long *>(tmpb);
    unsigned long long *k_out = k_in + nn;
    int32_t *v_in = reinterpret_cast<int32_t *>(k_out + nn);
    int32_t *v_out = v_in + nn;
    int32_t *o_seq = v_out + nn;
    int32_t *o_beg = o_seq + nn;
    int32_t *o_end = o_beg + nn;
    double *o_score = reinterpret_cast<double *>((reinterpret_cast<uintptr_t>(o_end + nn) + 7) & ~(uintptr_t)7);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_region_keys, dim3(g), dim3(256), 0, st, rb.beg, n, pre, k_in, v_in);
    KS_HIP(hipGetLastError());
    int end_bit = 1;
    while (end_bit < 64 && ((unsigned long long)total >> end_bit)) ++end_bit;
    size_t tb = 0;
    KS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k_in, k_out, v_in, v_out, (int)n, 0, end_bit, st));
    void *tmp = nullptr;
    KS_TRY(ensure(ctx, SLOT_SORT_TMP, tb, &tmp));
    KS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k_in, k_out, v_in, v_out, (int)n, 0, end_bit, st));
    hipLaunchKernelGGL(k_region_gather, dim3(g), dim3(256), 0, st, rb, v_out, n, s->offsets_dev, mode.trlr, o_seq, o_beg,
                       o_end, o_score);
    KS_HIP(hipGetLastError());
    // a kept (>= 1 MiB) output block is pinned: the rows go straight into it
    // by DMA (config 3's 1.09 M regions: no 30 MB staging copy on the host);
    // else one D2H of the contiguous [seq | beg | end | score] block into
    // pinned staging, then host copies into the caller-owned arrays
    KS_TRY(alloc_out());
    if (regions_pin(out)) {
      KS_HIP(hipMemcpyAsync(out->seq_id, o_seq, nn * 12, hipMemcpyDeviceToHost, st));  // (the three int32 rows)
      KS_HIP(hipMemcpyAsync(out->score, o_score, nn * 8, hipMemcpyDeviceToHost, st));
      KS_HIP(hipEventRecord(ctx->ev[6], st));
      memset(out->score + nn, 0, nn * 8);  // second row of `score` (overlaps the copies)
      KS_HIP(hipStreamSynchronize(st));
    } else {
      const size_t blk = (size_t)(reinterpret_cast<char *>(o_score + nn) - reinterpret_cast<char *>(o_seq));
      void *hp = nullptr;
      KS_TRY(ensure_pinned(ctx, blk, &hp));
      KS_HIP(hipMemcpyAsync(hp, o_seq, blk, hipMemcpyDeviceToHost, st));
      KS_HIP(hipEventRecord(ctx->ev[6], st));
      memset(out->score + nn, 0, nn * 8);  // second row of `score` (overlaps the device work)
      KS_HIP(hipStreamSynchronize(st));
      const char *h = static_cast<const char *>(hp);
      memcpy(out->seq_id, h, nn * 4);
      memcpy(out->beg, h + (reinterpret_cast<char *>(o_beg) - reinterpret_cast<char *>(o_seq)), nn * 4);
      memcpy(out->end, h + (reinterpret_cast<char *>(o_end) - reinterpret_cast<char *>(o_seq)), nn * 4);
      memcpy(out->score, h + (reinterpret_cast<char *>(o_score) - reinterpret_cast<char *>(o_seq)), nn * 8);
    }
  } else {
    KS_TRY(alloc_out());
    KS_HIP(hipEventRecord(ctx->ev[6], st));
    KS_HIP(hipStreamSynchronize(st));
  }
  S->n_regions = n;
  {
    float ms_runs = 0;
    KS_HIP(hipEventElapsedTime(&ms_runs, ctx->ev[0], ctx->ev[1]));  // (find_runs' events)
    S->ms_runs = ms_runs;
  }
  if (algo == 1) KS_TRY(chunked_phase_times(ctx, S));
  float ms_fin = 0, ms_tot = 0;
  KS_HIP(hipEventElapsedTime(&ms_fin, ctx->ev[5], ctx->ev[6]));
  KS_HIP(hipEventElapsedTime(&ms_tot, ctx->ev[2], ctx->ev[6]));
  S->ms_finish = ms_fin;
  S->ms_total = ms_tot;
  return KS_OK;
}


// Scan of one call.  With the visit histogram on the chunked path, the
// top-level count runs concurrently on the sub-context (below).  (The
// staggered two-part scan of round 4 -- the input cut at a sequence boundary,
// the later part on a context of its own -- measured no gain and is gone:
// DESIGN.md section 6.)
ks_status scan_impl(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, const ks_table *t,
                    int32_t min_width, double min_score, int32_t *visits_dev, ks_regions *out,
                    ks_scan_stats *stats, const ScanMode &mode) {
  {
    // Visits of the one-part chunked scan: the top-level count (the k-mer
    // histogram, ~24 ms at k = 13, streaming + LDS work) runs on the
    // sub-context's stream from a second host thread while the scan's gather
    // pass (random requests) runs here; the count lands in the sub-context's
    // histogram and is added once both are done (the count after the scan on
    // this stream: 42.2 vs 37.3 ms in round 2, retired).
    // Only when the chunked path is certain or likely: forced, or some
    // sequence longer than the lane kernel's limit (a run longer than 2^15
    // needs one); otherwise the lane kernel counts its own visits and a
    // concurrent count would be thrown away.
    int64_t longest_seq = 0;
    for (int32_t q = 0; q < s->nseq; ++q)
      longest_seq = std::max<int64_t>(longest_seq, s->offsets_host[q + 1] - s->offsets_host[q]);
    const bool chunked_likely = ctx->scan_algo == 1 || (ctx->scan_algo < 0 && longest_seq > (1 << 15));
    const bool vis_conc = visits_dev && !mode.trlr && !mode.visits_counted && chunked_likely && total > 0 &&
                          getenv("KS_VISITS_ATOMIC") == nullptr;
    if (!vis_conc) return scan_core(ctx, s, total, k, t, min_width, min_score, visits_dev, out, stats, mode);
    ks_ctx *vsub = nullptr;
    KS_TRY(ctx_sub(ctx, &vsub));
    const size_t nb = (size_t)4 << (2 * k);
    KS_HIP(hipEventRecord(ctx->ev[19], ctx->stream));  // the count starts after the caller's uploads
    KS_HIP(hipStreamWaitEvent(vsub->stream, ctx->ev[19], 0));
    ks_status rc_c = KS_OK;
    std::string err_c;
    void *cbuf = nullptr;
    std::thread th([&] {
      rc_c = activate(vsub);
      if (rc_c == KS_OK) rc_c = ensure(vsub, SLOT_COUNTS, nb, &cbuf);
      if (rc_c == KS_OK && hipMemsetAsync(cbuf, 0, nb, vsub->stream) != hipSuccess)
        rc_c = fail(KS_ERR_DEVICE, "hipMemsetAsync failed");
      double words = 0;
      Runs none;
      if (rc_c == KS_OK) rc_c = launch_count(vsub, s, total, none, k, static_cast<int32_t *>(cbuf), &words);
      if (rc_c != KS_OK) err_c = ks_last_error();  // (thread-local)
    });
    ctx->vis_count_ext = true;
    ctx->vis_count_ext_used = false;
    const ks_status rc = scan_core(ctx, s, total, k, t, min_width, min_score, visits_dev, out, stats, mode);
    ctx->vis_count_ext = false;
    th.join();  // (launch_count ended with a synchronisation of the sub-context's stream)
    if (rc != KS_OK) return rc;
    if (rc_c != KS_OK) {
      ks_regions_free(out);
      set_error("%s", err_c.c_str());
      return rc_c;
    }
    if (ctx->vis_count_ext_used) {  // (a lane-kernel fallback counted every visit itself)
      const int64_t n = (int64_t)1 << (2 * k);
      hipLaunchKernelGGL(k_add_hist, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0,
                         ctx->stream, reinterpret_cast<uint32_t *>(visits_dev), static_cast<const uint32_t *>(cbuf), n);
      KS_HIP(hipGetLastError());
      KS_HIP(hipStreamSynchronize(ctx->stream));
    }
    return KS_OK;
  }
}

}  // namespace ks
