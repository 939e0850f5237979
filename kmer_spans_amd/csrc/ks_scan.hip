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
#include <algorithm>
#include <numeric>

#include "ks_scan_common.h"

namespace ks {

ks_status scan_chunked(ks_ctx *ctx, const ks_dev_seqs *s, const Runs &runs, int k, const TableView &tv,
                       uint64_t mw, double min_score, uint32_t *visits, const RegionBuf &rb,
                       ks_scan_stats *stats);

namespace {

// Values of a batch of kBatch consecutive scan indices are gathered before
// the sequential state machine consumes them, so a lane keeps kBatch random
// table reads in flight instead of one (the gathers do not depend on S).
constexpr int kBatch = 16;

__global__ void __launch_bounds__(64) k_scan_lane(const uint8_t *__restrict__ seq,
                                                  const int64_t *__restrict__ ra,
                                                  const int64_t *__restrict__ rbnd,
                                                  const int32_t *__restrict__ rseq, int64_t nruns,
                                                  int k, TableView tv, uint64_t mw, double min_score,
                                                  uint32_t *__restrict__ visits, RegionBuf out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  const int64_t a = ra[r], b = rbnd[r];
  if (b - a <= k) return;
  const int32_t sid = rseq[r];
  const uint32_t mask = (1u << (2 * k)) - 1u;
  int64_t i = a;  // priming point
  for (;;) {
    uint32_t code = prime_code(seq, i, k);  // k-mer scored at index i + k
    double S = 0.0, prev = 0.0, best = 0.0;
    int64_t beg = 0, arg = 0;
    bool restart = false;
    for (int64_t p0 = i + k; p0 < b && !restart; p0 += kBatch) {
      const int n = (int)((b - p0) < kBatch ? (b - p0) : kBatch);
      double v[kBatch];
      uint32_t c[kBatch];
      uint32_t cc = code;
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        c[j] = cc;
        if (j < n) v[j] = tv_get(tv, cc);
        if (j < n) cc = ((cc << 2) | enc(seq[p0 + j])) & mask;
      }
      code = cc;
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {  // fully unrolled: v[]/c[] stay in registers
        if (j < n && !restart) {
          const int64_t p = p0 + j;
          if (visits) atomicAdd(&visits[c[j]], 1u);
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

__global__ void k_add_hist(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

}  // namespace

ks_status launch_scan_lane(ks_ctx *ctx, const uint8_t *seq, const int64_t *ra, const int64_t *rb,
                           const int32_t *rs, int64_t n, int k, const TableView &tv, uint64_t mw,
                           double min_score, uint32_t *visits, const RegionBuf &out) {
  if (n <= 0) return KS_OK;
  hipLaunchKernelGGL(k_scan_lane, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, ctx->stream, seq, ra, rb, rs, n, k,
                     tv, mw, min_score, visits, out);
  KS_HIP(hipGetLastError());
  return KS_OK;
}

ks_status scan_impl(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, const ks_table *t,
                    int32_t min_width, double min_score, int32_t *visits_dev, ks_regions *out,
                    ks_scan_stats *stats) {
  hipStream_t st = ctx->stream;
  ks_scan_stats local{};
  ks_scan_stats *S = stats ? stats : &local;
  *S = ks_scan_stats{};
  KS_HIP(hipEventRecord(ctx->ev[2], st));
  Runs runs;
  float ms_runs = 0;
  KS_TRY(find_runs(ctx, s, total, &runs, &ms_runs));
  S->ms_runs = ms_runs;
  // host view of runs for statistics and algorithm choice
  std::vector<int64_t> ha(runs.n), hb(runs.n);
  if (runs.n) {
    KS_HIP(hipMemcpyAsync(ha.data(), runs.a, runs.n * 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipMemcpyAsync(hb.data(), runs.b, runs.n * 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
  }
  int64_t longest = 0, scored = 0, nscan = 0;
  for (int64_t r = 0; r < runs.n; ++r) {
    const int64_t L = hb[r] - ha[r];
    if (L > k) { scored += L - k; ++nscan; longest = std::max(longest, L); }
  }
  S->n_scored = scored;
  S->n_runs = nscan;
  for (int32_t q = 0; q < s->nseq; ++q) {
    const int64_t L = s->offsets_host[q + 1] - s->offsets_host[q];
    if (L >= k) S->n_bases += L;
  }

  TableView tv{t->d_vals, t->d_codes, t->d_lut, t->compressed ? 1 : 0, t->d_ext, t->ext_J};
  const uint64_t mw = (uint64_t)(int64_t)min_width;
  int algo = ctx->scan_algo;
  if (algo < 0) algo = (longest > (1 << 15)) ? 1 : 0;
  S->scan_algo = algo;

  int64_t cap = std::max<int64_t>(4096, (int64_t)(ctx->slots[SLOT_REGIONS].bytes / 28));
  unsigned long long n_reg = 0;
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_rcount = reinterpret_cast<unsigned long long *>(scal) + 2;
  RegionBuf rb{};
  uint32_t *vis = reinterpret_cast<uint32_t *>(visits_dev);
  for (int attempt = 0; attempt < 3; ++attempt) {
    void *rp = nullptr;
    KS_TRY(ensure(ctx, SLOT_REGIONS, (size_t)cap * 28 + 64, &rp));
    rb.beg = reinterpret_cast<int64_t *>(rp);
    rb.end = rb.beg + cap;
    rb.score = reinterpret_cast<double *>(rb.end + cap);
    rb.seq = reinterpret_cast<int32_t *>(rb.score + cap);
    rb.count = d_rcount;
    rb.cap = cap;
    KS_HIP(hipMemsetAsync(d_rcount, 0, 8, st));
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
      ks_status rc = scan_chunked(ctx, s, runs, k, tv, mw, min_score, vscr, rb, S);
      if (rc == KS_OK) {
        if (vis) {
          const int64_t n = (int64_t)1 << (2 * k);
          hipLaunchKernelGGL(k_add_hist, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)), dim3(256), 0, st,
                             vis, vscr, n);
          KS_HIP(hipGetLastError());
        }
      } else if (rc == KS_ERR_INTERNAL) {
        fprintf(stderr, "kmer_spans_amd: chunked scan fell back to the lane kernel: %s\n", ks_last_error());
        algo = 0;
        S->scan_algo = 0;
        KS_HIP(hipMemsetAsync(d_rcount, 0, 8, st));
      } else {
        return rc;
      }
    }
    if (algo == 0) {
      if (runs.n) KS_TRY(launch_scan_lane(ctx, s->seq, runs.a, runs.b, runs.seq, runs.n, k, tv, mw, min_score, vis, rb));
    }
    KS_HIP(hipEventRecord(ctx->ev[4], st));
    KS_HIP(hipMemcpyAsync(&n_reg, d_rcount, 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
    float ms = 0;
    KS_HIP(hipEventElapsedTime(&ms, ctx->ev[3], ctx->ev[4]));
    if (algo == 0) S->ms_scan = ms;
    if ((int64_t)n_reg <= cap) break;
    cap = (int64_t)n_reg + 1024;
    vis = nullptr;  // visits were complete on the first pass
  }
  if ((int64_t)n_reg > cap) return fail(KS_ERR_INTERNAL, "region buffer overflow");

  // Order regions by global begin == (seq_id, beg); convert to local coords.
  KS_HIP(hipEventRecord(ctx->ev[5], st));
  const int64_t n = (int64_t)n_reg;
  std::vector<int64_t> gb(n), ge(n);
  std::vector<double> sc(n);
  std::vector<int32_t> sq(n);
  if (n) {
    KS_HIP(hipMemcpyAsync(gb.data(), rb.beg, n * 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipMemcpyAsync(ge.data(), rb.end, n * 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipMemcpyAsync(sc.data(), rb.score, n * 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipMemcpyAsync(sq.data(), rb.seq, n * 4, hipMemcpyDeviceToHost, st));
  }
  KS_HIP(hipEventRecord(ctx->ev[6], st));
  KS_HIP(hipStreamSynchronize(st));
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return gb[x] < gb[y]; });
  out->n = n;
  out->seq_id = (int32_t *)malloc(std::max<int64_t>(n, 1) * 4);
  out->beg = (int32_t *)malloc(std::max<int64_t>(n, 1) * 4);
  out->end = (int32_t *)malloc(std::max<int64_t>(n, 1) * 4);
  out->score = (double *)malloc(std::max<int64_t>(n, 1) * 8);
  if (!out->seq_id || !out->beg || !out->end || !out->score) {
    ks_regions_free(out);
    return fail(KS_ERR_NOMEM, "out of host memory for %lld regions", (long long)n);
  }
  for (int64_t j = 0; j < n; ++j) {
    const int64_t o = order[j];
    const int64_t base = s->offsets_host[sq[o]];
    out->seq_id[j] = sq[o];
    out->beg[j] = (int32_t)(gb[o] - base);
    out->end[j] = (int32_t)(ge[o] - base);
    out->score[j] = sc[o];
  }
  S->n_regions = n;
  float ms_fin = 0, ms_tot = 0;
  KS_HIP(hipEventElapsedTime(&ms_fin, ctx->ev[5], ctx->ev[6]));
  KS_HIP(hipEventElapsedTime(&ms_tot, ctx->ev[2], ctx->ev[6]));
  S->ms_finish = ms_fin;
  S->ms_total = ms_tot;
  return KS_OK;
}

}  // namespace ks
