// ks_windowed.hip -- windowed k-mer count distributions:
// windowed_kmer_count_distributions (kmer_spans.c:413-449) behind
// windowed_kmer_count_distributions_r (:717-793).
//
// Reference semantics: in every N-free run of a sequence longer than the
// window, each window of `window` consecutive bases [s, s + window) inside
// the run holds the window - k + 1 k-mers ending at s + k - 1 .. s + window - 1.
// For every query k-mer i, dist[i][c] counts the windows in which it occurs
// c times, and (ret_flag & 1) scores[seq][i][s - seq start] = c.
//
// Here: the windows of every run are cut into segments of R consecutive
// window starts; one lane per (segment, group of 16 queries) primes the
// counts over its first window and then slides (one k-mer leaves, one
// enters per step).  Counts change rarely, so the histogram gets one add per
// run of equal counts (LDS-privatised per block when 16 x (window + 1)
// counters fit 64 KiB, global atomics otherwise).
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr int kWG = 16;  // queries per lane
constexpr int kWThreads = 256;

// Window segments per run (0 if the run or its sequence is too short).
__global__ void k_win_segs(const int64_t *__restrict__ ra, const int64_t *__restrict__ rb,
                           const int32_t *__restrict__ rs, const int64_t *__restrict__ offs, int64_t n, int window,
                           int64_t R, int64_t *__restrict__ nseg) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > n) return;
  if (r == n) {
    nseg[n] = 0;
    return;
  }
  const int32_t q = rs[r];
  const int64_t slen = offs[q + 1] - offs[q];
  const int64_t W = rb[r] - ra[r] - window + 1;
  nseg[r] = (slen > window && W > 0) ? (W + R - 1) / R : 0;
}

template <bool kLds, bool kPos>
__global__ void __launch_bounds__(kWThreads) k_window(
    const uint8_t *__restrict__ seq, const int64_t *__restrict__ ra, const int64_t *__restrict__ rb,
    const int32_t *__restrict__ rs, const int64_t *__restrict__ segbase, int64_t nruns, int64_t R, int k, int window,
    const uint32_t *__restrict__ qcodes, int kmer_n, uint32_t *__restrict__ dist, int32_t *__restrict__ pos,
    const int64_t *__restrict__ offs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t h[];  // kLds: [kWG][window + 1]
  const int group = blockIdx.y;
  const int wp1 = window + 1;
  if (kLds) {
    for (int i = threadIdx.x; i < kWG * wp1; i += kWThreads) h[i] = 0;
    __syncthreads();
  }
  const int64_t nseg = segbase[nruns];
  const int64_t seg = (int64_t)blockIdx.x * kWThreads + threadIdx.x;
  uint32_t q[kWG];
#pragma unroll
  for (int g = 0; g < kWG; ++g) q[g] = qcodes[group * kWG + g];
  const int nq = min(kWG, kmer_n - group * kWG);
  if (seg < nseg) {
    int64_t lo = 0, hi = nruns - 1;  // last run with segbase <= seg
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (segbase[mid] <= seg) lo = mid; else hi = mid - 1;
    }
    const int64_t run = lo;
    const int64_t a = ra[run];
    const int64_t W = rb[run] - a - window + 1;
    const int64_t s0 = a + (seg - segbase[run]) * R;
    const int64_t s1 = min(s0 + R, a + W);
    const uint32_t mask = (1u << (2 * k)) - 1u;
    // prime: counts over the k-mers ending at s0 + k - 1 .. s0 + window - 1
    uint32_t cnt[kWG];
#pragma unroll
    for (int g = 0; g < kWG; ++g) cnt[g] = 0;
    uint32_t rcode = 0, lcode = 0;
    for (int64_t p = s0; p < s0 + window; ++p) {
      rcode = ((rcode << 2) | enc(seq[p])) & mask;
      if (p == s0 + k - 1) lcode = rcode;
      if (p >= s0 + k - 1) {
#pragma unroll
        for (int g = 0; g < kWG; ++g) cnt[g] += (rcode == q[g]) ? 1u : 0u;
      }
    }
    uint32_t cur[kWG], len[kWG];
#pragma unroll
    for (int g = 0; g < kWG; ++g) {
      cur[g] = cnt[g];
      len[g] = 0;
    }
    const int32_t sq = rs[run];
    const int64_t sbase = offs[sq], slen = offs[sq + 1] - sbase;
    int32_t *pout = kPos ? pos + (size_t)kmer_n * sbase + (size_t)group * kWG * slen + (s0 - sbase) : nullptr;
    for (int64_t s = s0; s < s1; ++s) {
#pragma unroll
      for (int g = 0; g < kWG; ++g) {
        if (cnt[g] != cur[g]) {
          if (g < nq) {
            if (kLds) atomicAdd(&h[g * wp1 + cur[g]], len[g]);
            else atomicAdd(&dist[(size_t)(group * kWG + g) * wp1 + cur[g]], len[g]);
          }
          cur[g] = cnt[g];
          len[g] = 0;
        }
        ++len[g];
        if (kPos && g < nq) pout[(size_t)g * slen + (s - s0)] = (int32_t)cnt[g];
      }
      if (s + 1 < s1) {
        // the k-mer ending at s + k - 1 leaves, the one ending at s + window enters
        const uint32_t out = lcode;
        lcode = ((lcode << 2) | enc(seq[s + k])) & mask;
        rcode = ((rcode << 2) | enc(seq[s + window])) & mask;
#pragma unroll
        for (int g = 0; g < kWG; ++g) cnt[g] += (uint32_t)(rcode == q[g]) - (uint32_t)(out == q[g]);
      }
    }
#pragma unroll
    for (int g = 0; g < kWG; ++g)
      if (g < nq && len[g]) {
        if (kLds) atomicAdd(&h[g * wp1 + cur[g]], len[g]);
        else atomicAdd(&dist[(size_t)(group * kWG + g) * wp1 + cur[g]], len[g]);
      }
  }
  if (kLds) {
    __syncthreads();
    for (int i = threadIdx.x; i < nq * wp1; i += kWThreads) {
      const uint32_t v = h[i];
      if (v) atomicAdd(&dist[(size_t)group * kWG * wp1 + i], v);
    }
  }
}

__global__ void k_seq_included(const int64_t *__restrict__ offs, int32_t nseq, int window, int32_t *__restrict__ inc) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nseq) inc[q] = (offs[q + 1] - offs[q]) > window ? 1 : 0;
}

}  // namespace

ks_status windowed_impl(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const uint32_t *qcodes_host, int kmer_n,
                        int k, int window, int32_t *dist_dev, int32_t *included_dev, int32_t *pos_dev) {
  hipStream_t st = ctx->stream;
  if (included_dev && s->nseq > 0) {
    hipLaunchKernelGGL(k_seq_included, dim3((s->nseq + 255) / 256), dim3(256), 0, st, s->offsets_dev, s->nseq,
                       window, included_dev);
    KS_HIP(hipGetLastError());
  }
  if (kmer_n == 0 || total == 0) return KS_OK;
  Runs runs;
  KS_TRY(find_runs(ctx, s, total, &runs, nullptr));
  if (runs.n == 0) return KS_OK;
  const int ngroups = (kmer_n + kWG - 1) / kWG;
  const int64_t R = std::max<int64_t>(1024, 2 * (int64_t)window);
  void *w = nullptr;
  KS_TRY(ensure(ctx, SLOT_WORK_A, ((size_t)runs.n + 1) * 16 + (size_t)ngroups * kWG * 4 + 64, &w));
  int64_t *nseg = static_cast<int64_t *>(w);
  int64_t *segbase = nseg + runs.n + 1;
  uint32_t *d_q = reinterpret_cast<uint32_t *>(segbase + runs.n + 1);
  std::vector<uint32_t> q((size_t)ngroups * kWG, 0xffffffffu);  // padding never matches a code
  for (int i = 0; i < kmer_n; ++i) q[i] = qcodes_host[i];
  KS_HIP(hipMemcpyAsync(d_q, q.data(), q.size() * 4, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_win_segs, dim3((unsigned)((runs.n + 1 + 255) / 256)), dim3(256), 0, st, runs.a, runs.b,
                     runs.seq, s->offsets_dev, runs.n, window, R, nseg);
  KS_HIP(hipGetLastError());
  size_t tb = 0;
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, nseg, segbase, (int)(runs.n + 1), st));
  void *tmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_SORT_TMP, tb + 16, &tmp));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, nseg, segbase, (int)(runs.n + 1), st));
  int64_t total_seg = 0;
  KS_HIP(hipMemcpyAsync(&total_seg, segbase + runs.n, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  if (total_seg == 0) return KS_OK;
  const size_t lds = (size_t)kWG * (window + 1) * 4;
  const bool use_lds = lds <= 65536;
  const dim3 grid((unsigned)((total_seg + kWThreads - 1) / kWThreads), (unsigned)ngroups);
  if (use_lds) {
    if (pos_dev)
      hipLaunchKernelGGL((k_window<true, true>), grid, dim3(kWThreads), lds, st, s->seq, runs.a, runs.b, runs.seq,
                         segbase, runs.n, R, k, window, d_q, kmer_n, (uint32_t *)dist_dev, pos_dev, s->offsets_dev);
    else
      hipLaunchKernelGGL((k_window<true, false>), grid, dim3(kWThreads), lds, st, s->seq, runs.a, runs.b, runs.seq,
                         segbase, runs.n, R, k, window, d_q, kmer_n, (uint32_t *)dist_dev, nullptr, s->offsets_dev);
  } else {
    if (pos_dev)
      hipLaunchKernelGGL((k_window<false, true>), grid, dim3(kWThreads), 0, st, s->seq, runs.a, runs.b, runs.seq,
                         segbase, runs.n, R, k, window, d_q, kmer_n, (uint32_t *)dist_dev, pos_dev, s->offsets_dev);
    else
      hipLaunchKernelGGL((k_window<false, false>), grid, dim3(kWThreads), 0, st, s->seq, runs.a, runs.b, runs.seq,
                         segbase, runs.n, R, k, window, d_q, kmer_n, (uint32_t *)dist_dev, nullptr, s->offsets_dev);
  }
  KS_HIP(hipGetLastError());
  KS_HIP(hipStreamSynchronize(st));
  return KS_OK;
}

}  // namespace ks
