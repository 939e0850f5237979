// ks_runs.hip -- N-free run segmentation of device-resident sequences.
//
// The reference discovers runs on the fly (skip_n + init_kmer,
// kmer_spans.c:111-132).  Here runs are materialised once per call so that
// counting and scanning can parallelise over them: a run is a maximal
// [a, b) of non-N bytes inside one sequence.  Boundaries are sparse (N gaps,
// sequence ends), so the kernel emits (position, START/END) events with a
// wave-aggregated atomic append and a radix sort restores position order;
// END sorts before START at the same position (sequence boundary between two
// non-N bytes), so the sorted events alternate START, END, START, ...
#include <hipcub/hipcub.hpp>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr int kTile = 4096;        // positions per block
constexpr int kPerThread = 16;     // 256 threads x 16 bytes

__device__ __forceinline__ bool bit_at(const uint32_t *m, int r) { return (m[r >> 5] >> (r & 31)) & 1u; }

// Emits key = (p << 1) | is_start for every run START (first byte) and END
// (one past the last byte) in positions [t0, t0 + kTile) intersect [0, total].
__global__ void __launch_bounds__(256) k_run_events(const uint8_t *__restrict__ seq, int64_t total,
                                                    const int64_t *__restrict__ offs, int32_t nseq,
                                                    unsigned long long *__restrict__ ev,
                                                    unsigned long long *__restrict__ ev_count,
                                                    int64_t cap) {
  __shared__ uint32_t bmask[kTile / 32 + 1];
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  for (int i = threadIdx.x; i < kTile / 32 + 1; i += blockDim.x) bmask[i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {  // sequence boundaries (offsets) falling in this tile
    int lo = 0, hi = nseq + 1;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (offs[mid] < t0) lo = mid + 1; else hi = mid;
    }
    for (int q = lo; q <= nseq && offs[q] < t0 + kTile; ++q) {
      const int r = (int)(offs[q] - t0);
      bmask[r >> 5] |= 1u << (r & 31);
    }
  }
  __syncthreads();

  const int64_t p0 = t0 + (int64_t)threadIdx.x * kPerThread;
  uint8_t b[kPerThread + 1];
  b[0] = (p0 >= 1 && p0 - 1 < total) ? seq[p0 - 1] : (uint8_t)'N';
  if (p0 + kPerThread <= total) {
    const uint4 v = *reinterpret_cast<const uint4 *>(seq + p0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) b[j + 1] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
  } else {
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) b[j + 1] = (p0 + j < total) ? seq[p0 + j] : (uint8_t)'N';
  }
  uint32_t starts = 0, ends = 0;  // bit j: event at p0 + j
  int cnt = 0;
  if (p0 <= total) {
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
      const int64_t p = p0 + j;
      if (p > total) break;
      const bool v = (p < total) && !is_n(b[j + 1]);
      const bool vp = (p >= 1) && !is_n(b[j]);
      const bool bd = bit_at(bmask, (int)(p - t0));
      if (v && (bd || !vp)) { starts |= 1u << j; ++cnt; }
      if (vp && (bd || !v)) { ends |= 1u << j; ++cnt; }
    }
  }
  // wave-aggregated append
  const unsigned long long any = __ballot(cnt > 0);
  if (any == 0) return;
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
  for (int j = 0; j < kPerThread; ++j) {
    const unsigned long long p = (unsigned long long)(p0 + j);
    if ((ends >> j) & 1u) { if ((int64_t)slot < cap) ev[slot] = (p << 1); ++slot; }
    if ((starts >> j) & 1u) { if ((int64_t)slot < cap) ev[slot] = (p << 1) | 1ull; ++slot; }
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

}  // namespace

ks_status find_runs(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, Runs *runs, float *ms) {
  hipStream_t st = ctx->stream;
  KS_HIP(hipEventRecord(ctx->ev[0], st));
  void *scal = nullptr;
  KS_TRY(ensure(ctx, SLOT_SCALARS, 4096, &scal));
  unsigned long long *d_count = reinterpret_cast<unsigned long long *>(scal);
  const int64_t nblocks = (total + 1 + kTile - 1) / kTile;
  int64_t cap = 1 << 20;
  if (ctx->slots[SLOT_EVENTS].bytes / 8 > (size_t)cap) cap = ctx->slots[SLOT_EVENTS].bytes / 8;
  unsigned long long n_ev = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    void *evp = nullptr;
    KS_TRY(ensure(ctx, SLOT_EVENTS, (size_t)cap * 8, &evp));
    KS_HIP(hipMemsetAsync(d_count, 0, 8, st));
    hipLaunchKernelGGL(k_run_events, dim3((unsigned)nblocks), dim3(256), 0, st, s->seq, total,
                       s->offsets_dev, s->nseq, (unsigned long long *)evp, d_count, cap);
    KS_HIP(hipGetLastError());
    KS_HIP(hipMemcpyAsync(&n_ev, d_count, 8, hipMemcpyDeviceToHost, st));
    KS_HIP(hipStreamSynchronize(st));
    if ((int64_t)n_ev <= cap) break;
    cap = (int64_t)n_ev;
  }
  if (n_ev & 1ull) return fail(KS_ERR_INTERNAL, "run segmentation produced an odd event count");
  const int64_t nruns = (int64_t)(n_ev / 2);
  runs->n = nruns;
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
