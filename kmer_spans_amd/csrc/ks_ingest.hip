// ks_ingest.hip -- FASTA parsing on the device.
//
// The reference reads sequence files with Biostrings::readDNAStringSet in
// kmers.to.file (kmer_spans.R:127-160) and hands the strings to kmer_counts.
// Here the raw file bytes are copied to HBM unparsed and three byte-parallel
// passes turn them into the ks_dev_seqs layout every scan consumes (one
// contiguous buffer + record offsets), so the host does no per-byte work:
//
//   A  k_fa_lastnl   per 4096-byte tile: position of its last '\n'
//      (device max-scan over tiles: the last line break before each tile)
//   B  k_fa_tile<0>  classify every byte by the first byte of its line
//      ('>' description, ';' comment, else sequence), count kept bytes and
//      description lines per tile, record the first invalid byte
//      (device exclusive sums: output base and record base per tile)
//   C  k_fa_tile<1>  same classification, write the kept bytes upper-cased
//      and, per description line, the record's output offset and the
//      line's byte position (for the names)
//
// Line rules (Biostrings' FASTA reader as documented; no fixture pins them,
// DESIGN.md section 6b): a line ends at '\n', one '\r' before it (or before
// EOF) is dropped, empty lines are skipped, ';' lines are comments, sequence
// bytes must be IUPAC DNA letters (either case) or '-', '+', '.'; anything
// else, or sequence before the first description line, is an error.  The
// kept bytes are upper-cased as as.character(DNAStringSet) returns them (the
// scan's encoding is case-blind either way, kmer_spans.c:34-35).
//
// A fourth kernel (k_fa_select) drops records shorter than min_len
// (kmer_spans.R:141) by a record-indexed gather.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr int kFT = 4096;  // bytes per tile
constexpr int kFPer = 16;  // bytes per thread
constexpr int kFThreads = kFT / kFPer;

// Biostrings DNA_ALPHABET: A C G T M R W S Y K V H D B N - + . (letters in
// either case).  256-bit set.
struct Alphabet {
  uint32_t w[8];
};
constexpr Alphabet make_alphabet() {
  Alphabet a{};
  const char *s = "ACGTMRWSYKVHDBNacgtmrwsykvhdbn-+.";
  for (int i = 0; s[i]; ++i) a.w[(uint8_t)s[i] >> 5] |= 1u << ((uint8_t)s[i] & 31);
  return a;
}
__constant__ Alphabet c_alpha = make_alphabet();

__device__ __forceinline__ bool valid_byte(uint8_t c) { return (c_alpha.w[c >> 5] >> (c & 31)) & 1u; }

// 16 bytes starting at p (zero beyond n) and the byte after them.
__device__ __forceinline__ void load16(const uint8_t *__restrict__ raw, int64_t n, int64_t p, uint8_t b[kFPer + 1]) {
  if (p + kFPer + 1 <= n) {
    const uint4 v = *reinterpret_cast<const uint4 *>(raw + p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < kFPer; ++j) b[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    b[kFPer] = raw[p + kFPer];
  } else {
#pragma unroll
    for (int j = 0; j <= kFPer; ++j) b[j] = (p + j < n) ? raw[p + j] : (uint8_t)0;
  }
}

template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, Op op) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d, 64);
    if ((int)(threadIdx.x & 63) >= d) v = op(v, o);
  }
  return v;
}

// Exclusive block scan (256 threads, 4 waves); ident is the identity of op.
template <typename T, typename Op>
__device__ __forceinline__ T block_excl_scan(T v, T ident, Op op, T *lds4, T *total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const T inc = wave_incl_scan(v, op);
  if (lane == 63) lds4[wave] = inc;
  __syncthreads();
  T before = ident;
  for (int w = 0; w < wave; ++w) before = op(before, lds4[w]);
  T all = ident;
  for (int w = 0; w < kFThreads / 64; ++w) all = op(all, lds4[w]);
  __syncthreads();
  T ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = ident;
  *total = all;
  return op(before, ex);
}

struct MaxOp {
  __device__ __forceinline__ int64_t operator()(int64_t a, int64_t b) const { return a > b ? a : b; }
};
struct SumOp {
  __device__ __forceinline__ int64_t operator()(int64_t a, int64_t b) const { return a + b; }
};

__global__ void __launch_bounds__(kFThreads) k_fa_lastnl(const uint8_t *__restrict__ raw, int64_t n,
                                                         int64_t *__restrict__ lastnl) {
  __shared__ int64_t lds4[4];
  const int64_t p0 = (int64_t)blockIdx.x * kFT + (int64_t)threadIdx.x * kFPer;
  uint8_t b[kFPer + 1];
  load16(raw, n, p0, b);
  int64_t m = -1;
#pragma unroll
  for (int j = 0; j < kFPer; ++j)
    if (b[j] == '\n' && p0 + j < n) m = p0 + j;
  int64_t all;
  (void)block_excl_scan<int64_t>(m, (int64_t)-1, MaxOp(), lds4, &all);
  if (threadIdx.x == 0) lastnl[blockIdx.x] = all;
}

// err[0] = first invalid byte, err[1] = first kept byte, err[2] = first
// description line (all atomicMin over positions; n = none).
template <int kEmit>
__global__ void __launch_bounds__(kFThreads) k_fa_tile(
    const uint8_t *__restrict__ raw, int64_t n, const int64_t *__restrict__ nl_incl,
    int64_t *__restrict__ kept_tile, int64_t *__restrict__ hdr_tile, unsigned long long *__restrict__ err,
    const int64_t *__restrict__ kept_base, const int64_t *__restrict__ hdr_base, uint8_t *__restrict__ out,
    int64_t *__restrict__ rec_out, int64_t *__restrict__ rec_pos) {
  __shared__ int64_t lds4[4];
  const int64_t t = blockIdx.x;
  const int64_t p0 = t * kFT + (int64_t)threadIdx.x * kFPer;
  uint8_t b[kFPer + 1];
  load16(raw, n, p0, b);
  int64_t mynl = -1;
#pragma unroll
  for (int j = 0; j < kFPer; ++j)
    if (b[j] == '\n' && p0 + j < n) mynl = p0 + j;
  int64_t dummy;
  int64_t before = block_excl_scan<int64_t>(mynl, (int64_t)-1, MaxOp(), lds4, &dummy);
  const int64_t incoming = t > 0 ? nl_incl[t - 1] : -1;
  if (incoming > before) before = incoming;
  // class of the line holding byte p0: 0 sequence, 1 skipped (description
  // or comment); a line starting at p0 is classified in the loop.
  int cls = 0;
  int64_t ls = before + 1;
  if (ls < p0 && ls < n) {
    const uint8_t c0 = raw[ls];
    cls = (c0 == '>' || c0 == ';') ? 1 : 0;
  }
  int nkeep = 0, nhdr = 0;
  int64_t bad = -1, firstk = -1, firsth = -1;
  uint32_t keepmask = 0;
#pragma unroll
  for (int j = 0; j < kFPer; ++j) {
    const int64_t p = p0 + j;
    if (p < n) {
      const uint8_t c = b[j];
      if (p == ls) {
        cls = (c == '>' || c == ';') ? 1 : 0;
        if (c == '>') {
          ++nhdr;
          if (firsth < 0) firsth = p;
        }
      }
      bool keep = false;
      if (c == '\n') {
        ls = p + 1;
      } else if (cls == 0) {
        keep = !(c == '\r' && (p + 1 == n || b[j + 1] == '\n'));
      }
      if (keep) {
        keepmask |= 1u << j;
        ++nkeep;
        if (firstk < 0) firstk = p;
        if (!valid_byte(c) && bad < 0) bad = p;
      }
    }
  }
  int64_t ktot, htot;
  const int64_t kex = block_excl_scan<int64_t>(nkeep, 0, SumOp(), lds4, &ktot);
  const int64_t hex = block_excl_scan<int64_t>(nhdr, 0, SumOp(), lds4, &htot);
  if (!kEmit) {
    // block minima first; one atomic per block, and only when it can lower
    // the current value (after the first tiles, none do)
    unsigned long long m[3] = {(unsigned long long)bad, (unsigned long long)firstk, (unsigned long long)firsth};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(m[i], d, 64);
        m[i] = o < m[i] ? o : m[i];
      }
    }
    __shared__ unsigned long long wmin[3][kFThreads / 64];
    if ((threadIdx.x & 63) == 0)
      for (int i = 0; i < 3; ++i) wmin[i][threadIdx.x >> 6] = m[i];
    __syncthreads();
    if (threadIdx.x < 3) {
      unsigned long long v = wmin[threadIdx.x][0];
      for (int w = 1; w < kFThreads / 64; ++w) v = wmin[threadIdx.x][w] < v ? wmin[threadIdx.x][w] : v;
      if (v != ~0ull && v < __hip_atomic_load(&err[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(&err[threadIdx.x], v);
    }
    if (threadIdx.x == 0) {
      kept_tile[t] = ktot;
      hdr_tile[t] = htot;
    }
    return;
  }
  int64_t o = kept_base[t] + kex;
  int64_t r = hdr_base[t] + hex;
  // replay the line starts to find description lines (ls restarts from the
  // value before this thread's bytes)
  int64_t ls2 = before + 1;
#pragma unroll
  for (int j = 0; j < kFPer; ++j) {
    const int64_t p = p0 + j;
    if (p < n) {
      const uint8_t c = b[j];
      if (p == ls2 && c == '>') {
        rec_out[r] = o;
        rec_pos[r] = p;
        ++r;
      }
      if (c == '\n') ls2 = p + 1;
      if ((keepmask >> j) & 1u) out[o++] = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    }
  }
}

// Gather the kept records: dst[new_off[i] + x] = src[src_off[i] + x].
__global__ void __launch_bounds__(256) k_fa_select(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                   const int64_t *__restrict__ src_off,
                                                   const int64_t *__restrict__ new_off, int32_t nkeep,
                                                   int64_t total) {
  const int64_t p0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * kFPer;
  if (p0 >= total) return;
  int lo = 0, hi = nkeep - 1;  // last record with new_off <= p0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (new_off[mid] <= p0) lo = mid; else hi = mid - 1;
  }
  int rec = lo;
  for (int j = 0; j < kFPer; ++j) {
    const int64_t p = p0 + j;
    if (p >= total) break;
    while (p >= new_off[rec + 1]) ++rec;
    dst[p] = src[src_off[rec] + (p - new_off[rec])];
  }
}

}  // namespace

ks_status fasta_parse_dev(ks_ctx *ctx, const uint8_t *raw, int64_t n, FastaParse *fp) {
  hipStream_t st = ctx->stream;
  fp->n_records = 0;
  fp->total = 0;
  fp->err_pos = -1;
  fp->first_kept = -1;
  fp->first_hdr = -1;
  fp->out = nullptr;
  fp->offsets.assign(1, 0);
  fp->hdr_pos.clear();
  const int64_t nt = (n + kFT - 1) / kFT;
  if (nt == 0) return KS_OK;
  // scratch: 6 int64 per tile + 3 error words
  void *scr = nullptr;
  KS_TRY(ensure(ctx, SLOT_EVENTS, (size_t)nt * 6 * 8 + 64, &scr));
  int64_t *lastnl = static_cast<int64_t *>(scr);
  int64_t *incl = lastnl + nt;
  int64_t *kept = incl + nt;
  int64_t *hdr = kept + nt;
  int64_t *kbase = hdr + nt;
  int64_t *hbase = kbase + nt;
  unsigned long long *err = reinterpret_cast<unsigned long long *>(hbase + nt);
  KS_HIP(hipMemsetAsync(err, 0xff, 3 * 8, st));
  hipLaunchKernelGGL(k_fa_lastnl, dim3((unsigned)nt), dim3(kFThreads), 0, st, raw, n, lastnl);
  KS_HIP(hipGetLastError());
  size_t tb = 0, tb2 = 0, tb3 = 0;
  KS_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, lastnl, incl, hipcub::Max(), (int)nt, st));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, kept, kbase, (int)nt, st));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, hdr, hbase, (int)nt, st));
  tb = std::max(tb, std::max(tb2, tb3));
  void *tmp = nullptr;
  KS_TRY(ensure(ctx, SLOT_SORT_TMP, tb, &tmp));
  KS_HIP(hipcub::DeviceScan::InclusiveScan(tmp, tb, lastnl, incl, hipcub::Max(), (int)nt, st));
  hipLaunchKernelGGL(k_fa_tile<0>, dim3((unsigned)nt), dim3(kFThreads), 0, st, raw, n, incl, kept, hdr, err,
                     nullptr, nullptr, nullptr, nullptr, nullptr);
  KS_HIP(hipGetLastError());
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, kept, kbase, (int)nt, st));
  KS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, hdr, hbase, (int)nt, st));
  int64_t tail[4];
  unsigned long long e[3];
  KS_HIP(hipMemcpyAsync(&tail[0], kbase + nt - 1, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(&tail[1], kept + nt - 1, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(&tail[2], hbase + nt - 1, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(&tail[3], hdr + nt - 1, 8, hipMemcpyDeviceToHost, st));
  KS_HIP(hipMemcpyAsync(e, err, 24, hipMemcpyDeviceToHost, st));
  KS_HIP(hipStreamSynchronize(st));
  const int64_t total = tail[0] + tail[1], nrec = tail[2] + tail[3];
  auto pos = [&](unsigned long long v) { return v == ~0ull ? (int64_t)-1 : (int64_t)v; };
  fp->err_pos = pos(e[0]);
  fp->first_kept = pos(e[1]);
  fp->first_hdr = pos(e[2]);
  if (fp->err_pos >= 0) return KS_OK;                     // caller reports the byte
  if (fp->first_kept >= 0 && (fp->first_hdr < 0 || fp->first_kept < fp->first_hdr)) return KS_OK;
  if (nrec > INT32_MAX - 1) return fail(KS_ERR_ARG, "too many FASTA records (%lld)", (long long)nrec);
  uint8_t *out = nullptr;
  if (hipMalloc(&out, (size_t)total + 32) != hipSuccess)
    return fail(KS_ERR_NOMEM, "hipMalloc(%lld) for FASTA sequences failed", (long long)total + 32);
  void *recs = nullptr;
  ks_status rc = ensure(ctx, SLOT_WORK_A, (size_t)(nrec + 1) * 16, &recs);
  if (rc != KS_OK) {
    (void)hipFree(out);
    return rc;
  }
  int64_t *rec_out = static_cast<int64_t *>(recs);
  int64_t *rec_pos = rec_out + nrec + 1;
  if (hipMemsetAsync(out + total, 'N', 32, st) != hipSuccess) {
    (void)hipFree(out);
    return fail(KS_ERR_DEVICE, "hipMemsetAsync failed");
  }
  hipLaunchKernelGGL(k_fa_tile<1>, dim3((unsigned)nt), dim3(kFThreads), 0, st, raw, n, incl, kept, hdr, err,
                     kbase, hbase, out, rec_out, rec_pos);
  fp->offsets.assign((size_t)nrec + 1, 0);
  fp->hdr_pos.assign((size_t)nrec, 0);
  hipError_t he = hipGetLastError();
  if (he == hipSuccess && nrec)
    he = hipMemcpyAsync(fp->offsets.data(), rec_out, (size_t)nrec * 8, hipMemcpyDeviceToHost, st);
  if (he == hipSuccess && nrec)
    he = hipMemcpyAsync(fp->hdr_pos.data(), rec_pos, (size_t)nrec * 8, hipMemcpyDeviceToHost, st);
  if (he == hipSuccess) he = hipStreamSynchronize(st);
  if (he != hipSuccess) {
    (void)hipFree(out);
    return fail(KS_ERR_DEVICE, "FASTA parse failed: %s", hipGetErrorString(he));
  }
  fp->offsets[(size_t)nrec] = total;
  fp->n_records = nrec;
  fp->total = total;
  fp->out = out;
  return KS_OK;
}

ks_status fasta_select_dev(ks_ctx *ctx, FastaParse *fp, const std::vector<int32_t> &keep) {
  hipStream_t st = ctx->stream;
  const int32_t nk = (int32_t)keep.size();
  std::vector<int64_t> so((size_t)nk), no((size_t)nk + 1, 0);
  for (int32_t i = 0; i < nk; ++i) {
    so[i] = fp->offsets[keep[i]];
    no[i + 1] = no[i] + (fp->offsets[keep[i] + 1] - fp->offsets[keep[i]]);
  }
  const int64_t total = no[(size_t)nk];
  uint8_t *out = nullptr;
  if (hipMalloc(&out, (size_t)total + 32) != hipSuccess)
    return fail(KS_ERR_NOMEM, "hipMalloc(%lld) for FASTA sequences failed", (long long)total + 32);
  void *d = nullptr;
  ks_status rc = ensure(ctx, SLOT_WORK_B, ((size_t)nk * 2 + 1) * 8, &d);
  hipError_t he = hipSuccess;
  if (rc == KS_OK) {
    int64_t *d_so = static_cast<int64_t *>(d), *d_no = d_so + nk;
    he = hipMemsetAsync(out + total, 'N', 32, st);
    if (he == hipSuccess && nk) he = hipMemcpyAsync(d_so, so.data(), (size_t)nk * 8, hipMemcpyHostToDevice, st);
    if (he == hipSuccess) he = hipMemcpyAsync(d_no, no.data(), ((size_t)nk + 1) * 8, hipMemcpyHostToDevice, st);
    if (he == hipSuccess && total > 0) {
      const int64_t blocks = (total + 256 * kFPer - 1) / (256 * kFPer);
      hipLaunchKernelGGL(k_fa_select, dim3((unsigned)blocks), dim3(256), 0, st, fp->out, out, d_so, d_no, nk, total);
      he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipStreamSynchronize(st);
    if (he != hipSuccess) rc = fail(KS_ERR_DEVICE, "FASTA record selection failed: %s", hipGetErrorString(he));
  }
  if (rc != KS_OK) {
    (void)hipFree(out);
    return rc;
  }
  (void)hipFree(fp->out);
  fp->out = out;
  fp->offsets.swap(no);
  fp->total = total;
  return KS_OK;
}

}  // namespace ks
