// ks_scan_common.h -- device helpers shared by the scan kernels.
#pragma once
#include "ks_internal.h"

namespace ks {

// Read-only view of a device score table: s = w[code] - thr (bitwise as the
// reference computes it, kmer_spans.c:268), either a full FP64 table or a
// uint16 code table + FP64 LUT of the distinct values.
struct TableView {
  const double *vals;
  const uint16_t *codes;
  const double *lut;
  int compressed;
  const void *ext;  // expanded table (see ks_table), nullptr if absent
  int ext_J;
};

__device__ __forceinline__ double tv_get(const TableView &t, uint32_t code) {
  return t.compressed ? t.lut[t.codes[code]] : t.vals[code];
}

// Append one region record (global coordinates); drops it (but counts it)
// when the buffer is full so the host can retry with a larger one.
__device__ __forceinline__ void push_region(const RegionBuf &rb, int32_t seq, int64_t beg, int64_t end,
                                            double score) {
  const unsigned long long slot = atomicAdd(rb.count, 1ull);
  if ((int64_t)slot < rb.cap) {
    rb.seq[slot] = seq;
    rb.beg[slot] = beg;
    rb.end[slot] = end;
    rb.score[slot] = score;
  }
}

// Encode the n bases [p, p + n), reading 'N' beyond total (only the bases
// inside the run matter; the rest feed k-mers of indices past the run end).
__device__ __forceinline__ uint32_t prime_code_guarded(const uint8_t *__restrict__ seq, int64_t p, int n,
                                                       int64_t total) {
  uint32_t c = 0;
  for (int j = 0; j < n; ++j) c = (c << 2) | enc(p + j < total ? seq[p + j] : (uint8_t)'N');
  return c;
}

// Encode the k bases [p, p + k) (all non-N, inside one run).
__device__ __forceinline__ uint32_t prime_code(const uint8_t *__restrict__ seq, int64_t p, int k) {
  uint32_t c = 0;
  for (int j = 0; j < k; ++j) c = (c << 2) | enc(seq[p + j]);
  return c;
}

}  // namespace ks
