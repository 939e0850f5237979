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
  int nlut;         // compressed: LUT entries (distinct values)
  int ext_bits;     // 12: J = 5 narrow codes (lut12 / map12, 0xFFF escapes)
  const double *lut12;
  const uint16_t *map12;
  const uint16_t *approx;  // fp16 prefix means (ks_table::d_approx), nullptr if absent
  int approx_k;
  const uint8_t *line;     // line table (ks_table line_kind), nullptr if absent; ext is then nullptr
  int line_kind;           // 1: uint16 codes, 2: FP64 values
  int line_own;
  int exact;               // ks_table::int_exact
  // weighted-rank code lines of pass 1 (ks_table::d_rlines, k_pass1r), nullptr if absent
  const uint8_t *rline = nullptr;
  const unsigned long long *rpc = nullptr;  // pieces: (base bits, increment) pairs, hottest first
  int nrpc = 0;
  double rthr = 0.0;                         // s = R - thr
};

// LUT entries that fit the LDS copy used by the streaming passes (64 KiB).
constexpr int kLdsLutMax = 8192;

__device__ __forceinline__ double tv_get(const TableView &t, uint32_t code) {
  return t.compressed ? t.lut[t.codes[code]] : t.vals[code];
}

// The own + 1 values one line-table read serves (ks_table line_kind; the
// passes after pass 1): the line of the m-mer key >> 2 (m = k + OWN - 1), its
// OWN own entries and the L1 entry of continuation key & 3, from the line's
// first 16-32 B.  key: the (k + OWN)-mer ending at the last index's k-mer.
// s_lut: the LUT in LDS, or nullptr (global).
template <int OWN>
__device__ __forceinline__ void line_entries(const TableView &t, uint64_t key, double lv[OWN + 1],
                                             const double *s_lut) {
  constexpr int JL = OWN + 1;
  const uint8_t *ln = t.line + (size_t)(key >> 2) * (t.line_kind == 3 ? 128 : 64);
  const uint32_t c1 = (uint32_t)key & 3u;
  if (t.line_kind == 2) {  // FP64 values: the own ones in 16-B loads, the L1 one alone
    const double2 *d2 = reinterpret_cast<const double2 *>(ln);
#pragma unroll
    for (int q = 0; q < OWN; q += 2) {
      const double2 e = d2[q >> 1];
      lv[q] = e.x;
      if (q + 1 < OWN) lv[q + 1] = e.y;
    }
    lv[OWN] = reinterpret_cast<const double *>(ln)[OWN + c1];
    return;
  }
  uint32_t cs[JL];
  const uint4 q0 = *reinterpret_cast<const uint4 *>(ln);
  if (t.line_kind == 3) {  // wide: 13-bit own / L1 codes in the first 16 B
    const uint64_t lo = (uint64_t)q0.x | ((uint64_t)q0.y << 32), hi = (uint64_t)q0.z | ((uint64_t)q0.w << 32);
    auto f13 = [&](int b) -> uint32_t {
      const uint64_t w = b < 64 ? ((lo >> b) | (b > 51 ? (hi << (64 - b)) : 0ull)) : (hi >> (b - 64));
      return (uint32_t)w & 0x1fffu;
    };
#pragma unroll
    for (int q = 0; q < OWN; ++q) cs[q] = f13(13 * q);
    const uint32_t l0 = f13(13 * OWN), l1 = f13(13 * (OWN + 1)), l2 = f13(13 * (OWN + 2)), l3 = f13(13 * (OWN + 3));
    cs[OWN] = c1 == 0 ? l0 : (c1 == 1 ? l1 : (c1 == 2 ? l2 : l3));
  } else {  // uint16 codes
    uint32_t h[16];
    h[0] = q0.x & 0xffffu; h[1] = q0.x >> 16; h[2] = q0.y & 0xffffu; h[3] = q0.y >> 16;
    h[4] = q0.z & 0xffffu; h[5] = q0.z >> 16; h[6] = q0.w & 0xffffu; h[7] = q0.w >> 16;
    if (OWN + 4 > 8) {
      const uint4 q1 = *reinterpret_cast<const uint4 *>(ln + 16);
      h[8] = q1.x & 0xffffu; h[9] = q1.x >> 16; h[10] = q1.y & 0xffffu; h[11] = q1.y >> 16;
      h[12] = q1.z & 0xffffu; h[13] = q1.z >> 16; h[14] = q1.w & 0xffffu; h[15] = q1.w >> 16;
    }
#pragma unroll
    for (int q = 0; q < OWN; ++q) cs[q] = h[q];
    cs[OWN] = c1 == 0 ? h[OWN] : (c1 == 1 ? h[OWN + 1] : (c1 == 2 ? h[OWN + 2] : h[OWN + 3]));
  }
#pragma unroll
  for (int q = 0; q < JL; ++q) lv[q] = s_lut ? s_lut[cs[q]] : t.lut[cs[q]];
}

// The J values of one expanded-table read: scan indices served by the
// (k+J-1)-mer `gcode` (J = 1: the base table entry of the k-mer).  J = 5
// (compressed) holds 12-bit codes; 0xFFF escapes to the base table.
template <int J, bool kCompressed, typename GC>
__device__ __forceinline__ void gather_group(const TableView &t, GC gcode, uint32_t kmask, double v[J]) {
  if (J >= 2 && t.line) {  // line table (the dispatch sets J = own + 1): gcode is the (k + own)-mer
    line_entries<(J >= 2 ? J - 1 : 1)>(t, (uint64_t)gcode, v, nullptr);
    return;
  }
  if (J == 1) {
    v[0] = kCompressed ? t.lut[t.codes[gcode]] : t.vals[gcode];
  } else if (kCompressed && J == 5) {
    const uint64_t e = reinterpret_cast<const uint64_t *>(t.ext)[gcode];
#pragma unroll
    for (int q = 0; q < J; ++q) {
      const uint32_t c12 = (uint32_t)(e >> (12 * q)) & 0xfffu;
      v[q] = (c12 != 0xfffu) ? t.lut12[c12] : t.lut[t.codes[(uint32_t)(gcode >> (2 * (J - 1 - q))) & kmask]];
    }
  } else if (kCompressed) {
    const uint64_t e = (J <= 2) ? (uint64_t)reinterpret_cast<const uint32_t *>(t.ext)[gcode]
                                : reinterpret_cast<const uint64_t *>(t.ext)[gcode];
#pragma unroll
    for (int q = 0; q < J; ++q) v[q] = t.lut[(uint16_t)(e >> (16 * q))];
  } else {
    const double2 *E = reinterpret_cast<const double2 *>(t.ext);
    double2 e0, e1 = make_double2(0.0, 0.0);
    if (J <= 2) {
      e0 = E[gcode];
    } else {
      e0 = E[2 * (size_t)gcode];
      e1 = E[2 * (size_t)gcode + 1];
    }
    const double ev[4] = {e0.x, e0.y, e1.x, e1.y};
#pragma unroll
    for (int q = 0; q < J && q < 4; ++q) v[q] = ev[q];
  }
}

// Segment of the append buffers used by the calling wave.
__device__ __forceinline__ int append_seg() {
  return (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kSegs - 1));
}

// Slot for one appended element, or -1 when its segment is full (the
// element is still counted so the host can retry with larger segments).
__device__ __forceinline__ int64_t append_one(unsigned long long *count, int64_t segcap) {
  const int s = append_seg();
  const unsigned long long i = atomicAdd(&count[s], 1ull);
  return (int64_t)i < segcap ? (int64_t)s * segcap + (int64_t)i : -1;
}

// Append one region record (global coordinates).
__device__ __forceinline__ void push_region(const RegionBuf &rb, int32_t seq, int64_t beg, int64_t end,
                                            double score) {
  const int64_t slot = append_one(rb.count, rb.segcap);
  if (slot >= 0) {
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

// 64-bit form for (k+J-1)-mers of up to 32 bases.
__device__ __forceinline__ uint64_t prime_code_guarded64(const uint8_t *__restrict__ seq, int64_t p, int n,
                                                         int64_t total) {
  uint64_t c = 0;
  for (int j = 0; j < n; ++j) c = (c << 2) | enc(p + j < total ? seq[p + j] : (uint8_t)'N');
  return c;
}

// Encode the k bases [p, p + k) (all non-N, inside one run).
__device__ __forceinline__ uint32_t prime_code(const uint8_t *__restrict__ seq, int64_t p, int k) {
  uint32_t c = 0;
  for (int j = 0; j < k; ++j) c = (c << 2) | enc(seq[p + j]);
  return c;
}

// 64 bits of 2-bit base codes from base q0 on (first base most significant),
// read from the packed codes of find_runs (Runs::packed, three words); false
// where those words are past the end of the packed array (callers then roll
// the bytes).
__device__ __forceinline__ bool packed_bits(const uint32_t *__restrict__ packed, int64_t total, int64_t q0,
                                            uint64_t &x) {
  if (!packed || q0 < 0 || (q0 >> 4) + 2 > (total >> 4)) return false;
  const uint32_t *w = packed + (q0 >> 4);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  const uint32_t bp = 2u * (uint32_t)(q0 & 15);
  x = ((((uint64_t)w0 << 32) | w1) << bp) | (((uint64_t)w2 << bp) >> 32);
  return true;
}

}  // namespace ks
