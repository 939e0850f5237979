// ks_kmer_swar.h -- the counted k-mers of one lane's 16 positions, computed
// word-parallel (SWAR) from its 32 bytes instead of a byte-serial walk.
//
// A count lane holds bytes 0..31 = positions p0 - 16 .. p0 + 15 and counts
// the k-mers ending at bytes 16..31 (kmer_spans.c:135-155).  The byte-serial
// form (round 1-6 `lane_kmers`) rolled the 2-bit code and the N-free run
// length byte by byte: ~40 VALU instructions per position in `k_part` and
// ~90 in `k_part_scatter_st` (SQ counters, profiles/r5/rank/
// sq_counters_rank_k13.txt), which made both passes VALU-bound.  Here:
//   codes   enc(c) = (c >> 1) & 3 (UPDATE_OFFSET, :33) of four bytes at once,
//           gathered into 8 bits by one multiply, first base most significant;
//           the code of the k-mer ending at byte 16 + i is a funnel shift of
//           the 64-bit (bytes 0-15 : bytes 16-31) code word (v_alignbit_b32);
//   breaks  N flags ((c | 0x20) == 'n', LC at :34) of four bytes by an exact
//           zero-byte test; sequence starts from the block's start bitmap;
//   windows a k-mer ending at byte j is counted when bytes j-k+1..j hold no N
//           and no sequence starts inside (j-k+1, j] -- both masks "smeared"
//           over the window length by doubling shifts -- except quirk Q1
//           (:142-144): the first window of a run (byte j-k is N, or byte
//           j-k+1 starts its sequence) is dropped when byte j+1 starts the
//           next sequence (the end of the string).
// Host and device (tests/test_swar_kmers.py checks it against the byte walk).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KS_SWAR_FN __host__ __device__ __forceinline__
#else
#define KS_SWAR_FN static inline
#endif

namespace ks {

struct SwarWin {
  uint32_t hi, lo;  // 2-bit codes of bytes 0-15 / 16-31, the earlier byte more significant
  uint32_t emit;    // bit 16 + i: the k-mer ending at byte 16 + i is counted
};

// bit j of the result = OR of x's bits j - L + 1 .. j (L in [0, 16])
KS_SWAR_FN uint32_t swar_smear(uint32_t x, int L) {
  if (L <= 0) return 0u;
  uint32_t r = x;
  int l = 1;
  if (L >= 2) r |= r << 1, l = 2;
  if (L >= 4) r |= r << 2, l = 4;
  if (L >= 8) r |= r << 4, l = 8;
  if (L >= 16) r |= r << 8, l = 16;
  return r | (r << (L - l));
}

// x: the 32 bytes as little-endian words (byte j = bits 8(j%4) of x[j/4]);
// sm: bit j (j = 0..32) set when byte j starts a sequence (0 without starts);
// jend: bytes >= jend lie past the input; k in [1, 15].
KS_SWAR_FN SwarWin swar_window(const uint32_t (&x)[8], uint64_t sm, int jend, int k) {
  SwarWin w;
  w.hi = w.lo = 0;
  uint32_t nm = 0;  // bit j: byte j is N
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t e = (x[q] >> 1) & 0x03030303u;
    const uint32_t c = (e * 0x40100401u) >> 24;  // e0 e1 e2 e3, e0 in bits 6-7
    if (q < 4) w.hi |= c << (8 * (3 - q));
    else w.lo |= c << (8 * (7 - q));
    const uint32_t t = (x[q] | 0x20202020u) ^ 0x6e6e6e6eu;
    const uint32_t z = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t) & 0x80808080u;  // 0x80 where t's byte is 0
    nm |= (((z >> 7) * 0x10204080u) >> 28) << (4 * q);
  }
  const uint32_t s32 = (uint32_t)sm;
  uint32_t ok = ~(swar_smear(nm, k) | swar_smear(s32, k - 1));
  if (sm) {
    const uint32_t next = (s32 >> 1) | ((uint32_t)(sm >> 32) << 31);  // bit j: byte j + 1 starts a sequence
    const uint32_t first = (nm << k) | (s32 << (k - 1));              // bit j: the window is its run's first
    ok &= ~(first & next);
  }
  const uint32_t in = jend >= 32 ? 0xffff0000u : (jend <= 16 ? 0u : (((1u << jend) - 1u) & 0xffff0000u));
  w.emit = ok & in;
  return w;
}

// the code of the k-mer ending at byte 16 + i (mask = 4^k - 1)
KS_SWAR_FN uint32_t swar_code(const SwarWin &w, int i, uint32_t mask) {
  return (uint32_t)((((uint64_t)w.hi << 32) | w.lo) >> (2 * (15 - i))) & mask;
}

}  // namespace ks
