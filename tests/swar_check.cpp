// Host check of ks_kmer_swar.h against the byte-serial k-mer walk it
// replaced in the count kernels (kmer_spans.c:111-155 semantics: N-free runs,
// sequence starts, quirk Q1).  Random 32-byte lane windows over an alphabet
// with upper/lower-case bases, N/n and other bytes, random start bits (bit 32
// included), every k in [1, 15], every jend.  Prints "ok <cases>" or the
// first mismatch and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <random>

#include "../kmer_spans_amd/csrc/ks_kmer_swar.h"

static bool is_n(uint8_t c) { return (c | 0x20) == 'n'; }
static uint32_t enc(uint8_t c) { return (c >> 1) & 3u; }

// the round-6 lane_kmers byte walk: emit bit 16 + i and the code of position i
static void walk(const uint8_t *b, uint64_t sm, int jend, int k, uint32_t mask, uint32_t *emit, uint32_t *codes) {
  *emit = 0;
  uint32_t code = 0;
  int len = 0;
  for (int j = 1; j < 32; ++j) {
    if ((sm >> j) & 1u) len = 0;
    if (!is_n(b[j])) {
      code = ((code << 2) | enc(b[j])) & mask;
      ++len;
    } else {
      len = 0;
    }
    if (j >= 16 && j < jend && len >= k) {
      const bool q1 = (len == k) && ((sm >> (j + 1)) & 1u);
      if (!q1) {
        *emit |= 1u << j;
        codes[j - 16] = code;
      }
    }
  }
}

int main(int argc, char **argv) {
  const long trials = argc > 1 ? atol(argv[1]) : 200000;
  std::mt19937_64 rng(12345);
  const char alpha[] = "ACGTACGTACGTacgtNnRYKM";
  long cases = 0;
  for (long t = 0; t < trials; ++t) {
    uint8_t b[32];
    const int npct = (int)(rng() % 4);  // N density class
    for (int j = 0; j < 32; ++j) {
      const uint64_t r = rng();
      if ((int)(r % 16) < npct) b[j] = (r >> 8) & 1 ? 'N' : 'n';
      else if (r % 97 == 0) b[j] = (uint8_t)(r >> 16);  // any byte value
      else b[j] = alpha[(r >> 24) % 22];
    }
    uint64_t sm = 0;
    const int ns = (int)(rng() % 4);
    for (int s = 0; s < ns; ++s) sm |= 1ull << (rng() % 33);
    if (rng() % 3 == 0) sm = 0;
    uint32_t x[8];
    for (int q = 0; q < 8; ++q) x[q] = b[4 * q] | (b[4 * q + 1] << 8) | (b[4 * q + 2] << 16) | ((uint32_t)b[4 * q + 3] << 24);
    for (int k = 1; k <= 15; ++k) {
      const uint32_t mask = (1u << (2 * k)) - 1u;
      const int jend = (rng() % 4 == 0) ? 16 + (int)(rng() % 17) : 32;
      uint32_t e0, c0[16] = {0};
      walk(b, sm, jend, k, mask, &e0, c0);
      const ks::SwarWin w = ks::swar_window(x, sm, jend, k);
      bool bad = w.emit != e0;
      for (int i = 0; i < 16 && !bad; ++i)
        if ((e0 >> (16 + i)) & 1u) bad = ks::swar_code(w, i, mask) != c0[i];
      ++cases;
      if (bad) {
        printf("mismatch k=%d jend=%d sm=%llx emit %08x vs %08x bytes:", k, jend, (unsigned long long)sm, w.emit, e0);
        for (int j = 0; j < 32; ++j) printf(" %02x", b[j]);
        printf("\n");
        return 1;
      }
    }
  }
  printf("ok %ld\n", cases);
  return 0;
}
