/* ASan + UBSan run of the CPU oracle (TEST INFRASTRUCTURE): every oracle
 * entry point on random inputs with N runs, lowercase, IUPAC bytes, empty
 * and length < k sequences, special weights (NaN, +-Inf), k = 1..8. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ks_oracle.h"

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

int main(void) {
  const char *alpha[] = {"ACGT", "ACGTN", "ACGTNacgtn", "ACGTRYKM", "A", "NNNNACGT"};
  for (int it = 0; it < 400; ++it) {
    const int k = 1 + (int)(rnd() % 8);
    const int nseq = 1 + (int)(rnd() % 4);
    char *seqs[4];
    int64_t lens[4];
    for (int q = 0; q < nseq; ++q) {
      const int64_t L = (int64_t)(rnd() % 600);
      const char *a = alpha[rnd() % 6];
      const size_t na = strlen(a);
      seqs[q] = malloc((size_t)L + 1);
      for (int64_t i = 0; i < L; ++i) seqs[q][i] = a[rnd() % na];
      seqs[q][L] = 0;
      lens[q] = L;
    }
    const int64_t n = (int64_t)1 << (2 * k);
    double *w = malloc((size_t)n * 8), *r = malloc((size_t)n * 8), *w2 = malloc((size_t)n * 8);
    int32_t *c = malloc((size_t)n * 4), *vis = malloc((size_t)n * 4);
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t x = rnd() % 40;
      w[i] = x == 0 ? NAN : x == 1 ? INFINITY : x == 2 ? -INFINITY : ((double)(rnd() % 2001) - 1200.0) / 500.0;
    }
    double nw = 0, nb = 0, nn[2];
    orc_regions out = {0};
    if (orc_kmer_counts((const char *const *)seqs, lens, nseq, k, c, &nw)) return 1;
    if (orc_kmer_regions((const char *const *)seqs, lens, nseq, k, w, (int32_t)(rnd() % 8) - 1, 1.0, vis, &nb, &out))
      return 2;
    orc_regions_free(&out);
    if (orc_low_comp((const char *const *)seqs, lens, nseq, k, 3, 2.0, 0.75, c, r, nn, &out)) return 3;
    orc_regions_free(&out);
    if (orc_log2_table(c, k, w2) || orc_pm1_table(c, k, w2) || orc_rank_table(c, k, nw > 0 ? nw : 1.0, r)) return 4;
    if (k <= 6) {
      char *names = malloc((size_t)n * (k + 1));
      const char **kp = malloc((size_t)n * sizeof(char *));
      orc_kmer_seq(k, names);
      for (int64_t i = 0; i < n; ++i) kp[i] = names + i * (k + 1);
      double *ks = malloc((size_t)n * 8), *tr = malloc((size_t)n * 8);
      orc_trlr_remap(kp, k, w, w, ks, tr);
      orc_tr_lr_regions((const char *const *)seqs, lens, nseq, k, (int32_t)(rnd() % 5), ks, tr, &out);
      orc_regions_free(&out);
      const int window = 2 * k + (int)(rnd() % 20);
      int32_t *dist = malloc((size_t)(window + 1) * 2 * 4), inc[4];
      orc_windowed_dist((const char *const *)seqs, lens, nseq, kp, 2, k, window, dist, inc, NULL);
      free(dist);
      free(ks);
      free(tr);
      free(kp);
      free(names);
    }
    for (int q = 0; q < nseq; ++q) free(seqs[q]);
    free(w);
    free(w2);
    free(r);
    free(c);
    free(vis);
  }
  const char *fa = ">a desc\r\nACGTN\n;comment\n\nacgt-+.\n>b\nRYKM\n";
  orc_fasta f;
  memset(&f, 0, sizeof f);
  if (orc_fasta_parse(fa, (int64_t)strlen(fa), 0, &f) != 0) return 5;
  orc_fasta_free(&f);
  printf("oracle sanitizer run ok\n");
  return 0;
}
