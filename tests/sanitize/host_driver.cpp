// ASan + UBSan run of the library's host-side C++ (TEST INFRASTRUCTURE):
// the exact table builders (ks_tables.cpp: counting sort, closed-form rank
// prefix, R median), count files (ks_io.cpp), k-mer names, and the
// argument validation of every entry point (ks_abi.cpp), which must fail
// before any device work.  No GPU is touched.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmer_spans.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

int main() {
  for (int it = 0; it < 60; ++it) {
    const int k = 1 + (int)(rnd() % 10);
    const size_t n = (size_t)1 << (2 * k);
    std::vector<int32_t> c(n);
    const int kind = it % 4;
    for (size_t i = 0; i < n; ++i) {
      if (kind == 0) c[i] = (int32_t)(rnd() % 50);
      else if (kind == 1) c[i] = (int32_t)((1u << 30) + 2 * (rnd() % 300) + 1);  // rank sums past 2^53
      else if (kind == 2) c[i] = (rnd() % 7 == 0) ? (int32_t)(rnd() % 5000000) : 0;  // wide span
      else c[i] = -(int32_t)(rnd() % 3);  // wrapped counts: sequential fallback
    }
    std::vector<double> w(n), r(n);
    double tot = 0;
    for (size_t i = 0; i < n; ++i) tot += c[i];
    if (ks_rank_table(c.data(), k, tot != 0 ? tot : 1.0, r.data()) != KS_OK) return 1;
    if (ks_log2_table(c.data(), k, w.data()) != KS_OK) return 2;
    if (ks_pm1_table(c.data(), k, w.data()) != KS_OK) return 3;
    std::vector<char> names(n * (k + 1));
    if (ks_kmer_seq(k, names.data(), names.size()) != KS_OK) return 4;
  }
  // count files round trip
  const char *path = "ks_san_counts.bin";
  std::vector<int32_t> a(16, 7), b(256, 3);
  const int32_t ks[2] = {2, 4};
  const int32_t *cs[2] = {a.data(), b.data()};
  if (ks_count_file_write(path, 310572, 2, ks, cs) != KS_OK) return 5;
  ks_count_file f;
  memset(&f, 0, sizeof f);
  if (ks_count_file_read(path, 310572, &f) != KS_OK || !f.valid || f.nk != 2 || f.counts[1][255] != 3) return 6;
  ks_count_file_free(&f);
  if (ks_count_file_read(path, 12345, &f) != KS_OK || f.valid) return 7;
  ks_count_file_free(&f);
  remove(path);
  // validation paths (must return errors without device work)
  const char *seqs[1] = {"ACGT"};
  const int64_t lens[1] = {4};
  int32_t counts[4];
  double nw = 0, nb = 0, nn[2], wv[3] = {0, 0, 0};
  ks_regions out;
  if (ks_kmer_counts(nullptr, seqs, lens, 1, 0, counts, &nw) == KS_OK) return 8;
  if (ks_kmer_counts(nullptr, seqs, lens, 0, 2, counts, &nw) == KS_OK) return 9;
  if (ks_kmer_regions(nullptr, seqs, lens, 1, 1, wv, 3, 0, 0.0, nullptr, &nb, &out) == KS_OK) return 10;
  if (ks_kmer_regions(nullptr, seqs, lens, 1, 16, wv, 3, 0, 0.0, nullptr, &nb, &out) == KS_OK) return 11;
  if (ks_low_comp_regions(nullptr, seqs, lens, 1, 2, 0, 0.0, 1.5, counts, wv, nn, &out) == KS_OK) return 12;
  if (std::string(ks_last_error()).find("threshold") == std::string::npos) return 13;
  if (ks_table_from_counts(nullptr, nullptr, 13, 1, 0, 0, 0, 0, nullptr, nullptr) == KS_OK) return 14;
  // multi-device shard plan and merge (ks_multi.cpp, host only): random
  // sequences with N gaps, every part's regions synthesised in its pieces'
  // coordinates, merged back
  for (int it = 0; it < 40; ++it) {
    const int nseq = 1 + (int)(rnd() % 5), nparts = 1 + (int)(rnd() % 6);
    std::vector<std::string> ss(nseq);
    for (auto &s : ss) {
      const int segs = (int)(rnd() % 6);
      for (int g = 0; g < segs; ++g) {
        s.append((size_t)(rnd() % 3000), 'A' + (char)(rnd() % 2) * 2);
        s.append((size_t)(rnd() % 2) ? 1200 : 7, 'N');
      }
    }
    std::vector<const char *> ptr(nseq);
    std::vector<int64_t> len(nseq);
    for (int q = 0; q < nseq; ++q) {
      ptr[q] = ss[q].data();
      len[q] = (int64_t)ss[q].size();
    }
    const int64_t np = ks_shard_plan(ptr.data(), len.data(), nseq, nparts, nullptr, 0);
    if (np < 0) return 15;
    std::vector<int64_t> plan(4 * (size_t)np + 4);
    if (ks_shard_plan(ptr.data(), len.data(), nseq, nparts, plan.data(), np) != np) return 16;
    std::vector<int32_t> sid, beg, end;
    std::vector<double> sc;
    std::vector<ks_regions> parts(nparts);
    std::vector<std::vector<int32_t>> ps(nparts), pb(nparts), pe(nparts);
    std::vector<std::vector<double>> pc(nparts);
    for (int p = 0; p < nparts; ++p) {
      int32_t local = 0;
      for (int64_t i = 0; i < np; ++i) {
        if (plan[4 * i] != p) continue;
        const int64_t L = plan[4 * i + 3] - plan[4 * i + 2];
        if (L > 10) {
          ps[p].push_back(local);
          pb[p].push_back(1);
          pe[p].push_back((int32_t)(L - 2));
          pc[p].push_back(0.5 * (double)i);
        }
        ++local;
      }
      parts[p].n = (int64_t)ps[p].size();
      parts[p].seq_id = ps[p].data();
      parts[p].beg = pb[p].data();
      parts[p].end = pe[p].data();
      parts[p].score = pc[p].data();
    }
    ks_regions merged;
    if (ks_merge_parts(plan.data(), np, nparts, parts.data(), &merged) != KS_OK) return 17;
    for (int64_t i = 1; i < merged.n; ++i)
      if (merged.seq_id[i] < merged.seq_id[i - 1] ||
          (merged.seq_id[i] == merged.seq_id[i - 1] && merged.beg[i] <= merged.beg[i - 1]))
        return 18;
    ks_regions_free(&merged);
  }
  std::printf("host sanitizer run ok (%s)\n", ks_version());
  return 0;
}
