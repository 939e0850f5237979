// ks_multi.cpp -- the host-buffer entry points over several GPUs of one node.
//
// N-free runs never interact (the reference restarts after every N and never
// across a sequence, kmer_spans.c:261-265, 281, 303), so a call's input splits
// into shards that are counted and scanned independently:
//  - the pieces are whole sequences, except that a sequence longer than a
//    shard's fair share is cut in the middle of its N gaps of >= kMinGap bases
//    (both sides of a cut are N, so the pieces have exactly the sequence's
//    runs and the count's end-of-string quirk, :142-144, cannot apply at a
//    cut);
//  - pieces go to shards by LPT (longest processing time first) on length;
//  - one host thread and one context per listed device run the single-device
//    body on their shard (the pieces passed as sequences);
//  - counts and visit histograms add exactly (uint32 wrap-around, as the
//    reference's int counters and the single-device path); the weighted-rank
//    table of kmer_low_comp_regions needs the whole input's counts, so its
//    shards count first, the host adds the counts, and every shard builds the
//    table from the sum before scanning;
//  - region records return in each piece's coordinates and are mapped back
//    (sequence id, + piece start) and put in (seq_id, beg) order.
// The device list (ks_set_devices, or KS_DEVICES="0,1,..." at first use) may
// repeat a device: two contexts on one card run the shards side by side (the
// tests use [0, 0]).  Only NULL-context calls spread; a call with an explicit
// context runs on that context's device, as before.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr int kMaxDevices = 64;
constexpr int64_t kMinGap = 1000;  // N gaps a long sequence may be cut in (dist.gap_cuts)

std::mutex g_mu;
bool g_init = false;
std::vector<int32_t> g_devs;       // the list (empty: device 0 alone)
std::vector<ks_ctx *> g_ctx;       // one context per list entry, created on first use

void init_locked() {
  if (g_init) return;
  g_init = true;
  const char *e = getenv("KS_DEVICES");
  if (!e) return;
  std::string s(e);
  size_t p = 0;
  while (p < s.size() && (int)g_devs.size() < kMaxDevices) {
    const size_t q = s.find(',', p);
    const std::string tok = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
    if (!tok.empty()) g_devs.push_back((int32_t)atoi(tok.c_str()));
    if (q == std::string::npos) break;
    p = q + 1;
  }
}

struct Piece {
  int32_t seq;
  int64_t lo, hi;
};

// Cut points of sequence s (length n): the middle of every N gap of at least
// kMinGap bases that is not at either end of the sequence.  Eight bytes per
// step (SWAR N test) outside the gaps and inside them.
std::vector<int64_t> gap_cuts(const char *s, int64_t n) {
  std::vector<int64_t> cuts;
  constexpr uint64_t kOnes = 0x0101010101010101ull, kHigh = 0x8080808080808080ull, kLc = 0x2020202020202020ull,
                     kN = 0x6e6e6e6e6e6e6e6eull;
  auto word = [&](int64_t i) {
    uint64_t w;
    memcpy(&w, s + i, 8);
    return (w | kLc) ^ kN;  // zero bytes: N / n
  };
  int64_t i = 0;
  while (i < n) {
    // to the next N
    while (i + 8 <= n) {
      const uint64_t t = word(i);
      if (((t - kOnes) & ~t & kHigh) != 0) break;  // a zero byte: an N in these eight
      i += 8;
    }
    while (i < n && !is_n((uint8_t)s[i])) ++i;
    if (i >= n) break;
    // to the end of the gap
    int64_t j = i;
    while (j + 8 <= n && word(j) == 0) j += 8;
    while (j < n && is_n((uint8_t)s[j])) ++j;
    if (j - i >= kMinGap && i > 0 && j < n) cuts.push_back((i + j) / 2);
    i = j;
  }
  return cuts;
}

// LPT: pieces to parts, longest first, each to the least loaded part; each
// part's pieces then ordered by (seq, lo).
std::vector<std::vector<Piece>> lpt(const std::vector<Piece> &pieces, int nparts, int64_t *max_load) {
  std::vector<size_t> order(pieces.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {
    return pieces[x].hi - pieces[x].lo > pieces[y].hi - pieces[y].lo;
  });
  std::vector<std::vector<Piece>> parts((size_t)std::max(nparts, 1));
  std::vector<int64_t> load(parts.size(), 0);
  for (size_t i : order) {
    const size_t p = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
    parts[p].push_back(pieces[i]);
    load[p] += pieces[i].hi - pieces[i].lo;
  }
  for (auto &v : parts)
    std::sort(v.begin(), v.end(), [](const Piece &x, const Piece &y) { return x.seq != y.seq ? x.seq < y.seq : x.lo < y.lo; });
  *max_load = *std::max_element(load.begin(), load.end());
  return parts;
}

// The shard plan: whole sequences by LPT, unless that leaves a part more than
// 5 % above the fair share; then the sequences longer than half a share are
// cut in their N gaps first.
std::vector<std::vector<Piece>> shard_plan(const char *const *seqs, const int64_t *lens, int32_t nseq, int nparts) {
  int64_t total = 0;
  for (int32_t q = 0; q < nseq; ++q) total += std::max<int64_t>(lens[q], 0);
  nparts = std::max(nparts, 1);
  const int64_t fair = (total + nparts - 1) / nparts;
  std::vector<Piece> whole;
  for (int32_t q = 0; q < nseq; ++q)
    if (lens[q] > 0) whole.push_back(Piece{q, 0, lens[q]});  // (an empty sequence counts and scans nothing)
  int64_t worst = 0;
  auto parts = lpt(whole, nparts, &worst);
  if (nparts == 1 || worst <= fair + fair / 20) return parts;
  std::vector<Piece> pieces;
  for (const Piece &w : whole) {
    std::vector<int64_t> cuts;
    if (w.hi > fair / 2 && w.hi >= 2 * kMinGap) cuts = gap_cuts(seqs[w.seq], w.hi);
    int64_t a = 0;
    for (int64_t c : cuts) {
      pieces.push_back(Piece{w.seq, a, c});
      a = c;
    }
    pieces.push_back(Piece{w.seq, a, w.hi});
  }
  return lpt(pieces, nparts, &worst);
}

// One part's input as sequences (pointers into the caller's strings).
struct PartIn {
  std::vector<const char *> ptr;
  std::vector<int64_t> len;
};
PartIn part_input(const char *const *seqs, const std::vector<Piece> &pieces) {
  PartIn in;
  for (const Piece &p : pieces) {
    in.ptr.push_back(seqs[p.seq] + p.lo);
    in.len.push_back(p.hi - p.lo);
  }
  return in;
}

// Regions of every part (in its pieces' coordinates) in the caller's
// coordinates, ordered by (seq_id, beg); one output block.
ks_status merge_parts(const std::vector<std::vector<Piece>> &parts, const std::vector<ks_regions> &rs,
                      ks_regions *out) {
  int64_t n = 0;
  for (const ks_regions &r : rs) n += r.n;
  struct Rec {
    int32_t seq;
    int64_t beg, end;
    double score;
  };
  std::vector<Rec> all;
  all.reserve((size_t)n);
  for (size_t p = 0; p < rs.size(); ++p)
    for (int64_t i = 0; i < rs[p].n; ++i) {
      const int32_t j = rs[p].seq_id[i];
      if (j < 0 || (size_t)j >= parts[p].size()) return fail(KS_ERR_INTERNAL, "merge: piece %d of part %zu", j, p);
      const Piece &pc = parts[p][(size_t)j];
      all.push_back(Rec{pc.seq, pc.lo + rs[p].beg[i], pc.lo + rs[p].end[i], rs[p].score[i]});
    }
  std::stable_sort(all.begin(), all.end(),
                   [](const Rec &a, const Rec &b) { return a.seq != b.seq ? a.seq < b.seq : a.beg < b.beg; });
  KS_TRY(regions_alloc(out, n));
  for (int64_t i = 0; i < n; ++i) {
    out->seq_id[i] = all[(size_t)i].seq;
    out->beg[i] = (int32_t)all[(size_t)i].beg;
    out->end[i] = (int32_t)all[(size_t)i].end;
    out->score[i] = all[(size_t)i].score;
  }
  if (n > 0) memset(out->score + n, 0, (size_t)n * 8);  // second row of `score`
  return KS_OK;
}

// The contexts of the list (created on first use, kept for the process).
ks_status list_contexts(std::vector<ks_ctx *> *out) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  if (g_ctx.size() != g_devs.size()) {
    for (ks_ctx *c : g_ctx) ks_ctx_destroy(c);
    g_ctx.assign(g_devs.size(), nullptr);
  }
  for (size_t i = 0; i < g_devs.size(); ++i) {
    if (g_ctx[i] && g_ctx[i]->pid != (int)getpid()) g_ctx[i] = nullptr;  // inherited across fork()
    if (!g_ctx[i]) KS_TRY(ks_ctx_create(g_devs[i], &g_ctx[i]));
  }
  *out = g_ctx;
  return KS_OK;
}

// Runs fn(part index) on one host thread per non-empty part; the first
// failure's status and message are returned.
template <typename F>
ks_status run_parts(size_t nparts, const std::vector<std::vector<Piece>> &parts, F fn) {
  std::vector<ks_status> rc(nparts, KS_OK);
  std::vector<std::string> err(nparts);
  std::vector<std::thread> th;
  for (size_t p = 0; p < nparts; ++p) {
    if (parts[p].empty()) continue;
    th.emplace_back([&, p] {
      rc[p] = fn(p);
      if (rc[p] != KS_OK) err[p] = ks_last_error();  // (thread-local)
    });
  }
  for (auto &t : th) t.join();
  for (size_t p = 0; p < nparts; ++p)
    if (rc[p] != KS_OK) {
      set_error("device list entry %zu: %s", p, err[p].c_str());
      return rc[p];
    }
  return KS_OK;
}

}  // namespace

int multi_devices() {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  return (int)g_devs.size();
}

ks_status multi_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t *counts,
                            double *n_words) {
  std::vector<ks_ctx *> ctx;
  KS_TRY(list_contexts(&ctx));
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t nk = (size_t)1 << (2 * k);
  std::vector<std::vector<int32_t>> c(parts.size());
  std::vector<double> w(parts.size(), 0.0);
  KS_TRY(run_parts(parts.size(), parts, [&](size_t p) -> ks_status {
    const PartIn in = part_input(seqs, parts[p]);
    c[p].assign(nk, 0);
    return kmer_counts_on(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k, c[p].data(), &w[p]);
  }));
  memset(counts, 0, nk * 4);
  double words = 0;
  for (size_t p = 0; p < parts.size(); ++p) {
    if (parts[p].empty()) continue;
    words += w[p];
    uint32_t *dst = reinterpret_cast<uint32_t *>(counts);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(c[p].data());
    for (size_t i = 0; i < nk; ++i) dst[i] += src[i];
  }
  *n_words = words;
  return KS_OK;
}

ks_status multi_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, const double *w,
                             int32_t min_width, double min_score, int32_t *visits, ks_regions *out) {
  std::vector<ks_ctx *> ctx;
  KS_TRY(list_contexts(&ctx));
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t nk = (size_t)1 << (2 * k);
  std::vector<std::vector<int32_t>> v(parts.size());
  std::vector<ks_regions> rs(parts.size());
  for (ks_regions &r : rs) memset(&r, 0, sizeof(r));
  ks_status rc = run_parts(parts.size(), parts, [&](size_t p) -> ks_status {
    const PartIn in = part_input(seqs, parts[p]);
    if (visits) v[p].assign(nk, 0);
    return kmer_regions_on(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k, w, min_width, min_score,
                           visits ? v[p].data() : nullptr, &rs[p]);
  });
  if (rc == KS_OK) rc = merge_parts(parts, rs, out);
  for (ks_regions &r : rs) ks_regions_free(&r);
  if (rc != KS_OK) return rc;
  if (visits) {
    memset(visits, 0, nk * 4);
    uint32_t *dst = reinterpret_cast<uint32_t *>(visits);
    for (size_t p = 0; p < parts.size(); ++p) {
      if (v[p].empty()) continue;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(v[p].data());
      for (size_t i = 0; i < nk; ++i) dst[i] += src[i];
    }
  }
  return KS_OK;
}

ks_status multi_low_comp_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                                 int32_t min_width, double min_score, double thr, int32_t *counts, double *ranks,
                                 double *n, ks_regions *out) {
  std::vector<ks_ctx *> ctx;
  KS_TRY(list_contexts(&ctx));
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t np = parts.size();
  const size_t nk = (size_t)1 << (2 * k), nb = nk * 4, rb = nk * 8;
  // The contexts stay this call's until the end: phase 1 stages and counts
  // each shard, the host adds the counts, phase 2 builds every shard's rank
  // table from the sum and scans; the staged bases stay on the devices
  // between the phases.
  struct Shard {
    Staged st;
    std::vector<int32_t> cnt;
    double words = 0;
  };
  std::vector<Shard> sh(np);
  for (size_t p = 0; p < np; ++p)
    if (!parts[p].empty() && ctx[p]->user.load() != std::thread::id()) return ctx_busy();
  struct End {  // the host-entry memory policy of every context, at the end of the call
    std::vector<ks_ctx *> &c;
    ~End() {
      for (ks_ctx *x : c) host_call_end(x);
    }
  } const end{ctx};
  KS_TRY(run_parts(np, parts, [&](size_t p) -> ks_status {
    KS_ENTER(ctx[p]);
    const PartIn in = part_input(seqs, parts[p]);
    void *d_counts = nullptr;
    KS_TRY(ensure(ctx[p], SLOT_COUNTS, nb, &d_counts));
    KS_TRY(stage_counted(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k,
                         static_cast<int32_t *>(d_counts), &sh[p].st, &sh[p].words));
    sh[p].cnt.resize(nk);
    return copy_out(ctx[p], sh[p].cnt.data(), d_counts, nb);
  }));
  memset(counts, 0, nb);
  double words = 0;
  for (size_t p = 0; p < np; ++p) {
    if (parts[p].empty()) continue;
    words += sh[p].words;
    uint32_t *dst = reinterpret_cast<uint32_t *>(counts);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(sh[p].cnt.data());
    for (size_t i = 0; i < nk; ++i) dst[i] += src[i];
  }
  n[0] = words;
  n[1] = 0;  // Q8 (:613)
  size_t first = np;
  for (size_t p = 0; p < np && first == np; ++p)
    if (!parts[p].empty()) first = p;
  std::vector<ks_regions> rs(np);
  for (ks_regions &r : rs) memset(&r, 0, sizeof(r));
  ks_status rc = run_parts(np, parts, [&](size_t p) -> ks_status {
    KS_ENTER(ctx[p]);
    void *d_counts = nullptr, *d_rk = nullptr;
    KS_TRY(ensure(ctx[p], SLOT_COUNTS, nb, &d_counts));
    KS_TRY(ensure(ctx[p], SLOT_RANKS, rb, &d_rk));
    KS_HIP(hipMemcpy(d_counts, counts, nb, hipMemcpyHostToDevice));
    ks_table *t = nullptr;
    KS_TRY(ks_table_from_counts(ctx[p], static_cast<const int32_t *>(d_counts), k, KS_SCORE_RANK, words, thr,
                                KS_TABLE_EXPAND, host_ext_cap(sh[p].st.total), static_cast<double *>(d_rk), &t));
    ks_status r = KS_OK;
    if (p == first) r = copy_out(ctx[p], ranks, d_rk, rb);  // (every shard's ranks are the same)
    if (r == KS_OK) r = scan_impl(ctx[p], &sh[p].st.dev, sh[p].st.total, k, t, min_width, min_score, nullptr, &rs[p],
                                  nullptr);
    ks_table_destroy(t);
    return r;
  });
  if (first == np) memset(ranks, 0, rb);  // (no sequence: no ranks were built)
  if (rc == KS_OK) rc = merge_parts(parts, rs, out);
  for (ks_regions &r : rs) ks_regions_free(&r);
  return rc;
}

}  // namespace ks

using namespace ks;

extern "C" ks_status ks_set_devices(const int32_t *devices, int32_t n) {
  if (n < 0 || n > kMaxDevices || (n > 0 && !devices))
    return fail(KS_ERR_ARG, "a device list holds 0 to %d devices", kMaxDevices);
  for (int32_t i = 0; i < n; ++i)
    if (devices[i] < 0) return fail(KS_ERR_ARG, "device %d out of range", devices[i]);
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  for (ks_ctx *c : g_ctx) ks_ctx_destroy(c);
  g_ctx.clear();
  g_devs.assign(devices, devices + n);
  return KS_OK;
}

extern "C" int32_t ks_get_devices(int32_t *devices, int32_t cap) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  for (int32_t i = 0; i < cap && (size_t)i < g_devs.size(); ++i) devices[i] = g_devs[i];
  return (int32_t)g_devs.size();
}

extern "C" int64_t ks_shard_plan(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t nparts,
                                 int64_t *out, int64_t cap) {
  if (!seqs || !lens || nseq < 1 || nparts < 1) return -1;
  const auto parts = shard_plan(seqs, lens, nseq, nparts);
  int64_t i = 0;
  for (size_t p = 0; p < parts.size(); ++p)
    for (const Piece &pc : parts[p]) {
      if (out && i < cap) {
        out[4 * i] = (int64_t)p;
        out[4 * i + 1] = pc.seq;
        out[4 * i + 2] = pc.lo;
        out[4 * i + 3] = pc.hi;
      }
      ++i;
    }
  return i;
}

extern "C" ks_status ks_merge_parts(const int64_t *plan, int64_t npieces, int32_t nparts, const ks_regions *parts,
                                    ks_regions *out) {
  if (!plan || npieces < 0 || nparts < 1 || !parts || !out) return fail(KS_ERR_ARG, "null argument");
  memset(out, 0, sizeof(*out));
  std::vector<std::vector<Piece>> pl((size_t)nparts);
  for (int64_t i = 0; i < npieces; ++i) {
    const int64_t p = plan[4 * i];
    if (p < 0 || p >= nparts) return fail(KS_ERR_ARG, "plan row %lld names part %lld", (long long)i, (long long)p);
    pl[(size_t)p].push_back(Piece{(int32_t)plan[4 * i + 1], plan[4 * i + 2], plan[4 * i + 3]});
  }
  std::vector<ks_regions> rs(parts, parts + nparts);
  return merge_parts(pl, rs, out);
}
