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
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
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
// 0.5 % above the fair share; then the sequences longer than half a share are
// cut in their N gaps first (the gap scans on up to 16 host threads).  The
// one planner of the library and of bench.py / dist.py (ks_shard_plan).
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
  if (nparts == 1 || worst <= fair + fair / 200) return parts;
  std::vector<std::vector<int64_t>> cuts(whole.size());
  std::vector<size_t> todo;
  for (size_t i = 0; i < whole.size(); ++i)
    if (whole[i].hi > fair / 2 && whole[i].hi >= 2 * kMinGap) todo.push_back(i);
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  const size_t nt = std::min<size_t>(16, todo.size());
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (size_t j = next++; j < todo.size(); j = next++) {
        const Piece &w = whole[todo[j]];
        cuts[todo[j]] = gap_cuts(seqs[w.seq], w.hi);
      }
    });
  for (auto &x : th) x.join();
  std::vector<Piece> pieces;
  for (size_t i = 0; i < whole.size(); ++i) {
    const Piece &w = whole[i];
    int64_t a = 0;
    for (int64_t c : cuts[i]) {
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

// dst[i] += src[i] (uint32 wrap-around: the reference's int counters)
__global__ void k_add_u32(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

// Peer access between the list's distinct devices (xGMI copies of the count
// stripes, multi_low_comp_regions); a device pair without it still copies
// (the runtime stages through the host).
void enable_peers(const std::vector<int32_t> &devs) {
  for (int32_t a : devs)
    for (int32_t b : devs) {
      if (a == b) continue;
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, a, b) != hipSuccess || !ok) continue;
      if (hipSetDevice(a) != hipSuccess) continue;
      (void)hipDeviceEnablePeerAccess(b, 0);  // (already enabled: an error we ignore)
      (void)hipGetLastError();
    }
}

// The contexts of the list: one immutable set per list, shared by the calls
// that use it.  ks_set_devices (or a change of the list's length) replaces the
// set; the old one is destroyed when its last call drops it, never under a
// running call.
struct CtxSet {
  std::vector<ks_ctx *> c;
  ~CtxSet() {
    for (ks_ctx *x : c) ks_ctx_destroy(x);  // (a no-op for contexts inherited across fork())
  }
};
std::shared_ptr<CtxSet> g_set;
// One multi-device call at a time: its threads own every context of the set
// from its first phase to its end; a second thread's call meanwhile is
// refused (as a second thread on one context is, include/kmer_spans.h).
std::mutex g_call_mu;

ks_status list_contexts(std::shared_ptr<CtxSet> *out) {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  bool fresh = !g_set || g_set->c.size() != g_devs.size();
  for (size_t i = 0; !fresh && i < g_set->c.size(); ++i)
    fresh = g_set->c[i]->pid != (int)getpid();  // inherited across fork(): a new set
  if (fresh) {
    auto set = std::make_shared<CtxSet>();
    for (size_t i = 0; i < g_devs.size(); ++i) {
      ks_ctx *c = nullptr;
      KS_TRY(ks_ctx_create(g_devs[i], &c));  // (on failure the partial set destroys what it made)
      set->c.push_back(c);
    }
    g_set = std::move(set);
    enable_peers(g_devs);
  }
  *out = g_set;
  return KS_OK;
}

// Phase times of the last multi-device call (ks_multi_last_stats).
struct MultiStats {
  double total = 0, phase1 = 0, host_sum = 0, phase2 = 0, merge = 0;
  std::vector<double> part;  // per part: body, staging + count, table upload, scan (ms)
};
std::mutex g_stats_mu;
MultiStats g_stats;

// A barrier of the call's part threads; a part that fails breaks it for all.
class PartBarrier {
 public:
  explicit PartBarrier(int n) : n_(n) {}
  // false: a part failed (the caller returns at once)
  bool arrive(bool ok) {
    std::unique_lock<std::mutex> g(mu_);
    if (!ok) broken_ = true;
    const int gen = gen_;
    if (++here_ == n_) {
      here_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(g, [&] { return gen_ != gen; });
    }
    return !broken_;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, here_ = 0, gen_ = 0;
  bool broken_ = false;
};

// Runs fn(part index) on one host thread per non-empty part, each holding
// its part's context (KS_ENTER) for the whole of fn; the first failure's
// status and message are returned.
template <typename F>
ks_status run_parts(const std::vector<ks_ctx *> &ctx, const std::vector<std::vector<Piece>> &parts, F fn) {
  const size_t nparts = parts.size();
  std::vector<ks_status> rc(nparts, KS_OK);
  std::vector<std::string> err(nparts);
  std::vector<std::thread> th;
  for (size_t p = 0; p < nparts; ++p) {
    if (parts[p].empty()) continue;
    th.emplace_back([&, p] {
      rc[p] = [&]() -> ks_status {
        KS_ENTER(ctx[p]);
        return fn(p);
      }();
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

// dst += every src (uint32 wrap-around, the reference's int counters), on up
// to 16 threads over stripes of the histogram
void add_hists(int32_t *dst, const std::vector<const int32_t *> &src, size_t n) {
  const size_t nt = std::max<size_t>(1, std::min<size_t>(16, n >> 20));
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      const size_t a = n * t / nt, b = n * (t + 1) / nt;
      uint32_t *d = reinterpret_cast<uint32_t *>(dst);
      for (const int32_t *s : src) {
        const uint32_t *u = reinterpret_cast<const uint32_t *>(s);
        for (size_t i = a; i < b; ++i) d[i] += u[i];
      }
    });
  for (auto &x : th) x.join();
}

size_t live_parts(const std::vector<std::vector<Piece>> &parts) {
  size_t n = 0;
  for (const auto &v : parts) n += !v.empty();
  return n;
}

void record_stats(const MultiStats &m) {
  std::lock_guard<std::mutex> g(g_stats_mu);
  g_stats = m;
}

}  // namespace

int multi_devices() {
  std::lock_guard<std::mutex> g(g_mu);
  init_locked();
  return (int)g_devs.size();
}

ks_status multi_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t *counts,
                            double *n_words) {
  std::unique_lock<std::mutex> call(g_call_mu, std::try_to_lock);
  if (!call.owns_lock()) return ctx_busy();
  std::shared_ptr<CtxSet> set;
  KS_TRY(list_contexts(&set));
  const std::vector<ks_ctx *> &ctx = set->c;
  const double t0 = now_ms();
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t nk = (size_t)1 << (2 * k);
  std::vector<std::vector<int32_t>> c(parts.size());
  std::vector<double> w(parts.size(), 0.0);
  KS_TRY(run_parts(ctx, parts, [&](size_t p) -> ks_status {
    const PartIn in = part_input(seqs, parts[p]);
    c[p].assign(nk, 0);
    return kmer_counts_on(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k, c[p].data(), &w[p]);
  }));
  const double t1 = now_ms();
  memset(counts, 0, nk * 4);
  double words = 0;
  std::vector<const int32_t *> src;
  for (size_t p = 0; p < parts.size(); ++p)
    if (!parts[p].empty()) {
      words += w[p];
      src.push_back(c[p].data());
    }
  add_hists(counts, src, nk);
  *n_words = words;
  MultiStats m;
  m.phase1 = t1 - t0;
  m.host_sum = now_ms() - t1;
  m.total = now_ms() - t0;
  record_stats(m);
  return KS_OK;
}

ks_status multi_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, const double *w,
                             int32_t min_width, double min_score, int32_t *visits, ks_regions *out) {
  std::unique_lock<std::mutex> call(g_call_mu, std::try_to_lock);
  if (!call.owns_lock()) return ctx_busy();
  std::shared_ptr<CtxSet> set;
  KS_TRY(list_contexts(&set));
  const std::vector<ks_ctx *> &ctx = set->c;
  const double t0 = now_ms();
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t nk = (size_t)1 << (2 * k);
  std::vector<std::vector<int32_t>> v(parts.size());
  std::vector<ks_regions> rs(parts.size());
  for (ks_regions &r : rs) memset(&r, 0, sizeof(r));
  MultiStats m;
  m.part.assign(4 * parts.size(), 0.0);
  ks_status rc = run_parts(ctx, parts, [&](size_t p) -> ks_status {
    const PartIn in = part_input(seqs, parts[p]);
    if (visits) v[p].assign(nk, 0);
    const ks_status r = kmer_regions_on(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k, w, min_width,
                                        min_score, visits ? v[p].data() : nullptr, &rs[p]);
    m.part[4 * p] = ctx[p]->host_ms[3];
    m.part[4 * p + 1] = ctx[p]->host_ms[0];
    m.part[4 * p + 2] = ctx[p]->host_ms[1];
    m.part[4 * p + 3] = ctx[p]->host_ms[2];
    return r;
  });
  const double t1 = now_ms();
  if (rc == KS_OK) rc = merge_parts(parts, rs, out);
  const double t2 = now_ms();
  for (ks_regions &r : rs) ks_regions_free(&r);
  if (rc != KS_OK) return rc;
  if (visits) {
    memset(visits, 0, nk * 4);
    std::vector<const int32_t *> src;
    for (size_t p = 0; p < parts.size(); ++p)
      if (!v[p].empty()) src.push_back(v[p].data());
    add_hists(visits, src, nk);
  }
  m.phase1 = t1 - t0;
  m.merge = t2 - t1;
  m.host_sum = now_ms() - t2;
  m.total = now_ms() - t0;
  record_stats(m);
  return KS_OK;
}

ks_status multi_low_comp_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                                 int32_t min_width, double min_score, double thr, int32_t *counts, double *ranks,
                                 double *n, ks_regions *out) {
  std::unique_lock<std::mutex> call(g_call_mu, std::try_to_lock);
  if (!call.owns_lock()) return ctx_busy();
  std::shared_ptr<CtxSet> set;
  KS_TRY(list_contexts(&set));
  const std::vector<ks_ctx *> &ctx = set->c;
  const double t0 = now_ms();
  const auto parts = shard_plan(seqs, lens, nseq, (int)ctx.size());
  const size_t np = parts.size();
  const size_t nk = (size_t)1 << (2 * k), nb = nk * 4, rb = nk * 8;
  // One thread per part holds its context from the first phase to the end
  // (run_parts): phase 1 stages and counts the part's bases; then the parts
  // sum their histograms on the devices (a reduce-scatter and an all-gather
  // of stripes, device-to-device, with barriers between); every part builds
  // the rank table from the sum and scans the bases it still holds.  (Round
  // 5 summed on the host from a full host copy per part; round 6's first form
  // summed stripes on the host: 114 ms for two parts at the metric genome.)
  struct Shard {
    Staged st;
    double words = 0;
    int32_t *d_counts = nullptr;
  };
  std::vector<Shard> sh(np);
  size_t first = np;
  for (size_t p = 0; p < np && first == np; ++p)
    if (!parts[p].empty()) first = p;
  const size_t nlive = live_parts(parts);
  PartBarrier bar((int)nlive);
  std::vector<size_t> live;
  for (size_t p = 0; p < np; ++p)
    if (!parts[p].empty()) live.push_back(p);
  std::vector<ks_regions> rs(np);
  for (ks_regions &r : rs) memset(&r, 0, sizeof(r));
  double t_p1 = 0, t_sum = 0;
  ks_status rc = run_parts(ctx, parts, [&](size_t p) -> ks_status {
    struct End {  // the host-entry memory policy, at the end of the part's call
      ks_ctx *c;
      ~End() { host_call_end(c); }
    } const end{ctx[p]};
    debug_poison_workspace(ctx[p]);  // (KS_DEBUG_POISON)
    // ---- phase 1: stage + count
    ks_status r = [&]() -> ks_status {
      const PartIn in = part_input(seqs, parts[p]);
      void *d = nullptr;
      KS_TRY(ensure(ctx[p], SLOT_COUNTS, nb, &d));
      sh[p].d_counts = static_cast<int32_t *>(d);
      KS_TRY(stage_counted(ctx[p], in.ptr.data(), in.len.data(), (int32_t)in.len.size(), k, sh[p].d_counts, &sh[p].st,
                           &sh[p].words));
      KS_HIP(hipStreamSynchronize(ctx[p]->stream));
      return KS_OK;
    }();
    if (!bar.arrive(r == KS_OK)) return r != KS_OK ? r : fail(KS_ERR_DEVICE, "another device list entry failed");
    // KS_DEBUG_MULTI_PHASE_SLEEP_MS (tests): a long gap between the phases,
    // during which the contexts must stay this call's (janitor, other threads)
    if (const char *e = getenv("KS_DEBUG_MULTI_PHASE_SLEEP_MS"))
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min(10000, std::max(0, atoi(e)))));
    // ---- the count sum on the devices: each part adds its stripe of every
    // other part's counts into its own (device-to-device copies, xGMI between
    // GPUs), then, after a barrier, copies every other part's summed stripe
    // into its own histogram -- every part then holds the whole input's
    // counts, and the caller's copy comes from one part
    const size_t ip = (size_t)(std::find(live.begin(), live.end(), p) - live.begin());
    if (ip == 0) t_p1 = now_ms() - t0;
    auto stripe = [&](size_t i, size_t *a, size_t *b) {
      *a = nk * i / nlive;
      *b = nk * (i + 1) / nlive;
    };
    hipStream_t sp = ctx[p]->stream;
    r = [&]() -> ks_status {
      size_t a = 0, b = 0;
      stripe(ip, &a, &b);
      if (b <= a || nlive < 2) return KS_OK;
      void *tmp = nullptr;
      KS_TRY(ensure(ctx[p], SLOT_TABLE_TMP, (b - a) * 4, &tmp));
      for (size_t q : live) {
        if (q == p) continue;
        KS_HIP(hipMemcpyAsync(tmp, sh[q].d_counts + a, (b - a) * 4, hipMemcpyDeviceToDevice, sp));
        hipLaunchKernelGGL(k_add_u32, dim3((unsigned)std::min<size_t>((b - a + 255) / 256, 8192)), dim3(256), 0, sp,
                           reinterpret_cast<uint32_t *>(sh[p].d_counts + a), static_cast<const uint32_t *>(tmp),
                           (int64_t)(b - a));
        KS_HIP(hipGetLastError());
      }
      KS_HIP(hipStreamSynchronize(sp));
      return KS_OK;
    }();
    if (!bar.arrive(r == KS_OK)) return r != KS_OK ? r : fail(KS_ERR_DEVICE, "another device list entry failed");
    r = [&]() -> ks_status {
      for (size_t j = 0; j < nlive && nlive > 1; ++j) {
        if (j == ip) continue;
        size_t a = 0, b = 0;
        stripe(j, &a, &b);
        if (b > a)
          KS_HIP(hipMemcpyAsync(sh[p].d_counts + a, sh[live[j]].d_counts + a, (b - a) * 4, hipMemcpyDeviceToDevice,
                                sp));
      }
      KS_HIP(hipStreamSynchronize(sp));
      return KS_OK;
    }();
    // (every part has read its stripes before any part's phase 2 touches its histogram)
    if (!bar.arrive(r == KS_OK)) return r != KS_OK ? r : fail(KS_ERR_DEVICE, "another device list entry failed");
    if (ip == 0) t_sum = now_ms() - t0 - t_p1;
    // ---- phase 2: the rank table from the sum, the scan
    KS_TRY(activate(ctx[p]));
    double words = 0;
    for (size_t q : live) words += sh[q].words;
    void *d_rk = nullptr;
    KS_TRY(ensure(ctx[p], SLOT_RANKS, rb, &d_rk));
    if (p == first) KS_TRY(copy_out(ctx[p], counts, sh[p].d_counts, nb));  // (the summed counts: the caller's)
    ks_table *t = nullptr;
    KS_TRY(ks_table_from_counts(ctx[p], sh[p].d_counts, k, KS_SCORE_RANK, words, thr, KS_TABLE_EXPAND,
                                host_ext_cap(sh[p].st.total), static_cast<double *>(d_rk), &t));
    r = KS_OK;
    if (p == first) r = copy_out(ctx[p], ranks, d_rk, rb);  // (every part's ranks are the same)
    if (r == KS_OK) r = scan_impl(ctx[p], &sh[p].st.dev, sh[p].st.total, k, t, min_width, min_score, nullptr, &rs[p],
                                  nullptr);
    ks_table_destroy(t);
    return r;
  });
  const double t1 = now_ms();
  double words = 0;
  for (size_t q : live) words += sh[q].words;
  if (nlive == 0) memset(counts, 0, nb);
  n[0] = words;
  n[1] = 0;  // Q8 (:613)
  if (first == np) memset(ranks, 0, rb);  // (no sequence: no ranks were built)
  if (rc == KS_OK) rc = merge_parts(parts, rs, out);
  for (ks_regions &r : rs) ks_regions_free(&r);
  MultiStats m;
  m.phase1 = t_p1;
  m.host_sum = t_sum;
  m.phase2 = t1 - t0 - t_p1 - t_sum;
  m.merge = now_ms() - t1;
  m.total = now_ms() - t0;
  record_stats(m);
  return rc;
}

}  // namespace ks

using namespace ks;

extern "C" ks_status ks_set_devices(const int32_t *devices, int32_t n) {
  if (n < 0 || n > kMaxDevices || (n > 0 && !devices))
    return fail(KS_ERR_ARG, "a device list holds 0 to %d devices", kMaxDevices);
  for (int32_t i = 0; i < n; ++i)
    if (devices[i] < 0) return fail(KS_ERR_ARG, "device %d out of range", devices[i]);
  std::shared_ptr<CtxSet> old;  // destroyed outside the lock, after any call still using it
  {
    std::lock_guard<std::mutex> g(g_mu);
    init_locked();
    old = std::move(g_set);
    g_set.reset();
    g_devs.assign(devices, devices + n);
  }
  return KS_OK;
}

extern "C" int32_t ks_multi_last_stats(double *out, int32_t cap) {
  std::lock_guard<std::mutex> g(g_stats_mu);
  std::vector<double> v = {g_stats.total, g_stats.phase1, g_stats.host_sum, g_stats.phase2, g_stats.merge,
                           (double)(g_stats.part.size() / 4)};
  v.insert(v.end(), g_stats.part.begin(), g_stats.part.end());
  for (int32_t i = 0; out && i < cap && (size_t)i < v.size(); ++i) out[i] = v[(size_t)i];
  return (int32_t)v.size();
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
