// ks_internal.h -- shared definitions of libkmerspans (HIP, gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <sys/types.h>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kmer_spans.h"

namespace ks {

// Internal status (never returned through the C ABI): the region buffer was
// too small for a pass whose partial results cannot be kept; grow and rerun.
constexpr ks_status KS_INTERNAL_RETRY = static_cast<ks_status>(100);


// ---------------------------------------------------------------- errors
void set_error(const char *fmt, ...);
ks_status fail(ks_status st, const char *fmt, ...);

#define KS_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      return ::ks::fail(KS_ERR_DEVICE, "%s failed: %s (%s:%d)", #call,                \
                        hipGetErrorString(e_), __FILE__, __LINE__);                   \
  } while (0)

#define KS_TRY(expr)                 \
  do {                               \
    ks_status s_ = (expr);           \
    if (s_ != KS_OK) return s_;      \
  } while (0)

// ------------------------------------------------------ device workspace
// Grow-only device buffers, one per slot.  Never freed inside a call, so a
// call sequence can be captured or replayed without allocation.
enum Slot : int {
  SLOT_SEQ = 0,     // staged sequence bytes (host entry points)
  SLOT_OFFS,        // staged offsets
  SLOT_EVENTS,      // run boundary events
  SLOT_EVENTS_TMP,
  SLOT_RUNS,        // run table
  SLOT_REGIONS,     // region records
  SLOT_REG_TMP,
  SLOT_SCALARS,     // small counters
  SLOT_SORT_TMP,    // hipcub temp storage
  SLOT_COUNTS,      // count / visit histograms
  SLOT_CHUNK_A,     // chunk summaries
  SLOT_CHUNK_B,
  SLOT_CHUNK_C,
  SLOT_CHUNK_D,
  SLOT_WORK_A,      // rescan work lists
  SLOT_WORK_B,
  SLOT_TABLE_TMP,
  SLOT_LAYOUT,      // run layout (chunk / tile bases)
  SLOT_PACKED,      // 2-bit base codes of the whole buffer (find_runs, want_packed)
  SLOT_STAGE_NIB,   // host entry staging: 4-bit base classes as sent over PCIe
  SLOT_RANKS,       // host low-comp entry: the weighted-rank vector (FP64 [4^k]) on its way out
  SLOT_COUNT
};

// SLOT_SCALARS (4 KiB = 512 u64 words): every user's offset, in one place.
// Users on one context run in order on its streams; none of these ranges
// overlap, so a count and a scan may share a context's slot.
constexpr int kScEvents = 0;       // find_runs: run-event count
constexpr int kScWords = 1;        // launch_count: words counted
constexpr int kScLayout = 8;       // run_layout: 8 aggregates [8, 16)
constexpr int kScRegions = 16;     // scan_core: region counters [16, 16 + kSegs)
constexpr int kScSumWords = 96;    // count_words: sum of a histogram
constexpr int kScMultiWords = 104; // launch_count_multi: words per k of a batch [104, 112)
constexpr int kScEnd = 112;

struct DevBuf {
  void *ptr = nullptr;
  size_t bytes = 0;
};

}  // namespace ks

struct ks_ctx {
  std::atomic<std::thread::id> user{};  // the thread inside an entry point (CtxUse)
  // 1 while the library itself holds `user` to return this context's memory
  // (the policy-2 janitor, ks_release_cache): an entry point that finds the
  // context taken then waits for the release instead of failing as busy
  std::atomic<int> reclaim{0};
  uint32_t scan_epoch = 0;  // chunked scans on this context (the pass-1 epoch stamp, ks_scan_chunked.hip)
  // phases of the last host-buffer kmer_regions call on this context (ms):
  // staging + count, score-table upload + compression, scan, whole body
  double host_ms[4] = {};
  int device = 0;
  int pid = 0;  // creating process (fork check)
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int scan_algo = -1;
  int num_cus = 256;
  ks::DevBuf slots[ks::SLOT_COUNT];
  // pinned host staging
  void *pinned = nullptr;
  size_t pinned_bytes = 0;
  hipEvent_t ev[24] = {};
  hipStream_t side = nullptr;  // forked work that overlaps the main stream (joined by events; lowest priority)
  hipStream_t hi = nullptr;    // highest-priority stream: the first half's pass 1 (ks_scan_chunked.hip)
  ks_ctx *sub = nullptr;       // second context of the same device (host entries' table / count / output copies)
  unsigned long long hreg[64] = {};  // region counters per segment read back with the chunked scan's counters
  bool hreg_ok = false;              // (kSegs entries, valid until the next scan attempt)
  int64_t rescan_segcap = 0;  // grow-only rescan capacity per segment (tr_lr rescans outnumber regions)
  // top-level visits counted by another context concurrently with the scan
  // (scan_impl): scan_core leaves the count out and says whether it did
  bool vis_count_ext = false;
  bool chunked_events = false;  // the last scan_chunked recorded its phase events (ev[7..11], ev[14..15])
  bool vis_count_ext_used = false;
};

struct ks_table {
  ks_ctx *ctx = nullptr;
  int k = 0;
  double thr = 0;
  bool compressed = false;
  bool codes_pooled = false;  // d_codes came from / goes back to the per-device code-array pool
  int64_t distinct = 0;
  double *d_vals = nullptr;     // full table s = w - thr (uncompressed), 4^k doubles
  uint16_t *d_codes = nullptr;  // compressed: 4^k u16 codes
  double *d_lut = nullptr;      // compressed: distinct s values
  // Expanded table: one entry per (k+J-1)-mer holding the values (or uint16
  // codes) of its J consecutive k-mers, so one random request serves J scan
  // indices.  J = 1: not built.
  int ext_J = 1;
  void *d_ext = nullptr;        // uint64 (J <= 4 codes) or double[4] (J <= 3 values), or a line table
  // Line table (line_kind != 0; d_ext holds it, ext_J = its positions per
  // line): one 64-B line per m-mer (m = k + line_own - 1) with the values of
  // its line_own k-mers and of every one- and two-base continuation (uint16
  // codes, line_kind 1, ext_J = own + 2) or one-base continuation (FP64,
  // line_kind 2, ext_J = own + 1); see k_build_line_u16 / k_pass1l.
  int line_kind = 0;
  int line_own = 0;
  size_t ext_bytes = 0;
  size_t ext_cap = 0;           // bytes of the allocation (a pooled buffer may be larger)
  int device = 0;
  // setup time (ms, host wall clock around synchronised device work)
  double ms_upload = 0;         // w -> device, s = w - thr, finiteness scan
  double ms_compress = 0;       // distinct values: radix sort + unique + code assignment
  double ms_codes12 = 0;        // 12-bit code choice: weight histogram + renumbering
  double ms_ext_alloc = 0;      // hipMalloc of the expanded table
  double ms_ext = 0;            // expanded-table build kernel (hipEvents)
  double ms_total = 0;
  bool no_nan_posinf = true;    // no s is NaN or +Inf (-Inf allowed: it clamps to 0)
  double max_abs = 0.0;         // max |s| over the finite values
  // every s is a finite integer of magnitude <= 2^20 (+-1 tables, integer
  // scores): FP64 sums of up to 2^32 of them are exact, so the chunked scan's
  // max-plus prescan is the exact carry (no binade summaries, no replays)
  bool int_exact = false;
  // Narrow codes (ext_bits = 12, J = 5): the uint16 codes are numbered by
  // position weight, so the 4095 values covering most positions have codes
  // 0..4094, which are also their 12-bit codes (d_map12 is the identity,
  // d_lut12 = d_lut[0..4096)); 0xFFF escapes to the base uint16 table.
  int ext_bits = 16;
  uint16_t *d_map12 = nullptr;  // [4096]
  double *d_lut12 = nullptr;    // [4096]
  double escape_frac = 0.0;     // estimated share of positions that escape
  // Approximate value per (approx_k)-base prefix of the k-mer (fp16 bits):
  // the position-weighted mean of s over the k-mers sharing the prefix.  Only
  // predicts which binade the exact carry will be in (k_predict); never a result.
  uint16_t *d_approx = nullptr;
  int approx_k = 0;
  // Weighted-rank code lines for pass 1 (k_pass1r; k = 13 rank tables from
  // counts, ks_table_from_counts): each k-mer's rank as a 32-bit code
  // (piece << 18 | offset) of the closed-form prefix (RankPiece), decoded as
  // bits(R) = base[piece] + offset * inc[piece]; 128-B lines of the codes of
  // own 3 + L1 4 + L2 16 (J = 5 per read, against 4 for the FP64 64-B lines
  // that the later passes keep reading).  Pieces in weight order: the first
  // ones are the hottest (k_pass1r stages them in LDS).
  uint32_t *d_rcodes = nullptr;             // [4^k] (freed once the lines are built)
  unsigned long long *d_rpieces = nullptr;  // [2 * n_rpieces]: base bits, increment
  int32_t n_rpieces = 0;
  double rpieces_cover = 0.0;               // share of the positions whose piece is LDS-staged
  void *d_rlines = nullptr;
  size_t rlines_bytes = 0, rlines_cap = 0;
  double ms_rlines = 0;                     // code build + verification + line build (ms)
};

namespace ks {

// Host wall clock in milliseconds (setup timings).
inline double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

ks_status ensure(ks_ctx *ctx, Slot s, size_t bytes, void **out);
// KS_DEBUG_POISON (diagnostics): fill n bytes at p with the poison byte
// (synchronous; no-op unless set), and every workspace slot of ctx and its
// sub / part contexts
void debug_poison(void *p, size_t n);
void debug_poison_workspace(ks_ctx *ctx);
ks_status ensure_pinned(ks_ctx *ctx, size_t bytes, void **out);
// Host sequences staged on the device for a host entry point (ks_stage.cpp).
struct Staged {
  ks_dev_seqs dev{};
  std::vector<int64_t> offs;
  int64_t total = 0;
};
// Stage into the ctx's SLOT_SEQ (16-byte aligned; 32 B of slack after the
// bases).  compact: the bases cross PCIe as 2-bit codes + N runs / 4-bit
// classes and are rewritten as bytes of the same class on the device.
// on_bytes (optional): called on the host after each chunk is queued, with
// the end of the bases queued so far, which are then ready in ctx->side
// order; st->dev is valid from the first call.  Synchronises ctx->stream at
// the end (work the caller queued on ctx->side is the caller's to join).
ks_status stage(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, Staged *st,
                bool compact = false, const std::function<ks_status(int64_t)> &on_bytes = nullptr);
int64_t stage_chunk_bases();
// memcpy with up to 16 threads
void par_memcpy(void *dst, const void *src, size_t n);
// device -> pageable host through the ctx's pinned buffer (synchronises)
ks_status copy_out(ks_ctx *ctx, void *dst, const void *src_dev, size_t n);
// pageable host -> device through the ctx's pinned buffer, nthr fill threads
// (synchronises ctx->stream)
ks_status h2d_pinned(ks_ctx *ctx, void *dst_dev, const void *src, size_t n, int nthr);
ks_status activate(ks_ctx *ctx);  // fork check + hipSetDevice
// A context is used by one thread at a time (include/kmer_spans.h): an entry
// point marks its context as in use for its duration (nested entry points
// of the same thread pass), and a call from a second thread meanwhile fails
// with KS_ERR_ARG instead of racing on the workspace.
struct CtxUse {
  ks_ctx *c = nullptr;
  bool owner = false, busy = false;
  explicit CtxUse(ks_ctx *ctx) : c(ctx) {
    if (!c) return;
    const std::thread::id me = std::this_thread::get_id();
    for (int tries = 0;; ++tries) {
      std::thread::id none{};
      if (c->user.compare_exchange_strong(none, me)) {
        owner = true;
        return;
      }
      if (none == me) return;  // nested entry point of the same thread
      // the library is returning the context's memory (janitor): wait for it;
      // one more try after that, as a release may have ended just now
      if (c->reclaim.load() != 0) {
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        continue;
      }
      if (tries == 0) continue;
      busy = true;
      return;
    }
  }
  ~CtxUse() {
    if (owner) c->user.store(std::thread::id());
  }
  CtxUse(const CtxUse &) = delete;
  CtxUse &operator=(const CtxUse &) = delete;
};
ks_status ctx_busy();  // the KS_ERR_ARG of a context used by another thread
#define KS_ENTER(ctx)                        \
  CtxUse ks_use_(ctx);                       \
  if (ks_use_.busy) return ks::ctx_busy();   \
  KS_TRY(activate(ctx))
ks_status ctx_sub(ks_ctx *ctx, ks_ctx **sub);  // ctx->sub, created on first use
void pool_release_device(int dev);             // free the device's pooled expanded-table buffer
// End of a host-buffer entry point: unless ks_set_host_cache(1), the call's
// device memory (ctx's and its sub-context's workspace, the pooled table
// buffer) goes back to the driver.
void host_call_end(ks_ctx *ctx);
void janitor_forget(ks_ctx *ctx);  // (ks_ctx_destroy) off the timed-release list
void janitor_release_all();        // (ks_release_cache) the listed contexts' memory back now
ks_status default_ctx(ks_ctx **ctx);  // *ctx or the process default context (fork-checked)
bool hip_usable_here();  // false in a child forked after HIP was initialised
// Region output block (ks_regions_free frees it): [seq_id | beg | end] int32,
// then [score | 0.0] doubles.
ks_status regions_alloc(ks_regions *out, int64_t n);
// Pins out's block for direct D2H copies (hipHostRegister, once per kept
// block); false when it cannot (small block, registration refused).
bool regions_pin(ks_regions *out);
void regions_cache_release();  // the kept output blocks (ks_release_cache)
struct Staged;
// Host entry bodies on one context, arguments validated (ks_abi.cpp); the
// multi-device forms (ks_multi.cpp) run them on a shard of the input each.
ks_status kmer_counts_on(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                         int32_t *counts, double *n_words);
ks_status kmer_regions_on(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                          const double *w, int32_t min_width, double min_score, int32_t *visits, ks_regions *out);
// Stage host sequences and count their k-mers into d_cnt (zeroed here), the
// count overlapping the PCIe transfer where it can; ctx->stream is ordered
// after the count on return; *words (nullable) = the words counted.
ks_status stage_counted(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int k,
                        int32_t *d_cnt, Staged *st, double *words);
// Devices of the NULL-context host entry points (ks_set_devices, KS_DEVICES);
// > 1: the multi-device forms below take the call.
int multi_devices();
ks_status multi_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t *counts,
                            double *n_words);
ks_status multi_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, const double *w,
                             int32_t min_width, double min_score, int32_t *visits, ks_regions *out);
ks_status multi_low_comp_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                                 int32_t min_width, double min_score, double thr, int32_t *counts, double *ranks,
                                 double *n, ks_regions *out);
// GPU broker for fork children (ks_broker.cpp): broker_before_hip() forks it
// right before a process's first HIP use (when enabled); use_broker() is true
// in a child forked after that, whose host-buffer calls the broker_* forward.
void broker_before_hip();
bool broker_wanted(pid_t hip_pid);
bool use_broker();
void broker_reset_locks();
ks_status broker_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t *counts,
                             double *n_words);
ks_status broker_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, const double *w,
                              int64_t w_len, int32_t min_width, double min_score, int32_t *visits, double *n_bases,
                              ks_regions *out);
ks_status broker_low_comp(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t min_width,
                          double min_score, double thr, int32_t *counts, double *ranks, double *n, ks_regions *out);
ks_status broker_tr_lr(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t min_length,
                       const char *const *kmers, const double *kmer_scores, const double *trans_scores,
                       int64_t n_scores, double *spectra, ks_regions *out);
ks_status broker_windowed(const char *const *seqs, const int64_t *lens, int32_t nseq, const char *const *kmers,
                          int32_t kmer_n, int32_t k, int32_t window, int32_t ret_flag, int32_t *dist,
                          int32_t *seq_included, int32_t *const *scores);
ks_status broker_kmers_to_file(const char *seq_path, const char *out_prefix, const int32_t *ks, int32_t nk,
                               double min_l, int32_t magic, ks_kmer_file_info *info);

// -------------------------------------------------------------- encoding
__host__ __device__ __forceinline__ bool is_n(uint8_t c) { return (c | 0x20) == 'n'; }
__host__ __device__ __forceinline__ uint32_t enc(uint8_t c) { return (c >> 1) & 3u; }

// Run table produced by run segmentation: maximal N-free runs [a, b) inside
// one sequence (SoA).
struct Runs {
  int64_t *a = nullptr;
  int64_t *b = nullptr;
  int32_t *seq = nullptr;
  int64_t n = 0;
  // optional: enc() of every byte, 16 per word, first base most significant
  // (word p >> 4, bits 30 - 2 * (p & 15)); total / 16 + 1 words
  const uint32_t *packed = nullptr;
};

// Scan indices per chunk of the chunked scan, chunks per stitch tile.
constexpr int kChunk = 256;
constexpr int kTileChunks = 64;

// Chunk layout of the runs, computed on the device (run_layout): chunk and
// tile bases per run (device, n + 1 entries) and host totals.
struct RunLayout {
  int64_t *cbase = nullptr;
  int64_t *tbase = nullptr;
  int64_t nch = 0, ntiles = 0;
  int64_t scored = 0;   // scan indices (sum over runs of len - k)
  int64_t nscan = 0;    // runs longer than k
  int64_t longest = 0;  // longest run (bases)
  // split of the runs into two halves of about nch / 2 chunks (the chunked
  // scan overlaps the second half's pass 1 with the first half's later
  // passes): runs [0, split_r), chunks [0, split_c), tiles [0, split_t)
  int64_t split_r = 0, split_c = 0, split_t = 0;
};
// trlr: one more scan index per run (the first k-mer's own step) and the
// :341 skip of runs whose first k-mer ends within two bytes of the string end.
ks_status run_layout(ks_ctx *ctx, const Runs &runs, int k, RunLayout *lay, int trlr = 0,
                     const int64_t *offs_dev = nullptr);

// Region record buffer written by scan kernels.
// Append buffers (regions, rescans, candidates) are split into kSegs
// segments of segcap slots, each with its own counter, so that appends from
// thousands of waves do not serialise on one address; slot s*segcap + i.
constexpr int kSegs = 64;
static_assert(kScRegions + kSegs <= kScSumWords && kScEnd * 8 <= 4096, "SLOT_SCALARS layout");
static_assert(kSegs <= 64, "ks_ctx::hreg holds kSegs counters");

struct RegionBuf {
  int32_t *seq;
  int64_t *beg;
  int64_t *end;
  double *score;
  unsigned long long *count;  // [kSegs] device counters
  int64_t cap;                // kSegs * segcap
  int64_t segcap;
};

// Launch wrappers (defined in the .hip files).
ks_status find_runs(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, Runs *runs, float *ms,
                    bool want_packed = false, int64_t p_lo = 0, int64_t p_hi = -1);
ks_status launch_count(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const Runs &runs, int k,
                       int32_t *counts_dev, double *n_words);
// The partitioned count of the k-mers ending at [p_lo, p_hi) on stream st
// (accumulated into counts_dev; p_lo a multiple of count_range_align(); no
// synchronisation): the host entry counts each staged piece while the next
// one is still crossing PCIe.  Only where count_range_ok(k, total).
bool count_range_ok(int k, int64_t total);
int64_t count_range_align();
ks_status launch_count_range(ks_ctx *ctx, hipStream_t st, const ks_dev_seqs *s, int64_t p_lo, int64_t p_hi, int k,
                             int32_t *counts_dev);
// Words counted into a histogram (the sum of its counts as uint32: exact for
// totals < 2^32, i.e. wherever count_range_ok); synchronises st.
ks_status count_words(ks_ctx *ctx, hipStream_t st, const int32_t *counts_dev, int k, double *n_words);
// Which span scan a call performs.  trlr = 0: kmer_regions (kmer_spans.c:
// 243-307).  trlr = 1: find_kmer_tr_lr_regions (:329-395): the table holds the
// transition scores, ks the first-k-mer scores, regions need
// (max_pos - begin) >= min_len, every closed excursion restarts, output is
// 1-based.  finite / maxabs describe both tr_lr tables: the chunked path
// needs scores without NaN or +Inf whose partial sums cannot overflow (the
// reference's clamp keeps NaN, the chunked path's does not; -Inf clamps to 0
// in both); otherwise the literal lane kernel runs.
struct ScanMode {
  int trlr = 0;
  const double *ks = nullptr;
  int64_t min_len = 0;
  int finite = 1;
  double maxabs = 0.0;
  // visits_dev already holds the top-level k-mer count of the input
  // (sequence_kmer_count's histogram, e.g. the one the caller built the
  // table's hint from): the scan applies its corrections and rescans only
  bool visits_counted = false;
};

ks_status scan_impl(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, int k, const ks_table *t,
                    int32_t min_width, double min_score, int32_t *visits_dev, ks_regions *out,
                    ks_scan_stats *stats, const ScanMode &mode = ScanMode());

// FASTA parse of raw file bytes in HBM (ks_ingest.hip).  On return either
// err_pos >= 0 (first byte outside the DNA alphabet), first_kept <
// first_hdr (sequence before the first description line), or out holds the
// records' bytes (hipMalloc'd, total + 32 bytes, 'N' padded) with host
// offsets (n_records + 1) and description-line positions.
struct FastaParse {
  int64_t n_records = 0, total = 0;
  int64_t err_pos = -1, first_kept = -1, first_hdr = -1;
  uint8_t *out = nullptr;
  std::vector<int64_t> offsets, hdr_pos;
};
ks_status fasta_parse_dev(ks_ctx *ctx, const uint8_t *raw, int64_t n, FastaParse *fp);
// Keep only the records listed (ascending); replaces out / offsets / total.
ks_status fasta_select_dev(ks_ctx *ctx, FastaParse *fp, const std::vector<int32_t> &keep);
// Batched k-mer counting (ks_count.hip): one pass for nk values of k.
ks_status launch_count_multi(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const int32_t *ks, int nk,
                             int32_t *const *counts_dev, double *n_words);

// Windowed k-mer count distributions (ks_windowed.hip).  dist_dev: int32
// [(window + 1) x kmer_n] accumulated; included_dev (nullable): int32[nseq];
// pos_dev (nullable, zeroed by the caller): per sequence q an int32
// [len_q x kmer_n] column-major matrix at kmer_n * offsets[q].
ks_status windowed_impl(ks_ctx *ctx, const ks_dev_seqs *s, int64_t total, const uint32_t *qcodes_host, int kmer_n,
                        int k, int window, int32_t *dist_dev, int32_t *included_dev, int32_t *pos_dev);

// ks_table_create_hint with a cap on the expanded table (<= 0: default).
ks_status table_create(ks_ctx *ctx, const double *w_host, int32_t k, double thr, int32_t flags,
                       const int32_t *freq_dev, int64_t max_ext_bytes, ks_table **out);
// Expanded-table cap of the host entry points, whose table is built per
// call: 16 B per input base (3.1 Gbp at k = 13: J = 4 (32 GiB, ~7 ms to
// build) rather than J = 5 (128 GiB)), so the build stays a fraction of the
// scan it speeds up.
inline int64_t host_ext_cap(int64_t total_bases) { return std::max<int64_t>(16 * total_bases, (int64_t)1 << 20); }
// Build the expanded table of t (no-op if it exists or does not fit).
ks_status table_expand(ks_ctx *ctx, ks_table *t, size_t max_bytes, const int32_t *freq_dev);

// Host table builders (ks_tables.cpp).
ks_status rank_table_host(const int32_t *counts, int k, double total, double *ranks);
ks_status log2_table_host(const int32_t *counts, int k, double *w);
ks_status pm1_table_host(const int32_t *counts, int k, double *w);

// The weighted-rank prefix of rank_kmers_w (kmer_spans.c:196-200) in closed
// form.  In the stable (count, index) order, position j holds
// R_j = fl(R_{j-1} + c_{j-1} / total), R_0 = 0.  Equal counts are adjacent, so
// over a run of equal counts the same d is added again and again; while R
// stays in one binade [2^e, 2^(e+1)), R = m * 2^(e-52) and fl(R + d) adds
// RN(d * 2^(52-e)) to the integer m (an exact half rounds to the even
// result: after one such step m is even and the increment is constant).  So a
// run is a few arithmetic progressions of m, cut where R leaves the binade;
// those crossing steps are FP64 additions done here exactly as the reference
// does them.  A piece covers sorted positions [j0, next j0):
//   kind 0: R = r0 throughout;
//   kind 1: R = r0 at j0, then m(r0) + inc1 + (j - j0 - 1) * inc in binade e.
struct RankPiece {
  int64_t j0;
  double r0;
  int64_t inc1, inc;
  int32_t e, kind;
};
__host__ __device__ __forceinline__ double rank_piece_value(const RankPiece &p, int64_t j) {
  if (p.kind == 0 || j == p.j0) return p.r0;
  union { double d; int64_t i; } u;
  u.d = p.r0;
  const int64_t m = (u.i & ((1LL << 52) - 1)) | (1LL << 52);
  const int64_t mt = m + p.inc1 + (j - p.j0 - 1) * p.inc;
  u.i = ((int64_t)(p.e + 1023) << 52) | (mt - (1LL << 52));
  return u.d;
}
// Weighted-rank codes (ks_table::d_rcodes): a code is piece << kRankOffBits |
// offset; at most 2^(32 - kRankOffBits) pieces; the first kRankPieceLds
// (the hottest) are staged in LDS by k_pass1r.
constexpr int kRankOffBits = 18;
constexpr int kRankPieceLds = 7040;  // 110 KiB beside k_pass1r's 48 KiB ring
// Pieces of the whole prefix from the distinct counts (ascending) and their
// multiplicities.  Empty if a count is negative (wrapped int32 counts: the
// caller then runs the sequential prefix).
std::vector<RankPiece> rank_pieces(const int32_t *vals, const int64_t *mult, int64_t nu, double total);
// log2(f / f_med) (score 1) or +-1 (score 2) of each distinct count, with f
// and f_med as log2_table_host / pm1_table_host compute them (bit-identical).
void score_of_counts(int score, const int32_t *vals, const int64_t *mult, int64_t nu, double *w);

}  // namespace ks
