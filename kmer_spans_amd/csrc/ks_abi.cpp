// ks_abi.cpp -- the C ABI (include/kmer_spans.h): contexts, workspace,
// argument validation and the host-buffer entry points that stand in for the
// reference's .Call routines (kmer_spans.c:452-639).
//
// Validation happens before any device work, with the reference's error
// strings, because R's error() longjmps out of the caller.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include <unistd.h>

#include "ks_internal.h"

namespace ks {

static thread_local char g_err[512];

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

ks_status fail(ks_status st, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return st;
}

// The process that first touched HIP through this library.  HIP state does
// not survive fork(): a child (R's mclapply, test.R:550-567) that inherits a
// context must not use it -- a HIP call there can hang -- so every entry
// point refuses it with a clear status instead.
static pid_t g_hip_pid = 0;

static ks_status fork_check(const ks_ctx *ctx) {
  const pid_t me = getpid();
  if ((ctx && ctx->pid != me) || (g_hip_pid != 0 && g_hip_pid != me))
    return fail(KS_ERR_DEVICE,
                "HIP was initialised in process %d before fork(); this child (%d) cannot use the GPU: "
                "make the first kmer_spans call inside each worker (see INTEGRATION.md, fork safety)",
                (int)(ctx ? ctx->pid : g_hip_pid), (int)me);
  return KS_OK;
}

bool hip_usable_here() { return g_hip_pid == 0 || g_hip_pid == getpid(); }

bool use_broker() { return broker_wanted(g_hip_pid); }


// Region output blocks carry their capacity (and whether they are pinned) in
// a 64-B header.  The last two freed blocks of >= 1 MiB are kept and handed
// to the next allocation they fit (up to 4x its size): a fresh block of tens
// of MB pays its page faults in the host copy-out (config 3: 1.09 M regions,
// 30 MB, ~1.5 ms per call); ks_release_cache frees them.  A kept block the
// scan pinned (regions_pin) stays pinned, so the regions land in it by DMA
// with no staging copy (round 6: the 30 MB host copy of config 3).
namespace {
constexpr size_t kBlkHdr = 64;
std::mutex g_blk_mu;
struct FreeBlk {
  char *base = nullptr;
  size_t cap = 0;
};
FreeBlk g_blk[2];
size_t &blk_cap(char *base) { return *reinterpret_cast<size_t *>(base); }
size_t &blk_pinned(char *base) { return *reinterpret_cast<size_t *>(base + 8); }
void blk_free(char *base) {
  if (!base) return;
  if (blk_pinned(base) && hip_usable_here()) (void)hipHostUnregister(base);
  free(base);
}
}  // namespace

void regions_cache_release() {
  std::lock_guard<std::mutex> g(g_blk_mu);
  for (FreeBlk &b : g_blk) {
    blk_free(b.base);
    b = FreeBlk();
  }
}

bool regions_pin(ks_regions *out) {
  if (!out || !out->seq_id) return false;
  char *base = reinterpret_cast<char *>(out->seq_id) - kBlkHdr;
  if (blk_pinned(base)) return true;
  if (blk_cap(base) < ((size_t)1 << 20)) return false;
  if (hipHostRegister(base, kBlkHdr + blk_cap(base), hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  blk_pinned(base) = 1;
  return true;
}

ks_status regions_alloc(ks_regions *out, int64_t n) {
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  const size_t ioff = (3 * nn * 4 + 7) & ~(size_t)7;
  const size_t need = ioff + 2 * nn * 8;
  char *base = nullptr;
  {
    std::lock_guard<std::mutex> g(g_blk_mu);
    for (FreeBlk &b : g_blk)
      if (b.base && b.cap >= need && b.cap <= 4 * need) {
        base = b.base;
        b = FreeBlk();
        break;
      }
  }
  if (!base) {
    base = static_cast<char *>(malloc(kBlkHdr + need));
    if (!base) {
      memset(out, 0, sizeof(*out));
      return fail(KS_ERR_NOMEM, "out of host memory for %lld regions", (long long)n);
    }
    blk_cap(base) = need;
    blk_pinned(base) = 0;
  }
  char *blk = base + kBlkHdr;
  out->n = n;
  out->seq_id = reinterpret_cast<int32_t *>(blk);
  out->beg = out->seq_id + nn;
  out->end = out->beg + nn;
  out->score = reinterpret_cast<double *>(blk + ioff);
  if (n == 0) out->score[0] = 0.0;  // (n > 0: the caller fills the second row with zeros)
  return KS_OK;
}

ks_status activate(ks_ctx *ctx) {
  KS_TRY(fork_check(ctx));
  KS_HIP(hipSetDevice(ctx->device));
  return KS_OK;
}

ks_status ctx_busy() {
  return fail(KS_ERR_ARG, "this ks_ctx is in use by another thread: a context takes one call at a time "
                          "(create one context per thread)");
}

// KS_DEBUG_POISON=<byte> (tests, diagnostics): device memory the library
// allocates or reuses is filled with that byte before the call writes it, so
// a read of memory the call did not write shows up reproducibly: fresh
// workspace slots (ensure), every slot at the start of a host entry call
// (debug_poison_workspace), and the table-side allocations (ks_table.hip:
// table values / codes / LUT, predictor table, expanded and line tables
// including pooled buffers taken again).
int debug_poison_byte() {
  static const int poison = getenv("KS_DEBUG_POISON") ? (int)strtol(getenv("KS_DEBUG_POISON"), nullptr, 0) : -1;
  return poison;
}

void debug_poison(void *p, size_t n) {
  const int poison = debug_poison_byte();
  if (poison < 0 || !p || !n) return;
  (void)hipDeviceSynchronize();
  (void)hipMemset(p, poison & 0xff, n);
  (void)hipDeviceSynchronize();
}

void debug_poison_workspace(ks_ctx *ctx) {
  if (debug_poison_byte() < 0 || !ctx) return;
  for (ks_ctx *c : {ctx, ctx->sub})
    if (c)
      for (auto &b : c->slots) debug_poison(b.ptr, b.bytes);
}

// The free-ordering probe (diagnostics, tests only).
// KS_DEBUG_SPIN_MS=<ms>: right before the library drains a context's streams
// and frees one of its buffers (a workspace slot growing in ensure, the
// workspace returned at the end of a host call), a kernel that spins for
// that long is queued on the context's side and high-priority streams --
// where the round-4 report put the unordered use.  The drain and the
// hipFree are timed and reported to stderr: a hipFree that lasts the spin
// although only the main stream was drained (KS_DEBUG_DRAIN_MAIN_ONLY=1, the
// round-4 ensure) waits for the device's other streams itself.
__global__ void k_debug_spin(long long ticks) {
  const long long t0 = wall_clock64();  // (100 MHz constant clock)
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

double debug_spin(ks_ctx *ctx) {
  const char *e = getenv("KS_DEBUG_SPIN_MS");
  const double ms = e ? std::min(2000.0, std::max(0.0, atof(e))) : 0.0;
  if (ms <= 0) return 0.0;
  for (hipStream_t x : {ctx->side, ctx->hi})
    if (x) hipLaunchKernelGGL(k_debug_spin, dim3(1), dim3(64), 0, x, (long long)(ms * 1e5));
  return ms;
}

bool debug_drain_main_only() { return getenv("KS_DEBUG_DRAIN_MAIN_ONLY") != nullptr; }

void debug_spin_report(const char *where, int slot, double spin_ms, double drain_ms, double free_ms) {
  fprintf(stderr, "[spin] %s slot %d: spin %.1f ms queued on side+hi, drain (%s) %.2f ms, hipFree %.2f ms\n", where,
          slot, spin_ms, debug_drain_main_only() ? "main stream only" : "all streams", drain_ms, free_ms);
}

ks_status ensure(ks_ctx *ctx, Slot s, size_t bytes, void **out) {
  DevBuf &b = ctx->slots[s];
  if (b.bytes < bytes) {
    if (b.ptr) {
      // every stream of the context may still use the old buffer (the
      // piecewise count of a host entry runs on the side stream, pass 1's
      // first half on the high-priority one): all three drain before the free
      // (KS_DEBUG_SPIN_MS / KS_DEBUG_DRAIN_MAIN_ONLY: the ordering probe, below)
      const double spin = debug_spin(ctx);
      const double t0 = spin > 0 ? now_ms() : 0.0;
      if (debug_drain_main_only()) {
        KS_HIP(hipStreamSynchronize(ctx->stream));
      } else {
        for (hipStream_t x : {ctx->stream, ctx->side, ctx->hi})
          if (x) KS_HIP(hipStreamSynchronize(x));
      }
      const double t1 = spin > 0 ? now_ms() : 0.0;
      KS_HIP(hipFree(b.ptr));
      if (spin > 0) debug_spin_report("ensure", (int)s, spin, t1 - t0, now_ms() - t1);
      b.ptr = nullptr;
      b.bytes = 0;
    }
    size_t want = std::max<size_t>(bytes, 256);
    want = (want + 4095) & ~(size_t)4095;
    hipError_t e = hipMalloc(&b.ptr, want);
    if (e != hipSuccess) {
      b.ptr = nullptr;
      return fail(KS_ERR_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
    }
    b.bytes = want;
    debug_poison(b.ptr, want);  // (KS_DEBUG_POISON)
  }
  *out = b.ptr;
  return KS_OK;
}

ks_status ensure_pinned(ks_ctx *ctx, size_t bytes, void **out) {
  if (ctx->pinned_bytes < bytes) {
    if (ctx->pinned) {
      KS_HIP(hipStreamSynchronize(ctx->stream));
      KS_HIP(hipHostFree(ctx->pinned));
      ctx->pinned = nullptr;
      ctx->pinned_bytes = 0;
    }
    size_t want = (std::max<size_t>(bytes, 4096) + 4095) & ~(size_t)4095;
    hipError_t e = hipHostMalloc(&ctx->pinned, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      ctx->pinned = nullptr;
      return fail(KS_ERR_NOMEM, "hipHostMalloc(%zu) failed: %s", want, hipGetErrorString(e));
    }
    ctx->pinned_bytes = want;
  }
  *out = ctx->pinned;
  return KS_OK;
}

namespace {

struct HostEnd {  // host_call_end when a host-buffer entry point returns
  ks_ctx *c;
  ~HostEnd() { host_call_end(c); }
};

ks_status check_seqs(const char *const *seqs, const int64_t *lens, int32_t nseq) {
  if (nseq < 1 || !seqs || !lens)
    return fail(KS_ERR_ARG, "seq_r must be a character vector of length at least one");
  for (int32_t q = 0; q < nseq; ++q) {
    if (lens[q] < 0 || lens[q] > INT32_MAX) return fail(KS_ERR_ARG, "sequence %d has an invalid length", q);
    if (lens[q] > 0 && !seqs[q]) return fail(KS_ERR_ARG, "sequence %d is NULL", q);
  }
  return KS_OK;
}

ks_status check_dev_seqs(const ks_dev_seqs *s) {
  if (!s || s->nseq < 1 || !s->offsets_host || !s->offsets_dev)
    return fail(KS_ERR_ARG, "seq_r must be a character vector of length at least one");
  if (s->offsets_host[s->nseq] > 0 && !s->seq) return fail(KS_ERR_ARG, "null device sequence buffer");
  if (((uintptr_t)s->seq & 15u) != 0) return fail(KS_ERR_ARG, "device sequence buffer must be 16-byte aligned");
  for (int32_t q = 0; q < s->nseq; ++q)
    if (s->offsets_host[q + 1] < s->offsets_host[q]) return fail(KS_ERR_ARG, "offsets must be non-decreasing");
  return KS_OK;
}

std::mutex g_default_mu;
ks_ctx *g_default = nullptr;

}  // namespace

// In the broker right after fork(): the forking thread held the default
// context's lock (ks_default_ctx -> ks_ctx_create -> broker_before_hip).
void broker_reset_locks() { new (&g_default_mu) std::mutex(); }
}  // namespace ks

using namespace ks;

extern "C" const char *ks_last_error(void) { return g_err; }

extern "C" void ks_regions_free(ks_regions *r) {
  if (!r) return;
  if (r->seq_id) {  // one block holds all four arrays (regions_alloc)
    char *base = reinterpret_cast<char *>(r->seq_id) - kBlkHdr;
    const size_t cap = blk_cap(base);
    if (cap >= ((size_t)1 << 20)) {  // keep it for the next call (the smaller of the two kept goes)
      std::lock_guard<std::mutex> g(g_blk_mu);
      FreeBlk &v = !g_blk[0].base ? g_blk[0] : !g_blk[1].base ? g_blk[1] : (g_blk[0].cap <= g_blk[1].cap ? g_blk[0] : g_blk[1]);
      blk_free(v.base);
      v.base = base;
      v.cap = cap;
    } else {
      blk_free(base);
    }
  }
  memset(r, 0, sizeof(*r));
}

extern "C" ks_status ks_ctx_create(int32_t device, ks_ctx **out) {
  if (!out) return fail(KS_ERR_ARG, "null output");
  KS_TRY(fork_check(nullptr));
  if (g_hip_pid == 0) {
    broker_before_hip();  // (a copy of this process before it touches HIP, when enabled)
    g_hip_pid = getpid();
  }
  int ndev = 0;
  KS_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(KS_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
  ks_ctx *c = new ks_ctx();
  c->device = device;
  c->pid = getpid();
  KS_HIP(hipSetDevice(device));
  KS_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  c->own_stream = true;
  hipDeviceProp_t prop;
  KS_HIP(hipGetDeviceProperties(&prop, device));
  c->num_cus = prop.multiProcessorCount;
  for (auto &e : c->ev) KS_HIP(hipEventCreate(&e));
  int least = 0, greatest = 0;
  KS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  KS_HIP(hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, least));
  KS_HIP(hipStreamCreateWithPriority(&c->hi, hipStreamNonBlocking, greatest));
  *out = c;
  return KS_OK;
}

extern "C" void ks_ctx_destroy(ks_ctx *c) {
  if (!c) return;
  if (c->pid != getpid()) return;  // inherited across fork(): its HIP handles are not ours
  ks::janitor_forget(c);
  if (c->sub) {
    ks_ctx_destroy(c->sub);
    c->sub = nullptr;
  }
  (void)hipSetDevice(c->device);
  // every stream drains before anything it may still use is freed
  for (hipStream_t x : {c->stream, c->side, c->hi})
    if (x) (void)hipStreamSynchronize(x);
  for (auto &b : c->slots)
    if (b.ptr) (void)hipFree(b.ptr);
  if (c->pinned) (void)hipHostFree(c->pinned);
  for (auto &e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t x : {c->side, c->hi})
    if (x) (void)hipStreamDestroy(x);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  ks::pool_release_device(c->device);  // a destroyed table's pooled expanded-table buffer (ks_table.hip)
  delete c;
}

namespace ks {
ks_status ctx_sub(ks_ctx *ctx, ks_ctx **sub) {
  if (!ctx->sub) KS_TRY(ks_ctx_create(ctx->device, &ctx->sub));
  *sub = ctx->sub;
  return KS_OK;
}


// Memory policy of the host-buffer entry points (ks_set_host_cache): 0 returns
// a call's device memory when it ends, 1 keeps it, 2 (the default) keeps it
// while calls keep coming and returns it once the context has been idle for
// g_idle_ms (a janitor thread).  Fresh VRAM is slow to get: the driver clears
// it (tools/probes/alloc_probe.py: 4-6 s for 128 GiB), so a default of "return at
// once" made every host call pay its workspace and table buffer again.
static std::atomic<int> g_host_cache{-1};    // -1: KS_HOST_CACHE decides on first use
static std::atomic<double> g_idle_ms{-1.0};  // -1: KS_HOST_CACHE_SECONDS (default 20 s)

static int host_cache_mode() {
  int m = g_host_cache.load();
  if (m < 0) {
    const char *e = getenv("KS_HOST_CACHE");
    m = e ? std::max(0, std::min(2, atoi(e))) : 2;
    g_host_cache.store(m);
  }
  return m;
}

static double idle_ms() {
  double v = g_idle_ms.load();
  if (v < 0) {
    const char *e = getenv("KS_HOST_CACHE_SECONDS");
    v = 1000.0 * (e ? std::max(0.0, atof(e)) : 20.0);
    g_idle_ms.store(v);
  }
  return v;
}

static void free_workspace(ks_ctx *c) {
  (void)hipSetDevice(c->device);
  bool any = false;
  for (auto &b : c->slots) any = any || b.ptr;
  const double spin = any ? debug_spin(c) : 0.0;  // (KS_DEBUG_SPIN_MS: the ordering probe, ensure)
  const double t0 = spin > 0 ? now_ms() : 0.0;
  if (debug_drain_main_only()) {
    (void)hipStreamSynchronize(c->stream);
  } else {
    for (hipStream_t x : {c->stream, c->side, c->hi})
      if (x) (void)hipStreamSynchronize(x);
  }
  const double t1 = spin > 0 ? now_ms() : 0.0;
  for (auto &b : c->slots) {
    if (b.ptr) (void)hipFree(b.ptr);
    b = DevBuf();
  }
  if (spin > 0) debug_spin_report("host_call_end", -1, spin, t1 - t0, now_ms() - t1);
}

static void release_ctx_memory(ks_ctx *c) {
  free_workspace(c);
  if (c->sub) free_workspace(c->sub);
  pool_release_device(c->device);
}

namespace {
// Contexts whose memory goes back at a deadline (policy 2).  The janitor
// takes a context only when no thread is inside a call on it (the CtxUse
// ownership word); a busy context is dropped from the list, and its call's
// end lists it again.  Never destroyed (a process exit joins the thread).
struct Janitor {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::pair<ks_ctx *, double>> due;  // (context, now_ms() deadline)
  std::thread th;
  bool started = false, exiting = false;
};
Janitor &janitor() {
  static Janitor *j = new Janitor();
  return *j;
}

// The library takes a context to return its memory: `reclaim` is raised
// before the ownership word is taken and lowered after it is given back, so an
// entry point that finds the word taken meanwhile waits (CtxUse) instead of
// failing as busy.
bool reclaim_begin(ks_ctx *c) {
  c->reclaim.store(1);
  std::thread::id none{};
  if (c->user.compare_exchange_strong(none, std::this_thread::get_id())) return true;
  c->reclaim.store(0);
  return false;
}

void reclaim_end(ks_ctx *c) {
  // KS_DEBUG_JANITOR_HOLD_MS (tests): hold the context that long after its
  // memory went back, so a test can call into it during a release
  if (const char *e = getenv("KS_DEBUG_JANITOR_HOLD_MS"))
    std::this_thread::sleep_for(std::chrono::milliseconds(std::min(10000, std::max(0, atoi(e)))));
  c->user.store(std::thread::id());
  c->reclaim.store(0);
}

void janitor_loop() {
  Janitor &J = janitor();
  std::unique_lock<std::mutex> g(J.mu);
  while (!J.exiting) {
    if (J.due.empty()) {
      J.cv.wait(g);
      continue;
    }
    double next = J.due.front().second;
    for (auto &d : J.due) next = std::min(next, d.second);
    const double now = now_ms();
    if (std::isinf(next)) {  // (policy 1: kept until ks_release_cache)
      J.cv.wait(g);
      continue;
    }
    if (now < next) {
      J.cv.wait_for(g, std::chrono::duration<double, std::milli>(next - now));
      continue;
    }
    for (size_t i = 0; i < J.due.size();) {
      if (J.due[i].second > now) {
        ++i;
        continue;
      }
      ks_ctx *c = J.due[i].first;
      if (reclaim_begin(c)) {
        release_ctx_memory(c);
        reclaim_end(c);
      }
      J.due.erase(J.due.begin() + (long)i);
    }
  }
}

void janitor_exit() {
  Janitor &J = janitor();
  {
    std::lock_guard<std::mutex> g(J.mu);
    J.exiting = true;
  }
  J.cv.notify_all();
  if (J.th.joinable() && J.th.get_id() != std::this_thread::get_id()) J.th.join();
}

void janitor_list(ks_ctx *c, double deadline) {
  Janitor &J = janitor();
  {
    std::lock_guard<std::mutex> g(J.mu);
    if (J.exiting) return;
    bool found = false;
    for (auto &d : J.due)
      if (d.first == c) {
        d.second = deadline;
        found = true;
      }
    if (!found) J.due.emplace_back(c, deadline);
    if (!J.started) {
      J.started = true;
      J.th = std::thread(janitor_loop);
      atexit(janitor_exit);
    }
  }
  J.cv.notify_all();
}
}  // namespace

// (ks_ctx_destroy) a destroyed context leaves the janitor's list
void janitor_forget(ks_ctx *c) {
  Janitor &J = janitor();
  std::lock_guard<std::mutex> g(J.mu);
  for (size_t i = 0; i < J.due.size();)
    if (J.due[i].first == c) J.due.erase(J.due.begin() + (long)i);
    else ++i;
}

// (ks_release_cache) every listed context's memory back now, where no call holds it
void janitor_release_all() {
  Janitor &J = janitor();
  std::lock_guard<std::mutex> g(J.mu);
  for (size_t i = 0; i < J.due.size();) {
    ks_ctx *c = J.due[i].first;
    if (c->pid == getpid() && reclaim_begin(c)) {
      release_ctx_memory(c);
      reclaim_end(c);
      J.due.erase(J.due.begin() + (long)i);
    } else {
      ++i;
    }
  }
}

void host_call_end(ks_ctx *ctx) {
  if (!ctx || ctx->pid != getpid()) return;
  const int mode = host_cache_mode();
  if (mode != 0) {  // (policy 1: listed for ks_release_cache, never due)
    janitor_list(ctx, mode == 1 ? HUGE_VAL : now_ms() + idle_ms());
    return;
  }
  release_ctx_memory(ctx);
}
}  // namespace ks

extern "C" ks_status ks_set_host_cache(int32_t keep) {
  if (keep < 0 || keep > 2) return fail(KS_ERR_ARG, "host cache policy must be 0, 1 or 2");
  ks::g_host_cache.store(keep);
  return KS_OK;
}

extern "C" ks_status ks_set_host_cache_idle(double seconds) {
  if (!(seconds >= 0) || seconds > 1e6) return fail(KS_ERR_ARG, "idle time must be between 0 and 1e6 seconds");
  ks::g_idle_ms.store(1000.0 * seconds);
  return KS_OK;
}

extern "C" ks_status ks_ctx_set_stream(ks_ctx *c, void *stream) {
  if (!c) return fail(KS_ERR_ARG, "null ctx");
  if (c->own_stream && c->stream) {
    KS_HIP(hipStreamSynchronize(c->stream));
    KS_HIP(hipStreamDestroy(c->stream));
    c->own_stream = false;
    c->stream = nullptr;
  }
  c->stream = static_cast<hipStream_t>(stream);  // nullptr: the default (null) stream
  return KS_OK;
}

extern "C" ks_status ks_ctx_set_scan_algo(ks_ctx *c, int32_t algo) {
  if (!c || algo < -1 || algo > 1) return fail(KS_ERR_ARG, "invalid scan algorithm");
  c->scan_algo = algo;
  return KS_OK;
}

extern "C" ks_ctx *ks_default_ctx(void) {
  std::lock_guard<std::mutex> g(g_default_mu);
  if (g_default && fork_check(g_default) != KS_OK) return nullptr;
  if (!g_default) {
    if (ks_ctx_create(0, &g_default) != KS_OK) g_default = nullptr;
  }
  return g_default;
}

namespace ks {
// *ctx, or the process default context; the error of a failed creation (no
// device, inherited across fork) is kept for ks_last_error().
ks_status default_ctx(ks_ctx **ctx) {
  if (*ctx) return fork_check(*ctx);
  g_err[0] = 0;
  *ctx = ks_default_ctx();
  if (!*ctx) {
    if (g_err[0] == 0) return fail(KS_ERR_DEVICE, "no HIP device available");
    return KS_ERR_DEVICE;
  }
  return KS_OK;
}
}  // namespace ks

// ------------------------------------------------------------ host entries

extern "C" ks_status ks_kmer_seq(int32_t k, char *out, size_t out_len) {
  if (k < 1 || k > KS_MAX_K)  // kmer_spans.c:627-628
    return fail(KS_ERR_ARG, "k_r (%d) should be smaller than MAX_K (%d) and larger than 0", k, KS_MAX_K + 1);
  const size_t n = (size_t)1 << (2 * k);
  if (!out || out_len < n * (size_t)(k + 1)) return fail(KS_ERR_ARG, "output buffer too small");
  static const char nuc[4] = {'A', 'C', 'T', 'G'};
  for (size_t i = 0; i < n; ++i) {
    char *o = out + i * (size_t)(k + 1);
    for (int p = 0; p < k; ++p) o[p] = nuc[(i >> (2 * (k - 1 - p))) & 3u];
    o[k] = 0;
  }
  return KS_OK;
}

extern "C" ks_status ks_rank_table(const int32_t *counts, int32_t k, double total, double *ranks) {
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  if (!counts || !ranks) return fail(KS_ERR_ARG, "null argument");
  return rank_table_host(counts, k, total, ranks);
}

extern "C" ks_status ks_log2_table(const int32_t *counts, int32_t k, double *w) {
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  if (!counts || !w) return fail(KS_ERR_ARG, "null argument");
  return log2_table_host(counts, k, w);
}

extern "C" ks_status ks_pm1_table(const int32_t *counts, int32_t k, double *w) {
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be between 1 and %d", KS_MAX_K);
  if (!counts || !w) return fail(KS_ERR_ARG, "null argument");
  return pm1_table_host(counts, k, w);
}

extern "C" ks_status ks_count_dev(ks_ctx *ctx, const ks_dev_seqs *s, int32_t k, int32_t *counts_dev,
                                  double *n_words) {
  if (!ctx) return fail(KS_ERR_ARG, "null ctx");
  KS_TRY(check_dev_seqs(s));
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k must be a positive integer less than 1+MAX_K");
  if (!counts_dev || !n_words) return fail(KS_ERR_ARG, "null argument");
  KS_ENTER(ctx);
  Runs none;
  return launch_count(ctx, s, s->offsets_host[s->nseq], none, k, counts_dev, n_words);
}

extern "C" ks_status ks_scan_dev(ks_ctx *ctx, const ks_dev_seqs *s, int32_t k, const ks_table *t,
                                 int32_t min_width, double min_score, int32_t *visits_dev,
                                 ks_regions *out, ks_scan_stats *stats) {
  if (!ctx || !t || !out) return fail(KS_ERR_ARG, "null argument");
  KS_TRY(check_dev_seqs(s));
  if (k < 1 || k > KS_MAX_K)
    return fail(KS_ERR_ARG, "kmer sizes larger than or equal to %d not currently supported", KS_MAX_K + 1);
  if (t->k != k) return fail(KS_ERR_ARG, "table built for k=%d used with k=%d", t->k, k);
  memset(out, 0, sizeof(*out));
  KS_ENTER(ctx);
  return scan_impl(ctx, s, s->offsets_host[s->nseq], k, t, min_width, min_score, visits_dev, out, stats);
}

extern "C" ks_status ks_tr_lr_dev(ks_ctx *ctx, const ks_dev_seqs *s, int32_t k, const ks_table *trans,
                                  const ks_table *init, int32_t min_length, ks_regions *out, ks_scan_stats *stats) {
  if (!ctx || !trans || !init || !out) return fail(KS_ERR_ARG, "null argument");
  KS_TRY(check_dev_seqs(s));
  if (k < 1 || k > KS_MAX_K) return fail(KS_ERR_ARG, "k should be a positive value less than MAX_K");
  if (min_length < 0) return fail(KS_ERR_ARG, "min_length should be a positive integer");
  if (trans->k != k || init->k != k) return fail(KS_ERR_ARG, "tables built for another k");
  if (!init->d_vals || init->thr != 0.0 || trans->thr != 0.0)
    return fail(KS_ERR_ARG, "tr_lr tables need threshold 0 and an uncompressed init table");
  memset(out, 0, sizeof(*out));
  KS_ENTER(ctx);
  ScanMode mode;
  mode.trlr = 1;
  mode.ks = init->d_vals;
  mode.min_len = min_length;
  mode.finite = trans->no_nan_posinf && init->no_nan_posinf;
  mode.maxabs = std::max(trans->max_abs, init->max_abs);
  return scan_impl(ctx, s, s->offsets_host[s->nseq], k, trans, 0, 0.0, nullptr, out, stats, mode);
}

// init_kmer (kmer_spans.c:119-132) on a NUL-terminated string from index 0:
// the code of the first k consecutive non-N bytes; returns the index past them
// (!= k when N bytes were skipped or the string is short).
static int64_t prime_string(const char *str, int k, uint64_t *code) {
  const unsigned char *s = (const unsigned char *)str;
  int64_t i = 0, j = 0;
  while (s[i]) {
    uint64_t c = 0;
    for (j = 0; j < k && s[i + j] && !is_n(s[i + j]); ++j) c = (c << 2) | enc(s[i + j]);
    *code = c;
    if (!s[i + j] || j == k) break;
    i += j;
    while (s[i] && is_n(s[i])) ++i;
    j = 0;
  }
  return i + j;
}

extern "C" ks_status ks_tr_lr_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq,
                                      int32_t k, int32_t min_length, const char *const *kmers,
                                      const double *kmer_scores, const double *trans_scores, int64_t n_scores,
                                      double *spectra, ks_regions *out) {
  if (nseq < 1 || !seqs || !lens)                             // :653-654
    return fail(KS_ERR_ARG, "seq_r should be a character vector of of positive length");
  KS_TRY(check_seqs(seqs, lens, nseq));
  if (!kmers) return fail(KS_ERR_ARG, "kmers_r should be a character vector");              // :657-658
  if (!kmer_scores || !trans_scores) return fail(KS_ERR_ARG, "freq_a and freq_b should be double vectors");
  if (k < 1 || k > KS_MAX_K + 1)                              // :663-664 (MAX_K = 16 allowed there)
    return fail(KS_ERR_ARG, "k should be a positive value less than MAX_K");
  if (k > KS_MAX_K) return fail(KS_ERR_ARG, "k = 16 overflows the reference's int shift; not supported");
  if (min_length < 0) return fail(KS_ERR_ARG, "min_length should be a positive integer");  // :665-666
  const int64_t nk = (int64_t)1 << (2 * k);
  if (n_scores != nk) return fail(KS_ERR_ARG, "kmers_r, freq_a, freq_b should all be 4^k long");  // :668-671
  if (!out) return fail(KS_ERR_ARG, "null output");
  memset(out, 0, sizeof(*out));
  // remap to 2-bit code order (:677-690)
  std::vector<double> ks((size_t)nk, 0.0), tr((size_t)nk, 0.0);
  int64_t bad = 0;
  for (int64_t i = 0; i < nk; ++i) {
    if (!kmers[i]) return fail(KS_ERR_ARG, "kmers_r should be a character vector");
    uint64_t code = 0;
    if (prime_string(kmers[i], k, &code) != k) ++bad;
    ks[code] = kmer_scores[i];
    tr[code] = trans_scores[i];
  }
  if (bad) fprintf(stderr, "kmer_spans_amd: %lld k-mer strings of tr_lr_regions do not spell %d bases\n",
                   (long long)bad, k);
  if (use_broker())
    return broker_tr_lr(seqs, lens, nseq, k, min_length, kmers, kmer_scores, trans_scores, n_scores, spectra, out);
  if (spectra) {
    memcpy(spectra, ks.data(), (size_t)nk * 8);
    memcpy(spectra + nk, tr.data(), (size_t)nk * 8);
  }
  KS_TRY(default_ctx(&ctx));
  KS_ENTER(ctx);
  const HostEnd host_end{ctx};  // (ks_set_host_cache)
  Staged st;
  KS_TRY(stage(ctx, seqs, lens, nseq, &st));
  ks_table *t_tr = nullptr, *t_ks = nullptr;
  KS_TRY(ks_table_create(ctx, tr.data(), k, 0.0, k >= 9 ? KS_TABLE_COMPRESS : 0, &t_tr));
  ks_status rc = ks_table_create(ctx, ks.data(), k, 0.0, 0, &t_ks);
  if (rc == KS_OK) {
    ScanMode mode;
    mode.trlr = 1;
    mode.ks = t_ks->d_vals;
    mode.min_len = min_length;
    mode.finite = t_tr->no_nan_posinf && t_ks->no_nan_posinf;
    mode.maxabs = std::max(t_tr->max_abs, t_ks->max_abs);
    rc = scan_impl(ctx, &st.dev, st.total, k, t_tr, 0, 0.0, nullptr, out, nullptr, mode);
  }
  ks_table_destroy(t_tr);
  ks_table_destroy(t_ks);
  if (rc != KS_OK) ks_regions_free(out);
  return rc;
}

extern "C" ks_status ks_kmer_counts(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                                    int32_t nseq, int32_t k, int32_t *counts, double *n_words) {
  KS_TRY(check_seqs(seqs, lens, nseq));                       // kmer_spans.c:454-455
  if (k < 1 || k > KS_MAX_K)                                  // :461-462 (and Q2)
    return fail(KS_ERR_ARG, "k must be a positive integer less than 1+MAX_K");
  if (!counts || !n_words) return fail(KS_ERR_ARG, "null output");
  if (use_broker()) return broker_kmer_counts(seqs, lens, nseq, k, counts, n_words);
  if (!ctx && multi_devices() > 1) return multi_kmer_counts(seqs, lens, nseq, k, counts, n_words);
  KS_TRY(default_ctx(&ctx));
  return kmer_counts_on(ctx, seqs, lens, nseq, k, counts, n_words);
}

// The body of ks_kmer_counts on one context (validated arguments).
ks_status ks::kmer_counts_on(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                             int32_t *counts, double *n_words) {
  KS_ENTER(ctx);
  const HostEnd host_end{ctx};  // (ks_set_host_cache)
  debug_poison_workspace(ctx);  // (KS_DEBUG_POISON)
  Staged st;
  KS_TRY(stage(ctx, seqs, lens, nseq, &st));
  const size_t nb = (size_t)4 << (2 * k);
  void *d_counts = nullptr;
  KS_TRY(ensure(ctx, SLOT_COUNTS, nb, &d_counts));
  KS_HIP(hipMemsetAsync(d_counts, 0, nb, ctx->stream));
  Runs none;
  KS_TRY(launch_count(ctx, &st.dev, st.total, none, k, (int32_t *)d_counts, n_words));
  KS_HIP(hipMemcpyAsync(counts, d_counts, nb, hipMemcpyDeviceToHost, ctx->stream));
  KS_HIP(hipStreamSynchronize(ctx->stream));
  return KS_OK;
}

// Stages the host sequences (compact forms, ks_stage.cpp) and counts their
// k-mers into d_cnt (zeroed here; sequence_kmer_count, kmer_spans.c:135-155).
// Where the partitioned count takes position ranges, each ~eighth of the
// staged bases is counted on the side stream while the rest crosses PCIe;
// otherwise the count follows the staging.  On return ctx->stream is ordered
// after the count; *words (nullable) = the words counted.
ks_status ks::stage_counted(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int k,
                           int32_t *d_cnt, Staged *st, double *words) {
  const size_t nb = (size_t)4 << (2 * k);
  int64_t total_in = 0;
  for (int32_t q = 0; q < nseq; ++q) total_in += std::max<int64_t>(lens[q], 0);
  KS_HIP(hipMemsetAsync(d_cnt, 0, nb, ctx->stream));
  const bool piecewise = count_range_ok(k, total_in) && !getenv("KS_HOST_COUNT_AFTER");
  const int64_t align = std::max<int64_t>(count_range_align(), stage_chunk_bases());
  const int64_t piece = std::max<int64_t>(align, (total_in / 8 + align - 1) / align * align);
  int64_t counted = 0;
  struct Ev {
    hipEvent_t e = nullptr;
    ~Ev() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev;
  if (piecewise) KS_HIP(hipEventCreateWithFlags(&ev.e, hipEventDisableTiming));
  auto on_bytes = [&](int64_t p1) -> ks_status {
    if (p1 < total_in && p1 - counted < piece) return KS_OK;
    KS_TRY(launch_count_range(ctx, ctx->side, &st->dev, counted, p1, k, d_cnt));
    counted = p1;
    return KS_OK;
  };
  KS_TRY(stage(ctx, seqs, lens, nseq, st, true, piecewise ? std::function<ks_status(int64_t)>(on_bytes) : nullptr));
  if (piecewise) {  // the main stream waits for the last piece's count
    KS_HIP(hipEventRecord(ev.e, ctx->side));
    KS_HIP(hipStreamWaitEvent(ctx->stream, ev.e, 0));
    if (words) KS_TRY(count_words(ctx, ctx->stream, d_cnt, k, words));
    return KS_OK;
  }
  double w = 0;
  Runs none;
  KS_TRY(launch_count(ctx, &st->dev, st->total, none, k, d_cnt, &w));
  if (words) *words = w;
  return KS_OK;
}

extern "C" ks_status ks_kmer_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                                     int32_t nseq, int32_t k, const double *w, int64_t w_len,
                                     int32_t min_width, double min_score, int32_t *visits,
                                     double *n_bases, ks_regions *out) {
  KS_TRY(check_seqs(seqs, lens, nseq));                       // :491-492
  if (!w) return fail(KS_ERR_ARG, "kmer_w_r must be a double vector of length k^4");  // :495-496
  if (k >= KS_MAX_K + 1)                                      // :504-505
    return fail(KS_ERR_ARG, "kmer sizes larger than or equal to %d not currently supported", KS_MAX_K + 1);
  if (k < 1) return fail(KS_ERR_ARG, "k must be a positive integer");
  const int64_t want = (int64_t)1 << (2 * k);
  if (w_len != want)                                          // :508-509
    return fail(KS_ERR_ARG, "kmer_w contains %lld elements but should have %lld", (long long)w_len,
                (long long)want);
  if (!out || !n_bases) return fail(KS_ERR_ARG, "null output");
  memset(out, 0, sizeof(*out));
  if (use_broker()) return broker_kmer_regions(seqs, lens, nseq, k, w, w_len, min_width, min_score, visits, n_bases, out);
  double n = 0;
  for (int32_t q = 0; q < nseq; ++q)
    if (lens[q] >= k) n += (double)lens[q];                   // :535
  *n_bases = n;
  if (!ctx && multi_devices() > 1) return multi_kmer_regions(seqs, lens, nseq, k, w, min_width, min_score, visits, out);
  KS_TRY(default_ctx(&ctx));
  return kmer_regions_on(ctx, seqs, lens, nseq, k, w, min_width, min_score, visits, out);
}

// The body of ks_kmer_regions on one context (validated arguments).
ks_status ks::kmer_regions_on(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k,
                              const double *w, int32_t min_width, double min_score, int32_t *visits,
                              ks_regions *out) {
  KS_ENTER(ctx);
  const HostEnd host_end{ctx};  // (ks_set_host_cache)
  debug_poison_workspace(ctx);  // (KS_DEBUG_POISON)
  const int64_t want = (int64_t)1 << (2 * k);
  static const bool dbg = getenv("KS_DEBUG_HOST") != nullptr;  // phase times to stderr
  const double t0 = now_ms();
  // The score table's upload and compression (host w, independent of the
  // sequences) run on the sub-context from a second host thread while the
  // sequences are staged; its expansion waits for the k-mer count.
  ks_ctx *sub = nullptr;
  KS_TRY(ctx_sub(ctx, &sub));
  ks_table *t = nullptr;
  ks_status rc_t = KS_OK;
  std::string err_t;
  double t_table = 0, t_stage = 0;
  std::thread th([&] {
    rc_t = activate(sub);
    if (rc_t == KS_OK) rc_t = table_create(sub, w, k, 0.0, k >= 9 ? KS_TABLE_COMPRESS : 0, nullptr, 0, &t);
    if (rc_t == KS_OK && hipStreamSynchronize(sub->stream) != hipSuccess)
      rc_t = fail(KS_ERR_DEVICE, "table upload failed");
    if (rc_t != KS_OK) err_t = ks_last_error();  // (thread-local)
    t_table = now_ms();
  });
  // the top-level visits: sequence_kmer_count's histogram (the partitioned
  // count), also the table's position-frequency hint (the binade predictor
  // of the scan's pass-1 summaries is built from it: without it a
  // metric-size scan spends ~27 ms more on summary fixes)
  const size_t nb = (size_t)4 << (2 * k);
  void *d_cnt = nullptr;
  Staged st;
  ks_status rc = ensure(ctx, SLOT_COUNTS, nb, &d_cnt);
  if (rc == KS_OK) rc = stage_counted(ctx, seqs, lens, nseq, k, static_cast<int32_t *>(d_cnt), &st, nullptr);
  t_stage = now_ms();
  if (th.joinable()) th.join();
  if (rc == KS_OK && rc_t != KS_OK) {
    set_error("%s", err_t.c_str());
    rc = rc_t;
  }
  if (rc != KS_OK) {
    ks_table_destroy(t);
    return rc;
  }
  const double t1 = now_ms();
  const double t2 = now_ms();
  static const bool verify = getenv("KS_DEBUG_VERIFY") != nullptr;  // (diagnostics, ks_scan_chunked.hip)
  if (verify && k <= 11) {  // the device table against the caller's w
    std::vector<double> dv((size_t)want);
    if (t->compressed) {
      std::vector<uint16_t> cd((size_t)want);
      std::vector<double> lut((size_t)t->distinct);
      KS_HIP(hipMemcpy(cd.data(), t->d_codes, cd.size() * 2, hipMemcpyDeviceToHost));
      KS_HIP(hipMemcpy(lut.data(), t->d_lut, lut.size() * 8, hipMemcpyDeviceToHost));
      for (int64_t i = 0; i < want; ++i) dv[i] = lut[cd[i]];
    } else {
      KS_HIP(hipMemcpy(dv.data(), t->d_vals, dv.size() * 8, hipMemcpyDeviceToHost));
    }
    long long bad = 0;
    for (int64_t i = 0; i < want; ++i)
      if (memcmp(&dv[i], &w[i], 8) != 0 && !(dv[i] != dv[i] && w[i] != w[i]) && ++bad <= 8)
        fprintf(stderr, "[verify] table entry %lld = %.17g, host %.17g\n", (long long)i, dv[i], w[i]);
    if (bad) fprintf(stderr, "[verify] %lld table entries differ\n", bad);
  }
  if (rc == KS_OK) {
    t->ctx = ctx;
    rc = table_expand(ctx, t, (size_t)host_ext_cap(st.total), static_cast<const int32_t *>(d_cnt));
  }
  const double t3 = now_ms();
  if (rc == KS_OK) {
    ScanMode mode;
    mode.visits_counted = true;
    rc = scan_impl(ctx, &st.dev, st.total, k, t, min_width, min_score, visits ? (int32_t *)d_cnt : nullptr, out,
                   nullptr, mode);
  }
  const double t4 = now_ms();
  if (rc == KS_OK && verify && st.total <= ((int64_t)64 << 20)) {  // the same scan again: same regions?
    ks_regions again{};
    ScanMode mode;
    const ks_status r2 = scan_impl(ctx, &st.dev, st.total, k, t, min_width, min_score, nullptr, &again, nullptr, mode);
    bool same = r2 == KS_OK && again.n == out->n;
    for (int64_t i = 0; same && i < out->n; ++i)
      same = again.seq_id[i] == out->seq_id[i] && again.beg[i] == out->beg[i] && again.end[i] == out->end[i] &&
             memcmp(&again.score[i], &out->score[i], 8) == 0;
    if (!same) {
      fprintf(stderr, "[verify] replay differs: first call %lld regions, replay %lld (rc %d), k %d total %lld\n",
              (long long)out->n, (long long)again.n, (int)r2, k, (long long)st.total);
      for (int64_t i = 0; i < std::max(out->n, again.n) && i < 8; ++i)
        fprintf(stderr, "[verify]   %lld: first %d %d %d %.17g | replay %d %d %d %.17g\n", (long long)i,
                i < out->n ? out->seq_id[i] : -1, i < out->n ? out->beg[i] : -1, i < out->n ? out->end[i] : -1,
                i < out->n ? out->score[i] : 0.0, i < again.n ? again.seq_id[i] : -1,
                i < again.n ? again.beg[i] : -1, i < again.n ? again.end[i] : -1, i < again.n ? again.score[i] : 0.0);
    }
    ks_regions_free(&again);
  }
  if (rc == KS_OK && visits) rc = copy_out(ctx, visits, d_cnt, nb);
  ctx->host_ms[0] = t_stage - t0;
  ctx->host_ms[1] = t_table - t0;
  ctx->host_ms[2] = t4 - t3;
  ctx->host_ms[3] = now_ms() - t0;
  if (dbg)
    fprintf(stderr, "[host kmer_regions] stage %.2f table %.2f (upload %.2f compress %.2f) (both %.2f) count %.2f "
            "expand %.2f (J %d) scan %.2f visits D2H %.2f ms\n", t_stage - t0, t_table - t0, t->ms_upload,
            t->ms_compress, t1 - t0, t2 - t1, t3 - t2, t->ext_J, t4 - t3, now_ms() - t4);
  ks_table_destroy(t);
  if (rc != KS_OK) ks_regions_free(out);
  return rc;
}

extern "C" ks_status ks_low_comp_regions(ks_ctx *ctx, const char *const *seqs, const int64_t *lens,
                                         int32_t nseq, int32_t k, int32_t min_width, double min_score,
                                         double thr, int32_t *counts, double *ranks, double *n,
                                         ks_regions *out) {
  KS_TRY(check_seqs(seqs, lens, nseq));                       // :549-550
  if (thr <= 0 || thr >= 1)                                   // :567-568
    return fail(KS_ERR_ARG, "the threshold must be between 0 and 1");
  if (k < 1 || k > KS_MAX_K)                                  // Q7: unchecked in the reference
    return fail(KS_ERR_ARG, "k must be a positive integer less than 1+MAX_K");
  if (!counts || !ranks || !n || !out) return fail(KS_ERR_ARG, "null output");
  memset(out, 0, sizeof(*out));
  if (use_broker()) return broker_low_comp(seqs, lens, nseq, k, min_width, min_score, thr, counts, ranks, n, out);
  if (!ctx && multi_devices() > 1)
    return multi_low_comp_regions(seqs, lens, nseq, k, min_width, min_score, thr, counts, ranks, n, out);
  KS_TRY(default_ctx(&ctx));
  KS_ENTER(ctx);
  const HostEnd host_end{ctx};  // (ks_set_host_cache)
  debug_poison_workspace(ctx);  // (KS_DEBUG_POISON)
  // the pipeline of ks_kmer_regions: the bases cross PCIe as 2-bit codes +
  // N runs and are counted in pieces meanwhile (:592-601); the weighted
  // ranks are built on the device (rank_kmers_w :602, closed-form exact
  // prefix) straight into the scan's FP64 line table; the counts and ranks
  // (768 MiB at k = 13) return over PCIe from a second host thread, through
  // the sub-context's pinned buffer, while the scan runs
  static const bool dbg = getenv("KS_DEBUG_HOST") != nullptr;
  const double t0 = now_ms();
  const size_t nb = (size_t)4 << (2 * k), rb = (size_t)8 << (2 * k);
  void *d_counts = nullptr, *d_rk = nullptr;
  KS_TRY(ensure(ctx, SLOT_COUNTS, nb, &d_counts));
  KS_TRY(ensure(ctx, SLOT_RANKS, rb, &d_rk));
  double *d_ranks = static_cast<double *>(d_rk);
  ks_ctx *sub = nullptr;
  KS_TRY(ctx_sub(ctx, &sub));
  Staged st;
  double words = 0;
  KS_TRY(stage_counted(ctx, seqs, lens, nseq, k, static_cast<int32_t *>(d_counts), &st, &words));
  n[0] = words;
  const double t1 = now_ms();
  ks_table *t = nullptr;
  ks_status rc = ks_table_from_counts(ctx, (const int32_t *)d_counts, k, KS_SCORE_RANK, words, thr, KS_TABLE_EXPAND,
                                      host_ext_cap(st.total), d_ranks, &t);
  const double t2 = now_ms();
  // the outputs' D2H on the sub-context (ordered after the table build)
  ks_status rc_o = KS_OK;
  std::string err_o;
  double t_out = 0;
  std::thread th;
  if (rc == KS_OK) {
    KS_HIP(hipEventRecord(ctx->ev[23], ctx->stream));
    th = std::thread([&] {
      rc_o = activate(sub);
      if (rc_o == KS_OK && hipStreamWaitEvent(sub->stream, ctx->ev[23], 0) != hipSuccess)
        rc_o = fail(KS_ERR_DEVICE, "output copy ordering failed");
      if (rc_o == KS_OK) rc_o = copy_out(sub, counts, d_counts, nb);
      if (rc_o == KS_OK) rc_o = copy_out(sub, ranks, d_ranks, rb);
      if (rc_o != KS_OK) err_o = ks_last_error();  // (thread-local)
      t_out = now_ms();
    });
  }
  if (rc == KS_OK) rc = scan_impl(ctx, &st.dev, st.total, k, t, min_width, min_score, nullptr, out, nullptr);
  const double t3 = now_ms();
  if (th.joinable()) th.join();
  if (rc == KS_OK && rc_o != KS_OK) {
    set_error("%s", err_o.c_str());
    rc = rc_o;
  }
  if (dbg)
    fprintf(stderr, "[host low_comp] stage+count %.2f rank table %.2f scan %.2f outputs D2H %.2f (from table end) ms\n",
            t1 - t0, t2 - t1, t3 - t2, t_out - t2);
  ks_table_destroy(t);
  n[1] = 0;                                                   // Q8 (:613)
  if (rc != KS_OK) ks_regions_free(out);
  return rc;
}

// ----------------------------------------------------------- windowed counts

static ks_status check_windowed(int32_t kmer_n, int32_t k, int32_t window) {
  if (kmer_n < 1) return fail(KS_ERR_ARG, "kmers_r should be a character vector with at least one element");  // :722-723
  if (k >= KS_MAX_K + 1)                                       // :729-731 (MAX_K = 16)
    return fail(KS_ERR_ARG, "kmer sizes larger than or equal to %d not currently supported", KS_MAX_K + 1);
  if (k < 1) return fail(KS_ERR_ARG, "k must be a positive integer");
  if (window < 2 * k) return fail(KS_ERR_ARG, "The window size must be at least two times k");  // :738-739
  return KS_OK;
}

extern "C" ks_status ks_windowed_dev(ks_ctx *ctx, const ks_dev_seqs *s, const uint32_t *kmer_codes, int32_t kmer_n,
                                     int32_t k, int32_t window, int32_t *dist_dev, int32_t *included_dev,
                                     int32_t *scores_dev) {
  if (!ctx || !kmer_codes || !dist_dev) return fail(KS_ERR_ARG, "null argument");
  KS_TRY(check_dev_seqs(s));
  KS_TRY(check_windowed(kmer_n, k, window));
  for (int32_t i = 0; i < kmer_n; ++i)
    if (kmer_codes[i] >> (2 * k)) return fail(KS_ERR_ARG, "k-mer code %u out of range for k=%d", kmer_codes[i], k);
  KS_ENTER(ctx);
  return windowed_impl(ctx, s, s->offsets_host[s->nseq], kmer_codes, kmer_n, k, window, dist_dev, included_dev,
                       scores_dev);
}

extern "C" ks_status ks_windowed_dist(ks_ctx *ctx, const char *const *seqs, const int64_t *lens, int32_t nseq,
                                      const char *const *kmers, int32_t kmer_n, int32_t k, int32_t window,
                                      int32_t ret_flag, int32_t *dist, int32_t *seq_included,
                                      int32_t *const *scores) {
  if (nseq < 1 || !seqs || !lens)                              // :720-721
    return fail(KS_ERR_ARG, "seq_r should be a character vector with at least one element");
  KS_TRY(check_seqs(seqs, lens, nseq));
  if (!kmers) return fail(KS_ERR_ARG, "kmers_r should be a character vector with at least one element");
  if (kmer_n >= 1 && k >= 1 && k <= KS_MAX_K)
    for (int32_t i = 0; i < kmer_n; ++i)                         // :733-736
      if (!kmers[i] || (int64_t)strlen(kmers[i]) != k) return fail(KS_ERR_ARG, "All kmers specified must be of the same length");
  KS_TRY(check_windowed(kmer_n, k, window));
  if (!dist || !seq_included) return fail(KS_ERR_ARG, "null output");
  const bool want_pos = (ret_flag & 1) != 0;                   // :763-766
  if (want_pos && !scores) return fail(KS_ERR_ARG, "null scores output");
  std::vector<uint32_t> codes((size_t)kmer_n, 0);
  for (int32_t i = 0; i < kmer_n; ++i) {                       // init_kmer on each query (:757-758)
    uint64_t c = 0;
    prime_string(kmers[i], k, &c);
    codes[i] = (uint32_t)c;
  }
  if (use_broker())
    return broker_windowed(seqs, lens, nseq, kmers, kmer_n, k, window, ret_flag, dist, seq_included, scores);
  KS_TRY(default_ctx(&ctx));
  KS_ENTER(ctx);
  const HostEnd host_end{ctx};  // (ks_set_host_cache)
  Staged st;
  KS_TRY(stage(ctx, seqs, lens, nseq, &st));
  const size_t dn = (size_t)(window + 1) * (size_t)kmer_n;
  void *d_dist = nullptr, *d_inc = nullptr;
  KS_TRY(ensure(ctx, SLOT_COUNTS, dn * 4, &d_dist));
  KS_TRY(ensure(ctx, SLOT_REG_TMP, (size_t)nseq * 4 + 16, &d_inc));
  KS_HIP(hipMemsetAsync(d_dist, 0, dn * 4, ctx->stream));
  int32_t *d_pos = nullptr;
  const size_t pn = want_pos ? (size_t)kmer_n * (size_t)st.total : 0;
  if (pn) {
    if (hipMalloc(&d_pos, pn * 4) != hipSuccess)
      return fail(KS_ERR_NOMEM, "hipMalloc(%zu) for window scores failed", pn * 4);
    if (hipMemsetAsync(d_pos, 0, pn * 4, ctx->stream) != hipSuccess) {
      (void)hipFree(d_pos);
      return fail(KS_ERR_DEVICE, "hipMemsetAsync failed");
    }
  }
  ks_status rc = windowed_impl(ctx, &st.dev, st.total, codes.data(), kmer_n, k, window, (int32_t *)d_dist,
                               (int32_t *)d_inc, d_pos);
  hipError_t he = hipSuccess;
  if (rc == KS_OK) he = hipMemcpyAsync(dist, d_dist, dn * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (rc == KS_OK && he == hipSuccess)
    he = hipMemcpyAsync(seq_included, d_inc, (size_t)nseq * 4, hipMemcpyDeviceToHost, ctx->stream);
  if (rc == KS_OK && he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
  if (rc == KS_OK && he == hipSuccess && pn) {
    for (int32_t q = 0; q < nseq && he == hipSuccess; ++q)
      if (seq_included[q] && scores[q])                        // :776-784 (matrix [len x kmer_n])
        he = hipMemcpy(scores[q], d_pos + (size_t)kmer_n * st.offs[q], (size_t)kmer_n * lens[q] * 4,
                       hipMemcpyDeviceToHost);
  }
  if (d_pos) (void)hipFree(d_pos);
  if (rc == KS_OK && he != hipSuccess) rc = fail(KS_ERR_DEVICE, "window result copy failed: %s", hipGetErrorString(he));
  return rc;
}
