// ks_broker.cpp -- the GPU broker for processes forked after the library used
// HIP (R's mclapply after a call in the parent: test.R:351 then :554-565).
//
// HIP state does not survive fork(): a child of a process that has used HIP
// must not make HIP calls.  With the broker on (ks_set_fork_broker(1), which
// the R shim's R_init_kmer_spans does, or KS_FORK_BROKER=1), the process
// forks a broker right before its own first HIP use -- the broker is then a
// copy of a process that has not touched HIP -- and keeps going on the GPU
// itself.  A later fork child (an mclapply worker) sends the host-buffer calls
// the .Call shim makes (kmer_counts, kmer_regions, kmer_low_comp_regions,
// tr_lr_regions, windowed distributions, kmers_to_file) over a Unix socket to
// the broker, which runs them and sends the outputs back.  Argument
// validation stays in the caller, so errors read the same either way.
//
// The broker serves up to KS_BROKER_THREADS (default 4) requests at once,
// each server thread on its own HIP context (its own streams and workspace,
// the device shared): test.R:554 runs 20 mclapply workers, whose calls would
// otherwise queue behind each other.  A connection is served by one thread at
// a time (its requests stay in order).
//
// Only the owner's own processes may use it: a connecting peer must have the
// broker's uid (SO_PEERCRED) and descend from the process that forked the
// broker; request lengths are capped per operation.  The broker ends when its
// parent is gone (getppid() polled every second: PR_SET_PDEATHSIG would fire
// when the forking *thread* ends, which may be a short-lived one).
//
// Wire format: request = u32 magic, u32 op, u64 payload bytes, payload;
// reply = u64 payload bytes, payload = i32 status, u32 message length,
// message, outputs.  Payloads are the arguments / outputs in call order,
// arrays as raw bytes (both ends are the same build on the same host).
#include <algorithm>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <dirent.h>
#include <fcntl.h>
#include <limits.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include "ks_internal.h"

namespace ks {
namespace {

constexpr uint32_t kMagic = 0x6b73626bu;  // "kbsk"
enum Op : uint32_t { OP_COUNTS = 1, OP_REGIONS, OP_LOWCOMP, OP_TRLR, OP_WINDOWED, OP_TOFILE };

std::mutex g_mu;
std::mutex g_call_mu;     // a worker's connection carries one request at a time
int g_on = -1;            // -1: KS_FORK_BROKER decides at the first HIP use
bool g_started = false;   // this process forked its broker
bool g_is_broker = false;
pid_t g_owner = 0;        // the process that forked the broker (and then used HIP)
char g_name[96] = {0};    // abstract socket name (without the leading NUL)
int g_fd = -1;            // this process's connection
pid_t g_fd_pid = 0;

struct Buf {
  std::vector<char> b;
  template <typename T>
  void put(const T &v) {
    const char *p = reinterpret_cast<const char *>(&v);
    b.insert(b.end(), p, p + sizeof(T));
  }
  void raw(const void *p, size_t n) {
    if (n) b.insert(b.end(), static_cast<const char *>(p), static_cast<const char *>(p) + n);
  }
  void str(const char *s) {
    const uint32_t n = s ? (uint32_t)strlen(s) : 0;
    put(n);
    raw(s, n);
  }
};

struct Rd {
  const char *p, *e;
  bool ok = true;
  template <typename T>
  T get() {
    T v{};
    if ((size_t)(e - p) < sizeof(T)) {
      ok = false;
      return v;
    }
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  const char *raw(size_t n) {
    if ((size_t)(e - p) < n) {
      ok = false;
      return nullptr;
    }
    const char *q = p;
    p += n;
    return q;
  }
  void copy(void *dst, size_t n) {
    const char *q = raw(n);
    if (q && n) memcpy(dst, q, n);
  }
  std::string str() {
    const uint32_t n = get<uint32_t>();
    const char *q = raw(n);
    return q ? std::string(q, n) : std::string();
  }
};

bool write_all(int fd, const void *p, size_t n) {
  const char *c = static_cast<const char *>(p);
  while (n) {
    const ssize_t w = send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    c += w;
    n -= (size_t)w;
  }
  return true;
}

bool read_all(int fd, void *p, size_t n) {
  char *c = static_cast<char *>(p);
  while (n) {
    const ssize_t r = recv(fd, c, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

sockaddr_un addr_of(socklen_t *len) {
  sockaddr_un a;
  memset(&a, 0, sizeof(a));
  a.sun_family = AF_UNIX;
  const size_t n = strlen(g_name);
  memcpy(a.sun_path + 1, g_name, n);  // abstract namespace: leading NUL
  *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
  return a;
}

// Whether the process already has the GPU driver open (e.g. torch made HIP
// calls before this library's first one).
bool hip_open_here() {
  bool open = false;
  if (DIR *d = opendir("/proc/self/fd")) {
    char path[64], tgt[256];
    while (dirent *e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      snprintf(path, sizeof(path), "/proc/self/fd/%s", e->d_name);
      const ssize_t n = readlink(path, tgt, sizeof(tgt) - 1);
      if (n > 0) {
        tgt[n] = 0;
        if (strcmp(tgt, "/dev/kfd") == 0) open = true;
      }
    }
    closedir(d);
  }
  return open;
}

// ---- the broker side

void put_seqs(Buf &o, const char *const *seqs, const int64_t *lens, int32_t nseq) {
  o.put(nseq);
  o.raw(lens, (size_t)nseq * 8);
  for (int32_t q = 0; q < nseq; ++q) o.raw(seqs[q], (size_t)lens[q]);
}

struct Seqs {
  std::vector<int64_t> lens;
  std::vector<const char *> ptr;
  int32_t n = 0;
};

void get_seqs(Rd &r, Seqs *s) {
  s->n = r.get<int32_t>();
  if (!r.ok || s->n < 0) {
    r.ok = false;
    return;
  }
  s->lens.resize((size_t)s->n);
  r.copy(s->lens.data(), (size_t)s->n * 8);
  s->ptr.resize((size_t)s->n);
  for (int32_t q = 0; q < s->n && r.ok; ++q) {
    if (s->lens[q] < 0) {
      r.ok = false;
      break;
    }
    s->ptr[q] = r.raw((size_t)s->lens[q]);
  }
}

void put_regions(Buf &o, const ks_regions &g) {
  o.put(g.n);
  const size_t n = (size_t)g.n;
  o.raw(g.seq_id, n * 4);
  o.raw(g.beg, n * 4);
  o.raw(g.end, n * 4);
  o.raw(g.score, n * 8);
}

ks_status get_regions(Rd &r, ks_regions *out) {
  const int64_t n = r.get<int64_t>();
  if (!r.ok || n < 0) return fail(KS_ERR_INTERNAL, "broker reply is malformed");
  KS_TRY(regions_alloc(out, n));
  const size_t m = (size_t)n;
  r.copy(out->seq_id, m * 4);
  r.copy(out->beg, m * 4);
  r.copy(out->end, m * 4);
  r.copy(out->score, m * 8);
  if (m) memset(out->score + m, 0, m * 8);
  if (!r.ok) {
    ks_regions_free(out);
    return fail(KS_ERR_INTERNAL, "broker reply is malformed");
  }
  return KS_OK;
}

// Largest request payload of an operation: the sequences and tables of a call
// (a genome, a 4^15 FP64 table) fit; a file request holds two paths.
uint64_t max_request(uint32_t op) {
  return op == OP_TOFILE ? ((uint64_t)1 << 20) : ((uint64_t)1 << 37);
}

// Runs one request in the broker on ctx; returns the reply payload.
Buf serve(ks_ctx *ctx, uint32_t op, Rd &r) {
  Buf o;
  ks_status st = KS_OK;
  Buf out;
  Seqs s;
  switch (op) {
    case OP_COUNTS: {
      get_seqs(r, &s);
      const int32_t k = r.get<int32_t>();
      if (!r.ok || k < 1 || k > KS_MAX_K) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<int32_t> counts((size_t)1 << (2 * k));
      double w = 0;
      st = ks_kmer_counts(ctx, s.ptr.data(), s.lens.data(), s.n, k, counts.data(), &w);
      if (st == KS_OK) {
        out.raw(counts.data(), counts.size() * 4);
        out.put(w);
      }
      break;
    }
    case OP_REGIONS: {
      get_seqs(r, &s);
      const int32_t k = r.get<int32_t>();
      const int64_t wl = r.get<int64_t>();
      if (!r.ok || wl < 0 || wl > ((int64_t)1 << 30)) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<double> w((size_t)wl);
      r.copy(w.data(), (size_t)wl * 8);
      const int32_t mw = r.get<int32_t>();
      const double ms = r.get<double>();
      const uint8_t want_vis = r.get<uint8_t>();
      if (!r.ok || k < 1 || k > KS_MAX_K) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<int32_t> vis(want_vis ? (size_t)1 << (2 * k) : 0);
      double nb = 0;
      ks_regions g;
      memset(&g, 0, sizeof(g));
      st = ks_kmer_regions(ctx, s.ptr.data(), s.lens.data(), s.n, k, w.data(), wl, mw, ms,
                           want_vis ? vis.data() : nullptr, &nb, &g);
      if (st == KS_OK) {
        out.put(nb);
        out.raw(vis.data(), vis.size() * 4);
        put_regions(out, g);
        ks_regions_free(&g);
      }
      break;
    }
    case OP_LOWCOMP: {
      get_seqs(r, &s);
      const int32_t k = r.get<int32_t>(), mw = r.get<int32_t>();
      const double ms = r.get<double>(), thr = r.get<double>();
      if (!r.ok || k < 1 || k > KS_MAX_K) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      const size_t nk = (size_t)1 << (2 * k);
      std::vector<int32_t> counts(nk);
      std::vector<double> ranks(nk);
      double n[2] = {0, 0};
      ks_regions g;
      memset(&g, 0, sizeof(g));
      st = ks_low_comp_regions(ctx, s.ptr.data(), s.lens.data(), s.n, k, mw, ms, thr, counts.data(), ranks.data(),
                               n, &g);
      if (st == KS_OK) {
        out.raw(counts.data(), nk * 4);
        out.raw(ranks.data(), nk * 8);
        out.raw(n, 16);
        put_regions(out, g);
        ks_regions_free(&g);
      }
      break;
    }
    case OP_TRLR: {
      get_seqs(r, &s);
      const int32_t k = r.get<int32_t>(), ml = r.get<int32_t>();
      const int64_t ns = r.get<int64_t>();
      if (!r.ok || ns < 0 || ns > ((int64_t)1 << 30)) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<std::string> km((size_t)ns);
      for (auto &x : km) x = r.str();
      std::vector<double> ksc((size_t)ns), tsc((size_t)ns);
      r.copy(ksc.data(), (size_t)ns * 8);
      r.copy(tsc.data(), (size_t)ns * 8);
      const uint8_t want_sp = r.get<uint8_t>();
      if (!r.ok) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<const char *> kp((size_t)ns);
      for (size_t i = 0; i < km.size(); ++i) kp[i] = km[i].c_str();
      std::vector<double> sp(want_sp ? (size_t)ns * 2 : 0);
      ks_regions g;
      memset(&g, 0, sizeof(g));
      st = ks_tr_lr_regions(ctx, s.ptr.data(), s.lens.data(), s.n, k, ml, kp.data(), ksc.data(), tsc.data(), ns,
                            want_sp ? sp.data() : nullptr, &g);
      if (st == KS_OK) {
        out.raw(sp.data(), sp.size() * 8);
        put_regions(out, g);
        ks_regions_free(&g);
      }
      break;
    }
    case OP_WINDOWED: {
      get_seqs(r, &s);
      const int32_t kn = r.get<int32_t>();
      if (!r.ok || kn < 0 || kn > (1 << 28)) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<std::string> km((size_t)kn);
      for (auto &x : km) x = r.str();
      const int32_t k = r.get<int32_t>(), win = r.get<int32_t>(), flag = r.get<int32_t>();
      std::vector<uint8_t> want_sc((size_t)s.n, 0);
      const uint8_t have_sc = r.get<uint8_t>();
      if (have_sc) r.copy(want_sc.data(), want_sc.size());
      if (!r.ok || win < 0) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<const char *> kp((size_t)kn);
      for (size_t i = 0; i < km.size(); ++i) kp[i] = km[i].c_str();
      std::vector<int32_t> dist((size_t)(win + 1) * (size_t)kn), inc((size_t)s.n);
      std::vector<std::vector<int32_t>> sc((size_t)s.n);
      std::vector<int32_t *> scp((size_t)s.n, nullptr);
      for (int32_t q = 0; q < s.n; ++q)
        if (have_sc && want_sc[q] && s.lens[q] > win) {
          sc[q].resize((size_t)s.lens[q] * (size_t)kn);
          scp[q] = sc[q].data();
        }
      st = ks_windowed_dist(ctx, s.ptr.data(), s.lens.data(), s.n, kp.data(), kn, k, win, flag, dist.data(),
                            inc.data(), have_sc ? scp.data() : nullptr);
      if (st == KS_OK) {
        out.raw(dist.data(), dist.size() * 4);
        out.raw(inc.data(), inc.size() * 4);
        for (int32_t q = 0; q < s.n; ++q) out.raw(sc[q].data(), sc[q].size() * 4);
      }
      break;
    }
    case OP_TOFILE: {
      const std::string path = r.str(), prefix = r.str();
      const int32_t nk = r.get<int32_t>();
      if (!r.ok || nk < 0 || nk > 64) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      std::vector<int32_t> ks((size_t)nk);
      r.copy(ks.data(), (size_t)nk * 4);
      const double ml = r.get<double>();
      const int32_t magic = r.get<int32_t>();
      if (!r.ok) {
        st = fail(KS_ERR_INTERNAL, "broker request is malformed");
        break;
      }
      ks_kmer_file_info info;
      st = ks_kmers_to_file(ctx, path.c_str(), prefix.c_str(), ks.data(), nk, ml, magic, &info);
      if (st == KS_OK) out.raw(&info, sizeof(info));
      break;
    }
    default:
      st = fail(KS_ERR_INTERNAL, "unknown broker request %u", op);
  }
  o.put((int32_t)st);
  o.str(st == KS_OK ? "" : ks_last_error());
  if (st == KS_OK) o.raw(out.b.data(), out.b.size());
  return o;
}

// The parent of pid from /proc (0 if unknown).
pid_t parent_of(pid_t pid) {
  char path[64], buf[512];
  snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE *f = fopen(path, "r");
  if (!f) return 0;
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char *p = strrchr(buf, ')');  // comm may hold spaces and parentheses
  int ppid = 0;
  char state = 0;
  if (!p || sscanf(p + 1, " %c %d", &state, &ppid) != 2) return 0;
  return (pid_t)ppid;
}

// A connecting peer is served only if it runs as this user and descends from
// the process that forked the broker (its fork children, e.g. mclapply
// workers, at any depth).
bool peer_allowed(int fd, pid_t owner) {
  ucred cr;
  socklen_t cl = sizeof(cr);
  if (getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &cr, &cl) != 0 || cl != sizeof(cr)) return false;
  if (cr.uid != getuid()) return false;
  pid_t p = cr.pid;
  for (int depth = 0; depth < 64 && p > 1; ++depth) {
    p = parent_of(p);
    if (p == owner) return true;
  }
  return false;
}

[[noreturn]] void broker_main(int lfd, pid_t owner) {
  // keep stdio and the listening socket; drop what else the owner had open
  if (DIR *d = opendir("/proc/self/fd")) {
    std::vector<int> fds;
    const int dfd = dirfd(d);
    while (dirent *e = readdir(d)) {
      const int fd = atoi(e->d_name);
      if (e->d_name[0] >= '0' && e->d_name[0] <= '9' && fd > 2 && fd != lfd && fd != dfd) fds.push_back(fd);
    }
    closedir(d);
    for (int fd : fds) close(fd);
  }
  int wake[2];  // server threads hand a served connection back to the poll loop
  if (pipe2(wake, O_CLOEXEC) != 0) _exit(1);
  std::mutex mu;
  std::condition_variable cv;
  std::deque<int> ready;  // connections with a request waiting, for the server threads
  int nthreads = 4;
  if (const char *e = getenv("KS_BROKER_THREADS")) nthreads = std::max(1, std::min(64, atoi(e)));
  std::mutex ctx_mu;  // (context creation: the process's first HIP use)
  for (int t = 0; t < nthreads; ++t) {
    std::thread([&, t] {
      ks_ctx *ctx = nullptr;
      for (;;) {
        int fd;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return !ready.empty(); });
          fd = ready.front();
          ready.pop_front();
        }
        uint32_t hdr[2];
        uint64_t len = 0;
        bool ok = read_all(fd, hdr, 8) && read_all(fd, &len, 8) && hdr[0] == kMagic && len <= max_request(hdr[1]);
        std::vector<char> pay;
        if (ok) {
          try {
            pay.resize(len);
          } catch (const std::bad_alloc &) {
            ok = false;
          }
        }
        if (ok) ok = read_all(fd, pay.data(), len);
        if (ok) {
          if (!ctx) {
            std::lock_guard<std::mutex> g(ctx_mu);
            if (ks_ctx_create(0, &ctx) != KS_OK) ctx = nullptr;
          }
          Rd r{pay.data(), pay.data() + pay.size()};
          Buf o;
          if (ctx) {
            o = serve(ctx, hdr[1], r);
          } else {
            o.put((int32_t)KS_ERR_DEVICE);
            o.str(ks_last_error());
          }
          const uint64_t ol = o.b.size();
          ok = write_all(fd, &ol, 8) && write_all(fd, o.b.data(), o.b.size());
        }
        const int msg[2] = {fd, ok ? 1 : 0};  // back to the poll loop (or dropped: a worker ended / sent garbage)
        if (write(wake[1], msg, sizeof(msg)) != (ssize_t)sizeof(msg)) _exit(1);
      }
      (void)t;
    }).detach();
  }
  std::vector<pollfd> pf{{lfd, POLLIN, 0}, {wake[0], POLLIN, 0}};
  for (;;) {
    if (getppid() != owner) _exit(0);  // the owner is gone
    for (auto &p : pf) p.revents = 0;
    const int n = poll(pf.data(), pf.size(), 1000);
    if (n < 0 && errno != EINTR) _exit(1);
    if (n <= 0) continue;
    std::vector<pollfd> back;
    if (pf[1].revents & POLLIN) {  // served connections: listen to them again, or close them
      int msg[2];
      if (read(wake[0], msg, sizeof(msg)) == (ssize_t)sizeof(msg)) {
        if (msg[1]) back.push_back({msg[0], POLLIN, 0});
        else close(msg[0]);
      }
    }
    for (size_t i = pf.size(); i-- > 2;) {
      if (!pf[i].revents) continue;
      const int fd = pf[i].fd;
      pf.erase(pf.begin() + (long)i);  // (a server thread owns it until it comes back)
      {
        std::lock_guard<std::mutex> g(mu);
        ready.push_back(fd);
      }
      cv.notify_one();
    }
    for (const pollfd &p : back) pf.push_back(p);
    if (pf[0].revents & POLLIN) {
      const int c = accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (c >= 0) {
        if (peer_allowed(c, owner)) pf.push_back({c, POLLIN, 0});
        else close(c);
      }
    }
  }
}

// ---- the worker side

ks_status connect_broker(int *out) {
  const pid_t me = getpid();
  if (g_fd >= 0 && g_fd_pid == me) {
    *out = g_fd;
    return KS_OK;
  }
  if (g_fd >= 0 && g_fd_pid != me) g_fd = -1;  // the parent's connection (shared stream): not ours
  const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return fail(KS_ERR_DEVICE, "broker socket failed: %s", strerror(errno));
  socklen_t al = 0;
  const sockaddr_un a = addr_of(&al);
  if (connect(fd, reinterpret_cast<const sockaddr *>(&a), al) != 0) {
    const int e = errno;
    close(fd);
    return fail(KS_ERR_DEVICE, "the GPU broker of process %d is not reachable (%s)", (int)g_owner, strerror(e));
  }
  g_fd = fd;
  g_fd_pid = me;
  *out = fd;
  return KS_OK;
}

// Sends one request, returns the reply's outputs in *rep (status and message
// already taken: a failure in the broker comes back as that status with the
// broker's message).
ks_status call(uint32_t op, const Buf &req, std::vector<char> *rep, Rd *r) {
  std::lock_guard<std::mutex> g(g_call_mu);  // threads of one worker share its connection
  int fd = -1;
  KS_TRY(connect_broker(&fd));
  const uint32_t hdr[2] = {kMagic, op};
  const uint64_t len = req.b.size();
  uint64_t rl = 0;
  if (!write_all(fd, hdr, 8) || !write_all(fd, &len, 8) || !write_all(fd, req.b.data(), req.b.size()) ||
      !read_all(fd, &rl, 8)) {
    close(fd);
    g_fd = -1;
    return fail(KS_ERR_DEVICE, "the GPU broker of process %d went away", (int)g_owner);
  }
  rep->resize(rl);
  if (!read_all(fd, rep->data(), rl)) {
    close(fd);
    g_fd = -1;
    return fail(KS_ERR_DEVICE, "the GPU broker of process %d went away", (int)g_owner);
  }
  *r = Rd{rep->data(), rep->data() + rep->size()};
  const int32_t st = r->get<int32_t>();
  const std::string msg = r->str();
  if (!r->ok) return fail(KS_ERR_INTERNAL, "broker reply is malformed");
  if (st != KS_OK) return fail((ks_status)st, "%s", msg.c_str());
  return KS_OK;
}

}  // namespace

void broker_before_hip() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_started || g_is_broker) return;
  if (g_on < 0) g_on = getenv("KS_FORK_BROKER") && atoi(getenv("KS_FORK_BROKER")) != 0;
  if (!g_on) return;
  g_started = true;
  if (hip_open_here()) return;  // a fork now would copy someone else's HIP state
  const pid_t owner = getpid();
  static int seq = 0;
  snprintf(g_name, sizeof(g_name), "kmer_spans_amd.broker.%d.%d.%d", (int)getuid(), (int)owner, seq++);
  const int lfd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd < 0) {
    g_name[0] = 0;
    return;
  }
  socklen_t al = 0;
  const sockaddr_un a = addr_of(&al);
  if (bind(lfd, reinterpret_cast<const sockaddr *>(&a), al) != 0 || listen(lfd, 64) != 0) {
    close(lfd);
    g_name[0] = 0;
    return;
  }
  const pid_t pid = fork();
  if (pid == 0) {
    // the only thread here held these two locks at the fork
    new (&g_mu) std::mutex();
    broker_reset_locks();
    g_is_broker = true;
    broker_main(lfd, owner);
  }
  close(lfd);
  if (pid < 0) {
    g_name[0] = 0;
    return;
  }
  g_owner = owner;
}

bool broker_wanted(pid_t hip_pid) {
  return g_on == 1 && g_owner != 0 && g_name[0] != 0 && hip_pid == g_owner && getpid() != g_owner;
}

ks_status broker_kmer_counts(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t *counts,
                             double *n_words) {
  Buf q;
  put_seqs(q, seqs, lens, nseq);
  q.put(k);
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_COUNTS, q, &rep, &r));
  r.copy(counts, (size_t)4 << (2 * k));
  *n_words = r.get<double>();
  return r.ok ? KS_OK : fail(KS_ERR_INTERNAL, "broker reply is malformed");
}

ks_status broker_kmer_regions(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, const double *w,
                              int64_t w_len, int32_t min_width, double min_score, int32_t *visits, double *n_bases,
                              ks_regions *out) {
  Buf q;
  put_seqs(q, seqs, lens, nseq);
  q.put(k);
  q.put(w_len);
  q.raw(w, (size_t)w_len * 8);
  q.put(min_width);
  q.put(min_score);
  q.put((uint8_t)(visits != nullptr));
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_REGIONS, q, &rep, &r));
  *n_bases = r.get<double>();
  if (visits) r.copy(visits, (size_t)4 << (2 * k));
  return get_regions(r, out);
}

ks_status broker_low_comp(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t min_width,
                          double min_score, double thr, int32_t *counts, double *ranks, double *n, ks_regions *out) {
  Buf q;
  put_seqs(q, seqs, lens, nseq);
  q.put(k);
  q.put(min_width);
  q.put(min_score);
  q.put(thr);
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_LOWCOMP, q, &rep, &r));
  r.copy(counts, (size_t)4 << (2 * k));
  r.copy(ranks, (size_t)8 << (2 * k));
  r.copy(n, 16);
  return get_regions(r, out);
}

ks_status broker_tr_lr(const char *const *seqs, const int64_t *lens, int32_t nseq, int32_t k, int32_t min_length,
                       const char *const *kmers, const double *kmer_scores, const double *trans_scores,
                       int64_t n_scores, double *spectra, ks_regions *out) {
  Buf q;
  put_seqs(q, seqs, lens, nseq);
  q.put(k);
  q.put(min_length);
  q.put(n_scores);
  for (int64_t i = 0; i < n_scores; ++i) q.str(kmers[i]);
  q.raw(kmer_scores, (size_t)n_scores * 8);
  q.raw(trans_scores, (size_t)n_scores * 8);
  q.put((uint8_t)(spectra != nullptr));
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_TRLR, q, &rep, &r));
  if (spectra) r.copy(spectra, (size_t)n_scores * 16);
  return get_regions(r, out);
}

ks_status broker_windowed(const char *const *seqs, const int64_t *lens, int32_t nseq, const char *const *kmers,
                          int32_t kmer_n, int32_t k, int32_t window, int32_t ret_flag, int32_t *dist,
                          int32_t *seq_included, int32_t *const *scores) {
  Buf q;
  put_seqs(q, seqs, lens, nseq);
  q.put(kmer_n);
  for (int32_t i = 0; i < kmer_n; ++i) q.str(kmers[i]);
  q.put(k);
  q.put(window);
  q.put(ret_flag);
  const bool have = scores != nullptr && (ret_flag & 1);
  q.put((uint8_t)have);
  if (have)
    for (int32_t i = 0; i < nseq; ++i) q.put((uint8_t)(scores[i] != nullptr));
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_WINDOWED, q, &rep, &r));
  r.copy(dist, (size_t)(window + 1) * (size_t)kmer_n * 4);
  r.copy(seq_included, (size_t)nseq * 4);
  if (have)
    for (int32_t i = 0; i < nseq; ++i)
      if (scores[i] && lens[i] > window) r.copy(scores[i], (size_t)lens[i] * (size_t)kmer_n * 4);
  return r.ok ? KS_OK : fail(KS_ERR_INTERNAL, "broker reply is malformed");
}

ks_status broker_kmers_to_file(const char *seq_path, const char *out_prefix, const int32_t *ks, int32_t nk,
                               double min_l, int32_t magic, ks_kmer_file_info *info) {
  // relative paths are the worker's: the broker's working directory is the
  // one the owner had when it first used HIP
  auto absolute = [](const char *p) {
    std::string a = p ? p : "";
    if (!a.empty() && a[0] != '/') {
      char cwd[PATH_MAX];
      if (getcwd(cwd, sizeof(cwd))) a = std::string(cwd) + "/" + a;
    }
    return a;
  };
  const std::string sp = absolute(seq_path), op = absolute(out_prefix);
  Buf q;
  q.str(sp.c_str());
  q.str(op.c_str());
  q.put(nk);
  q.raw(ks, (size_t)nk * 4);
  q.put(min_l);
  q.put(magic);
  std::vector<char> rep;
  Rd r{nullptr, nullptr};
  KS_TRY(call(OP_TOFILE, q, &rep, &r));
  r.copy(info, sizeof(*info));
  return r.ok ? KS_OK : fail(KS_ERR_INTERNAL, "broker reply is malformed");
}

}  // namespace ks

extern "C" ks_status ks_set_fork_broker(int32_t on) {
  std::lock_guard<std::mutex> g(ks::g_mu);
  ks::g_on = on ? 1 : 0;
  return KS_OK;
}
