// ks_io.cpp -- sequence-file ingest and the binary count-file format
// (SURVEY 8(f) #2 and #4).
//
// kmers.to.file (kmer_spans.R:127-160) reads a sequence file, drops records
// shorter than min.l, counts k-mers for every k and writes
//   int32 magic (kmer.magic() = 310572, :5), int32 n, n x int32 4^k,
//   then the n count vectors (int32, native byte order, R writeBin);
// read.kmers (:162-186) reads it back (FALSE on a wrong magic or n < 1).
//
// Ingest: the file is memory-mapped (or inflated, for gzip) and streamed to
// HBM through two pinned staging halves, so the copy of one half overlaps the
// fill of the other; the device parses it (ks_ingest.hip).  Names come from
// the host view at the description-line positions the device reports.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "ks_internal.h"

namespace ks {
namespace {

// The bytes of a sequence file: mapped, inflated, or borrowed.
struct HostView {
  const uint8_t *p = nullptr;
  size_t n = 0;
  void *map = nullptr;
  size_t map_len = 0;
  std::vector<uint8_t> buf;
  HostView() = default;
  HostView(const HostView &) = delete;
  HostView &operator=(const HostView &) = delete;
  ~HostView() {
    if (map) munmap(map, map_len);
  }
};

ks_status open_view(const char *path, HostView *v) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(KS_ERR_ARG, "cannot open '%s'", path);
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return fail(KS_ERR_ARG, "cannot stat '%s'", path);
  }
  uint8_t magic[2] = {0, 0};
  const bool gz = sb.st_size >= 2 && pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
  if (!gz) {
    v->n = (size_t)sb.st_size;
    if (v->n) {
      v->map = mmap(nullptr, v->n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (v->map == MAP_FAILED) {
        v->map = nullptr;
        close(fd);
        return fail(KS_ERR_ARG, "cannot map '%s'", path);
      }
      v->map_len = v->n;
      madvise(v->map, v->n, MADV_SEQUENTIAL);
      v->p = static_cast<const uint8_t *>(v->map);
    }
    close(fd);
    return KS_OK;
  }
  close(fd);
  gzFile g = gzopen(path, "rb");
  if (!g) return fail(KS_ERR_ARG, "cannot open '%s'", path);
  gzbuffer(g, 1 << 20);
  v->buf.resize(std::max<size_t>((size_t)sb.st_size * 4, (size_t)1 << 20));
  size_t have = 0;
  for (;;) {
    if (have == v->buf.size()) v->buf.resize(v->buf.size() * 2);
    const size_t want = std::min<size_t>(v->buf.size() - have, (size_t)1 << 30);
    const int got = gzread(g, v->buf.data() + have, (unsigned)want);
    if (got < 0) {
      int e = 0;
      const char *m = gzerror(g, &e);
      gzclose(g);
      return fail(KS_ERR_ARG, "'%s': gzip error: %s", path, m ? m : "?");
    }
    if (got == 0) break;
    have += (size_t)got;
  }
  gzclose(g);
  v->buf.resize(have);
  v->p = v->buf.data();
  v->n = have;
  return KS_OK;
}

// Host bytes -> device buffer (n + 32 bytes) through two pinned halves.
ks_status upload(ks_ctx *ctx, const uint8_t *src, size_t n, uint8_t **d_out) {
  void *d = nullptr;
  KS_TRY(ensure(ctx, SLOT_SEQ, n + 32, &d));
  *d_out = static_cast<uint8_t *>(d);
  if (!n) return KS_OK;
  const size_t half = std::min<size_t>((size_t)64 << 20, (n + 4095) & ~(size_t)4095);
  void *pin = nullptr;
  KS_TRY(ensure_pinned(ctx, 2 * half, &pin));
  hipEvent_t ev[2];
  KS_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
  KS_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
  const unsigned hw = std::thread::hardware_concurrency();
  const int nt = (int)std::max(1u, std::min(hw ? hw : 1u, 8u));
  ks_status rc = KS_OK;
  size_t i = 0;
  for (size_t off = 0; off < n && rc == KS_OK; off += half, ++i) {
    const size_t len = std::min(half, n - off);
    uint8_t *h = static_cast<uint8_t *>(pin) + (i & 1) * half;
    if (i >= 2 && hipEventSynchronize(ev[i & 1]) != hipSuccess) {
      rc = fail(KS_ERR_DEVICE, "staging event failed");
      break;
    }
    if (len >= ((size_t)4 << 20) && nt > 1) {
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t) {
        const size_t a = len * t / nt, b = len * (t + 1) / nt;
        th.emplace_back([=] { memcpy(h + a, src + off + a, b - a); });
      }
      for (auto &x : th) x.join();
    } else {
      memcpy(h, src + off, len);
    }
    if (hipMemcpyAsync(*d_out + off, h, len, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipEventRecord(ev[i & 1], ctx->stream) != hipSuccess)
      rc = fail(KS_ERR_DEVICE, "sequence upload failed");
  }
  if (rc == KS_OK && hipMemsetAsync(*d_out + n, 0, 32, ctx->stream) != hipSuccess)
    rc = fail(KS_ERR_DEVICE, "hipMemsetAsync failed");
  if (rc == KS_OK && hipStreamSynchronize(ctx->stream) != hipSuccess)
    rc = fail(KS_ERR_DEVICE, "sequence upload failed");
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  return rc;
}

int64_t line_of(const HostView &v, int64_t pos) {
  int64_t line = 1;
  const uint8_t *p = v.p, *e = v.p + pos;
  while ((p = static_cast<const uint8_t *>(memchr(p, '\n', (size_t)(e - p)))) != nullptr) {
    ++line;
    ++p;
  }
  return line;
}

void fasta_reset(ks_fasta *f) { memset(f, 0, sizeof(*f)); }

// Parse the view on the device and fill *out (kept records only).
ks_status fasta_from_view(ks_ctx *ctx, const HostView &v, const char *what, int64_t min_len, ks_fasta *out) {
  const double t0 = now_ms();
  uint8_t *d_raw = nullptr;
  KS_TRY(upload(ctx, v.p, v.n, &d_raw));
  const double t1 = now_ms();
  FastaParse fp;
  KS_TRY(fasta_parse_dev(ctx, d_raw, (int64_t)v.n, &fp));
  if (fp.err_pos >= 0) {
    const uint8_t c = v.p[fp.err_pos];
    return fail(KS_ERR_ARG, "reading FASTA %s: invalid one-letter sequence code '%c' (0x%02x) at line %lld", what,
                (c >= 32 && c < 127) ? c : '?', c, (long long)line_of(v, fp.err_pos));
  }
  if (fp.first_kept >= 0 && (fp.first_hdr < 0 || fp.first_kept < fp.first_hdr))
    return fail(KS_ERR_ARG, "reading FASTA %s: sequence data before the first description line (line %lld)", what,
                (long long)line_of(v, fp.first_kept));
  struct Guard {
    FastaParse *fp;
    ~Guard() {
      if (fp->out) (void)hipFree(fp->out);
    }
  } guard{&fp};
  out->n_records = fp.n_records;
  out->bases_all = fp.total;
  std::vector<int32_t> keep;
  keep.reserve((size_t)fp.n_records);
  for (int64_t r = 0; r < fp.n_records; ++r)
    if (fp.offsets[r + 1] - fp.offsets[r] >= min_len) keep.push_back((int32_t)r);
  std::vector<int64_t> hdr;
  hdr.reserve(keep.size());
  for (int32_t r : keep) hdr.push_back(fp.hdr_pos[r]);
  if ((int64_t)keep.size() != fp.n_records) KS_TRY(fasta_select_dev(ctx, &fp, keep));
  const int32_t nseq = (int32_t)keep.size();
  for (int32_t q = 0; q < nseq; ++q)
    if (fp.offsets[q + 1] - fp.offsets[q] > INT32_MAX)
      return fail(KS_ERR_ARG, "reading FASTA %s: record %d is longer than 2^31-1 bases", what, q + 1);
  int64_t *oh = static_cast<int64_t *>(malloc(((size_t)nseq + 1) * 8));
  char **names = static_cast<char **>(calloc((size_t)nseq + 1, sizeof(char *)));
  int64_t *od = nullptr;
  if (!oh || !names || hipMalloc(&od, ((size_t)nseq + 1) * 8) != hipSuccess) {
    free(oh);
    free(names);
    return fail(KS_ERR_NOMEM, "out of memory for %d FASTA records", nseq);
  }
  memcpy(oh, fp.offsets.data(), ((size_t)nseq + 1) * 8);
  for (int32_t q = 0; q < nseq; ++q) {
    const uint8_t *a = v.p + hdr[q] + 1, *e = v.p + v.n;
    const uint8_t *nl = static_cast<const uint8_t *>(memchr(a, '\n', (size_t)(e - a)));
    const uint8_t *b = nl ? nl : e;
    if (b > a && b[-1] == '\r') --b;
    names[q] = static_cast<char *>(malloc((size_t)(b - a) + 1));
    if (names[q]) {
      memcpy(names[q], a, (size_t)(b - a));
      names[q][b - a] = 0;
    }
  }
  if (hipMemcpyAsync(od, oh, ((size_t)nseq + 1) * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    for (int32_t q = 0; q < nseq; ++q) free(names[q]);
    free(names);
    free(oh);
    (void)hipFree(od);
    return fail(KS_ERR_DEVICE, "offset upload failed");
  }
  out->seqs.seq = fp.out;
  out->seqs.offsets_host = oh;
  out->seqs.offsets_dev = od;
  out->seqs.nseq = nseq;
  out->names = names;
  out->bases_kept = fp.total;
  out->device = ctx->device;
  out->ms_upload = t1 - t0;
  out->ms_parse = now_ms() - t1;
  fp.out = nullptr;  // now owned by *out
  return KS_OK;
}

}  // namespace
}  // namespace ks

using namespace ks;

extern "C" void ks_fasta_free(ks_fasta *f) {
  if (!f) return;
  if (hip_usable_here()) {  // (a child forked after HIP init leaves the parent's device memory alone)
    if (f->seqs.seq || f->seqs.offsets_dev) (void)hipSetDevice(f->device);
    if (f->seqs.seq) (void)hipFree((void *)f->seqs.seq);
    if (f->seqs.offsets_dev) (void)hipFree((void *)f->seqs.offsets_dev);
  }
  if (f->names)
    for (int32_t q = 0; q < f->seqs.nseq; ++q) free(f->names[q]);
  free(f->names);
  free((void *)f->seqs.offsets_host);
  fasta_reset(f);
}

extern "C" ks_status ks_fasta_load(ks_ctx *ctx, const char *path, int64_t min_len, ks_fasta *out) {
  if (!path || !out) return fail(KS_ERR_ARG, "null argument");
  fasta_reset(out);
  KS_TRY(default_ctx(&ctx));
  HostView v;
  KS_TRY(open_view(path, &v));
  KS_ENTER(ctx);
  return fasta_from_view(ctx, v, path, min_len, out);
}

extern "C" ks_status ks_fasta_parse(ks_ctx *ctx, const char *buf, int64_t n, int64_t min_len, ks_fasta *out) {
  if (!out || n < 0 || (n > 0 && !buf)) return fail(KS_ERR_ARG, "null argument");
  fasta_reset(out);
  KS_TRY(default_ctx(&ctx));
  HostView v;
  v.p = reinterpret_cast<const uint8_t *>(buf);
  v.n = (size_t)n;
  KS_ENTER(ctx);
  return fasta_from_view(ctx, v, "buffer", min_len, out);
}

extern "C" ks_status ks_fasta_copy_seqs(const ks_fasta *f, uint8_t *dst) {
  if (!f || !dst) return fail(KS_ERR_ARG, "null argument");
  const int64_t n = f->seqs.nseq ? f->seqs.offsets_host[f->seqs.nseq] : 0;
  if (!n) return KS_OK;
  KS_HIP(hipSetDevice(f->device));
  KS_HIP(hipMemcpy(dst, f->seqs.seq, (size_t)n, hipMemcpyDeviceToHost));
  return KS_OK;
}

extern "C" ks_status ks_count_multi_dev(ks_ctx *ctx, const ks_dev_seqs *s, const int32_t *ks, int32_t nk,
                                        int32_t *const *counts_dev, double *n_words) {
  if (!ctx || !s || (nk > 0 && (!ks || !counts_dev || !n_words)) || nk < 0) return fail(KS_ERR_ARG, "null argument");
  if (s->nseq < 1 || !s->offsets_host || !s->offsets_dev)
    return fail(KS_ERR_ARG, "seq_r must be a character vector of length at least one");
  if (((uintptr_t)s->seq & 15u) != 0) return fail(KS_ERR_ARG, "device sequence buffer must be 16-byte aligned");
  for (int32_t i = 0; i < nk; ++i) {
    if (ks[i] < 1 || ks[i] > KS_MAX_K) return fail(KS_ERR_ARG, "k must be a positive integer less than 1+MAX_K");
    if (!counts_dev[i]) return fail(KS_ERR_ARG, "null count buffer");
  }
  KS_ENTER(ctx);
  return launch_count_multi(ctx, s, s->offsets_host[s->nseq], ks, nk, counts_dev, n_words);
}

extern "C" ks_status ks_count_file_write(const char *path, int32_t magic, int32_t nk, const int32_t *ks,
                                         const int32_t *const *counts) {
  if (!path || nk < 0 || (nk > 0 && (!ks || !counts))) return fail(KS_ERR_ARG, "null argument");
  for (int32_t i = 0; i < nk; ++i)
    if (ks[i] < 1 || ks[i] > KS_MAX_K || !counts[i]) return fail(KS_ERR_ARG, "invalid k (%d)", ks[i]);
  FILE *f = fopen(path, "wb");
  if (!f) return fail(KS_ERR_ARG, "cannot open '%s' for writing", path);
  bool ok = fwrite(&magic, 4, 1, f) == 1 && fwrite(&nk, 4, 1, f) == 1;  // kmer_spans.R:153-154
  for (int32_t i = 0; ok && i < nk; ++i) {
    const int32_t len = 1 << (2 * ks[i]);                                // :155-156
    ok = fwrite(&len, 4, 1, f) == 1;
  }
  for (int32_t i = 0; ok && i < nk; ++i) {                               // :157-158
    const size_t len = (size_t)1 << (2 * ks[i]);
    ok = fwrite(counts[i], 4, len, f) == len;
  }
  if (fclose(f) != 0) ok = false;
  return ok ? KS_OK : fail(KS_ERR_ARG, "write to '%s' failed", path);
}

extern "C" void ks_count_file_free(ks_count_file *c) {
  if (!c) return;
  if (c->counts)
    for (int32_t i = 0; i < c->nk; ++i) free(c->counts[i]);
  free(c->counts);
  free(c->k);
  free(c->lens);
  memset(c, 0, sizeof(*c));
}

extern "C" ks_status ks_count_file_read(const char *path, int32_t magic, ks_count_file *out) {
  if (!path || !out) return fail(KS_ERR_ARG, "null argument");
  memset(out, 0, sizeof(*out));
  FILE *f = fopen(path, "rb");
  if (!f) return fail(KS_ERR_ARG, "cannot open file '%s'", path);
  int32_t m = 0, kn = 0;
  if (fread(&m, 4, 1, f) != 1 || m != magic || fread(&kn, 4, 1, f) != 1 || kn < 1) {  // :163-172
    fclose(f);
    return KS_OK;  // valid = 0: read.kmers returns FALSE
  }
  std::vector<int32_t> lens((size_t)kn, 0);
  const size_t got = fread(lens.data(), 4, (size_t)kn, f);  // readBin stops at EOF
  lens.resize(got);
  out->nk = (int32_t)got;
  out->k = static_cast<int32_t *>(calloc(got ? got : 1, 4));
  out->lens = static_cast<int64_t *>(calloc(got ? got : 1, 8));
  out->counts = static_cast<int32_t **>(calloc(got ? got : 1, sizeof(int32_t *)));
  if (!out->k || !out->lens || !out->counts) {
    fclose(f);
    ks_count_file_free(out);
    return fail(KS_ERR_NOMEM, "out of memory");
  }
  for (size_t i = 0; i < got; ++i) {
    if (lens[i] < 0) {
      fclose(f);
      ks_count_file_free(out);
      return fail(KS_ERR_ARG, "invalid 'n' argument");  // readBin(n < 0)
    }
    // k = as.integer(log2(n) / 2) (:184); n = 0 gives -Inf -> NA (-1 here)
    out->k[i] = lens[i] > 0 ? (int32_t)(std::log2((double)lens[i]) / 2) : -1;
    out->counts[i] = static_cast<int32_t *>(malloc((size_t)std::max(lens[i], 1) * 4));
    if (!out->counts[i]) {
      fclose(f);
      ks_count_file_free(out);
      return fail(KS_ERR_NOMEM, "out of memory");
    }
    out->lens[i] = (int64_t)fread(out->counts[i], 4, (size_t)lens[i], f);
  }
  fclose(f);
  out->valid = 1;
  return KS_OK;
}

extern "C" ks_status ks_kmers_to_file(ks_ctx *ctx, const char *seq_path, const char *out_prefix, const int32_t *ks,
                                      int32_t nk, double min_l, int32_t magic, ks_kmer_file_info *info) {
  if (!seq_path || !out_prefix || !info || nk < 0 || (nk > 0 && !ks)) return fail(KS_ERR_ARG, "null argument");
  memset(info, 0, sizeof(*info));
  // out.f <- paste0(out.prefix, "counts_", paste(k, collapse="_"), ".bin") (:128)
  std::string of = std::string(out_prefix) + "counts_";
  for (int32_t i = 0; i < nk; ++i) of += (i ? "_" : "") + std::to_string(ks[i]);
  of += ".bin";
  if (of.size() >= sizeof(info->out_path)) return fail(KS_ERR_ARG, "output path too long");
  memcpy(info->out_path, of.c_str(), of.size() + 1);
  if (use_broker()) return broker_kmers_to_file(seq_path, out_prefix, ks, nk, min_l, magic, info);
  KS_TRY(default_ctx(&ctx));
  // (the context is this thread's before the end-of-call guard exists: a
  // refused call must not release another thread's workspace)
  KS_ENTER(ctx);
  struct End {  // a host-buffer entry point: ks_set_host_cache policy
    ks_ctx *c;
    ~End() { host_call_end(c); }
  } const host_end{ctx};
  // read.count() inside try(): any failure there is the NA result (:145-148)
  auto na = [&](const char *why) {
    info->written = 0;
    snprintf(info->message, sizeof(info->message), "%s", why);
    return KS_OK;
  };
  HostView v;
  if (open_view(seq_path, &v) != KS_OK) return na(ks_last_error());
  ks_fasta fa;
  fasta_reset(&fa);
  const int64_t ml = std::isfinite(min_l) ? (int64_t)std::ceil(min_l) : (min_l > 0 ? INT64_MAX : INT64_MIN);
  ks_status rc = fasta_from_view(ctx, v, seq_path, ml, &fa);
  if (rc == KS_ERR_DEVICE || rc == KS_ERR_NOMEM) return rc;
  if (rc != KS_OK) return na(ks_last_error());
  info->seq_size = (double)fa.bases_all;   // :139
  info->seq_fsize = (double)fa.bases_kept; // :141
  info->seq_fl = (double)fa.seqs.nseq;     // :142
  if (fa.seqs.nseq < 1) {
    ks_fasta_free(&fa);
    return na("No sequence after length filtering");  // :143-144
  }
  for (int32_t i = 0; i < nk; ++i)
    if (ks[i] < 1 || ks[i] > KS_MAX_K) {
      ks_fasta_free(&fa);
      return na("k must be a positive integer less than 1+MAX_K");  // kmer_counts :461-462
    }
  std::vector<int32_t *> d_counts((size_t)nk, nullptr);
  std::vector<std::vector<int32_t>> h_counts((size_t)nk);
  std::vector<double> words((size_t)nk, 0.0);
  rc = KS_OK;
  for (int32_t i = 0; i < nk && rc == KS_OK; ++i) {
    const size_t nb = (size_t)4 << (2 * ks[i]);
    if (hipMalloc(&d_counts[i], nb) != hipSuccess || hipMemsetAsync(d_counts[i], 0, nb, ctx->stream) != hipSuccess)
      rc = fail(KS_ERR_NOMEM, "hipMalloc for k=%d counts failed", ks[i]);
  }
  if (rc == KS_OK && nk) rc = launch_count_multi(ctx, &fa.seqs, fa.bases_kept, ks, nk, d_counts.data(), words.data());
  for (int32_t i = 0; i < nk && rc == KS_OK; ++i) {
    h_counts[i].resize((size_t)1 << (2 * ks[i]));
    if (hipMemcpy(h_counts[i].data(), d_counts[i], h_counts[i].size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(KS_ERR_DEVICE, "count copy failed");
  }
  for (auto p : d_counts)
    if (p) (void)hipFree(p);
  ks_fasta_free(&fa);
  if (rc != KS_OK) return rc;
  std::vector<const int32_t *> cp((size_t)nk);
  for (int32_t i = 0; i < nk; ++i) cp[i] = h_counts[i].data();
  KS_TRY(ks_count_file_write(info->out_path, magic, nk, ks, cp.data()));
  info->written = 1;
  return KS_OK;
}
