// alloc_race: does device memory fresh from hipMalloc keep what the first
// kernels after the allocation write into it?  (Hypothesis for the round-4
// intermittent host-entry failures: every wrong value seen was a field that
// read back as 0 -- a chunk's tail begin, a stitch state's begin, a chunk's
// carried entry -- in workspace the call had just allocated.  A clear of new
// VRAM that lands after the call's first writes would do exactly that.)
//
// Each round allocates a set of buffers of sizes not seen before (so they are
// new memory, not blocks the runtime kept), writes a pattern into each right
// after its allocation (a kernel, or an H2D copy from pinned memory), then
// checks every word on the device and counts mismatches and zero words.
// The buffers are freed at the end of the round, as the host entry points
// free their workspace at the end of each call.
//
// Build: hipcc -O2 --offload-arch=gfx950 tools/probes/alloc_race.hip -o tools/probes/alloc_race
// Run:   tools/probes/alloc_race [rounds] [bufs_per_round] [big_gib] [child_gib]
// child_gib > 0: before each round a separate process (this binary, "child
// G") allocates and writes G GiB and exits, so the round's buffers may land
// on VRAM another process just freed (which the driver must clear first).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <spawn.h>
#include <sys/wait.h>

extern char **environ;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

__host__ __device__ inline uint32_t pat(uint32_t seed, uint64_t i) {
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)seed << 32 | seed);
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 32;
  return (uint32_t)x | 1u;  // never 0
}

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = pat(seed, i);
}

// (in reverse order: a word is read by another block -- on another XCD, behind
// another L2 and TLB -- than the one that wrote it)
__global__ void k_check(const uint32_t *p, uint64_t n, uint32_t seed, unsigned long long *out) {
  unsigned long long bad = 0, zero = 0, first = ~0ull;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = n - 1 - j;
    const uint32_t v = p[i];
    if (v != pat(seed, i)) {
      ++bad;
      zero += v == 0;
      first = i < first ? i : first;
    }
  }
  if (bad) {
    atomicAdd(&out[0], bad);
    atomicAdd(&out[1], zero);
    atomicMin(&out[2], first);
  }
}

static int child_main(int gib) {
  void *p = nullptr;
  const size_t b = (size_t)gib << 30;
  CK(hipMalloc(&p, b));
  CK(hipMemset(p, 0x77, b));
  CK(hipDeviceSynchronize());
  return 0;  // (exit without freeing: the process's teardown returns it)
}

static void run_child(const char *self, int gib) {
  char a1[] = "child";
  char a2[16];
  snprintf(a2, sizeof a2, "%d", gib);
  char *argv[] = {const_cast<char *>(self), a1, a2, nullptr};
  pid_t pid = 0;
  if (posix_spawn(&pid, self, nullptr, nullptr, argv, environ) != 0) {
    fprintf(stderr, "spawn failed\n");
    exit(2);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
    fprintf(stderr, "child failed (%d)\n", st);
    exit(2);
  }
}

int main(int argc, char **argv) {
  if (argc > 2 && strcmp(argv[1], "child") == 0) return child_main(atoi(argv[2]));
  const int rounds = argc > 1 ? atoi(argv[1]) : 400;
  const int nb = argc > 2 ? atoi(argv[2]) : 16;
  hipStream_t st, st2;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  unsigned long long *cnt = nullptr;
  CK(hipMalloc(&cnt, 64 * 8 * nb));
  uint32_t *pin = nullptr;
  const size_t pin_words = (size_t)1 << 22;  // 16 MiB pinned source for the copy form
  CK(hipHostMalloc(&pin, pin_words * 4, hipHostMallocDefault));
  unsigned long long tot_bad = 0, tot_zero = 0, tot_bufs = 0, bad_bufs = 0;
  uint64_t rng = 12345;
  auto rnd = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  std::vector<void *> bufs(nb);
  std::vector<uint64_t> words(nb);
  std::vector<uint32_t> seeds(nb);
  std::vector<int> form(nb);
  const int big_gib = argc > 3 ? atoi(argv[3]) : 0;  // each round first dirties and frees this much VRAM
  const int child_gib = argc > 4 ? atoi(argv[4]) : 0;
  for (int r = 0; r < rounds; ++r) {
    if (child_gib > 0) run_child(argv[0], child_gib);
    if (big_gib > 0) {  // freshly freed, written VRAM: the small buffers below may land on it
      void *big = nullptr;
      const size_t bb = ((size_t)(1 + r % big_gib)) << 30;
      CK(hipMalloc(&big, bb));
      CK(hipMemsetAsync(big, 0x5a, bb, st));
      CK(hipStreamSynchronize(st));
      CK(hipFree(big));
    }
    CK(hipMemsetAsync(cnt, 0, 64 * 8 * nb, st));
    for (int j = 0; j < nb; ++j) {
      // sizes from 256 B to 64 MiB, log-uniform, odd multiples of 256 B
      const int lg = 8 + (int)(rnd() % 19);
      uint64_t bytes = ((uint64_t)1 << lg) + 256 * (rnd() % 64);
      words[j] = bytes / 4;
      seeds[j] = (uint32_t)(r * 131 + j * 7 + 1);
      form[j] = (int)(rnd() % 3);  // 0 kernel on st, 1 kernel on st2, 2 H2D copy (small) then kernel
      CK(hipMalloc(&bufs[j], bytes));
      uint32_t *p = static_cast<uint32_t *>(bufs[j]);
      const unsigned g = (unsigned)std::min<uint64_t>((words[j] + 255) / 256, 1024);
      if (form[j] == 2 && words[j] <= pin_words) {
        for (uint64_t i = 0; i < words[j]; ++i) pin[i] = pat(seeds[j], i);
        CK(hipMemcpyAsync(p, pin, words[j] * 4, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));  // (the pinned source is rewritten by the next buffer)
      } else {
        hipLaunchKernelGGL(k_fill, dim3(g), dim3(256), 0, form[j] == 1 ? st2 : st, p, words[j], seeds[j]);
        CK(hipGetLastError());
      }
    }
    CK(hipStreamSynchronize(st2));
    for (int j = 0; j < nb; ++j) {
      const unsigned g = (unsigned)std::min<uint64_t>((words[j] + 255) / 256, 1024);
      hipLaunchKernelGGL(k_check, dim3(g), dim3(256), 0, st, static_cast<const uint32_t *>(bufs[j]), words[j],
                         seeds[j], cnt + 8 * j);
    }
    std::vector<unsigned long long> h(8 * nb);
    CK(hipMemcpyAsync(h.data(), cnt, 64 * nb, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    for (int j = 0; j < nb; ++j) {
      ++tot_bufs;
      if (h[8 * j]) {
        ++bad_bufs;
        tot_bad += h[8 * j];
        tot_zero += h[8 * j + 1];
        if (bad_bufs <= 20)
          printf("round %d buf %d (%llu B at %p, form %d): %llu bad words (%llu zero), first at word %llu\n", r, j,
                 (unsigned long long)words[j] * 4, bufs[j], form[j], h[8 * j], h[8 * j + 1], h[8 * j + 2]);
      }
    }
    for (int j = 0; j < nb; ++j) CK(hipFree(bufs[j]));
    if ((r + 1) % 50 == 0) {
      printf("after %d rounds: %llu buffers, %llu bad (%llu bad words, %llu zero)\n", r + 1, tot_bufs, bad_bufs,
             tot_bad, tot_zero);
      fflush(stdout);
    }
  }
  printf("RESULT buffers %llu bad_buffers %llu bad_words %llu zero_words %llu\n", tot_bufs, bad_bufs, tot_bad,
         tot_zero);
  return bad_bufs ? 1 : 0;
}
