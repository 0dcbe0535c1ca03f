// xcd_stale_probe.hip -- diagnosis: can a line that XCD r's L2 cached in one kernel be read STALE by
// XCD r in a later kernel after a kernel in between rewrote it from XCD w (plain loads and stores,
// one stream, hipMalloc memory)?  The hand-offs of the engine are all kernel boundaries of this kind.
//
//   hipcc --offload-arch=gfx950 -O2 tools/xcd_stale_probe.hip -o /tmp/xcd_stale_probe && /tmp/xcd_stale_probe
//
// Per (reader r, writer w): memset B = 0; touch(B) on XCD r; write(B, v) on XCD w (whole lines, or
// only the first half of every 128-byte line, or every 2-byte element at odd positions); check(B, v)
// on XCD r counts words != expected.  Work-groups read their XCD from HW_REG_XCC_ID; the grid is large
// enough that every XCD gets some.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void touch(const unsigned* B, size_t n, int xcd, unsigned* sink) {
  if (xcc_id() != xcd) return;
  unsigned acc = 0;
  for (size_t i = threadIdx.x; i < n; i += NT) acc += B[i];
  if (acc == 0xdeadbeefu) sink[0] = acc;  // keeps the loads
}

// mode 0: every word; 1: words 0..15 of every 32-word line; 2: the odd 16-bit halves only
__global__ __launch_bounds__(NT) void writek(unsigned* B, size_t n, int xcd, unsigned v, int mode) {
  if (xcc_id() != xcd) return;
  if (blockIdx.x % 64 >= 8) return;  // a few writers per XCD
  for (size_t i = threadIdx.x; i < n; i += NT) {
    if (mode == 0) B[i] = v;
    else if (mode == 1) {
      if ((i & 31) < 16) B[i] = v;
    } else {
      reinterpret_cast<unsigned short*>(B)[2 * i + 1] = (unsigned short)v;
    }
  }
}

__global__ __launch_bounds__(NT) void check(const unsigned* B, size_t n, int xcd, unsigned v, int mode,
                                            unsigned* errs) {
  if (xcc_id() != xcd) return;
  unsigned bad = 0;
  for (size_t i = threadIdx.x; i < n; i += NT) {
    unsigned want = mode == 0 ? v : mode == 1 ? ((i & 31) < 16 ? v : 0u) : (v << 16);
    bad += B[i] != want;
  }
  if (bad) atomicAdd(errs, bad);
}

__global__ void census(int* cnt) { if (threadIdx.x == 0) atomicAdd(&cnt[xcc_id() & 7], 1); }

int main(int argc, char** argv) {
  const size_t n = (argc > 1 ? atol(argv[1]) : 64 * 1024) ;  // words (default 256 KiB)
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  unsigned *B, *sink, *errs;
  int* cnt;
  CK(hipMalloc(&B, n * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&errs, 4));
  CK(hipMalloc(&cnt, 8 * 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int G = 512;
  CK(hipMemsetAsync(cnt, 0, 32, s));
  census<<<G, 64, 0, s>>>(cnt);
  int hc[8];
  CK(hipMemcpyAsync(hc, cnt, 32, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  printf("census:");
  for (int i = 0; i < 8; i++) printf(" %d", hc[i]);
  printf("\n");
  for (int mode = 0; mode < 3; mode++) {
    long total = 0, same_total = 0;
    for (int r = 0; r < 8; r++)
      for (int w = 0; w < 8; w++) {
        long e_pair = 0;
        for (int it = 0; it < iters; it++) {
          const unsigned v = 0x100u + (unsigned)(it * 64 + r * 8 + w);
          CK(hipMemsetAsync(B, 0, n * 4, s));
          CK(hipMemsetAsync(errs, 0, 4, s));
          touch<<<G, NT, 0, s>>>(B, n, r, sink);
          writek<<<G, NT, 0, s>>>(B, n, w, v, mode);
          check<<<G, NT, 0, s>>>(B, n, r, v, mode, errs);
          unsigned he = 0;
          CK(hipMemcpyAsync(&he, errs, 4, hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          e_pair += he;
        }
        if (r == w) same_total += e_pair;
        else total += e_pair;
        if (e_pair) printf("mode %d reader %d writer %d: %ld stale words over %d iters\n", mode, r, w, e_pair, iters);
      }
    printf("mode %d: cross-XCD stale words %ld, same-XCD %ld\n", mode, total, same_total);
  }
  return 0;
}
