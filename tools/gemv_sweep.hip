// gemv_sweep.hip -- tuning sweep for the decode GEMV (mm_kernel) on the
// Llama-3-8B projection shapes.  Each configuration streams a rotating set of
// distinct weight matrices (> Infinity Cache) so no launch re-reads cached
// bytes; time per launch is measured with hipEvents over many launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemv_sweep.hip -o tools/gemv_sweep
//   ./tools/gemv_sweep            (prints one line per shape x config)
#include "../llama-p2p_amd/csrc/kernels.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

using namespace mx;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

struct Shape {
  const char* name;
  int N, K;
};

static uint16_t* g_w = nullptr;
static size_t g_wbytes = 0;
static uint16_t* g_x = nullptr;
static float* g_out = nullptr;

template <int KS, int RT, int NB, int U>
static void run(const Shape& sh, int M, const char* tag) {
  MMArgs a{};
  a.N = sh.N;
  a.K = sh.K;
  a.X = g_x;
  a.ldx = sh.K;
  a.M = M;
  a.out = g_out;
  a.ldo = sh.N;
  const size_t mbytes = (size_t)sh.N * sh.K * 2;
  const int nmat = (int)(g_wbytes / mbytes);
  const int grid = sh.N / (16 * RT);
  if (sh.N % (16 * RT)) return;
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int iters = 3 * nmat;
  for (int i = 0; i < nmat; i++) {
    a.W = g_w + (size_t)i * mbytes / 2;
    mm_kernel<KS, RT, NB, EPI_F32, U, false><<<grid, 64 * KS>>>(a);
  }
  CK(hipEventRecord(t0));
  for (int i = 0; i < iters; i++) {
    a.W = g_w + (size_t)(i % nmat) * mbytes / 2;
    mm_kernel<KS, RT, NB, EPI_F32, U, false><<<grid, 64 * KS>>>(a);
  }
  CK(hipEventRecord(t1));
  CK(hipEventSynchronize(t1));
  float ms;
  CK(hipEventElapsedTime(&ms, t0, t1));
  const double us = ms * 1e3 / iters;
  printf("%-6s M=%-3d KS=%-2d RT=%d NB=%d U=%-2d grid=%-6d  %8.2f us  %7.1f GB/s %s\n", sh.name, M, KS, RT, NB, U,
         grid, us, mbytes / us / 1e3, tag);
  fflush(stdout);
  hipEventDestroy(t0);
  hipEventDestroy(t1);
}

template <int NB>
static void sweep(const Shape& sh, int M) {
  run<4, 1, NB, 8>(sh, M, "");
  run<8, 1, NB, 8>(sh, M, "");
  run<16, 1, NB, 8>(sh, M, "");
  run<4, 1, NB, 16>(sh, M, "");
  run<8, 1, NB, 16>(sh, M, "");
  run<16, 1, NB, 4>(sh, M, "");
  run<4, 2, NB, 8>(sh, M, "");
  run<8, 2, NB, 8>(sh, M, "");
  run<2, 1, NB, 16>(sh, M, "");
  run<2, 2, NB, 8>(sh, M, "");
  run<4, 4, NB, 4>(sh, M, "");
  run<8, 4, NB, 4>(sh, M, "");
}

template <int W, int RTW>
static void runw(const Shape& sh, int M, int ksplit) {
  MMArgs a{};
  a.N = sh.N;
  a.K = sh.K;
  a.X = g_x;
  a.ldx = sh.K;
  a.M = M;
  a.out = g_out;
  a.ldo = sh.N;
  a.slab_stride = (size_t)64 * sh.N;
  const size_t mbytes = (size_t)sh.N * sh.K * 2;
  const int nmat = (int)(g_wbytes / mbytes);
  const int ntiles = sh.N / 16, KT = sh.K / 32;
  if (ntiles % (W * RTW) || KT % (ksplit * 4)) return;
  dim3 grid(ntiles / (W * RTW), ksplit);
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int iters = 3 * nmat;
  for (int i = 0; i < nmat; i++) {
    a.W = g_w + (size_t)i * mbytes / 2;
    mm_wide_kernel<W, RTW, 2, EPI_SLAB><<<grid, 64 * W>>>(a);
  }
  CK(hipEventRecord(t0));
  for (int i = 0; i < iters; i++) {
    a.W = g_w + (size_t)(i % nmat) * mbytes / 2;
    mm_wide_kernel<W, RTW, 2, EPI_SLAB><<<grid, 64 * W>>>(a);
  }
  CK(hipEventRecord(t1));
  CK(hipEventSynchronize(t1));
  float ms;
  CK(hipEventElapsedTime(&ms, t0, t1));
  const double us = ms * 1e3 / iters;
  printf("WIDE %-6s M=%-3d W=%d RTW=%d ksplit=%d grid=%-5dx%d  %8.2f us  %7.1f GB/s\n", sh.name, M, W, RTW, ksplit,
         grid.x, grid.y, us, mbytes / us / 1e3);
  fflush(stdout);
  hipEventDestroy(t0);
  hipEventDestroy(t1);
}

static void sweep_wide(const Shape& sh, int M) {
  for (int ks : {1, 2, 4, 8}) {
    runw<4, 1>(sh, M, ks);
    runw<8, 1>(sh, M, ks);
    runw<2, 1>(sh, M, ks);
    runw<4, 2>(sh, M, ks);
    runw<2, 2>(sh, M, ks);
    runw<8, 2>(sh, M, ks);
  }
}

static void sweep_wide_odd(const Shape& sh, int M) {
  for (int ks : {1, 2, 4, 8}) {
    runw<3, 1>(sh, M, ks);
    runw<6, 1>(sh, M, ks);
    runw<7, 1>(sh, M, ks);
    runw<3, 2>(sh, M, ks);
    runw<4, 2>(sh, M, ks);
    runw<2, 1>(sh, M, ks);
  }
}

int main(int argc, char** argv) {
  const bool odd = argc > 1 && argv[1][0] == 'o';
  const bool wide_only = argc > 1;
  g_wbytes = (size_t)6 << 30;  // 6 GiB of distinct weights to rotate through
  CK(hipMalloc(&g_w, g_wbytes));
  CK(hipMemset(g_w, 0x3c, g_wbytes));  // bf16 ~1.0: finite, non-zero data
  CK(hipMalloc(&g_x, (size_t)64 * 14336 * 2));
  CK(hipMemset(g_x, 0x3c, (size_t)64 * 14336 * 2));
  CK(hipMalloc(&g_out, (size_t)8 * 64 * 128256 * 4));  // room for 8 split-K slabs of the largest N
  const Shape shapes[] = {{"qkv", 6144, 4096}, {"wo", 4096, 4096}, {"gu", 28672, 4096},
                          {"down", 4096, 14336}, {"lmhead", 128256, 4096}};
  if (!wide_only && !odd) {
    for (const Shape& sh : shapes) sweep<1>(sh, 1);
    for (const Shape& sh : shapes) sweep<2>(sh, 32);
  }
  if (odd) {
    for (const Shape& sh : shapes) sweep_wide_odd(sh, 32);
    return 0;
  }
  for (const Shape& sh : shapes) sweep_wide(sh, 32);
  return 0;
}
