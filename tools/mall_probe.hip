// mall_probe.hip -- does streaming a weight matrix into the Infinity Cache (MALL) ahead of
// the GEMV that consumes it shorten that GEMV?  Measures, for the Llama-3-8B projection
// shapes at one token: cold GEMV (rotating > 256 MiB of matrices), warm GEMV (same matrix
// re-read), GEMV right after a prefetch kernel on the same stream, and a latency-bound
// "attention-like" kernel overlapped with a prefetch on a second stream, then the GEMV.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mall_probe.hip -o tools/mall_probe
#include "../llama-p2p_amd/csrc/kernels.hip"

#include <stdio.h>
#include <stdlib.h>

using namespace mx;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__);      \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void prefetch_kernel(const u32x4* p, size_t n16, unsigned* sink) {
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 a, b, c, d;
    if (NT) {
      a = __builtin_nontemporal_load(p + i); b = __builtin_nontemporal_load(p + i + stride);
      c = __builtin_nontemporal_load(p + i + 2 * stride); d = __builtin_nontemporal_load(p + i + 3 * stride);
    } else {
      a = p[i]; b = p[i + stride]; c = p[i + 2 * stride]; d = p[i + 3 * stride];
    }
    acc ^= a[0] ^ b[1] ^ c[2] ^ d[3];
  }
  for (; i < n16; i += stride) acc ^= p[i][0];
  if (acc == 0x9e3779b9u) *sink = acc;  // never true for the fill pattern; keeps the loads
}

// latency-bound stand-in for attention: G work-groups spin for `ns` nanoseconds
__global__ void spin_kernel(long long cycles) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
}

struct Shape {
  const char* name;
  int N, K;
};

int main() {
  const size_t pool = (size_t)4 << 30;
  uint16_t* w;
  CK(hipMalloc(&w, pool));
  CK(hipMemset(w, 0x3c, pool));
  uint16_t* x;
  float* out;
  unsigned* sink;
  CK(hipMalloc(&x, 64 * 14336 * 2));
  CK(hipMemset(x, 0x3c, 64 * 14336 * 2));
  CK(hipMalloc(&out, (size_t)64 * 128256 * 4));
  CK(hipMalloc(&sink, 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, ep;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&ep, hipEventDisableTiming));
  const Shape shapes[] = {{"qkv", 6144, 4096}, {"wo", 4096, 4096}, {"gu", 28672, 4096}, {"down", 4096, 14336}};
  for (const Shape& sh : shapes) {
    MMArgs a{};
    a.N = sh.N; a.K = sh.K; a.X = x; a.ldx = sh.K; a.M = 1; a.out = out; a.ldo = sh.N;
    const size_t mb = (size_t)sh.N * sh.K * 2;
    const int nmat = (int)(pool / mb);
    auto gemv = [&](int i, hipStream_t s) {
      a.W = w + (size_t)(i % nmat) * mb / 2;
      mm_kernel<16, 1, 1, EPI_F32, 4, false><<<sh.N / 16, 1024, 0, s>>>(a);
    };
    auto pf = [&](int i, hipStream_t s, bool nt, int grid) {
      const u32x4* p = reinterpret_cast<const u32x4*>(w + (size_t)(i % nmat) * mb / 2);
      if (nt) prefetch_kernel<true><<<grid, 256, 0, s>>>(p, mb / 16, sink);
      else prefetch_kernel<false><<<grid, 256, 0, s>>>(p, mb / 16, sink);
    };
    const int iters = 2 * nmat;
    float ms;
    // 1. cold
    for (int i = 0; i < nmat; i++) gemv(i, s1);
    CK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; i++) gemv(i, s1);
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double cold = ms * 1e3 / iters;
    // 2. warm (same matrix)
    CK(hipEventRecord(e0, s1));
    for (int i = 0; i < 20; i++) gemv(0, s1);
    CK(hipEventRecord(e1, s1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double warm = ms * 1e3 / 20;
    // 3. prefetch kernel alone (cold), plain and NT
    double pft[2];
    for (int nt = 0; nt < 2; nt++) {
      CK(hipEventRecord(e0, s1));
      for (int i = 0; i < iters; i++) pf(i, s1, nt, 1024);
      CK(hipEventRecord(e1, s1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      pft[nt] = ms * 1e3 / iters;
    }
    // 4. GEMV right after a prefetch of its matrix (time the GEMV only), plain / NT prefetch
    double after[2];
    for (int nt = 0; nt < 2; nt++) {
      double tot = 0;
      for (int i = 0; i < iters; i++) {
        pf(i, s1, nt, 1024);
        CK(hipEventRecord(e0, s1));
        gemv(i, s1);
        CK(hipEventRecord(e1, s1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
      }
      after[nt] = tot * 1e3 / iters;
    }
    // 5. spin(8us, 8 WGs) then GEMV, serial vs spin || prefetch(64 WGs) then GEMV
    const long long cyc = 8 * 100;  // wall_clock64 ticks at 100 MHz -> 8 us
    double ser, ovl;
    {
      CK(hipEventRecord(e0, s1));
      for (int i = 0; i < iters; i++) {
        spin_kernel<<<8, 64, 0, s1>>>(cyc);
        gemv(i, s1);
      }
      CK(hipEventRecord(e1, s1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ser = ms * 1e3 / iters;
      CK(hipEventRecord(e0, s1));
      for (int i = 0; i < iters; i++) {
        CK(hipEventRecord(ep, s1));
        CK(hipStreamWaitEvent(s2, ep, 0));
        pf(i, s2, false, 64);
        spin_kernel<<<8, 64, 0, s1>>>(cyc);
        CK(hipEventRecord(ep, s2));
        CK(hipStreamWaitEvent(s1, ep, 0));
        gemv(i, s1);
      }
      CK(hipEventRecord(e1, s1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ovl = ms * 1e3 / iters;
    }
    printf("%-5s %6.1f MB  cold %7.2f us (%6.0f GB/s)  warm %7.2f  prefetch plain %7.2f nt %7.2f  "
           "gemv-after-plain %7.2f after-nt %7.2f  spin+gemv serial %7.2f  spin||prefetch,gemv %7.2f\n",
           sh.name, mb / 1e6, cold, mb / cold / 1e3, warm, pft[0], pft[1], after[0], after[1], ser, ovl);
    fflush(stdout);
  }
  return 0;
}
