// phase_probe.hip -- what does a decode step pay per dependent GEMV phase on MI355X, and how much of
// it does a persistent kernel with grid barriers recover?
//
// A "phase" = every one of G work-groups (1024 threads) streams S bytes of its own weights and reads
// the whole activation vector the previous phase wrote (G x 16 floats), then writes its 16 floats --
// the dependency shape of a chain of decode GEMVs (each needs every output of the previous one).
//   kernels: P kernels captured in one hipGraph (the engine's launch structure)
//   persist: one kernel, P phases separated by grid barriers: each work-group issues its next
//            phase's weight loads, then waits for the barrier (sc1 write-through activations, one
//            relaxed agent-scope counter add per work-group, one polling lane, bounded spin), then
//            reads the activations with sc1 loads (no acquire fence needed)
// Both check the activation chain (value after P phases == P) and report us per phase.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/phase_probe.hip -o tools/phase_probe
//   tools/phase_probe [x]   (x: the XCD-local hand-off variants, round 6)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e = (x);                                                                   \
    if (e != hipSuccess) {                                                                \
      fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NT = 1024;
constexpr int SPIN_MAX = 1 << 22;

// weights of (phase, work-group): S bytes = NT threads x U x 16 B, summed into a value that is
// (almost) never stored, so the loads stay
template <int U>
__device__ __forceinline__ void wload(u32x4 (&r)[U], const u32x4* w, int p, int g, int G) {
  const u32x4* b = w + ((size_t)p * G + g) * NT * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = __builtin_nontemporal_load(b + u * NT);
}
template <int U>
__device__ __forceinline__ unsigned wsum(const u32x4 (&r)[U]) {
  unsigned s = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) s ^= r[u][0] ^ r[u][1] ^ r[u][2] ^ r[u][3];
  return s;
}

// the phase's activation work: mean of the previous G x 16 values (+1) -> this group's 16 values
__device__ __forceinline__ float reduce_block(float v) {
  __shared__ float part[NT / 64];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += part[i];
  __syncthreads();
  return s;
}

template <int U>
__global__ __launch_bounds__(NT) void phase_kernel(const u32x4* w, const float* ain, float* aout, int p, int G,
                                                   unsigned* sink) {
  u32x4 r[U];
  if (w) wload<U>(r, w, p, blockIdx.x, G);
  float v = 0.f;
  for (int i = threadIdx.x; i < G * 16; i += NT) v += ain[i];
  const float m = reduce_block(v) / (G * 16) + 1.f;
  if (threadIdx.x < 16) aout[blockIdx.x * 16 + threadIdx.x] = m;
  if (w && wsum<U>(r) == 0x9e3779b9u) *sink = 1;
}

template <int U>
__global__ __launch_bounds__(NT) void persist_kernel(const u32x4* w, float* act, int P, int G, unsigned* cnt,
                                                     unsigned* err, unsigned* sink) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(act, (short)0, (int)(2 * G * 16 * 4), 0x00020000);
  __shared__ int ok;
  unsigned acc = 0;
  for (int p = 0; p < P; ++p) {
    u32x4 r[U];
    if (w) wload<U>(r, w, p, blockIdx.x, G);  // issued before the wait: streams under the barrier
    if (p > 0) {  // barrier: every group has published phase p-1
      if (threadIdx.x == 0) {
        int s = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(G * p) && ++s < SPIN_MAX)
          __builtin_amdgcn_s_sleep(1);
        ok = s < SPIN_MAX;
        if (!ok) atomicOr(err, 1u);
      }
      __syncthreads();
      if (!ok) return;
    }
    const int src = (p & 1) ^ 1, dst = p & 1;
    float v = 0.f;
    for (int i = threadIdx.x; i < G * 16; i += NT) {  // sc1 loads: past this CU's L1 (written by other CUs)
      const unsigned off = (unsigned)((src * G * 16 + i) * 4);
      v += p > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 16)) : 0.f;
    }
    const float m = reduce_block(v) / (G * 16) + 1.f;
    if (threadIdx.x < 16)  // sc1 (write-through) store
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, m), rs, (unsigned)((dst * G * 16 + blockIdx.x * 16 + threadIdx.x) * 4), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w) acc ^= wsum<U>(r);
  }
  if (acc == 0x9e3779b9u) *sink = 1;
}

// XCD-local persistent chain (round 6): only the G work-groups of XCD 0 (blockIdx % 8 == 0 under the
// round-robin dispatch) take part; the others exit at once.  MODE 1: the cross-XCD protocol above
// (sc1 stores / loads, agent-scope counter); MODE 2: L2-coherent within the XCD -- plain stores (the
// vector L1 writes through to L2), sc0 loads that skip only the L1, a workgroup-scope counter add
// (executed at the XCD's L2) polled with an sc0 load.  What does a hand-off cost when it never
// leaves one XCD's L2?
template <int MODE>
__global__ __launch_bounds__(NT) void persist_xcd_kernel(float* act, int P, unsigned* cnt, unsigned* err) {
  if (blockIdx.x % 8) return;
  const int G = gridDim.x / 8, g = blockIdx.x / 8;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(act, (short)0, (int)(2 * G * 16 * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t cs = __builtin_amdgcn_make_buffer_rsrc(cnt, (short)0, 64, 0x00020000);
  constexpr int LD = MODE == 1 ? 16 : 1, ST = MODE == 1 ? 16 : 0;
  __shared__ int ok;
  for (int p = 0; p < P; ++p) {
    if (p > 0) {
      if (threadIdx.x == 0) {
        int sp = 0;
        if constexpr (MODE == 1) {
          while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(G * p) && ++sp < SPIN_MAX)
            __builtin_amdgcn_s_sleep(1);
        } else {
          while ((unsigned)__builtin_amdgcn_raw_buffer_load_b32(cs, 0, 0, 1) < (unsigned)(G * p) && ++sp < SPIN_MAX)
            __builtin_amdgcn_s_sleep(1);
        }
        ok = sp < SPIN_MAX;
        if (!ok) atomicOr(err, 1u);
      }
      __syncthreads();
      if (!ok) return;
    }
    const int src = (p & 1) ^ 1, dst = p & 1;
    float v = 0.f;
    for (int i = threadIdx.x; i < G * 16; i += NT) {
      const unsigned off = (unsigned)((src * G * 16 + i) * 4);
      v += p > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, LD)) : 0.f;
    }
    const float m = reduce_block(v) / (G * 16) + 1.f;
    if (threadIdx.x < 16)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, m), rs, (unsigned)((dst * G * 16 + g * 16 + threadIdx.x) * 4), 0, ST);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if constexpr (MODE == 1) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

template <int MODE>
static void run_xcd(int P) {
  const int GRID = 256, G = GRID / 8;
  float* act;
  unsigned *cnt, *err;
  CK(hipMalloc(&act, 2 * G * 16 * 4));
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CK(hipMemsetAsync(cnt, 0, 64, s));
    CK(hipMemsetAsync(act, 0, 2 * G * 16 * 4, s));
    CK(hipEventRecord(e0, s));
    persist_xcd_kernel<MODE><<<GRID, NT, 0, s>>>(act, P, cnt, err);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it) best = ms < best ? ms : best;
  }
  float hp[16];
  unsigned herr;
  CK(hipMemcpy(hp, act + ((P - 1) & 1) * G * 16, 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("{\"xcd_local_groups\": %d, \"mode\": \"%s\", \"phases\": %d, \"persist_us_per_phase\": %.3f, \"check\": %.1f, "
         "\"spin_timeout\": %u}\n", G, MODE == 1 ? "sc1 stores/loads, agent counter" : "L2-coherent: sc0 loads, workgroup counter",
         P, best * 1000.f / P, hp[0], herr);
  fflush(stdout);
  CK(hipFree(act));
  CK(hipFree(cnt));
  CK(hipFree(err));
  CK(hipStreamDestroy(s));
}

// Grid-wide (all 8 XCDs) chain with a two-level count (round 6): a work-group adds 1 to its XCD's
// counter (own 128-B line); the one that completes its XCD's count for the phase adds 1 to the global
// counter, which the next phase polls -- 32 + 8 serialised atomics per phase instead of 256 on one
// address.  Data as persist_kernel (sc1 write-through stores, sc1 loads).
__global__ __launch_bounds__(NT) void persist_hier_kernel(float* act, int P, unsigned* cnt, unsigned* err) {
  const int G = gridDim.x, g = blockIdx.x, xcd = g % 8, per = G / 8;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(act, (short)0, (int)(2 * G * 16 * 4), 0x00020000);
  unsigned* gcnt = cnt;                  // global count (line 0)
  unsigned* xcnt = cnt + 32 * (1 + xcd);  // this XCD's count (lines 1..8)
  __shared__ int ok;
  for (int p = 0; p < P; ++p) {
    if (p > 0) {
      if (threadIdx.x == 0) {
        int sp = 0;
        while (__hip_atomic_load(gcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(8 * p) && ++sp < SPIN_MAX)
          __builtin_amdgcn_s_sleep(1);
        ok = sp < SPIN_MAX;
        if (!ok) atomicOr(err, 1u);
      }
      __syncthreads();
      if (!ok) return;
    }
    const int src = (p & 1) ^ 1, dst = p & 1;
    float v = 0.f;
    for (int i = threadIdx.x; i < G * 16; i += NT) {
      const unsigned off = (unsigned)((src * G * 16 + i) * 4);
      v += p > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 16)) : 0.f;
    }
    const float m = reduce_block(v) / (G * 16) + 1.f;
    if (threadIdx.x < 16)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, m), rs, (unsigned)((dst * G * 16 + g * 16 + threadIdx.x) * 4), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned old = __hip_atomic_fetch_add(xcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (unsigned)(per * (p + 1) - 1)) __hip_atomic_fetch_add(gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static void run_hier(int G, int P) {
  float* act;
  unsigned *cnt, *err;
  CK(hipMalloc(&act, 2 * G * 16 * 4));
  CK(hipMalloc(&cnt, 9 * 128));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CK(hipMemsetAsync(cnt, 0, 9 * 128, s));
    CK(hipMemsetAsync(act, 0, 2 * G * 16 * 4, s));
    CK(hipEventRecord(e0, s));
    persist_hier_kernel<<<G, NT, 0, s>>>(act, P, cnt, err);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it) best = ms < best ? ms : best;
  }
  float hp[16];
  unsigned herr;
  CK(hipMemcpy(hp, act + ((P - 1) & 1) * G * 16, 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("{\"groups\": %d, \"mode\": \"two-level count (per-XCD then global)\", \"phases\": %d, \"persist_us_per_phase\": %.3f, "
         "\"check\": %.1f, \"spin_timeout\": %u}\n", G, P, best * 1000.f / P, hp[0], herr);
  fflush(stdout);
  CK(hipFree(act));
  CK(hipFree(cnt));
  CK(hipFree(err));
  CK(hipStreamDestroy(s));
}

// bare dependency chain with NTH threads per group: each group reads the previous kernel's G floats
// and writes one (the floor of a dependent launch by group count and size)
template <int NTH>
__global__ __launch_bounds__(NTH) void bare_kernel(const float* ain, float* aout, int G) {
  float v = 0.f;
  for (int i = threadIdx.x; i < G; i += NTH) v += ain[i];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __shared__ float part[NTH / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < NTH / 64; ++i) s += part[i];
    aout[blockIdx.x] = s / G + 1.f;
  }
}
template <int NTH>
static void run_bare(int G, int P) {
  float *a0, *a1;
  CK(hipMalloc(&a0, G * 4));
  CK(hipMalloc(&a1, G * 4));
  CK(hipMemset(a0, 0, G * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int p = 0; p < P; ++p) bare_kernel<NTH><<<G, NTH, 0, s>>>(p & 1 ? a1 : a0, p & 1 ? a0 : a1, G);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it) best = ms < best ? ms : best;
  }
  printf("{\"bare_groups\": %d, \"threads\": %d, \"kernels_us_per_phase\": %.3f}\n", G, NTH, best * 1000.f / P);
  fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(a0));
  CK(hipFree(a1));
  CK(hipStreamDestroy(s));
}

template <int U>
static void run(int G, int P, bool weights) {
  const size_t per = (size_t)NT * U * 16;  // bytes per group and phase
  u32x4* w = nullptr;
  if (weights) {
    CK(hipMalloc(&w, per * G * P));
    CK(hipMemset(w, 0x5a, per * G * P));
  }
  float *a0, *a1, *act;
  unsigned *cnt, *err, *sink;
  CK(hipMalloc(&a0, G * 16 * 4));
  CK(hipMalloc(&a1, G * 16 * 4));
  CK(hipMalloc(&act, 2 * G * 16 * 4));
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a0, 0, G * 16 * 4));
  CK(hipMemset(err, 0, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // kernels: P launches captured in a graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int p = 0; p < P; ++p)
    phase_kernel<U><<<G, NT, 0, s>>>(w, p & 1 ? a1 : a0, p & 1 ? a0 : a1, p, G, sink);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  float best_k = 1e30f, best_p = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CK(hipMemsetAsync(a0, 0, G * 16 * 4, s));
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it) best_k = ms < best_k ? ms : best_k;
  }
  float hk[16];
  CK(hipMemcpy(hk, P & 1 ? a1 : a0, 64, hipMemcpyDeviceToHost));
  for (int it = 0; it < 6; ++it) {
    CK(hipMemsetAsync(cnt, 0, 64, s));
    CK(hipMemsetAsync(act, 0, 2 * G * 16 * 4, s));
    CK(hipEventRecord(e0, s));
    persist_kernel<U><<<G, NT, 0, s>>>(w, act, P, G, cnt, err, sink);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it) best_p = ms < best_p ? ms : best_p;
  }
  float hp[16];
  unsigned herr;
  CK(hipMemcpy(hp, act + ((P - 1) & 1) * G * 16, 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  printf("{\"groups\": %d, \"phases\": %d, \"bytes_per_phase\": %zu, \"kernels_us_per_phase\": %.3f, "
         "\"persist_us_per_phase\": %.3f, \"kernels_check\": %.1f, \"persist_check\": %.1f, \"spin_timeout\": %u}\n",
         G, P, weights ? per * G : 0, best_k * 1000.f / P, best_p * 1000.f / P, hk[0], hp[0], herr);
  fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  if (w) CK(hipFree(w));
  CK(hipFree(a0));
  CK(hipFree(a1));
  CK(hipFree(act));
  CK(hipFree(cnt));
  CK(hipFree(err));
  CK(hipFree(sink));
  CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'x') {  // XCD-local hand-offs (round 6)
    run_xcd<1>(256);
    run_xcd<2>(256);
    run_bare<1024>(32, 128);  // 32 groups as dependent kernels, for comparison
    run<1>(256, 64, false);   // the flat grid-wide count (round 3's figure) in the same run
    run_hier(256, 64);
    return 0;
  }
  if (argc > 1) {  // the floor by group count and size
    for (int G : {1, 8, 64, 256, 512, 1024}) {
      run_bare<64>(G, 128);
      run_bare<256>(G, 128);
      run_bare<1024>(G, 128);
    }
    return 0;
  }
  run<1>(256, 64, false);  // bare dependency chain (16 KB of weights per group unread)
  run<4>(256, 64, true);   // 16 MB per phase (TinyLlama q|k|v / attn_output scale)
  run<12>(256, 48, true);  // 48 MB per phase (Llama-3-8B q|k|v scale)
  run<4>(128, 64, true);   // half the CUs
  return 0;
}
