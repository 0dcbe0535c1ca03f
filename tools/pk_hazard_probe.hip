// pk_hazard_probe.hip -- diagnosis for DESIGN.md §5 (round 6): does the packed-FP32 sequence that gave
// wrong lanes 32-63 in round 5 (profiles/round5_rope_packed_hazard.txt) fail on its own, and which
// wait states, if any, cure it?
//
//   hipcc --offload-arch=gfx950 -O2 -ffp-contract=off tools/pk_hazard_probe.hip -o /tmp/pk_probe && /tmp/pk_probe
//
// The victim kernel replays the round-5 instruction sequence with fixed physical registers (inline asm):
//   global_load_dwordx4 C, D(address), off ; v_mov_b32 D.lo, B.hi ; s_waitcnt vmcnt(0) ;
//   v_pk_mul_f32 T, A, C.lo op_sel:[1,1] op_sel_hi:[1,0] ; v_pk_mul_f32 U, D, C.hi op_sel:[0,1] op_sel_hi:[0,0] ;
//   four v_pk_fma_f32 (RoPE o0..o3)
// and compares the 8 results of every lane with the same arithmetic as scalar v_mul_f32 / v_fma_f32.
// Variants:
//   0  the round-5 sequence exactly (the load's address pair is overwritten by the v_mov)
//   1  + s_nop 1 after the v_mov (2 wait states before the packed read)
//   2  + s_nop 4 after the v_mov
//   3  load address in another pair (no overwrite of an in-flight load's address), otherwise as 0
//   4  no load in the sequence: v_mov then the packed chain directly
// Each variant runs alone (one stream) and shared (two victim streams + a streaming aggressor stream),
// 20 launches each.  Mismatches are counted per result slot and per half-wave.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int NT = 256, GRID = 2048, ITERS = 64, TABLE = 4096;

__device__ __forceinline__ float hfloat(unsigned x) {  // [-2, 2) from a hash, exact
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return (float)(int)(x >> 8) * (1.0f / 4194304.0f) - 2.0f;
}

#define PK_TAIL                                                                                             \
  "s_waitcnt vmcnt(0)\n\t"                                                                                  \
  "v_pk_mul_f32 v[210:211], v[200:201], v[204:205] op_sel:[1,1] op_sel_hi:[1,0]\n\t"                        \
  "v_pk_mul_f32 v[212:213], v[208:209], v[206:207] op_sel:[0,1] op_sel_hi:[0,0]\n\t"                        \
  "v_pk_fma_f32 v[214:215], v[200:201], v[204:205], v[210:211] op_sel_hi:[0,1,1] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t" \
  "v_pk_fma_f32 v[216:217], v[200:201], v[204:205], v[210:211] op_sel_hi:[0,1,1]\n\t"                       \
  "v_pk_fma_f32 v[218:219], v[202:203], v[206:207], v[212:213] op_sel_hi:[0,1,1] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t" \
  "v_pk_fma_f32 v[220:221], v[202:203], v[206:207], v[212:213] op_sel_hi:[0,1,1]\n\t"                       \
  "v_mov_b32 %0, v214\n\tv_mov_b32 %1, v215\n\tv_mov_b32 %2, v216\n\tv_mov_b32 %3, v217\n\t"               \
  "v_mov_b32 %4, v218\n\tv_mov_b32 %5, v219\n\tv_mov_b32 %6, v220\n\tv_mov_b32 %7, v221"

#define PK_OUTS "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5]), "=v"(o[6]), "=v"(o[7])
#define PK_CLOB                                                                                                \
  "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212",    \
      "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "memory"

#define PK_HEAD                                                                            \
  "v_mov_b32 v200, %8\n\tv_mov_b32 v201, %9\n\tv_mov_b32 v202, %10\n\tv_mov_b32 v203, %11\n\t" \
  "v_mov_b32 v208, %12\n\tv_mov_b32 v209, %13\n\tv_mov_b32 v222, %12\n\tv_mov_b32 v223, %13\n\ts_nop 4\n\t"

template <int V>
__device__ __forceinline__ void pk_seq(float (&o)[8], float a0, float a1, float b0, float b1, const float* cs,
                                       const float4& cq) {
  const unsigned long long ad = (unsigned long long)cs;
  const unsigned alo = (unsigned)ad, ahi = (unsigned)(ad >> 32);
  if constexpr (V == 0)
    asm volatile(PK_HEAD "global_load_dwordx4 v[204:207], v[208:209], off\n\tv_mov_b32 v208, v203\n\t" PK_TAIL
                 : PK_OUTS : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(alo), "v"(ahi) : PK_CLOB);
  else if constexpr (V == 1)
    asm volatile(PK_HEAD "global_load_dwordx4 v[204:207], v[208:209], off\n\tv_mov_b32 v208, v203\n\ts_nop 1\n\t" PK_TAIL
                 : PK_OUTS : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(alo), "v"(ahi) : PK_CLOB);
  else if constexpr (V == 2)
    asm volatile(PK_HEAD "global_load_dwordx4 v[204:207], v[208:209], off\n\tv_mov_b32 v208, v203\n\ts_nop 4\n\t" PK_TAIL
                 : PK_OUTS : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(alo), "v"(ahi) : PK_CLOB);
  else if constexpr (V == 3)
    asm volatile(PK_HEAD "global_load_dwordx4 v[204:207], v[222:223], off\n\tv_mov_b32 v208, v203\n\t" PK_TAIL
                 : PK_OUTS : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(alo), "v"(ahi) : PK_CLOB);
  else
    asm volatile(PK_HEAD "v_mov_b32 v204, %14\n\tv_mov_b32 v205, %15\n\tv_mov_b32 v206, %16\n\tv_mov_b32 v207, %17\n\t"
                 "s_nop 4\n\tv_mov_b32 v208, v203\n\t" PK_TAIL
                 : PK_OUTS : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(alo), "v"(ahi), "v"(cq.x), "v"(cq.y), "v"(cq.z),
                   "v"(cq.w) : PK_CLOB);
}

__device__ __forceinline__ float smul(float x, float y) {
  float r;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ float sfma(float x, float y, float z) {
  float r;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
__device__ __forceinline__ float sfms(float x, float y, float z) {  // x*y - z, one rounding
  float r;
  asm volatile("v_fma_f32 %0, %1, %2, -%3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}

template <int V>
__global__ __launch_bounds__(NT) void victim(const float4* table, unsigned* bad, float* sample, unsigned seed) {
  const unsigned tid = blockIdx.x * NT + threadIdx.x;
  const int half = (threadIdx.x & 63) >> 5;
  for (int it = 0; it < ITERS; ++it) {
    const unsigned h = (tid * 2654435761u) ^ (it * 0x9e3779b9u) ^ seed;
    const float a0 = hfloat(h), a1 = hfloat(h + 1), b0 = hfloat(h + 2), b1 = hfloat(h + 3);
    const float4* cp = table + ((tid + it * 97) % TABLE);
    const float4 cq = *cp;
    float o[8];
    pk_seq<V>(o, a0, a1, b0, b1, reinterpret_cast<const float*>(cp), cq);
    const float t0 = smul(a1, cq.y), t1 = smul(a1, cq.x), u0 = smul(b1, cq.w), u1 = smul(b1, cq.z);
    float r[8];
    r[0] = sfms(a0, cq.x, t0); r[1] = sfms(a0, cq.y, t1);
    r[2] = sfma(a0, cq.x, t0); r[3] = sfma(a0, cq.y, t1);
    r[4] = sfms(b0, cq.z, u0); r[5] = sfms(b0, cq.w, u1);
    r[6] = sfma(b0, cq.z, u0); r[7] = sfma(b0, cq.w, u1);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (__float_as_uint(o[j]) != __float_as_uint(r[j])) atomicAdd(bad + 2 * j + half, 1u);
    if (it == 0 && tid < 64) {
      float* s = sample + tid * 20;
      s[0] = a0; s[1] = a1; s[2] = b0; s[3] = b1; s[4] = cq.x; s[5] = cq.y; s[6] = cq.z; s[7] = cq.w;
      for (int j = 0; j < 8; ++j) s[8 + j] = o[j];
    }
  }
}

// aggressor: streaming loads + f32 VALU, on its own stream
__global__ __launch_bounds__(NT) void aggressor(const float4* src, size_t n, float* sink) {
  float4 acc = make_float4(0, 0, 0, 0);
  for (size_t i = blockIdx.x * NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT) {
    const float4 v = src[i];
    acc.x = fmaf(acc.x, 1.0001f, v.x); acc.y = fmaf(acc.y, 0.9999f, v.y);
    acc.z = fmaf(acc.z, 1.0001f, v.z); acc.w = fmaf(acc.w, 0.9999f, v.w);
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[0] = acc.x;
}

template <int V>
static void run(const char* name, const float4* table, unsigned* bad, float* sample, const float4* big, size_t nbig,
                float* sink, hipStream_t s1, hipStream_t s2, hipStream_t s3) {
  for (int shared = 0; shared < 2; ++shared) {
    CK(hipMemset(bad, 0, 64 * 4));
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 20; ++rep) {
      if (shared) aggressor<<<1024, NT, 0, s3>>>(big, nbig, sink);
      victim<V><<<GRID, NT, 0, s1>>>(table, bad, sample, 1000u + rep);
      if (shared) victim<V><<<GRID, NT, 0, s2>>>(table, bad + 16, sample, 5000u + rep);
    }
    CK(hipDeviceSynchronize());
    unsigned h[32];
    CK(hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost));
    unsigned long long tot = 0;
    for (int i = 0; i < 32; ++i) tot += h[i];
    const double n = 20.0 * GRID * NT * ITERS * (shared ? 2 : 1);
    printf("variant %-34s %-6s results %.3g  mismatches %llu", name, shared ? "shared" : "alone", n * 8, tot);
    if (tot) {
      printf("  [slot lanes0-31/lanes32-63:");
      for (int j = 0; j < 8; ++j) printf(" %u/%u", h[2 * j] + h[16 + 2 * j], h[2 * j + 1] + h[16 + 2 * j + 1]);
      printf("]");
    }
    printf("\n");
    fflush(stdout);
  }
}

int main() {
  std::vector<float> t(TABLE * 4);
  for (int i = 0; i < TABLE; ++i) {
    const double th = 0.001 * i;
    t[4 * i] = (float)cos(th); t[4 * i + 1] = (float)sin(th);
    t[4 * i + 2] = (float)cos(3 * th); t[4 * i + 3] = (float)sin(3 * th);
  }
  float4 *table, *big;
  unsigned* bad;
  float *sample, *sink;
  const size_t nbig = (size_t)64 << 20;  // 1 GiB of float4
  CK(hipMalloc(&table, TABLE * 16));
  CK(hipMalloc(&big, nbig * 16));
  CK(hipMalloc(&bad, 64 * 4));
  CK(hipMalloc(&sample, 64 * 20 * 4));
  CK(hipMalloc(&sink, 16));
  CK(hipMemcpy(table, t.data(), TABLE * 16, hipMemcpyHostToDevice));
  CK(hipMemset(big, 0, nbig * 16));
  hipStream_t s1, s2, s3;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));

  // the scalar reference's semantics, checked on the host for one launch's first 64 lanes
  victim<4><<<1, NT>>>(table, bad, sample, 7u);
  CK(hipDeviceSynchronize());
  std::vector<float> sm(64 * 20);
  CK(hipMemcpy(sm.data(), sample, sm.size() * 4, hipMemcpyDeviceToHost));
  int host_bad = 0;
  for (int l = 0; l < 64; ++l) {
    const float* s = &sm[l * 20];
    const float a0 = s[0], a1 = s[1], b0 = s[2], b1 = s[3], c0 = s[4], c1 = s[5], c2 = s[6], c3 = s[7];
    const float t0 = a1 * c1, t1 = a1 * c0, u0 = b1 * c3, u1 = b1 * c2;
    const float r[8] = {fmaf(a0, c0, -t0), fmaf(a0, c1, -t1), fmaf(a0, c0, t0), fmaf(a0, c1, t1),
                        fmaf(b0, c2, -u0), fmaf(b0, c3, -u1), fmaf(b0, c2, u0), fmaf(b0, c3, u1)};
    for (int j = 0; j < 8; ++j) host_bad += memcmp(&r[j], &s[8 + j], 4) != 0;
  }
  printf("host check of the packed sequence's semantics (64 lanes x 8 results): %d mismatches\n", host_bad);

  run<0>("0 round-5 sequence", table, bad, sample, big, nbig, sink, s1, s2, s3);
  run<1>("1 +s_nop 1 after v_mov", table, bad, sample, big, nbig, sink, s1, s2, s3);
  run<2>("2 +s_nop 4 after v_mov", table, bad, sample, big, nbig, sink, s1, s2, s3);
  run<3>("3 load address not overwritten", table, bad, sample, big, nbig, sink, s1, s2, s3);
  run<4>("4 no load, v_mov -> packed chain", table, bad, sample, big, nbig, sink, s1, s2, s3);
  return 0;
}
