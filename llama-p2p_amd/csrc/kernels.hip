// kernels.hip -- gfx950 (CDNA4) kernels of the MI355X-native LLaMA forward.
//
// They replace the ggml CPU ops that llama.cpp's llm_build_llama runs for the
// reference's hot call  self.model(prompt, max_tokens=100)
// (/root/reference/llama_p2p_network.py:125, model built at :19).  Numerics
// follow ggml's CPU semantics: bf16 weights, activations
// rounded to bf16 before each weight product, f32 accumulation, f16 K/V cache,
// f16-rounded q and probabilities in attention, double-sum RMSNorm.
//
// Decode is HBM-bound (≈1 flop/byte at one token, ≈32 at 32 tokens, both far
// below the ≈300 flop/byte ridge), so the design goal is streaming every
// weight byte once at full HBM rate:
//   * weights are pre-packed into 1 KiB MFMA A-operand tiles (kernels.h), so a
//     wave-instruction is one contiguous 1 KiB, non-temporal, 16 B/lane load;
//   * v_mfma_f32_16x16x32_bf16 does the dot products for 1..64 tokens (its
//     issue rate is ~25x what HBM can feed, so padding columns costs nothing);
//   * K is split across the waves of a work-group (register ring of U loads
//     in flight per wave), partial tiles are summed through LDS, and the
//     epilogue fuses RoPE + KV-cache store, SwiGLU, or the residual add.
#include "kernels.h"

#include <math.h>

namespace mx {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
// round-nearest-even f32 -> bf16 bits (ggml_compute_fp32_to_bf16 without the NaN branch)
__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float round_f16(float f) { return (float)(_Float16)f; }

// ---------------------------------------------------------------------------
// synthetic weights (llama-p2p_amd/synth.py is the spec; bit-identical)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float synth_value(uint64_t seed, uint64_t tid, uint64_t idx, float scale) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + tid * 0xD1B54A32D192ED03ull + idx;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  uint32_t s = (uint32_t)(z & 0xffff) + (uint32_t)((z >> 16) & 0xffff) + (uint32_t)((z >> 32) & 0xffff) +
               (uint32_t)(z >> 48);
  return (float)((int32_t)s - 131070) * scale;
}

// packed element p of a [N][K] matrix -> (row, col) of the logical matrix
__device__ __forceinline__ void packed_coords(size_t p, int KT, int& row, int& col, size_t& tile) {
  tile = p / TILE_ELEMS;
  int within = (int)(p % TILE_ELEMS);
  int lane = within >> 3, j = within & 7;
  int nt = (int)(tile / KT), kt = (int)(tile % KT);
  row = nt * TILE_N + (lane & 15);
  col = kt * TILE_K + (lane >> 4) * 8 + j;
}

__global__ void synth_packed_kernel(uint16_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale,
                                    int stride, int offset) {
  const int KT = K / TILE_K;
  const size_t total = (size_t)N * K;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < total; p += (size_t)gridDim.x * blockDim.x) {
    int row, col;
    size_t tile;
    packed_coords(p, KT, row, col, tile);
    size_t nt = tile / KT, kt = tile % KT;
    size_t dtile = (nt * stride + offset) * KT + kt;
    float v = synth_value(seed, tid, (uint64_t)row * K + col, scale);
    dst[dtile * TILE_ELEMS + (p % TILE_ELEMS)] = (uint16_t)f2bf(v);
  }
}

__global__ void pack_kernel(uint16_t* dst, const uint16_t* src, int N, int K, int stride, int offset) {
  const int KT = K / TILE_K;
  const size_t total = (size_t)N * K;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < total; p += (size_t)gridDim.x * blockDim.x) {
    int row, col;
    size_t tile;
    packed_coords(p, KT, row, col, tile);
    size_t nt = tile / KT, kt = tile % KT;
    size_t dtile = (nt * stride + offset) * KT + kt;
    dst[dtile * TILE_ELEMS + (p % TILE_ELEMS)] = src[(size_t)row * K + col];
  }
}

__global__ void synth_rowmajor_kernel(uint16_t* dst, size_t n, uint64_t seed, uint64_t tid, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (uint16_t)f2bf(synth_value(seed, tid, i, scale));
}

__global__ void synth_norm_kernel(float* dst, size_t n, uint64_t seed, uint64_t tid, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = 1.0f + synth_value(seed, tid, i, scale);
}

static int fill_grid(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g == 0 ? 1 : g));
}

void launch_synth_packed(uint16_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale, int stride,
                         int offset, hipStream_t s) {
  synth_packed_kernel<<<fill_grid((size_t)N * K), 256, 0, s>>>(dst, N, K, seed, tid, scale, stride, offset);
}
void launch_pack(uint16_t* dst, const uint16_t* src, int N, int K, int stride, int offset, hipStream_t s) {
  pack_kernel<<<fill_grid((size_t)N * K), 256, 0, s>>>(dst, src, N, K, stride, offset);
}
void launch_synth_rowmajor(uint16_t* dst, size_t n, uint64_t seed, uint64_t tid, float scale, hipStream_t s) {
  synth_rowmajor_kernel<<<fill_grid(n), 256, 0, s>>>(dst, n, seed, tid, scale);
}
void launch_synth_norm(float* dst, size_t n, uint64_t seed, uint64_t tid, float scale, hipStream_t s) {
  synth_norm_kernel<<<fill_grid(n), 256, 0, s>>>(dst, n, seed, tid, scale);
}

// ---------------------------------------------------------------------------
// GET_ROWS: token embedding, bf16 -> f32  
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed_kernel(float* x, const uint16_t* tok_embd, const int* ids, int n) {
  const int c = blockIdx.x;
  const int id = ids[c];
  const u32x4* src = reinterpret_cast<const u32x4*>(tok_embd + (size_t)id * n);
  f32x4* dst = reinterpret_cast<f32x4*>(x + (size_t)c * n);
  for (int i = threadIdx.x; i < n / 8; i += blockDim.x) {
    u32x4 v = src[i];
    f32x4 lo, hi;
    lo[0] = __uint_as_float(v[0] << 16); lo[1] = __uint_as_float(v[0] & 0xffff0000u);
    lo[2] = __uint_as_float(v[1] << 16); lo[3] = __uint_as_float(v[1] & 0xffff0000u);
    hi[0] = __uint_as_float(v[2] << 16); hi[1] = __uint_as_float(v[2] & 0xffff0000u);
    hi[2] = __uint_as_float(v[3] << 16); hi[3] = __uint_as_float(v[3] & 0xffff0000u);
    dst[2 * i] = lo;
    dst[2 * i + 1] = hi;
  }
}

void launch_embed(float* x, const uint16_t* tok_embd, const int* ids, int M, int n, hipStream_t s) {
  embed_kernel<<<M, 256, 0, s>>>(x, tok_embd, ids, n);
}

// ---------------------------------------------------------------------------
// RMS_NORM + MUL(norm weight) -> bf16 activation  
// ggml: sum of x*x in double, scale = 1/sqrtf(mean + eps), y = (x*scale)*w;
// the bf16 rounding is the conversion ggml applies to src1 of the next MUL_MAT.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rmsnorm_kernel(uint16_t* y, int ldy, const float* x, const float* w,
                                                      const int* row_map, int n, float eps) {
  const int c = blockIdx.x;
  const int r = row_map ? row_map[c] : c;
  const float* xr = x + (size_t)r * n;
  double acc = 0.0;
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(xr + i);
    acc += (double)(v[0] * v[0]);
    acc += (double)(v[1] * v[1]);
    acc += (double)(v[2] * v[2]);
    acc += (double)(v[3] * v[3]);
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  __shared__ double part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  double sum = part[0] + part[1] + part[2] + part[3];
  const float mean = (float)(sum / n);
  const float scale = 1.0f / sqrtf(mean + eps);
  uint16_t* yr = y + (size_t)c * ldy;
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(xr + i);
    f32x4 g = *reinterpret_cast<const f32x4*>(w + i);
    u32x2 o;
    o[0] = f2bf((v[0] * scale) * g[0]) | (f2bf((v[1] * scale) * g[1]) << 16);
    o[1] = f2bf((v[2] * scale) * g[2]) | (f2bf((v[3] * scale) * g[3]) << 16);
    *reinterpret_cast<u32x2*>(yr + i) = o;
  }
}

void launch_rmsnorm(uint16_t* y, int ldy, const float* x, const float* w, const int* row_map, int M, int n,
                    float eps, hipStream_t s) {
  rmsnorm_kernel<<<M, 256, 0, s>>>(y, ldy, x, w, row_map, n, eps);
}

// ---------------------------------------------------------------------------
// MUL_MAT with bf16 weights for 1..64 tokens (decode GEMV / skinny GEMM) with
// fused epilogues.  
//
// Work-group = KS waves = RT row tiles (16 rows each) x all K; wave w owns the
// K-tiles [KT*w/KS, KT*(w+1)/KS).  Per K-tile a wave issues RT weight loads
// (1 KiB each, contiguous, non-temporal) and NB activation loads (L2 hits),
// and RT*NB MFMAs.  A ring of U K-tiles per wave keeps U*(RT+NB) loads in flight.
// ---------------------------------------------------------------------------
template <int KS, int RT, int NB, int EPI, int U>
__global__ __launch_bounds__(64 * KS) void mm_kernel(MMArgs a) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int KT = a.K / TILE_K;
  const int tile0 = blockIdx.x * RT;
  const int kb = (KT * w) / KS, ke = (KT * (w + 1)) / KS;

  const u32x4* Wp[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
    Wp[r] = reinterpret_cast<const u32x4*>(a.W) + (size_t)(tile0 + r) * KT * 64 + lane;
  const u32x4* Xp[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    int col = n * 16 + (lane & 15);
    col = col < a.M ? col : a.M - 1;  // padded columns re-read a valid row; their outputs are dropped
    Xp[n] = reinterpret_cast<const u32x4*>(a.X + (size_t)col * a.ldx + (lane >> 4) * 8);
  }

  f32x4 acc[RT][NB];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[U][RT], rb[U][NB];
  int kt = kb;
  const int nfull = (ke - kb) / U;
  if (nfull > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < RT; ++r) ra[u][r] = __builtin_nontemporal_load(Wp[r] + (size_t)(kt + u) * 64);
#pragma unroll
      for (int n = 0; n < NB; ++n) rb[u][n] = Xp[n][(kt + u) * 4];
    }
    for (int ch = 1; ch < nfull; ++ch) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int r = 0; r < RT; ++r)
#pragma unroll
          for (int n = 0; n < NB; ++n)
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ra[u][r]),
                                                                 __builtin_bit_cast(bf16x8, rb[u][n]), acc[r][n],
                                                                 0, 0, 0);
#pragma unroll
        for (int r = 0; r < RT; ++r) ra[u][r] = __builtin_nontemporal_load(Wp[r] + (size_t)(kt + U + u) * 64);
#pragma unroll
        for (int n = 0; n < NB; ++n) rb[u][n] = Xp[n][(kt + U + u) * 4];
      }
      kt += U;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int n = 0; n < NB; ++n)
          acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ra[u][r]),
                                                               __builtin_bit_cast(bf16x8, rb[u][n]), acc[r][n], 0,
                                                               0, 0);
    kt += U;
  }
  for (; kt < ke; ++kt) {
    u32x4 sa[RT], sb[NB];
#pragma unroll
    for (int r = 0; r < RT; ++r) sa[r] = __builtin_nontemporal_load(Wp[r] + (size_t)kt * 64);
#pragma unroll
    for (int n = 0; n < NB; ++n) sb[n] = Xp[n][kt * 4];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, sa[r]),
                                                             __builtin_bit_cast(bf16x8, sb[n]), acc[r][n], 0, 0, 0);
  }

  // ---- sum the KS partial tiles through LDS
  __shared__ f32x4 red[KS][RT][NB][64];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) red[w][r][n][lane] = acc[r][n];
  __syncthreads();

  // ---- epilogue.  unit = (r, n, lane): rows 16*(tile0+r) + 4*(lane>>4) + i, i<4; col n*16 + (lane&15)
  constexpr int RU = (EPI == EPI_SWIGLU) ? 1 : RT;  // SWIGLU consumes the (gate, up) tile pair per unit
  constexpr int UNITS = RU * NB * 64;
  for (int u = threadIdx.x; u < UNITS; u += 64 * KS) {
    const int l = u & 63;
    const int n = (u >> 6) % NB;
    const int r = (u >> 6) / NB;
    const int col = n * 16 + (l & 15);
    if (col >= a.M) continue;
    f32x4 s = red[0][r][n][l];
#pragma unroll
    for (int ww = 1; ww < KS; ++ww) s += red[ww][r][n][l];

    if constexpr (EPI == EPI_F32) {
      const int row = (tile0 + r) * 16 + (l >> 4) * 4;
      *reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row) = s;
    } else if constexpr (EPI == EPI_RESID) {
      const int row = (tile0 + r) * 16 + (l >> 4) * 4;
      f32x4* px = reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row);
      *px = *px + s;
    } else if constexpr (EPI == EPI_SWIGLU) {
      f32x4 up = red[0][1][n][l];
#pragma unroll
      for (int ww = 1; ww < KS; ++ww) up += red[ww][1][n][l];
      const int row = blockIdx.x * 16 + (l >> 4) * 4;  // gate/up tile pair index == blockIdx.x
      uint32_t h[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float g = s[i];
        float sg = g / (1.0f + expf(-g));
        h[i] = f2bf(sg * up[i]);
      }
      u32x2 o;
      o[0] = h[0] | (h[1] << 16);
      o[1] = h[2] | (h[3] << 16);
      *reinterpret_cast<u32x2*>(a.act + (size_t)col * a.lda + row) = o;
    } else {  // EPI_QKV
      const int row = (tile0 + r) * 16 + (l >> 4) * 4;
      const int d = a.head_dim;
      const int pos = a.pos[col];
      if (pos < 0 || pos >= a.n_ctx) continue;  // never write outside the slot's KV rows
      if (row < a.n_q + a.n_kv) {
        // ROPE_EXT mode NORM: rotate adjacent pairs (2i, 2i+1) of each head
        const bool is_q = row < a.n_q;
        const int rl = is_q ? row : row - a.n_q;
        const int dd = rl % d;  // multiple of 4
        const float* cs = a.rope_cs + ((size_t)pos * (d / 2) + dd / 2) * 2;
        f32x4 csv = *reinterpret_cast<const f32x4*>(cs);  // cos0, sin0, cos1, sin1
        f32x4 o;
        o[0] = s[0] * csv[0] - s[1] * csv[1];
        o[1] = s[0] * csv[1] + s[1] * csv[0];
        o[2] = s[2] * csv[2] - s[3] * csv[3];
        o[3] = s[2] * csv[3] + s[3] * csv[2];
        if (is_q) {
          *reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row) = o;
        } else {
          const int kvh = rl / d;
          _Float16* dst = a.kc + (size_t)a.slot[col] * a.slot_stride + ((size_t)kvh * a.n_ctx + pos) * d + dd;
          *reinterpret_cast<f16x4*>(dst) = f16x4{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
        }
      } else {
        const int rl = row - a.n_q - a.n_kv;
        const int kvh = rl / d, dd = rl % d;
        _Float16* dst = a.vc + (size_t)a.slot[col] * a.slot_stride + ((size_t)kvh * a.n_ctx + pos) * d + dd;
        *reinterpret_cast<f16x4*>(dst) = f16x4{(_Float16)s[0], (_Float16)s[1], (_Float16)s[2], (_Float16)s[3]};
      }
    }
  }
}

template <int KS, int RT, int EPI, int U>
static int launch_mm_nb(const MMArgs& a, hipStream_t s) {
  const int nb = (a.M + 15) / 16;
  const int grid = a.N / (16 * RT);
  switch (nb) {
    case 1: mm_kernel<KS, RT, 1, EPI, U><<<grid, 64 * KS, 0, s>>>(a); break;
    case 2: mm_kernel<KS, RT, 2, EPI, U><<<grid, 64 * KS, 0, s>>>(a); break;
    case 3:
    case 4: mm_kernel<KS, RT, 4, EPI, U><<<grid, 64 * KS, 0, s>>>(a); break;
    default: return -1;
  }
  return 0;
}

int launch_mm(int epi, const MMArgs& a, hipStream_t s) {
  if (a.M < 1 || a.M > MAX_ROWS || a.K % TILE_K != 0 || a.N % TILE_N != 0) return -1;
  switch (epi) {
    case EPI_F32: return launch_mm_nb<4, 1, EPI_F32, 8>(a, s);
    case EPI_RESID: return launch_mm_nb<8, 1, EPI_RESID, 8>(a, s);
    case EPI_QKV: return launch_mm_nb<4, 1, EPI_QKV, 8>(a, s);
    case EPI_SWIGLU:
      if (a.N % 32 != 0) return -1;
      return launch_mm_nb<4, 2, EPI_SWIGLU, 4>(a, s);
  }
  return -1;
}

// ---------------------------------------------------------------------------
// Attention for one query token per row (decode, and prefill rows alike):
// KQ = f16(q).K -> SOFT_MAX_EXT(scale, causal) -> f16(P).V   
// Split over ATTN_CHUNK-position chunks (flash-decoding); each work-group does
// one (chunk, kv head, row) for all G query heads of the group (GQA), writing
// an unnormalised partial (m, l, O); attn_combine merges the chunks.
// ---------------------------------------------------------------------------
template <int D, int G>
__global__ __launch_bounds__(256) void attn_chunk_kernel(AttnArgs a) {
  constexpr int CH = ATTN_CHUNK;
  constexpr int DQ = D / 4;  // dims per lane-quarter in the score phase
  const int chunk = blockIdx.x, kvh = blockIdx.y, c = blockIdx.z;
  const int pos = a.pos[c];
  const int ctx = min(pos + 1, a.n_ctx);
  const int p0 = chunk * CH;
  if (p0 >= ctx) return;
  const int np = min(CH, ctx - p0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = a.slot[c];

  __shared__ float qs[G][4 * (DQ + 1)];  // padded per quarter: conflict-free broadcast reads
  __shared__ float S[G][CH];
  constexpr int DP = D / 2;
  constexpr int NG = 256 / DP;
  __shared__ float red[NG * G * D];

  const int ldq = a.n_head * D;
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, dd = i % D;
    qs[g][(dd / DQ) * (DQ + 1) + dd % DQ] = round_f16(a.q[(size_t)c * ldq + (kvh * G + g) * D + dd]);
  }
  __syncthreads();

  const _Float16* Kb = a.kc + (size_t)slot * a.slot_stride + (size_t)kvh * a.n_ctx * D;
  const _Float16* Vb = a.vc + (size_t)slot * a.slot_stride + (size_t)kvh * a.n_ctx * D;

  {  // scores: wave w -> positions [16w, 16w+16); 4 lanes per position
    const int pl = w * 16 + (lane >> 2);
    const int part = lane & 3;
    float accg[G];
#pragma unroll
    for (int g = 0; g < G; ++g) accg[g] = 0.f;
    if (pl < np) {
      const f16x8* kr = reinterpret_cast<const f16x8*>(Kb + (size_t)(p0 + pl) * D + part * DQ);
#pragma unroll
      for (int v = 0; v < DQ / 8; ++v) {
        f16x8 kv = kr[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float kf = (float)kv[j];
#pragma unroll
          for (int g = 0; g < G; ++g) accg[g] += qs[g][part * (DQ + 1) + v * 8 + j] * kf;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      accg[g] += __shfl_xor(accg[g], 1);
      accg[g] += __shfl_xor(accg[g], 2);
    }
    if (part == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) S[g][pl] = (pl < np) ? accg[g] * a.scale : -INFINITY;
    }
  }
  __syncthreads();

  // chunk-local softmax: one wave per head, one lane per position
  for (int g = w; g < G; g += 4) {
    const float sv = S[g][lane];
    float m = sv;
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float e = (lane < np) ? expf(sv - m) : 0.f;
    float l = e;
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
    S[g][lane] = round_f16(e);  // ggml rounds probabilities to f16 for the f16 V product
    if (lane == 0) {
      float* ml = a.ml_part + (((size_t)c * a.n_head + kvh * G + g) * a.n_chunks + chunk) * 2;
      ml[0] = m;
      ml[1] = l;
    }
  }
  __syncthreads();

  {  // O = P.V ; thread -> (dim pair dp, position group pg)
    const int dp = tid % DP, pg = tid / DP;
    float o0[G], o1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) o0[g] = o1[g] = 0.f;
    for (int pl = pg; pl < np; pl += NG) {
      const f16x2 v = *reinterpret_cast<const f16x2*>(Vb + (size_t)(p0 + pl) * D + 2 * dp);
      const float v0 = (float)v[0], v1 = (float)v[1];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = S[g][pl];
        o0[g] += p * v0;
        o1[g] += p * v1;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      red[(pg * G + g) * D + 2 * dp] = o0[g];
      red[(pg * G + g) * D + 2 * dp + 1] = o1[g];
    }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, dd = i % D;
    float sacc = 0.f;
#pragma unroll
    for (int pg = 0; pg < NG; ++pg) sacc += red[(pg * G + g) * D + dd];
    a.o_part[(((size_t)c * a.n_head + kvh * G + g) * a.n_chunks + chunk) * D + dd] = sacc;
  }
}

// merge chunk partials: O = sum_i e^(m_i-M) O_i / sum_i e^(m_i-M) l_i  -> bf16 (src1 of attn_output)
__global__ void attn_combine_kernel(AttnArgs a) {
  const int h = blockIdx.x, c = blockIdx.y;
  const int D = a.head_dim;
  const int nch = (min(a.pos[c] + 1, a.n_ctx) + ATTN_CHUNK - 1) / ATTN_CHUNK;
  const float* ml = a.ml_part + ((size_t)c * a.n_head + h) * a.n_chunks * 2;
  float M = -INFINITY;
  for (int i = 0; i < nch; ++i) M = fmaxf(M, ml[2 * i]);
  float L = 0.f;
  for (int i = 0; i < nch; ++i) L += expf(ml[2 * i] - M) * ml[2 * i + 1];
  const float inv = 1.0f / L;
  const float* op = a.o_part + ((size_t)c * a.n_head + h) * a.n_chunks * D;
  for (int dd = threadIdx.x; dd < D; dd += blockDim.x) {
    float o = 0.f;
    for (int i = 0; i < nch; ++i) o += expf(ml[2 * i] - M) * op[(size_t)i * D + dd];
    a.out[(size_t)c * a.ldo + h * D + dd] = (uint16_t)f2bf(o * inv);
  }
}

template <int D>
static void launch_attn_d(const AttnArgs& a, hipStream_t s) {
  dim3 grid(a.n_chunks, a.n_head_kv, a.M);
  switch (a.n_head / a.n_head_kv) {
    case 1: attn_chunk_kernel<D, 1><<<grid, 256, 0, s>>>(a); break;
    case 2: attn_chunk_kernel<D, 2><<<grid, 256, 0, s>>>(a); break;
    case 4: attn_chunk_kernel<D, 4><<<grid, 256, 0, s>>>(a); break;
    case 8: attn_chunk_kernel<D, 8><<<grid, 256, 0, s>>>(a); break;
  }
}

void launch_attention(const AttnArgs& a, hipStream_t s) {
  if (a.head_dim == 64)
    launch_attn_d<64>(a, s);
  else
    launch_attn_d<128>(a, s);
  attn_combine_kernel<<<dim3(a.n_head, a.M), 64, 0, s>>>(a);
}

// ---------------------------------------------------------------------------
// greedy sampler: argmax over the vocabulary, ties -> lowest id  
// ---------------------------------------------------------------------------
constexpr int ARGMAX_CHUNKS = 64;

__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

__global__ __launch_bounds__(256) void argmax_stage1(const float* logits, int ldl, int V, float* ws_val,
                                                     int* ws_idx) {
  const int ch = blockIdx.x, c = blockIdx.y;
  const int per = (V + ARGMAX_CHUNKS - 1) / ARGMAX_CHUNKS;
  const int b = ch * per, e = min(V, b + per);
  const float* lr = logits + (size_t)c * ldl;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = b + threadIdx.x; i < e; i += 256) better(bv, bi, lr[i], i);
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o);
    int oi = __shfl_xor(bi, o);
    better(bv, bi, ov, oi);
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x >> 6] = bv;
    si[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) better(bv, bi, sv[k], si[k]);
    ws_val[c * ARGMAX_CHUNKS + ch] = bv;
    ws_idx[c * ARGMAX_CHUNKS + ch] = bi;
  }
}

__global__ void argmax_stage2(const float* ws_val, const int* ws_idx, int* tok_out, int* ids_next, int* pos_next,
                              int* hist, int hist_stride, int* hist_count, int max_hist) {
  const int c = blockIdx.x, lane = threadIdx.x;
  float bv = ws_val[c * ARGMAX_CHUNKS + lane];
  int bi = ws_idx[c * ARGMAX_CHUNKS + lane];
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o);
    int oi = __shfl_xor(bi, o);
    better(bv, bi, ov, oi);
  }
  if (lane == 0) {
    if (bi == 0x7fffffff) bi = 0;  // all-NaN row
    if (tok_out) tok_out[c] = bi;
    if (ids_next) ids_next[c] = bi;
    if (pos_next) pos_next[c] += 1;
    if (hist) {
      int n = hist_count[c];
      if (n < max_hist) hist[(size_t)c * hist_stride + n] = bi;
      hist_count[c] = n + 1;
    }
  }
}

void launch_argmax(const float* logits, int ldl, int M, int V, float* ws_val, int* ws_idx, int* tok_out,
                   int* ids_next, int* pos_next, int* hist, int hist_stride, int* hist_count, int max_hist,
                   hipStream_t s) {
  argmax_stage1<<<dim3(ARGMAX_CHUNKS, M), 256, 0, s>>>(logits, ldl, V, ws_val, ws_idx);
  argmax_stage2<<<M, 64, 0, s>>>(ws_val, ws_idx, tok_out, ids_next, pos_next, hist, hist_stride, hist_count,
                                 max_hist);
}

}  // namespace mx
