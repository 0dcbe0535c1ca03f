// kquant.hip -- K-quant weights (GGUF Q4_K, Q5_K, Q6_K) on the int8 MFMA path  (SURVEY §8a a16).
//
// llama.cpp runs a K-quant MUL_MAT as ggml_vec_dot_q{4,5,6}_K_q8_K: the f32 activation row is
// quantised to Q8_K (per 256 values: iscale = -127/max, q = nearest_int(iscale*x), d = 1/iscale,
// bsums per 16), and every super-block of 256 weights contributes an exact int32
//   Q4_K / Q5_K:  S = sum_j sc_j * (q_w . q_x over 32-value sub-block j),  Mn = sum_j m_j * bsum32_j
//   Q6_K:         S = sum_g sc_g * (q_w . q_x over 16-value group g)        (q_w = 6-bit value - 32)
// scaled in f32:  acc += (f16(d) * d_x) * S  -  (f16(dmin) * d_x) * Mn.
// Here the q_w . q_x products run on v_mfma_i32_16x16x32_i8 (16 rows x 16 tokens x one 32-k
// sub-block; Q6_K two per sub-block, each with the lanes of the other 16-k group zeroed), the
// mins term on v_mfma_f32_16x16x4_f32 (exact: every operand and sum is an integer < 2^24) and the
// scale multiply-adds in int32 on the VALU -- so each super-block integer equals ggml's and only
// the f32 accumulation order differs (ggml's own SIMD paths differ from its scalar one the same way).
//
// Weights are repacked at load into tiles of 16 rows x 256 k (kernels.h kq_tile_bytes) whose byte
// order is the lane order of the MFMA operands: a wave reads each tile region as contiguous 16 B
// per lane, and the 4-bit fields unpack with two mask/shift operations per 8 values.  Bytes per
// weight equal the GGUF's (Q6_K exactly; Q4_K / Q5_K +2.8% / +2.3% for byte-aligned scales).
// Activation rows are Q8_K images made once per GEMV by the producer side (RMS_NORM + quantise, or
// quantise of the attention output / SwiGLU product), k permuted within each super-block so a
// lane's 8-byte B fragments of all 8 sub-blocks are one 64-byte run.
#include "device_common.h"

namespace mx {

// ---------------------------------------------------------------------------
// Packed tile layout, per 16 rows x 256 k (one super-block of 16 weight rows):
//   [0, 2048)   QS: lane l (row r = l&15, k-slice g = l>>4) owns 8 dwords D[0..7], D[j] holding
//               the low 4 bits of value (j, e) -- k = 32j + 8g + e -- in byte e&3, nibble e>>2;
//               D[0..3] at 16*l, D[4..7] at 1024 + 16*l
//   Q5_K  [2048, 2560): lane l's 2 dwords at 2048 + 8l: bit 4 of value (j, e) at bit
//               8*(e&3) + (u&7) of dword u>>3, u = 2j + (e>>2)
//   Q6_K  [2048, 3072): lane l's 4 dwords at 2048 + 16l: bits 4-5 of value (j, e) at bits
//               8*(e&3) + 2*(u&3) of dword u>>2
//   scales lane-major, row r = 4q + i (q = r >> 2): byte SC + 64q + 4c + i is lane c + 16q's
//   byte i (the rows of the MFMA C-layout lane group q), so one dword per lane holds its 4 rows:
//   Q4_K / Q5_K at SC = 2048 / 2560:  column c < 8: 6-bit scale of sub-block c, c >= 8: 6-bit min
//               of sub-block c - 8;  SC + 256 + 16q + 2i: f16 d of row r, SC + 264 + 16q + 2i: f16 dmin
//   Q6_K at SC = 3072:  column c: int8 scale of 16-value group c;  SC + 256 + 2r: f16 d of row r
// ---------------------------------------------------------------------------
template <int T>
struct KqTile;
template <>
struct KqTile<12> {
  static constexpr int BYTES = 2368, SC = 2048, BLOCK = 144;
};
template <>
struct KqTile<13> {
  static constexpr int BYTES = 2880, SC = 2560, BLOCK = 176;
};
template <>
struct KqTile<14> {
  static constexpr int BYTES = 3360, SC = 3072, BLOCK = 210;
};

int kq_tile_bytes(int type) {
  return type == 12 ? KqTile<12>::BYTES : type == 13 ? KqTile<13>::BYTES : type == 14 ? KqTile<14>::BYTES : 0;
}
int kq_block_bytes(int type) {
  return type == 12 ? KqTile<12>::BLOCK : type == 13 ? KqTile<13>::BLOCK : type == 14 ? KqTile<14>::BLOCK : 0;
}

// The 256 values of one GGUF super-block in k order (Q4_K 0..15, Q5_K 0..31, Q6_K 0..63 before
// the -32) -- ggml-common.h block_q4_K {d, dmin, scales[12], qs[128]}, block_q5_K {d, dmin,
// scales[12], qh[32], qs[128]}, block_q6_K {ql[128], qh[64], scales[16], d}.
__device__ __forceinline__ int kq_value(int type, const uint8_t* b, int k) {
  if (type == 14) {
    const int h = k >> 7, i = (k >> 5) & 3, l = k & 31;
    const int L = b[64 * h + 32 * (i & 1) + l];
    const int H = b[128 + 32 * h + l];
    return ((i < 2 ? L & 15 : L >> 4) | (((H >> (2 * i)) & 3) << 4));
  }
  const int g = k >> 6, hi = (k >> 5) & 1, l = k & 31;
  const uint8_t* qs = b + (type == 13 ? 48 : 16);
  int v = hi ? qs[32 * g + l] >> 4 : qs[32 * g + l] & 15;
  if (type == 13) v |= ((b[16 + l] >> (2 * g + hi)) & 1) << 4;
  return v;
}

// One thread per (row, super-block): decode the GGUF block, write the row's bytes of its tile.
template <int T>
__global__ void pack_kq_kernel(uint8_t* dst, const uint8_t* src, int N, int K, int mode, int offset) {
  const int SB = K / 256;
  const size_t total = (size_t)N * SB;
  for (size_t it = blockIdx.x * (size_t)blockDim.x + threadIdx.x; it < total; it += (size_t)gridDim.x * blockDim.x) {
    const int row = (int)(it / SB), sb = (int)(it % SB);
    const uint8_t* b = src + it * KqTile<T>::BLOCK;
    const int P = packed_row(row, mode, offset);
    uint8_t* tile = dst + ((size_t)(P >> 4) * SB + sb) * KqTile<T>::BYTES;
    const int r = P & 15;
    for (int g = 0; g < 4; ++g) {
      const int lane = r + 16 * g;
      uint32_t D[8] = {0, 0, 0, 0, 0, 0, 0, 0}, H[4] = {0, 0, 0, 0};
      for (int j = 0; j < 8; ++j)
        for (int e = 0; e < 8; ++e) {
          const int v = kq_value(T, b, 32 * j + 8 * g + e);
          D[j] |= (uint32_t)(v & 15) << (8 * (e & 3) + 4 * (e >> 2));
          const int u = 2 * j + (e >> 2);
          if (T == 13) H[u >> 3] |= (uint32_t)((v >> 4) & 1) << (8 * (e & 3) + (u & 7));
          if (T == 14) H[u >> 2] |= (uint32_t)((v >> 4) & 3) << (8 * (e & 3) + 2 * (u & 3));
        }
      for (int j = 0; j < 8; ++j) *reinterpret_cast<uint32_t*>(tile + (j >> 2) * 1024 + 16 * lane + 4 * (j & 3)) = D[j];
      if (T == 13)
        for (int c = 0; c < 2; ++c) *reinterpret_cast<uint32_t*>(tile + 2048 + 8 * lane + 4 * c) = H[c];
      if (T == 14)
        for (int c = 0; c < 4; ++c) *reinterpret_cast<uint32_t*>(tile + 2048 + 16 * lane + 4 * c) = H[c];
    }
    constexpr int SC = KqTile<T>::SC;
    uint8_t* scr = tile + SC + 64 * (r >> 2) + (r & 3);  // column c at scr[4c]
    if (T == 14) {
      for (int g = 0; g < 16; ++g) scr[4 * g] = b[192 + g];
      tile[SC + 256 + 2 * r] = b[208];
      tile[SC + 256 + 2 * r + 1] = b[209];
    } else {
      const uint8_t* q = b + 4;  // get_scale_min_k4
      uint8_t sc[8], mn[8];
      for (int j = 0; j < 8; ++j) {
        if (j < 4) {
          sc[j] = q[j] & 63;
          mn[j] = q[j + 4] & 63;
        } else {
          sc[j] = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
          mn[j] = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
        }
        scr[4 * j] = sc[j];
        scr[4 * (8 + j)] = mn[j];
      }
      uint8_t* dr = tile + SC + 256 + 16 * (r >> 2) + 2 * (r & 3);
      dr[0] = b[0];  // d
      dr[1] = b[1];
      dr[8] = b[2];  // dmin
      dr[9] = b[3];
    }
  }
}

int launch_pack_kq(uint8_t* dst, const uint8_t* src, int type, int N, int K, int mode, int offset, hipStream_t s) {
  if (K % 256 || N % 8) return -1;
  const int g = fill_grid((size_t)N * (K / 256));
  switch (type) {
    case 12: pack_kq_kernel<12><<<g, 256, 0, s>>>(dst, src, N, K, mode, offset); return 0;
    case 13: pack_kq_kernel<13><<<g, 256, 0, s>>>(dst, src, N, K, mode, offset); return 0;
    case 14: pack_kq_kernel<14><<<g, 256, 0, s>>>(dst, src, N, K, mode, offset); return 0;
  }
  return -1;
}

// Synthetic K-quant blocks (synth.py kq_blocks is the spec): byte i of the tensor's block stream
// is byte i%8 of the synthetic hash of i/8; the f16 scale fields are then fixed-exponent bit
// patterns with a random mantissa byte, Q6_K's int8 scales folded into [-24, 23].
__device__ __forceinline__ uint64_t synth_hash(uint64_t seed, uint64_t tid, uint64_t idx) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + tid * 0xD1B54A32D192ED03ull + idx;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void synth_kq_kernel(uint8_t* dst, int type, int bb, size_t nblocks, uint64_t seed, uint64_t tid) {
  for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < nblocks; b += (size_t)gridDim.x * blockDim.x) {
    uint8_t* p = dst + b * bb;
    for (int i = 0; i < bb; ++i) {
      const uint64_t gi = (uint64_t)b * bb + i;
      p[i] = (uint8_t)(synth_hash(seed, tid, gi >> 3) >> (8 * (gi & 7)));
    }
    if (type == 14) {
      for (int j = 0; j < 16; ++j) p[192 + j] = (uint8_t)(int8_t)((int)(p[192 + j] % 48) - 24);
      const uint32_t d = 0x0500u + p[208];
      p[208] = (uint8_t)d;
      p[209] = (uint8_t)(d >> 8);
    } else {
      const uint32_t d = 0x0500u + p[0], mn = (type == 13 ? 0x1500u : 0x1100u) + p[1];
      p[0] = (uint8_t)d;
      p[1] = (uint8_t)(d >> 8);
      p[2] = (uint8_t)mn;
      p[3] = (uint8_t)(mn >> 8);
    }
  }
}

int launch_synth_kq_blocks(uint8_t* dst, int type, size_t nblocks, uint64_t seed, uint64_t tid, hipStream_t s) {
  const int bb = kq_block_bytes(type);
  if (!bb) return -1;
  synth_kq_kernel<<<fill_grid(nblocks), 256, 0, s>>>(dst, type, bb, nblocks, seed, tid);
  return 0;
}

// GET_ROWS of a K-quant token_embd: dequantize_row_q{4,5,6}_K (f32, one rounding per operation);
// thread = 16 consecutive values
__global__ __launch_bounds__(256) void embed_kq_kernel(float* x, const uint8_t* tok, int type, int bb, const int* ids,
                                                       int n, float* ssq) {
#pragma clang fp contract(off)
  const int c = blockIdx.x;
  const uint8_t* row = tok + (size_t)ids[c] * (n / 256) * bb;
  for (int t = threadIdx.x; t < n / 16; t += blockDim.x) {
    f32x4 g[4];  // this 16-element tile's values: its RMS_NORM-on-load partial is ssq16 (device_common.h)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = 16 * t + i;
      const uint8_t* b = row + (size_t)(k / 256) * bb;
      const int kk = k % 256;
      const int v = kq_value(type, b, kk);
      float y;
      if (type == 14) {
        const float d = (float)__builtin_bit_cast(_Float16, (uint16_t)(b[208] | (b[209] << 8)));
        y = (d * (float)(int8_t)b[192 + kk / 16]) * (float)(v - 32);
      } else {
        const int j = kk / 32;
        const uint8_t* q = b + 4;
        const int sc = j < 4 ? q[j] & 63 : (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        const int mn = j < 4 ? q[j + 4] & 63 : (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
        const float d = (float)__builtin_bit_cast(_Float16, (uint16_t)(b[0] | (b[1] << 8)));
        const float dmin = (float)__builtin_bit_cast(_Float16, (uint16_t)(b[2] | (b[3] << 8)));
        y = (d * (float)sc) * (float)v - dmin * (float)mn;
      }
      x[(size_t)c * n + k] = y;
      g[i >> 2][i & 3] = y;
    }
    if (ssq) ssq[(size_t)c * (n / 16) + t] = ssq16(g[0], g[1], g[2], g[3]);
  }
}

int launch_embed_kq(float* x, const uint8_t* tok, int type, const int* ids, int M, int n, float* ssq, hipStream_t s) {
  const int bb = kq_block_bytes(type);
  if (!bb || n % 256) return -1;
  embed_kq_kernel<<<M, 256, 0, s>>>(x, tok, type, bb, ids, n, ssq);
  return 0;
}

// ---------------------------------------------------------------------------
// Q8_K activation rows.  xq int8 [M][K]: within super-block s, logical k = 256s + 32j + 8g + e
// sits at 256s + 64g + 8j + e (lane group g's 8 sub-block fragments contiguous); xd f32 [M][K/256]
// (d = 1/iscale); xb f32 [M][K/32]: the sum of the 32 q of sub-block j at 8s + 2(j&3) + (j>>2)
// (the B operand order of the mins MFMA).
// One DPP row (16 lanes) per super-block, lane t holding k = 16t .. 16t+15: the max and the
// first-max search are row16 DPP reductions (no LDS round trips), 4 super-blocks per wave.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void q8k_row(const float (&v)[16], int t, int8_t* qsb, float* dsb, float* xbsb) {
  float a = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) a = fmaxf(a, fabsf(v[i]));
  const float amax = row16_max(a);
  // ggml takes max = the signed value of the FIRST element with |x| == amax
  int first = 1 << 20;
#pragma unroll
  for (int i = 15; i >= 0; --i)
    if (fabsf(v[i]) == amax) first = 16 * t + i;
  const int key = (int)-row16_max(-(float)first);  // exact: keys < 2^24
  float mine = 0.f;
  if (first == key) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (16 * t + i == key) mine = v[i];
  }
  const float mx = row16_sum(mine);  // only the owner lane contributes
  int q[16];
  float d = 0.f;
  if (amax != 0.f) {
    const float iscale = -127.f / mx;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = (int)__builtin_rintf(iscale * v[i]);
      q[i] = r < 127 ? r : 127;
    }
    d = 1.f / iscale;
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) q[i] = 0;
  }
  // k = 16t + i: sub-block j = t >> 1, lane group g = 2(t&1) + (i >> 3), e = i & 7
  const int j = t >> 1;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    u32x2 w = u32x2{0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e >> 2] |= (uint32_t)(uint8_t)(int8_t)q[8 * h + e] << (8 * (e & 3));
    *reinterpret_cast<u32x2*>(qsb + 64 * (2 * (t & 1) + h) + 8 * j) = w;
  }
  int bs = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) bs += q[i];
  bs += __shfl_xor(bs, 1);
  if ((t & 1) == 0) xbsb[2 * (j & 3) + (j >> 2)] = (float)bs;
  if (t == 0) *dsb = d;
}

// grid (ceil(K/256/16), M), 256 threads: super-block s = 16*blockIdx.x + threadIdx.x/16 of row
// blockIdx.y; with norm_w, RMS_NORM + MUL first (sum of squares of the whole row in double, every
// work-group of the row computing it the same way: norm_q8_kernel's arithmetic)
// With nslab > 0 (NORM, one work-group per row, no row_map): src is the residual stream x and the
// split-K partial slabs of the GEMV that produced it are folded first -- x += slab 0 + slab 1 + ...
// (resid_norm's order), the sum of squares taken over the folded row and the folded values written
// back to x by the thread that quantises them.
template <bool NORM, bool FOLD>
__global__ __launch_bounds__(FOLD ? 1024 : 256) void q8k_kernel(int8_t* xq, float* xd, float* xb, const float* src,
                                                                int ld, const float* w, const int* row_map, int n,
                                                                float eps, const float* slabs, int nslab,
                                                                size_t sstride) {
  const int c = blockIdx.y;
  const int r = row_map ? row_map[c] : c;
  const float* xr = src + (size_t)r * ld;
  float scale = 1.0f;
  // FOLD (n <= 4096, 1024 threads, NORM): one 4-value piece per thread, x and every slab loaded at once,
  // folded x written back to x and staged in LDS for the quantisation below
  __shared__ __attribute__((aligned(16))) float xf[FOLD ? 4096 : 1];
  if constexpr (NORM) {
    double acc = 0.0;
    if constexpr (FOLD) {
      const int i = threadIdx.x * 4;
      if (i < n) {
        f32x4 sl[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k < nslab) sl[k] = *reinterpret_cast<const f32x4*>(slabs + k * sstride + (size_t)c * n + i);
        f32x4 t = sl[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
          if (k < nslab) t += sl[k];
        const f32x4 v = *reinterpret_cast<const f32x4*>(xr + i) + t;  // x + (s0 + s1 + ...): resid_norm's order
        *reinterpret_cast<f32x4*>(const_cast<float*>(xr) + i) = v;
        *reinterpret_cast<f32x4*>(xf + i) = v;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += (double)(v[j] * v[j]);
      }
    } else {
      for (int i = threadIdx.x * 4; i < n; i += 1024) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(xr + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += (double)(v[j] * v[j]);
      }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    constexpr int NWV = FOLD ? 16 : 4;
    __shared__ double part[NWV];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    double sum = 0.0;
#pragma unroll
    for (int k = 0; k < NWV; ++k) sum += part[k];
    scale = 1.0f / sqrtf((float)(sum / n) + eps);
  }
  const int s = 16 * blockIdx.x + (threadIdx.x >> 4);
  if (s >= n / 256) return;
  const int t = threadIdx.x & 15;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; i += 4) {
    const int k = 256 * s + 16 * t + i;
    const f32x4 x4 = FOLD ? *reinterpret_cast<const f32x4*>(xf + k) : *reinterpret_cast<const f32x4*>(xr + k);
    if constexpr (NORM) {
      const f32x4 g4 = *reinterpret_cast<const f32x4*>(w + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i + e] = (x4[e] * scale) * g4[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i + e] = x4[e];
    }
  }
  q8k_row(v, t, xq + (size_t)c * n + 256 * s, xd + (size_t)c * (n / 256) + s, xb + (size_t)c * (n / 32) + 8 * s);
}

int launch_rmsnorm_q8k(int8_t* xq, float* xd, float* xb, const float* x, const float* w, const int* row_map, int M, int n,
                       float eps, hipStream_t s, const float* slabs, int nslab, size_t slab_stride) {
  if (n % 256 || M < 1) return -1;
  if (nslab && (row_map || n > 16 * 256 || !slabs)) return -1;  // the fold needs one work-group per row
  if (nslab)
    q8k_kernel<true, true><<<dim3(1, M), 1024, 0, s>>>(xq, xd, xb, x, n, w, row_map, n, eps, slabs, nslab, slab_stride);
  else
    q8k_kernel<true, false><<<dim3((n / 256 + 15) / 16, M), 256, 0, s>>>(xq, xd, xb, x, n, w, row_map, n, eps,
                                                                        nullptr, 0, 0);
  return 0;
}
int launch_quantize_q8k(int8_t* xq, float* xd, float* xb, const float* src, int ld, int M, int n, hipStream_t s) {
  if (n % 256 || M < 1) return -1;
  q8k_kernel<false, false><<<dim3((n / 256 + 15) / 16, M), 256, 0, s>>>(xq, xd, xb, src, ld, nullptr, nullptr, n,
                                                                         0.f, nullptr, 0, 0);
  return 0;
}

// ---------------------------------------------------------------------------
// Dequantisation of packed K-quant tiles into packed bf16 tiles (kernels.h layout: 16 rows x 32 k
// per 1 KiB lane-linear A fragment) for the prefill GEMM.  ggml's dequantize_row_q{4,5,6}_K values
// in f32 (Q4_K/Q5_K: (d*sc)*q - dmin*m; Q6_K: (d*sc)*(q-32)), rounded to bf16 like the bf16 path's
// weights.  One wave per (16-row tile, super-block): lane l holds row l&15, k 8(l>>4)..+8 of each
// 32-k sub-block j -- the i8 MFMA A-operand bytes of kq_compute, which are also the bf16 A layout.
// ---------------------------------------------------------------------------
template <int T>
__global__ __launch_bounds__(256) void dequant_kq_kernel(uint16_t* dst, const uint8_t* src, int tile_begin, int ntiles,
                                                         int SB) {
#pragma clang fp contract(off)  // ggml's dequantize_row_q*_K values: one rounding per operation
  constexpr int TB = KqTile<T>::BYTES, SC = KqTile<T>::SC;
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);  // (tile in segment, super-block)
  if (unit >= ntiles * SB) return;
  const int tile = unit / SB, sb = unit % SB;
  const uint8_t* t = src + (size_t)unit * TB;  // tiles are [tile][super-block] in the segment
  const int r = lane & 15, g = lane >> 4;
  const u32x4 q0 = *reinterpret_cast<const u32x4*>(t + 16 * lane);
  const u32x4 q1 = *reinterpret_cast<const u32x4*>(t + 1024 + 16 * lane);
  const uint32_t D[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
  u32x4 H = u32x4{0u, 0u, 0u, 0u};
  if constexpr (T == 13) {
    const u32x2 hv = *reinterpret_cast<const u32x2*>(t + 2048 + 8 * lane);
    H = u32x4{hv[0], hv[1], 0u, 0u};
  }
  if constexpr (T == 14) H = *reinterpret_cast<const u32x4*>(t + 2048 + 16 * lane);
  const int KT = SB * 8;
  uint16_t* out = dst + ((size_t)(tile_begin + tile) * KT + 8 * sb) * 512 + 8 * lane;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t lo = D[j] & 0x0F0F0F0Fu, hi = (D[j] >> 4) & 0x0F0F0F0Fu;
    if constexpr (T == 13) {
      lo |= ((H[j >> 2] >> ((2 * j) & 7)) & 0x01010101u) << 4;
      hi |= ((H[j >> 2] >> ((2 * j + 1) & 7)) & 0x01010101u) << 4;
    }
    if constexpr (T == 14) {
      lo |= ((H[j >> 1] >> (4 * (j & 1))) & 0x03030303u) << 4;
      hi |= ((H[j >> 1] >> (4 * (j & 1) + 2)) & 0x03030303u) << 4;
    }
    float y[8];
    if constexpr (T == 14) {
      const float d = f16b(t + SC + 256 + 2 * r);
      const int sc = (int)(int8_t)t[SC + 64 * (r >> 2) + 4 * (2 * j + (g >> 1)) + (r & 3)];
      const float ds = d * (float)sc;
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = ds * (float)((int)(((e < 4 ? lo : hi) >> (8 * (e & 3))) & 0xFFu) - 32);
    } else {
      const float d = f16b(t + SC + 256 + 16 * (r >> 2) + 2 * (r & 3));
      const float dmin = f16b(t + SC + 264 + 16 * (r >> 2) + 2 * (r & 3));
      const float d1 = d * (float)t[SC + 64 * (r >> 2) + 4 * j + (r & 3)];
      const float m1 = dmin * (float)t[SC + 64 * (r >> 2) + 4 * (8 + j) + (r & 3)];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = d1 * (float)((((e < 4 ? lo : hi) >> (8 * (e & 3))) & 0xFFu)) - m1;
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(y[2 * e]) | (f2bf(y[2 * e + 1]) << 16);
    *reinterpret_cast<u32x4*>(out + (size_t)j * 512) = o;
  }
}

int launch_dequant_kq(uint16_t* dst, const void* W, int K, int kq_n, const int* type, const int* tile_end,
                      const size_t* off, hipStream_t s) {
  if (K % 256 || kq_n < 1 || kq_n > 3) return -1;
  const int SB = K / 256;
  for (int i = 0; i < kq_n; ++i) {
    const int t0 = i ? tile_end[i - 1] : 0, nt = tile_end[i] - t0;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(W) + off[i];
    const int blocks = (nt * SB + 3) / 4;
    switch (type[i]) {
      case 12: dequant_kq_kernel<12><<<blocks, 256, 0, s>>>(dst, src, t0, nt, SB); break;
      case 13: dequant_kq_kernel<13><<<blocks, 256, 0, s>>>(dst, src, t0, nt, SB); break;
      case 14: dequant_kq_kernel<14><<<blocks, 256, 0, s>>>(dst, src, t0, nt, SB); break;
      default: return -1;
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// K-quant x Q8_K MUL_MAT.  Work-group = RT row tiles of one segment (one ggml type) x NB column
// tiles of 16 tokens (grid.y: groups of 16*NB tokens); its KS waves split the K/256 super-blocks,
// each keeping a ring of U super-blocks' loads in flight; partial tiles are summed through LDS and
// finished by the same epilogues as the bf16 / Q8_0 GEMVs (kernels.hip epi_store).
// ---------------------------------------------------------------------------
template <int RT, int NB>
struct KqFrag {
  u32x4 qs[RT][2];
  u32x4 h[RT];      // Q5_K: dwords 0-1; Q6_K: 0-3
  u32x4 sc[RT][4];  // Q4_K / Q5_K: [0..1]; Q6_K: [0..3]
  u32x4 dm[RT];     // Q4_K / Q5_K: f16 d x 4 rows, then f16 dmin x 4 rows; Q6_K: dwords 0-1 = f16 d x 4 rows
  u32x2 mw[RT];     // Q4_K / Q5_K: mins dwords of sub-blocks g, g+4 (byte lane&3 = this lane's A row), raw
  u32x4 x[NB][4];
  float dx[NB];
  f32x2 xb[NB];
};

// One super-block of RT weight tiles (Wt[r] = tile r's bytes at this super-block) ...
template <int T, int RT, int NB>
__device__ __forceinline__ void kq_load_w(KqFrag<RT, NB>& f, const uint8_t* const (&Wt)[RT], int lane, int g) {
  constexpr int SC = KqTile<T>::SC;
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const uint8_t* t = Wt[r];
    f.qs[r][0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t) + lane);
    f.qs[r][1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t + 1024) + lane);
    if constexpr (T == 13) {
      const u32x2 hv = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(t + 2048) + lane);
      f.h[r] = u32x4{hv[0], hv[1], 0u, 0u};
    }
    if constexpr (T == 14) f.h[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t + 2048) + lane);
    if constexpr (T == 14) {
#pragma unroll
      for (int c = 0; c < 4; ++c) f.sc[r][c] = *reinterpret_cast<const u32x4*>(t + SC + 64 * g + 16 * c);
      const u32x2 dv = *reinterpret_cast<const u32x2*>(t + SC + 256 + 8 * g);
      f.dm[r] = u32x4{dv[0], dv[1], 0u, 0u};
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) f.sc[r][c] = *reinterpret_cast<const u32x4*>(t + SC + 64 * g + 16 * c);
      // the mins of this lane's A row (lane & 15) for sub-blocks g and g + 4 (the mins MFMA's k = g),
      // kept raw: extracting them here would wait for this load at once (draining the ring)
      const uint8_t* mq = t + SC + 64 * ((lane & 15) >> 2) + 32 + 4 * g;
      f.mw[r] = u32x2{*reinterpret_cast<const uint32_t*>(mq), *reinterpret_cast<const uint32_t*>(mq + 16)};
      f.dm[r] = *reinterpret_cast<const u32x4*>(t + SC + 256 + 16 * g);
    }
  }
}

// ... and NB column tiles of Q8_K activations (Xq/Xd/Xb at this lane's column, Xq/Xb offset by
// its k group; global memory, or a quantise-on-load LDS image through the same pointers)
template <int T, int RT, int NB>
__device__ __forceinline__ void kq_load_x(KqFrag<RT, NB>& f, const int8_t* const (&Xq)[NB],
                                          const float* const (&Xd)[NB], const float* const (&Xb)[NB], int sb) {
#pragma unroll
  for (int n = 0; n < NB; ++n) {
#pragma unroll
    for (int c = 0; c < 4; ++c) f.x[n][c] = *reinterpret_cast<const u32x4*>(Xq[n] + (size_t)sb * 256 + 16 * c);
    f.dx[n] = Xd[n][sb];
    if constexpr (T != 14) f.xb[n] = *reinterpret_cast<const f32x2*>(Xb[n] + 8 * sb);
  }
}

template <int T, int RT, int NB>
__device__ __forceinline__ void kq_load(KqFrag<RT, NB>& f, const uint8_t* const (&Wt)[RT], const int8_t* const (&Xq)[NB],
                                        const float* const (&Xd)[NB], const float* const (&Xb)[NB], int sb, int lane,
                                        int g) {
  kq_load_w<T, RT, NB>(f, Wt, lane, g);
  kq_load_x<T, RT, NB>(f, Xq, Xd, Xb, sb);
}

// Quantise-on-load (one token): this wave's K-slice of super-blocks [kb, kb + nsb), nsb <= 8, of
// the f32 row xf -- after RMS_NORM+MUL when norm_w (scale from the ssq partials of the residual
// writers: fixed-order double sum, as xs_build) -- as Q8_K into a wave-private LDS image laid out
// like the global Q8_K buffers: q [nsb*256] (permuted), d [nsb], b [nsb*8].  Row group rr = lane/16
// quantises super-blocks rr and rr + 4 with q8k_row (ggml quantize_row_q8_K).  The source values
// are loaded by ql_load BEFORE the weight ring is issued (a load behind the ring waits for it).
struct QlRegs {
  f32x4 x[2][4], w[2][4], sq[2];
};
// every load unconditional at a clamped address (ql_build ignores the extra values): a load behind a
// branch left hipcc's wait counts at the merge at zero, serialising the prologue (xs_load's note)
__device__ __forceinline__ void ql_load(QlRegs& r, const MMArgs& a, int kb, int nsb, int lane) {
  const int t = lane & 15, rr = lane >> 4;
  const float* wsrc = a.norm_w ? a.norm_w : a.xf;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int it = max(0, min(rr + 4 * q, nsb - 1));  // a wave may own no super-block (K < 256 * waves)
    const size_t k0 = (size_t)(kb + it) * 256 + 16 * t;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r.x[q][i] = *reinterpret_cast<const f32x4*>(a.xf + k0 + 4 * i);
      r.w[q][i] = *reinterpret_cast<const f32x4*>(wsrc + k0 + 4 * i);
    }
  }
  const float* qsrc = a.norm_w ? a.ssq : a.xf;
  const int np = a.norm_w ? a.np : 4;
#pragma unroll
  for (int p = 0; p < 2; ++p) r.sq[p] = *reinterpret_cast<const f32x4*>(qsrc + min(lane * 4 + 256 * p, np - 4));
}
__device__ __forceinline__ void ql_build(const QlRegs& r, const MMArgs& a, int nsb, int lane, int8_t* iq, float* id,
                                         float* ib) {
  const int t = lane & 15, rr = lane >> 4;
  float scale = 1.0f;
  if (a.norm_w) {
    double acc = 0.0;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (lane * 4 + 256 * p < a.np)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += (double)r.sq[p][j];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    scale = 1.0f / sqrtf((float)(acc / a.K) + a.eps);
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int it = rr + 4 * q;
    if (it < nsb) {  // a whole 16-lane row takes the branch together (q8k_row's DPP rows)
      float v[16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * i + e] = a.norm_w ? (r.x[q][i][e] * scale) * r.w[q][i][e] : r.x[q][i][e];
      q8k_row(v, t, iq + 256 * it, id + it, ib + 8 * it);
    }
  }
}
constexpr int QL_SB_MAX = 8;                        // super-blocks per wave slice
constexpr int QL_WAVE_BYTES = QL_SB_MAX * (256 + 4 + 32);  // q, d, b of one slice

// the super-block's contribution to acc (int8 MFMA per 32-k sub-block, f32 scales as ggml)
template <int T, int RT, int NB>
__device__ __forceinline__ void kq_compute(f32x4 (&acc)[RT][NB], const KqFrag<RT, NB>& f, int g) {
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    uint32_t D[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      D[c] = f.qs[r][0][c];
      D[4 + c] = f.qs[r][1][c];
    }
    uint32_t scw[16];
#pragma unroll
    for (int c = 0; c < (T == 14 ? 4 : 2); ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) scw[4 * c + e] = f.sc[r][c][e];
    // sub-block by sub-block: unpack its A operand and scales once, then one MFMA (Q6_K: two) per
    // column tile; each sub-block's products are scaled into the int32 super-block sums only after
    // the next sub-block's MFMAs are issued, so the VALU does not wait on an MFMA it just issued
    // (integer sums: the order changes nothing)
    i32x4 S[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) S[n] = i32x4{0, 0, 0, 0};
    i32x4 Pp[NB], Pp1[NB];  // previous sub-block's products (Q6_K: both 16-value groups)
    int sp[4], sp1[4];      // ... and its scales
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      i32x4 Pc[NB], Pc1[NB];
      int sc[4], sc1[4];
      if (j < 8) {
        uint32_t lo = D[j] & 0x0F0F0F0Fu, hi = (D[j] >> 4) & 0x0F0F0F0Fu;
        if constexpr (T == 13) {
          const uint32_t H = f.h[r][j >> 2];
          lo |= ((H >> ((2 * j) & 7)) & 0x01010101u) << 4;
          hi |= ((H >> ((2 * j + 1) & 7)) & 0x01010101u) << 4;
        }
        if constexpr (T == 14) {
          const uint32_t H = f.h[r][j >> 1];
          lo |= ((H >> (4 * (j & 1))) & 0x03030303u) << 4;
          hi |= ((H >> (4 * (j & 1) + 2)) & 0x03030303u) << 4;
          lo = ((lo | 0x80808080u) - 0x20202020u) ^ 0x80808080u;  // bytewise q - 32
          hi = ((hi | 0x80808080u) - 0x20202020u) ^ 0x80808080u;
        }
        const long A = (long)(((unsigned long)hi << 32) | lo);
        if constexpr (T == 14) {
          // int8 scales of row 4g+i, groups 2j and 2j+1: byte i of dwords 2j, 2j+1 of the row group's 64
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            sc[i] = (int)(int8_t)(scw[2 * j] >> (8 * i));
            sc1[i] = (int)(int8_t)(scw[2 * j + 1] >> (8 * i));
          }
          const long A0 = g < 2 ? A : 0l, A1 = g < 2 ? 0l : A;
#pragma unroll
          for (int n = 0; n < NB; ++n) {
            const u32x4& xc = f.x[n][j >> 1];
            const long B = (long)(((unsigned long)xc[2 * (j & 1) + 1] << 32) | xc[2 * (j & 1)]);
            Pc[n] = __builtin_amdgcn_mfma_i32_16x16x32_i8(A0, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
            Pc1[n] = __builtin_amdgcn_mfma_i32_16x16x32_i8(A1, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
          }
        } else {
          // 6-bit scales of row 4g+i, sub-block j: byte i of dword j of the row group's 32
#pragma unroll
          for (int i = 0; i < 4; ++i) sc[i] = (int)((scw[j] >> (8 * i)) & 0xFFu);
#pragma unroll
          for (int n = 0; n < NB; ++n) {
            const u32x4& xc = f.x[n][j >> 1];
            const long B = (long)(((unsigned long)xc[2 * (j & 1) + 1] << 32) | xc[2 * (j & 1)]);
            Pc[n] = __builtin_amdgcn_mfma_i32_16x16x32_i8(A, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
          }
        }
      }
      if (j > 0) {
#pragma unroll
        for (int n = 0; n < NB; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if constexpr (T == 14) S[n][i] += __mul24(sp[i], Pp[n][i]) + __mul24(sp1[i], Pp1[n][i]);  // |P| < 2^17
            else S[n][i] += __mul24(sp[i], Pp[n][i]);
          }
      }
      if (j < 8) {
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          Pp[n] = Pc[n];
          if constexpr (T == 14) Pp1[n] = Pc1[n];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sp[i] = sc[i];
          if constexpr (T == 14) sp1[i] = sc1[i];
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const float dx = f.dx[n];
      if constexpr (T == 14) {
        const f16x4 d4 = __builtin_bit_cast(f16x4, u32x2{f.dm[r][0], f.dm[r][1]});
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[r][n][i] += ((float)d4[i] * dx) * (float)S[n][i];
      } else {
        // mins: sum_j m[row][j] * bsum32[j][col] on the f32 MFMA (k = sub-block g, then g + 4)
        const int rb = 8 * (threadIdx.x & 3);  // this lane's A row within its mins dwords
        const float m0 = (float)((f.mw[r][0] >> rb) & 0xFFu);  // mins of sub-blocks g, g + 4
        const float m1 = (float)((f.mw[r][1] >> rb) & 0xFFu);
        f32x4 Mn = __builtin_amdgcn_mfma_f32_16x16x4f32(m0, f.xb[n][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        Mn = __builtin_amdgcn_mfma_f32_16x16x4f32(m1, f.xb[n][1], Mn, 0, 0, 0);
        const f16x8 dm = __builtin_bit_cast(f16x8, f.dm[r]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[r][n][i] += ((float)dm[i] * dx) * (float)S[n][i];
          acc[r][n][i] -= ((float)dm[4 + i] * dx) * Mn[i];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// One token, block-diagonal form.  With one token kq_compute fills one of the 16 B columns of every
// MFMA and spends its VALU on per-sub-block int32 scaling of the 15 empty ones too (VALU-bound at
// ~3.3 TB/s).  Here the 16 columns carry the super-block's sub-blocks instead: for sub-block j the
// B operand holds the token's 32 q of sub-block j in column j (Q6_K: its two 16-value groups in
// columns 2j, 2j+1) and zeros elsewhere, so the 8 MFMAs of a super-block accumulate into ONE C
// whose column c is the integer product sum of sub-block (group) c for the tile's 16 rows.  Then
// per lane (column c, rows 4q..4q+3): one scale byte per row from its dword of the lane-major scale
// layout, one int multiply, and a DPP row reduction over the columns --
//   Q4_K / Q5_K: columns 0-7 give S = sum_j sc_j * P_j (lane 7), columns 8-15 the mins term
//                Mn = sum_j m_j * bsum32_j (lane 15; the lane's bsum32 from the Q8_K image),
//   Q6_K:        S = sum_g sc_g * (P_g - 32 * bsum16_g) over all 16 columns (the -32 of every
//                6-bit value taken out of the A operand: an exact integer identity),
// which are ggml's super-block integers exactly; the f32 scaling is kq_compute's.  The result of a
// tile ends in lane 0 of each row group (kq_bd_finish), i.e. column 0 of the C layout: the token.
// ---------------------------------------------------------------------------
struct KqBdX {
  u32x2 X;    // this lane's 8 q of its column's sub-block (group) slice, zero where it carries none
  int bs;     // Q4_K / Q5_K lanes c >= 8: bsum32 of sub-block c - 8; Q6_K: bsum16 of group c
  float dx;   // the super-block's d
};

// the token's super-block sb (xq / xd / xb: the Q8_K row, or a wave image indexed the same way)
template <int T>
__device__ __forceinline__ KqBdX kq_bd_x(const int8_t* xq, const float* xd, const float* xb, int sb, int lane) {
  const int c = lane & 15, q = lane >> 4;
  KqBdX r;
  // permuted Q8_K order: k = 32j + 8q + e of the super-block at 64q + 8j + e
  if constexpr (T == 14) {
    const u32x2 v = *reinterpret_cast<const u32x2*>(xq + (size_t)sb * 256 + 64 * q + 8 * (c >> 1));
    const bool on = (q >> 1) == (c & 1);  // lanes q = 0,1 hold group 2j's 16 values, q = 2,3 group 2j+1's
    r.X = on ? v : u32x2{0u, 0u};
    int p = __builtin_amdgcn_sdot4((int)r.X[0], 0x01010101, 0, false);
    p = __builtin_amdgcn_sdot4((int)r.X[1], 0x01010101, p, false);
    p += __shfl_xor(p, 16);
    r.bs = p + __shfl_xor(p, 32);  // column c's 16 values: two lanes of the four
  } else {
    const int j = c & 7;
    const u32x2 v = *reinterpret_cast<const u32x2*>(xq + (size_t)sb * 256 + 64 * q + 8 * j);
    r.X = c < 8 ? v : u32x2{0u, 0u};
    r.bs = (int)xb[(size_t)sb * 8 + 2 * (j & 3) + (j >> 2)];  // exact: an integer sum
  }
  r.dx = xd[sb];
  return r;
}

// kq_bd_x for lane l of a wave without cross-lane operations (the LDS image builder; Q6_K's bsum16
// summed over both halves of the group from the row itself)
template <int T>
__device__ __forceinline__ KqBdX kq_bd_x_lane(const int8_t* xq, const float* xd, const float* xb, int sb, int l) {
  const int c = l & 15, q = l >> 4;
  KqBdX r;
  if constexpr (T == 14) {
    const int j = c >> 1, h = c & 1;
    const u32x2 v = *reinterpret_cast<const u32x2*>(xq + (size_t)sb * 256 + 64 * q + 8 * j);
    r.X = (q >> 1) == h ? v : u32x2{0u, 0u};
    int p = 0;
#pragma unroll
    for (int qq = 2 * h; qq < 2 * h + 2; ++qq) {  // group c = lanes q = 2h, 2h+1 of column c
      const u32x2 g = *reinterpret_cast<const u32x2*>(xq + (size_t)sb * 256 + 64 * qq + 8 * j);
      p = __builtin_amdgcn_sdot4((int)g[0], 0x01010101, p, false);
      p = __builtin_amdgcn_sdot4((int)g[1], 0x01010101, p, false);
    }
    r.bs = p;
  } else {
    const int j = c & 7;
    const u32x2 v = *reinterpret_cast<const u32x2*>(xq + (size_t)sb * 256 + 64 * q + 8 * j);
    r.X = c < 8 ? v : u32x2{0u, 0u};
    r.bs = (int)xb[(size_t)sb * 8 + 2 * (j & 3) + (j >> 2)];
  }
  r.dx = xd[sb];
  return r;
}

// weights of one super-block of one tile: the 4-bit planes and high bits as kq_load_w, the lane's
// scale dword (lane-major layout) and f16 d (lanes c >= 8 of Q4_K / Q5_K: dmin) of its 4 rows
template <int T>
__device__ __forceinline__ void kq_load_w_bd(KqFrag<1, 1>& f, const uint8_t* t, int lane) {
  constexpr int SC = KqTile<T>::SC;
  const int g = lane >> 4;
  f.qs[0][0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t) + lane);
  f.qs[0][1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t + 1024) + lane);
  if constexpr (T == 13) {
    const u32x2 hv = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(t + 2048) + lane);
    f.h[0] = u32x4{hv[0], hv[1], 0u, 0u};
  }
  if constexpr (T == 14) f.h[0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t + 2048) + lane);
  f.sc[0][0][0] = *reinterpret_cast<const uint32_t*>(t + SC + 4 * lane);
  const u32x2 dv = *reinterpret_cast<const u32x2*>(t + SC + 256 + (T == 14 ? 8 * g : 16 * g + (lane & 8)));
  f.dm[0] = u32x4{dv[0], dv[1], 0u, 0u};
}

// in-row DPP sums of 4 ints: lane l adds lane (l - n) mod 16 (row_ror), steps 4, 2, 1 (8-lane sums
// in lanes 7 and 15) or 8, 4, 2, 1 (the row sum in every lane)
#define KQ_ROR_ADD4(op, n)                                                               \
  op "_dpp %0, %0, %0 row_ror:" #n " row_mask:0xf bank_mask:0xf\n\t" op "_dpp %1, %1, %1 row_ror:" #n \
     " row_mask:0xf bank_mask:0xf\n\t" op "_dpp %2, %2, %2 row_ror:" #n " row_mask:0xf bank_mask:0xf\n\t" op \
     "_dpp %3, %3, %3 row_ror:" #n " row_mask:0xf bank_mask:0xf\n\t"
__device__ __forceinline__ void row8_isum4(int (&v)[4]) {
  asm volatile("s_nop 1\n\t" KQ_ROR_ADD4("v_add_u32", 4) KQ_ROR_ADD4("v_add_u32", 2) KQ_ROR_ADD4("v_add_u32", 1)
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
__device__ __forceinline__ void row16_isum4(int (&v)[4]) {
  asm volatile("s_nop 1\n\t" KQ_ROR_ADD4("v_add_u32", 8) KQ_ROR_ADD4("v_add_u32", 4) KQ_ROR_ADD4("v_add_u32", 2)
                   KQ_ROR_ADD4("v_add_u32", 1)
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}

template <int T>
__device__ __forceinline__ void kq_compute_bd(f32x4& acc, const KqFrag<1, 1>& f, const KqBdX& x, int lane) {
  const int c = lane & 15;
  const int jsel = T == 14 ? (c >> 1) : c;  // the sub-block whose MFMA this lane's column joins
  uint32_t D[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    D[k] = f.qs[0][0][k];
    D[4 + k] = f.qs[0][1][k];
  }
  i32x4 C0 = i32x4{0, 0, 0, 0}, C1 = i32x4{0, 0, 0, 0};  // two chains: no MFMA waits on the previous
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t lo = D[j] & 0x0F0F0F0Fu, hi = (D[j] >> 4) & 0x0F0F0F0Fu;
    if constexpr (T == 13) {
      const uint32_t H = f.h[0][j >> 2];
      lo |= ((H >> ((2 * j) & 7)) & 0x01010101u) << 4;
      hi |= ((H >> ((2 * j + 1) & 7)) & 0x01010101u) << 4;
    }
    if constexpr (T == 14) {  // 6-bit values 0..63 (the -32 is applied to the sums)
      const uint32_t H = f.h[0][j >> 1];
      lo |= ((H >> (4 * (j & 1))) & 0x03030303u) << 4;
      hi |= ((H >> (4 * (j & 1) + 2)) & 0x03030303u) << 4;
    }
    const long A = (long)(((unsigned long)hi << 32) | lo);
    const bool on = jsel == j;
    const long B = (long)(((unsigned long)(on ? x.X[1] : 0u) << 32) | (on ? x.X[0] : 0u));
    if (j & 1) C1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A, B, C1, 0, 0, 0);
    else C0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A, B, C0, 0, 0, 0);
  }
  const uint32_t s = f.sc[0][0][0];
  int t[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int P = C0[i] + C1[i];
    if constexpr (T == 14) t[i] = __mul24((int)(int8_t)(s >> (8 * i)), P - 32 * x.bs);  // |P - 32 bs| < 2^18
    else t[i] = __mul24((int)((s >> (8 * i)) & 0xFFu), c < 8 ? P : x.bs);                // < 2^17
  }
  if constexpr (T == 14) row16_isum4(t);
  else row8_isum4(t);
  // ggml: (f16(d) * d_x) * S, and for the mins (f16(dmin) * d_x) * Mn subtracted: lanes 8-15 carry
  // dmin and -d_x, so lane 15 accumulates -(dmin * d_x) * Mn exactly
  const f16x4 dd = __builtin_bit_cast(f16x4, u32x2{f.dm[0][0], f.dm[0][1]});
  const float dxs = (T != 14 && c >= 8) ? -x.dx : x.dx;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] += ((float)dd[i] * dxs) * (float)t[i];
}

// kq_compute_bd with the block-diagonal B operands read from LDS (Bs[j][lane], mkq_bd_tile_kernel)
template <int T>
__device__ __forceinline__ void kq_compute_bd_lds(f32x4& acc, const KqFrag<1, 1>& f, const u32x2 (*Bs)[64], int bs,
                                                  float dx, int lane) {
  const int c = lane & 15;
  uint32_t D[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    D[k] = f.qs[0][0][k];
    D[4 + k] = f.qs[0][1][k];
  }
  i32x4 C0 = i32x4{0, 0, 0, 0}, C1 = i32x4{0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t lo = D[j] & 0x0F0F0F0Fu, hi = (D[j] >> 4) & 0x0F0F0F0Fu;
    if constexpr (T == 13) {
      const uint32_t H = f.h[0][j >> 2];
      lo |= ((H >> ((2 * j) & 7)) & 0x01010101u) << 4;
      hi |= ((H >> ((2 * j + 1) & 7)) & 0x01010101u) << 4;
    }
    if constexpr (T == 14) {
      const uint32_t H = f.h[0][j >> 1];
      lo |= ((H >> (4 * (j & 1))) & 0x03030303u) << 4;
      hi |= ((H >> (4 * (j & 1) + 2)) & 0x03030303u) << 4;
    }
    const long A = (long)(((unsigned long)hi << 32) | lo);
    const u32x2 bv = Bs[j][lane];
    const long B = (long)(((unsigned long)bv[1] << 32) | bv[0]);
    if (j & 1) C1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A, B, C1, 0, 0, 0);
    else C0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(A, B, C0, 0, 0, 0);
  }
  const uint32_t s = f.sc[0][0][0];
  int t[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int P = C0[i] + C1[i];
    if constexpr (T == 14) t[i] = __mul24((int)(int8_t)(s >> (8 * i)), P - 32 * bs);
    else t[i] = __mul24((int)((s >> (8 * i)) & 0xFFu), c < 8 ? P : bs);
  }
  if constexpr (T == 14) row16_isum4(t);
  else row8_isum4(t);
  const f16x4 dd = __builtin_bit_cast(f16x4, u32x2{f.dm[0][0], f.dm[0][1]});
  const float dxs = (T != 14 && c >= 8) ? -dx : dx;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] += ((float)dd[i] * dxs) * (float)t[i];
}

// end of a tile: Q4_K / Q5_K hold d-terms in lane 7 and mins terms in lane 15 of each row; their
// sum goes to lane 0 (Q6_K: every lane already holds the row's total)
template <int T>
__device__ __forceinline__ void kq_bd_finish(f32x4& acc) {
  if constexpr (T != 14) {
    float v0 = acc[0], v1 = acc[1], v2 = acc[2], v3 = acc[3];
    asm volatile("s_nop 1\n\t" KQ_ROR_ADD4("v_add_f32", 8)
                 "s_nop 1\n\t"
                 "v_mov_b32_dpp %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b32_dpp %1, %1 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b32_dpp %2, %2 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b32_dpp %3, %3 row_ror:1 row_mask:0xf bank_mask:0xf"
                 : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
    acc = f32x4{v0, v1, v2, v3};
  }
}
#undef KQ_ROR_ADD4

template <int T, int KS, int RT, int NB, int EPI, int U, bool QL, bool BD>
__device__ __forceinline__ void mkq_body(const MMArgs& a, const uint8_t* W, int tile_in_seg, int tile0,
                                         f32x4 (*red)[RT][NB][64]) {
  static_assert(!BD || (RT == 1 && NB == 1), "block-diagonal form: one token, one tile");
  constexpr int TB = KqTile<T>::BYTES;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int SB = a.K / 256;
  const int kb = (SB * w) / KS, ke = (SB * (w + 1)) / KS;
  const int cb = blockIdx.y * 16 * NB;

  const uint8_t* Wr[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) Wr[r] = W + (size_t)(tile_in_seg + r) * SB * TB;
  const int8_t* Xq[NB];
  const float* Xd[NB];
  const float* Xb[NB];
  extern __shared__ __attribute__((aligned(16))) uint8_t kq_ql_dyn[];  // QL: per-wave Q8_K images
  int8_t* iq = reinterpret_cast<int8_t*>(kq_ql_dyn + w * QL_WAVE_BYTES);
  float* id = reinterpret_cast<float*>(iq + QL_SB_MAX * 256);
  float* ib = id + QL_SB_MAX;
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    int col = cb + n * 16 + (lane & 15);
    col = col < a.M ? col : a.M - 1;  // padded columns re-read a valid row (outputs dropped)
    if constexpr (QL) {  // one token: the image holds super-blocks kb .. ke-1
      Xq[n] = iq + 64 * g - kb * 256;
      Xd[n] = id - kb;
      Xb[n] = ib + 2 * g - kb * 8;
    } else {
      Xq[n] = a.xq + (size_t)col * a.K + 64 * g;
      Xd[n] = a.xd + (size_t)col * SB;
      Xb[n] = a.xb + (size_t)col * (a.K / 32) + 2 * g;
    }
  }

  f32x4 acc[RT][NB];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  using Frag = KqFrag<RT, NB>;
  auto load = [&](Frag& f, int sb) {
    const uint8_t* Wt[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) Wt[r] = Wr[r] + (size_t)sb * TB;
    kq_load<T, RT, NB>(f, Wt, Xq, Xd, Xb, sb, lane, g);
  };
  auto compute = [&](const Frag& f) { kq_compute<T, RT, NB>(acc, f, g); };

  int sb = kb;
  const int nfull = (ke - kb) / U;
  QlRegs qr;
  if constexpr (BD) {  // one token (kq_compute_bd): weights and activation operands ring together
    const int8_t* bq = QL ? iq - kb * 256 : a.xq;
    const float* bd = QL ? id - kb : a.xd;
    const float* bb = QL ? ib - kb * 8 : a.xb;
    Frag ring[U];
    KqBdX xr[U];
    if (U >= (a.K / 256 + KS - 1) / KS) {  // (uniform) the whole slice in flight: U loads, no ring turns
      const int n = ke - kb;
      auto sbi = [&](int u) { return max(min(kb + u, ke - 1), 0); };  // clamped: loads past the slice are unused
      if constexpr (QL) ql_load(qr, a, kb, n, lane);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kq_load_w_bd<T>(ring[u], Wr[0] + (size_t)sbi(u) * TB, lane);
        if constexpr (!QL) xr[u] = kq_bd_x<T>(bq, bd, bb, sbi(u), lane);
      }
      if constexpr (QL) {
        ql_build(qr, a, n, lane, iq, id, ib);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is in LDS
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) xr[u] = kq_bd_x<T>(bq, bd, bb, n > 0 ? sbi(u) : kb, lane);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < n) kq_compute_bd<T>(acc[0][0], ring[u], xr[u], lane);
      kq_bd_finish<T>(acc[0][0]);
    } else {
    if constexpr (QL) ql_load(qr, a, kb, ke - kb, lane);
    if (nfull > 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kq_load_w_bd<T>(ring[u], Wr[0] + (size_t)(sb + u) * TB, lane);
        if constexpr (!QL) xr[u] = kq_bd_x<T>(bq, bd, bb, sb + u, lane);
      }
    }
    if constexpr (QL) {
      ql_build(qr, a, ke - kb, lane, iq, id, ib);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is in LDS
      __builtin_amdgcn_wave_barrier();
      if (nfull > 0)
#pragma unroll
        for (int u = 0; u < U; ++u) xr[u] = kq_bd_x<T>(bq, bd, bb, sb + u, lane);
    }
    if (nfull > 0) {
      for (int ch = 1; ch < nfull; ++ch) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          kq_compute_bd<T>(acc[0][0], ring[u], xr[u], lane);
          kq_load_w_bd<T>(ring[u], Wr[0] + (size_t)(sb + U + u) * TB, lane);
          xr[u] = kq_bd_x<T>(bq, bd, bb, sb + U + u, lane);
        }
        sb += U;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) kq_compute_bd<T>(acc[0][0], ring[u], xr[u], lane);
      sb += U;
    }
    for (; sb < ke; ++sb) {
      Frag f;
      kq_load_w_bd<T>(f, Wr[0] + (size_t)sb * TB, lane);
      const KqBdX x = kq_bd_x<T>(bq, bd, bb, sb, lane);
      kq_compute_bd<T>(acc[0][0], f, x, lane);
    }
    kq_bd_finish<T>(acc[0][0]);
    }
  } else {
  Frag ring[U];
  if constexpr (QL) ql_load(qr, a, kb, ke - kb, lane);
  if (nfull > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (QL) {
        const uint8_t* Wt[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) Wt[r] = Wr[r] + (size_t)(sb + u) * TB;
        kq_load_w<T, RT, NB>(ring[u], Wt, lane, g);
      } else {
        load(ring[u], sb + u);
      }
    }
  }
  if constexpr (QL) {
    ql_build(qr, a, ke - kb, lane, iq, id, ib);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is in LDS
    __builtin_amdgcn_wave_barrier();
    if (nfull > 0)
#pragma unroll
      for (int u = 0; u < U; ++u) kq_load_x<T, RT, NB>(ring[u], Xq, Xd, Xb, sb + u);
  }
  if (nfull > 0) {
    for (int ch = 1; ch < nfull; ++ch) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        compute(ring[u]);
        load(ring[u], sb + U + u);
      }
      sb += U;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) compute(ring[u]);
    sb += U;
  }
  for (; sb < ke; ++sb) {
    Frag f;
    load(f, sb);
    compute(f);
  }
  }

#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) red[w][r][n][lane] = acc[r][n];
  __syncthreads();

  constexpr int LU = (EPI == EPI_SWIGLU) ? 32 : 64;
  constexpr int UNITS = RT * NB * LU;
  for (int u = threadIdx.x; u < UNITS; u += 64 * KS) {
    const int l = u % LU;
    const int n = (u / LU) % NB;
    const int r = (u / LU) / NB;
    const int col = cb + n * 16 + (l & 15);
    if (col >= a.M) continue;
    f32x4 s = red[0][r][n][l];
#pragma unroll
    for (int ww = 1; ww < KS; ++ww) s += red[ww][r][n][l];
    if constexpr (EPI == EPI_RESID) {
      // residual add, and this tile's share of the next RMS_NORM's sum of squares (quantise-on-load
      // consumers): lanes l, l^16, l^32, l^48 hold the tile's 16 rows of col (kernels.hip mm_body)
      f32x4* px = reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + (tile0 + r) * 16 + (l >> 4) * 4);
      const f32x4 xv = *px + s;
      *px = xv;
      if (a.ssq) {
        double q = ssq4(xv);
        q += __shfl_xor(q, 16);
        q += __shfl_xor(q, 32);
        if (l < 16) a.ssq[(size_t)col * a.np + tile0 + r] = (float)q;
      }
      continue;
    }
    f32x4 up = s;
    if constexpr (EPI == EPI_SWIGLU) {
      up = red[0][r][n][l + 32];
#pragma unroll
      for (int ww = 1; ww < KS; ++ww) up += red[ww][r][n][l + 32];
    }
    epi_store<EPI>(a, tile0 + r, l, col, s, up);
  }
}

template <int KS, int RT, int NB, int EPI, int U, bool QL, bool BD = false>
__global__ __launch_bounds__(64 * KS) void mkq_kernel(MMArgs a) {
  __shared__ f32x4 red[KS][RT][NB][64];
  const int tile0 = blockIdx.x * RT;
  int seg = 0;
  while (seg < a.kq_n - 1 && tile0 >= a.kq_tile_end[seg]) ++seg;
  const int t_begin = seg ? a.kq_tile_end[seg - 1] : 0;
  const uint8_t* W = reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[seg];
  switch (a.kq_type[seg]) {
    case 12: mkq_body<12, KS, RT, NB, EPI, U, QL, BD>(a, W, tile0 - t_begin, tile0, red); break;
    case 13: mkq_body<13, KS, RT, NB, EPI, U, QL, BD>(a, W, tile0 - t_begin, tile0, red); break;
    case 14: mkq_body<14, KS, RT, NB, EPI, U, QL, BD>(a, W, tile0 - t_begin, tile0, red); break;
  }
}

// Tile-persistent form for <= 16 tokens and a single-type matrix (gate/up, attn_output, ffn_down,
// lm_head of a K-quant file): mkq_kernel gives each work-group one 16-row tile, so gate/up (1792
// tiles) runs 7 rounds of short work-groups, each paying the first-load latency; here G work-groups
// walk tiles blockIdx.x, +G, ... with every wave's super-block ring running across the tile seams
// (kernels.hip mm_pers_kernel's scheme: partials meet in a double-buffered LDS array behind a raw
// barrier that waits for the LDS writes only; wave 0 finishes tile i while the others stream tile
// i+1).  Same K split (KS waves) and summation order per tile as mkq_kernel (hipcc's fma contraction
// of the scale arithmetic may still differ by an ulp).
// CONTIG: the work-group's tiles are blockIdx.x*TPW + i (one segment of the matrix, starting at
// tile tseg0, whose packed tiles start at Wseg) instead of blockIdx.x + i*G
// BD: one token in the block-diagonal form (kq_compute_bd; NB = 1, M = 1): the ring holds weights
// only, the wave's NKW super-blocks of activation operands stay in registers for all its tiles
template <int T, int KS, int NKW, int TPW, int NB, int EPI, int U, bool QL, bool CONTIG = false, bool BD = false>
__device__ __forceinline__ void mkq_pers_body(const MMArgs& a, const uint8_t* Wseg, int tseg0) {
  static_assert(!BD || NB == 1, "block-diagonal form: one token");
  constexpr int TB = KqTile<T>::BYTES;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = lane >> 4;
  const int SB = KS * NKW;
  const int kb = w * NKW;
  const int G = gridDim.x;
  const int ntiles = a.N / TILE_N;
  __shared__ f32x4 red[2][KS][NB][64];
  auto tile_of = [&](int i) { return CONTIG ? (int)blockIdx.x * TPW + i : (int)blockIdx.x + i * G; };

  const uint8_t* W = Wseg;
  const int8_t* Xq[NB];
  const float* Xd[NB];
  const float* Xb[NB];
  int colr[NB];
  extern __shared__ __attribute__((aligned(16))) uint8_t kq_ql_dyn[];  // QL: per-wave Q8_K images
  int8_t* iq = reinterpret_cast<int8_t*>(kq_ql_dyn + w * QL_WAVE_BYTES);
  float* id = reinterpret_cast<float*>(iq + QL_SB_MAX * 256);
  float* ib = id + QL_SB_MAX;
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    colr[n] = n * 16 + (lane & 15);
    const int col = colr[n] < a.M ? colr[n] : a.M - 1;
    if constexpr (QL) {
      Xq[n] = iq + 64 * g - kb * 256;
      Xd[n] = id - kb;
      Xb[n] = ib + 2 * g - kb * 8;
    } else {
      Xq[n] = a.xq + (size_t)col * a.K + 64 * g;
      Xd[n] = a.xd + (size_t)col * SB;
      Xb[n] = a.xb + (size_t)col * (a.K / 32) + 2 * g;
    }
  }
  using Frag = KqFrag<1, NB>;
  // flat ring position f = tile i of this work-group, super-block kb + k (phantom tiles past the
  // end re-read the last tile; their outputs are dropped)
  auto load_w = [&](Frag& fr, int f) {
    const int i = f / NKW, k = f % NKW;
    const int tile = min(tile_of(i), ntiles - 1) - tseg0;
    const uint8_t* Wt[1] = {W + ((size_t)tile * SB + kb + k) * TB};
    if constexpr (BD) kq_load_w_bd<T>(fr, Wt[0], lane);
    else kq_load_w<T, 1, NB>(fr, Wt, lane, g);
  };
  auto load = [&](Frag& fr, int f) {
    load_w(fr, f);
    if constexpr (!BD) kq_load_x<T, 1, NB>(fr, Xq, Xd, Xb, kb + f % NKW);
  };
  // BD activation operands: the Q8_K row (QL: the wave image) indexed by absolute super-block
  KqBdX bx[BD ? NKW : 1];
  auto load_bx = [&]() {
    if constexpr (BD) {
      const int8_t* bq = QL ? iq - kb * 256 : a.xq;
      const float* bd = QL ? id - kb : a.xd;
      const float* bb = QL ? ib - kb * 8 : a.xb;
#pragma unroll
      for (int k = 0; k < NKW; ++k) bx[k] = kq_bd_x<T>(bq, bd, bb, kb + k, lane);
    }
  };
  constexpr int LU = (EPI == EPI_SWIGLU) ? 32 : 64;
  // one token's q|k|v: pos / slot once, each tile's RoPE pairs when the tile starts (mm_pers_kernel's
  // prefetch: in the epilogue they were a chain of dependent round trips)
  int qpos = 0, qslot = 0;
  f32x4 qcs[TPW];
  if constexpr (EPI == EPI_QKV && NB == 1) {
    const int c0 = colr[0] < a.M ? colr[0] : a.M - 1;
    qpos = a.pos[c0], qslot = a.slot[c0];
  }
  auto finish = [&](int i) {
    const int tile = tile_of(i);
    if (w != 0 || tile >= ntiles) return;
    f32x4 (*rb)[NB][64] = red[i & 1];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      if (lane >= LU || colr[n] >= a.M) continue;
      f32x4 s = rb[0][n][lane];
      f32x4 up = (EPI == EPI_SWIGLU) ? rb[0][n][lane + 32] : s;
#pragma unroll 3
      for (int ww = 1; ww < KS; ++ww) {
        s += rb[ww][n][lane];
        if constexpr (EPI == EPI_SWIGLU) up += rb[ww][n][lane + 32];
      }
      if constexpr (EPI == EPI_QKV && NB == 1) qkv_store_pre(a, tile * 16 + (lane >> 4) * 4, colr[0], s, qpos, qslot, qcs[i]);
      else epi_store<EPI>(a, tile, lane, colr[n], s, up);
    }
  };

  Frag ring[U];
  QlRegs qr;
  if constexpr (QL) ql_load(qr, a, kb, NKW, lane);  // once per work-group: the slice is the same for every tile
  if constexpr (BD && !QL) load_bx();
#pragma unroll
  for (int f = 0; f < U; ++f) {
    if constexpr (QL) load_w(ring[f], f);
    else load(ring[f], f);
  }
  if constexpr (QL) {
    ql_build(qr, a, NKW, lane, iq, id, ib);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image is in LDS
    __builtin_amdgcn_wave_barrier();
    if constexpr (BD) load_bx();
    else
#pragma unroll
      for (int f = 0; f < U; ++f) kq_load_x<T, 1, NB>(ring[f], Xq, Xd, Xb, kb + f % NKW);
  }
  // fully unrolled over the TPW tiles (a loop back-edge renames the ring with moves that wait for
  // the loads, draining it)
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    f32x4 acc[1][NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_QKV && NB == 1) qcs[i] = qkv_cs(a, min(tile_of(i), ntiles - 1) * 16 + (lane >> 4) * 4, qpos);
#pragma unroll
    for (int k = 0; k < NKW; ++k) {
      const int f = i * NKW + k;
      if constexpr (BD) kq_compute_bd<T>(acc[0][0], ring[f % U], bx[k], lane);
      else kq_compute<T, 1, NB>(acc, ring[f % U], g);
      if (f + U < TPW * NKW) load(ring[f % U], f + U);
      // issue the refill here: left to itself the scheduler sinks a tile's refills below its last
      // compute, which then waits for vmcnt(0) (the ring empty once per tile)
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (BD) kq_bd_finish<T>(acc[0][0]);
#pragma unroll
    for (int n = 0; n < NB; ++n) red[i & 1][w][n][lane] = acc[0][n];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only: the ring stays in flight
    __builtin_amdgcn_s_barrier();
    finish(i);
    __builtin_amdgcn_sched_barrier(0);  // no hoisting across tiles (it spilled the ring)
  }
}

template <int T, int KS, int NKW, int TPW, int NB, int EPI, int U, bool QL, bool BD>
__global__ __launch_bounds__(64 * KS) void mkq_pers_kernel(MMArgs a) {
  mkq_pers_body<T, KS, NKW, TPW, NB, EPI, U, QL, false, BD>(a, reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[0], 0);
}

// One token of a matrix with row segments of different types (q|k Q4_K + v Q6_K): TPW contiguous
// tiles per work-group, every segment boundary a multiple of TPW, the body chosen per work-group
template <int KS, int NKW, int TPW, int EPI, int U>
__global__ __launch_bounds__(64 * KS) void mkq_pers_seg_kernel(MMArgs a) {
  const int t0 = blockIdx.x * TPW;
  int seg = 0;
  while (seg < a.kq_n - 1 && t0 >= a.kq_tile_end[seg]) ++seg;
  const int tb = seg ? a.kq_tile_end[seg - 1] : 0;
  const uint8_t* Ws = reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[seg];
  switch (a.kq_type[seg]) {
    case 12: mkq_pers_body<12, KS, NKW, TPW, 1, EPI, U, true, true, true>(a, Ws, tb); break;
    case 13: mkq_pers_body<13, KS, NKW, TPW, 1, EPI, U, true, true, true>(a, Ws, tb); break;
    case 14: mkq_pers_body<14, KS, NKW, TPW, 1, EPI, U, true, true, true>(a, Ws, tb); break;
  }
}

// One token, every wave owning whole tiles (the whole K): the tile-persistent kernels above split
// each tile's K over 8 waves, so every tile ends in an LDS reduction behind a work-group barrier,
// where the slowest wave and wave 0's epilogue hold up the rest.  Here wave w of work-group b walks
// tiles (b * W + w) + i * gridDim.x * W, i < TPW, its U-deep weight ring running across them, and
// finishes each tile from registers.  The token's activation operands are built once per
// work-group in LDS, already in block-diagonal form: the Q8_K row (RMS_NORM + quantise on load by
// the first SB/8 waves, ql_build), then per super-block s and sub-block j the B operand of every
// lane (its 8 q or zeros) and per lane its bsum -- so a super-block's B operands are 8 conflict-free
// ds_read_b64 and no VALU.  Two barriers per launch.  K = 256 * SB, SB 8 or 16.
template <int SB>
struct KqBdImg {
  int8_t q[SB * 256];  // Q8_K row (permuted), d, sub-block sums: ql_build's image
  float d[SB];
  float b[SB * 8];
  u32x2 B[SB][8][64];  // block-diagonal B operand of lane l for (super-block, sub-block)
  int bs[SB][64];      // kq_bd_x's bs of lane l
};

template <int T, int W, int SB, int TPW, int EPI, int U>
__global__ __launch_bounds__(64 * W) void mkq_bd_tile_kernel(MMArgs a) {
  static_assert(SB % 8 == 0 && SB / 8 <= W, "the first SB/8 waves quantise 8 super-blocks each");
  constexpr int TB = KqTile<T>::BYTES;
  constexpr int NF = TPW * SB;  // flat ring positions (tile i, super-block k)
  __shared__ KqBdImg<SB> im;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ntiles = a.N / TILE_N;
  const int G = gridDim.x * W;
  const uint8_t* W0 = reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[0];
  auto tile_of = [&](int i) { return (int)blockIdx.x * W + w + i * G; };
  using Frag = KqFrag<1, 1>;
  Frag ring[U];
  auto load_w = [&](Frag& f, int fl) {
    const int tile = min(tile_of(fl / SB), ntiles - 1);  // phantom tiles re-read the last (dropped)
    kq_load_w_bd<T>(f, W0 + ((size_t)tile * SB + fl % SB) * TB, lane);
  };

  // prologue: the quantising waves load their norm operands first, every wave issues its ring
  QlRegs qr;
  const bool quant = w < SB / 8;
  if (quant) ql_load(qr, a, 8 * w, 8, lane);
#pragma unroll
  for (int f = 0; f < U; ++f) load_w(ring[f], f);
  if (quant) ql_build(qr, a, 8, lane, im.q + 8 * w * 256, im.d + 8 * w, im.b + 8 * w * 8);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the image is written (the weight ring stays in flight)
  __builtin_amdgcn_s_barrier();
  // block-diagonal operands: thread t handles (super-block, lane) pairs t, t + 64W, ...
  for (int u = threadIdx.x; u < SB * 64; u += 64 * W) {
    const int sb = u >> 6, l = u & 63;
    const KqBdX x = kq_bd_x_lane<T>(im.q, im.d, im.b, sb, l);
    const int jsel = T == 14 ? ((l & 15) >> 1) : (l & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) im.B[sb][j][l] = jsel == j ? x.X : u32x2{0u, 0u};
    im.bs[sb][l] = x.bs;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();

  // tiles in a run-time loop, super-blocks unrolled: U divides SB, so every tile uses the ring
  // slots in the same order and the loop carries the ring without renaming it
  static_assert(SB % U == 0, "ring slots line up across tiles");
  for (int i = 0; i < TPW; ++i) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < SB; ++k) {
      kq_compute_bd_lds<T>(acc, ring[k % U], im.B[k], im.bs[k][lane], im.d[k], lane);
      const int fl = i * SB + k + U;
      if (fl < NF) load_w(ring[k % U], fl);
      __builtin_amdgcn_sched_barrier(0);  // the refill issues here, not sunk below the next compute
    }
    kq_bd_finish<T>(acc);
    const int tile = tile_of(i);
    f32x4 up = acc;
    if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) up[r] = __shfl_xor(acc[r], 32);
    }
    if (tile < ntiles && (lane & 15) == 0 && (EPI != EPI_SWIGLU || lane < 32)) epi_store<EPI>(a, tile, lane, 0, acc, up);
  }
}

// one token, q|k|v of a K-quant file (K 4096: 16 super-blocks = 8 waves x 2): 2 tiles per
// work-group (Llama-3-8B: 192 groups) quantising on load; -1 if the shape has no such form
static int launch_kq_qkv_pers(const MMArgs& a, hipStream_t s) {
  constexpr bool off = false;
  if (off || a.M != 1 || a.xq != nullptr || a.K != 4096 || (a.N / TILE_N) % 2) return -1;
  for (int i = 0; i < a.kq_n; ++i)
    if (a.kq_tile_end[i] % 2) return -1;
  mkq_pers_seg_kernel<8, 2, 2, EPI_QKV, 4><<<a.N / TILE_N / 2, 512, 8 * QL_WAVE_BYTES, s>>>(a);
  return 0;
}

// U: ring depth for 2..16 tokens; UB: one token (block-diagonal, weights only in the ring)
// (one token: KSB waves per work-group, each NKW * 8 / KSB super-blocks of every tile)
template <int T, int NKW, int TPW, int NB, int EPI, int U, int UB, int KSB = 8>
static void launch_kq_pers_t(const MMArgs& a, int ntiles, hipStream_t s) {
  const int grid = (ntiles + TPW - 1) / TPW;
  constexpr int NKB = NKW * 8 / KSB;
  if (a.xq == nullptr)  // one token, quantised on load
    mkq_pers_kernel<T, KSB, NKB, TPW, NB, EPI, UB, true, true><<<grid, 64 * KSB, KSB * QL_WAVE_BYTES, s>>>(a);
  else if (a.M == 1)
    mkq_pers_kernel<T, KSB, NKB, TPW, NB, EPI, UB, false, true><<<grid, 64 * KSB, 0, s>>>(a);
  else
    mkq_pers_kernel<T, 8, NKW, TPW, NB, EPI, U, false, false><<<grid, 512, 0, s>>>(a);
}

// single-type matrices of the Llama shapes: gate/up (K 4096, 1792 tiles / TinyLlama K 2048, 704),
// attn_output / ffn_down (h 4096: 256 tiles, one per work-group: the KS split is mkq_kernel's), the
// lm_head (128256 / 32000 rows); -1 = no instantiation (mkq_kernel runs)
template <int T, int NB, int EPI>
static int launch_kq_pers_ty(const MMArgs& a, int ntiles, hipStream_t s) {
  const int SB = a.K / 256;
  if constexpr (EPI == EPI_SWIGLU) {
    if (SB == 16 && ntiles == 1792) return launch_kq_pers_t<T, 2, 7, NB, EPI, 2, 4>(a, ntiles, s), 0;
    if (SB == 8 && ntiles == 704) return launch_kq_pers_t<T, 1, 3, NB, EPI, 2, 3>(a, ntiles, s), 0;
  } else {
    if (SB == 16 && ntiles > 256 * 8) return launch_kq_pers_t<T, 2, 8, NB, EPI, 2, 4>(a, ntiles, s), 0;  // 16: spills
    if (SB == 8 && ntiles > 256 * 4) return launch_kq_pers_t<T, 1, 8, NB, EPI, 2, 4>(a, ntiles, s), 0;
  }
  return -1;
}

// one token quantised on load, single-type gate/up or lm_head: mkq_bd_tile_kernel when the shape has
// an instantiation (K 4096 / 2048: Llama-3-8B, TinyLlama; K 8192 spills), else -1
template <int T, int EPI>
static int launch_kq_bd_tile_t(const MMArgs& a, int ntiles, hipStream_t s) {
  const int SB = a.K / 256;
  auto go = [&](auto wc, auto sbc, auto tc) {
    constexpr int W = decltype(wc)::value, S = decltype(sbc)::value, TP = decltype(tc)::value;
    const int grid = (ntiles + W * TP - 1) / (W * TP);
    mkq_bd_tile_kernel<T, W, S, TP, EPI, 8><<<grid, 64 * W, 0, s>>>(a);
    return 0;
  };
  using std::integral_constant;
  if constexpr (EPI == EPI_SWIGLU) {
    if (SB == 16 && ntiles <= 1792) return go(integral_constant<int, 7>{}, integral_constant<int, 16>{}, integral_constant<int, 1>{});
    if (SB == 8 && ntiles <= 768) return go(integral_constant<int, 3>{}, integral_constant<int, 8>{}, integral_constant<int, 1>{});
  } else {
    if (SB == 16 && ntiles <= 8192) return go(integral_constant<int, 8>{}, integral_constant<int, 16>{}, integral_constant<int, 4>{});
    if (SB == 8 && ntiles <= 2048) return go(integral_constant<int, 8>{}, integral_constant<int, 8>{}, integral_constant<int, 1>{});
  }
  return -1;
}
static int launch_kq_bd_tile(int epi, const MMArgs& a, int ntiles, hipStream_t s) {
  static const bool off = getenv("MX_NO_KQ_BD_TILE") != nullptr;  // tests: the K-split persistent kernel's path
  if (off || a.M != 1 || a.xq != nullptr || a.kq_n != 1 || !a.xf || (a.norm_w && (!a.ssq || a.np * 16 != a.K)))
    return -1;
  const int t = a.kq_type[0];
  if (epi == EPI_SWIGLU)
    return t == 12 ? launch_kq_bd_tile_t<12, EPI_SWIGLU>(a, ntiles, s)
         : t == 13 ? launch_kq_bd_tile_t<13, EPI_SWIGLU>(a, ntiles, s)
                   : launch_kq_bd_tile_t<14, EPI_SWIGLU>(a, ntiles, s);
  if (epi == EPI_F32)
    return t == 12 ? launch_kq_bd_tile_t<12, EPI_F32>(a, ntiles, s)
         : t == 13 ? launch_kq_bd_tile_t<13, EPI_F32>(a, ntiles, s)
                   : launch_kq_bd_tile_t<14, EPI_F32>(a, ntiles, s);
  return -1;
}

static int launch_kq_pers(int epi, const MMArgs& a, int ntiles, hipStream_t s) {
  // MX_NO_KQ_PERS: the one-tile-per-work-group kernel (read per launch: tests compare the two)
  static const bool off = getenv("MX_NO_KQ_PERS") != nullptr;  // tests: the grouped kernel's path
  if (off || a.kq_n != 1 || a.M > 16) return -1;  // 17-32 rows (two column tiles): spills
  if (launch_kq_bd_tile(epi, a, ntiles, s) == 0) return 0;
  const int t = a.kq_type[0];
  auto by_nb = [&](auto nb) -> int {
    constexpr int NB = decltype(nb)::value;
    switch (epi) {
      case EPI_SWIGLU:
        return t == 12 ? launch_kq_pers_ty<12, NB, EPI_SWIGLU>(a, ntiles, s)
             : t == 13 ? launch_kq_pers_ty<13, NB, EPI_SWIGLU>(a, ntiles, s)
                       : launch_kq_pers_ty<14, NB, EPI_SWIGLU>(a, ntiles, s);
      case EPI_F32:
        return t == 12 ? launch_kq_pers_ty<12, NB, EPI_F32>(a, ntiles, s)
             : t == 13 ? launch_kq_pers_ty<13, NB, EPI_F32>(a, ntiles, s)
                       : launch_kq_pers_ty<14, NB, EPI_F32>(a, ntiles, s);
    }
    return -1;
  };
  return by_nb(std::integral_constant<int, 1>{});
}

// one token, one tile per work-group: 8 waves split K, each with its whole slice of super-blocks in
// flight (U >= slice: 1, 2, 4, 7, 8); longer slices ring 2 deep
template <int EPI, bool QL>
static void launch_mkq_bd(const MMArgs& a, int ntiles, hipStream_t s) {
  const int per = (a.K / 256 + 7) / 8;
  const dim3 grid(ntiles, 1);
  const size_t lds = QL ? 8 * QL_WAVE_BYTES : 0;
  if (per <= 1) mkq_kernel<8, 1, 1, EPI, 1, QL, true><<<grid, 512, lds, s>>>(a);
  else if (per <= 2) mkq_kernel<8, 1, 1, EPI, 2, QL, true><<<grid, 512, lds, s>>>(a);
  else if (per <= 4) mkq_kernel<8, 1, 1, EPI, 4, QL, true><<<grid, 512, lds, s>>>(a);
  else if (QL && per <= 7) mkq_kernel<8, 1, 1, EPI, QL ? 7 : 2, QL, true><<<grid, 512, lds, s>>>(a);
  else if (QL && per <= 8) mkq_kernel<8, 1, 1, EPI, QL ? 8 : 2, QL, true><<<grid, 512, lds, s>>>(a);
  else mkq_kernel<8, 1, 1, EPI, 2, QL, true><<<grid, 512, lds, s>>>(a);  // (quantise-on-load slices are <= 8)
}

template <int EPI>
static void launch_mkq_epi(const MMArgs& a, int ntiles, hipStream_t s) {
  if (a.xq == nullptr) {  // one token, quantised on load (launch_mkq checked the slice fits)
    launch_mkq_bd<EPI, true>(a, ntiles, s);
  } else if (a.M == 1) {
    launch_mkq_bd<EPI, false>(a, ntiles, s);
  } else if (a.M <= 16) {
    mkq_kernel<8, 1, 1, EPI, 2, false><<<dim3(ntiles, 1), 512, 0, s>>>(a);
  } else if (a.M <= 32) {  // (a 2-deep ring spills ~460 B/lane at two column tiles: U = 1)
    mkq_kernel<8, 1, 2, EPI, 1, false><<<dim3(ntiles, 1), 512, 0, s>>>(a);
  } else {
    mkq_kernel<8, 1, 2, EPI, 1, false><<<dim3(ntiles, (a.M + 31) / 32), 512, 0, s>>>(a);
  }
}

// ---------------------------------------------------------------------------
// K-quant GEMV for 17..64 tokens (32-sequence decode) with the Q8_K activations shared through LDS.
//
// mkq_kernel at two column tiles gives every wave its own copy of the activation fragments: per
// super-block 8 KB of Q8_K per wave against 2.4 KB of Q4_K weights, so it streams ~3x more bytes
// from L2 than weights from HBM, and with a one-deep ring it waits on both.  Here (as mm_wide_kernel
// does for bf16) the W waves of a work-group each own one 16-row tile over the whole K and share
// one staged super-block of activations [16*NB tokens][256 q + 8 sub-block sums + d] in LDS
// (double-buffered, one barrier per super-block; the next-but-one super-block's pieces are loaded
// into registers while this one computes), and each wave keeps a U-deep ring of its weight tiles in
// flight.  Per super-block and tile the arithmetic is kq_compute's (ggml's integer super-block sums,
// f32 scaling), and the whole K stays in one wave, so the epilogue runs from registers.
// Single-type matrices (one segment): gate/up and the lm_head of a K-quant file.
// ---------------------------------------------------------------------------
// 17-32 rows, Q4_K: the 6-bit sub-block scales folded into the int8 A operand.  kq_compute scales
// every sub-block's int32 products per output (NB column tiles x 4 values x 8 sub-blocks of VALU
// per super-block: VALU-bound at ~2.9 TB/s).  Here each 6-bit scale is split sc = 8h + l (l, h < 8),
// so q * l and q * h (q < 16) are int8 values <= 105: every lane multiplies its 4-bit row values by
// l and by h (v_pk_mul_lo_u16 on byte pairs: no product reaches a carry), and two accumulators take
// sum_j (q_j * l_j) . x_j and sum_j (q_j * h_j) . x_j over the whole super-block -- on
// v_mfma_i32_16x16x64_i8, two sub-blocks per MFMA (the K order inside one MFMA is the lanes' own, the
// same for A and B).  S = C_l + 8 C_h is ggml's integer sum_j sc_j (q_j . x_j) exactly; the mins and
// the f32 scaling are kq_compute's.
template <int NB>
__device__ __forceinline__ void kq_load_w_fold(KqFrag<1, NB>& f, const uint8_t* t, int lane) {
  constexpr int SC = KqTile<12>::SC;
  const int g = lane >> 4, rq = (lane & 15) >> 2;
  f.qs[0][0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t) + lane);
  f.qs[0][1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t + 1024) + lane);
  // the scales of this lane's A row (lane & 15): byte lane & 3 of dwords 0..7 of its row group
  f.sc[0][0] = *reinterpret_cast<const u32x4*>(t + SC + 64 * rq);
  f.sc[0][1] = *reinterpret_cast<const u32x4*>(t + SC + 64 * rq + 16);
  const uint8_t* mq = t + SC + 64 * rq + 32 + 4 * g;
  f.mw[0] = u32x2{*reinterpret_cast<const uint32_t*>(mq), *reinterpret_cast<const uint32_t*>(mq + 16)};
  f.dm[0] = *reinterpret_cast<const u32x4*>(t + SC + 256 + 16 * g);
}

template <int NB>
__device__ __forceinline__ void kq_compute_fold(f32x4 (&acc)[1][NB], const KqFrag<1, NB>& f, int lane) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const int g = lane >> 4;
  const uint32_t sel = 0x0C000C00u | (uint32_t)(lane & 3) * 0x00010001u;  // byte lane&3 -> bytes 0 and 2
  i32x4 Cl[NB], Ch[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) Cl[n] = Ch[n] = i32x4{0, 0, 0, 0};
#pragma unroll
  for (int m = 0; m < 4; ++m) {  // sub-blocks 2m, 2m+1
    u32x4 Al, Ah;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int j = 2 * m + hh;
      const uint32_t D = f.qs[0][j >> 2][j & 3];
      const uint32_t lo = D & 0x0F0F0F0Fu, hi = (D >> 4) & 0x0F0F0F0Fu;
      const uint32_t s2 = __builtin_amdgcn_perm(0u, f.sc[0][j >> 2][j & 3], sel);  // (sc, sc) as u16 pair
      const u16x2 l2 = __builtin_bit_cast(u16x2, s2 & 0x00070007u), h2 = __builtin_bit_cast(u16x2, (s2 >> 3) & 0x00070007u);
      Al[2 * hh] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, lo) * l2);
      Al[2 * hh + 1] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, hi) * l2);
      Ah[2 * hh] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, lo) * h2);
      Ah[2 * hh + 1] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, hi) * h2);
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const i32x4 B = __builtin_bit_cast(i32x4, f.x[n][m]);
      Cl[n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, Al), B, Cl[n], 0, 0, 0);
      Ch[n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, Ah), B, Ch[n], 0, 0, 0);
    }
  }
  const int rb = 8 * (lane & 3);
  const float m0 = (float)((f.mw[0][0] >> rb) & 0xFFu), m1 = (float)((f.mw[0][1] >> rb) & 0xFFu);
  const f16x8 dm = __builtin_bit_cast(f16x8, f.dm[0]);
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const float dx = f.dx[n];
    f32x4 Mn = __builtin_amdgcn_mfma_f32_16x16x4f32(m0, f.xb[n][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    Mn = __builtin_amdgcn_mfma_f32_16x16x4f32(m1, f.xb[n][1], Mn, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int S = Cl[n][i] + 8 * Ch[n][i];
      acc[0][n][i] += ((float)dm[i] * dx) * (float)S;
      acc[0][n][i] -= ((float)dm[4 + i] * dx) * Mn[i];
    }
  }
  (void)g;
}

template <int T, int W, int NB, int EPI, int U>
__device__ __forceinline__ void mkq_wide_body(const MMArgs& a, int tile, const uint8_t* Wseg, int tile_in_seg) {
  constexpr int TB = KqTile<T>::BYTES;
  constexpr int ROWS = 16 * NB;
  constexpr int QP = 256 + 16;  // int8 per LDS row: +16 B keeps the 16 token rows' fragment reads conflict-free
  constexpr int NQ = ROWS * 16;  // 16-B pieces of q per super-block
  constexpr int NBS = ROWS * 2;  // 16-B pieces of the sub-block sums (8 floats per token)
  constexpr int PIECES = NQ + NBS;
  constexpr int NT = 64 * W;
  constexpr int PPT = (PIECES + NT - 1) / NT;
  static_assert((U == 2 || U == 4) && ROWS <= NT, "ring depth in activation-set pairs; one d per thread");
  __shared__ __attribute__((aligned(16))) int8_t sq[2][ROWS][QP];
  __shared__ __attribute__((aligned(16))) float ssb[2][ROWS][8];
  __shared__ float sdx[2][ROWS];

  const int lane = threadIdx.x & 63, g = lane >> 4, tid = threadIdx.x;
  const int SB = a.K / 256;
  // grid.y > 1 (EPI_SLAB): this work-group's K range of super-blocks [kb, kb + nsb)
  const int kb = SB * blockIdx.y / gridDim.y, nsb = SB * (blockIdx.y + 1) / gridDim.y - kb;
  const uint8_t* Wr = Wseg + ((size_t)tile_in_seg * SB + kb) * TB;

  // staging: piece p < NQ = 16 B of q (token row p/16, segment p%16), else 16 B of the sums; tokens
  // >= M re-read token M-1 (outputs dropped); the ragged tail re-stages the last piece
  const u32x4* xsrc[PPT];
  int xstep[PPT], xdst[PPT];
  bool xq_piece[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int p = min(tid + i * NT, PIECES - 1);
    if (p < NQ) {
      const int row = p / 16, rr = row < a.M ? row : a.M - 1;
      xsrc[i] = reinterpret_cast<const u32x4*>(a.xq + (size_t)rr * a.K + (size_t)kb * 256 + (p % 16) * 16);
      xstep[i] = 16;  // u32x4 per super-block
      xdst[i] = row * QP + (p % 16) * 16;
      xq_piece[i] = true;
    } else {
      const int q = p - NQ, row = q / 2, rr = row < a.M ? row : a.M - 1;
      xsrc[i] = reinterpret_cast<const u32x4*>(a.xb + (size_t)rr * (a.K / 32) + kb * 8 + (q % 2) * 4);
      xstep[i] = 2;
      xdst[i] = row * 32 + (q % 2) * 16;
      xq_piece[i] = false;
    }
  }
  const int drow = tid < ROWS ? (tid < a.M ? tid : a.M - 1) : 0;
  const float* dsrc = a.xd + (size_t)drow * SB + kb;
  u32x4 xr[2][PPT];
  float xdr[2];
  auto load_x = [&](int set, int sb) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) xr[set][i] = xsrc[i][sb * xstep[i]];
    if (tid < ROWS) xdr[set] = dsrc[sb];
  };
  auto store_x = [&](int set, int buf) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      uint8_t* base = xq_piece[i] ? reinterpret_cast<uint8_t*>(&sq[buf][0][0])
                                  : reinterpret_cast<uint8_t*>(&ssb[buf][0][0]);
      *reinterpret_cast<u32x4*>(base + xdst[i]) = xr[set][i];
    }
    if (tid < ROWS) sdx[buf][tid] = xdr[set];
  };

  using Frag = KqFrag<1, NB>;
  Frag ring[U];
  constexpr bool FOLD = T == 12;  // Q4_K: scales folded into the A operand (kq_compute_fold)
  auto load_w = [&](Frag& f, int sb) {
    const uint8_t* Wt[1] = {Wr + (size_t)sb * TB};
    if constexpr (FOLD) kq_load_w_fold<NB>(f, Wt[0], lane);
    else kq_load_w<T, 1, NB>(f, Wt, lane, g);
  };
  f32x4 acc[1][NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) acc[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // super-block indices below are relative to kb
  load_x(0, 0);
  load_x(1, nsb > 1 ? 1 : 0);
#pragma unroll
  for (int u = 0; u < U; ++u) load_w(ring[u], u < nsb ? u : nsb - 1);
  store_x(0, 0);
  __syncthreads();

  // super-block sb: activation set H = sb & 1 receives sb + 2; set 1 - H (sb + 1) goes to LDS at the end
  auto step = [&](auto Hc, auto Rc, int sb) {
    constexpr int H = decltype(Hc)::value;
    constexpr int R = decltype(Rc)::value;
    const int buf = sb & 1;
    load_x(H, sb + 2 < nsb ? sb + 2 : nsb - 1);
    Frag& f = ring[R];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int row = n * 16 + (lane & 15);
#pragma unroll
      for (int c = 0; c < 4; ++c) f.x[n][c] = *reinterpret_cast<const u32x4*>(&sq[buf][row][64 * g + 16 * c]);
      f.dx[n] = sdx[buf][row];
      if constexpr (T != 14) f.xb[n] = *reinterpret_cast<const f32x2*>(&ssb[buf][row][2 * g]);
    }
    if constexpr (FOLD) kq_compute_fold<NB>(acc, f, lane);
    else kq_compute<T, 1, NB>(acc, f, g);
    load_w(f, min(sb + U, nsb - 1));  // past the end: re-read the last super-block (no branch)
    store_x(1 - H, buf ^ 1);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);  // nothing moves across super-blocks (interleaving them spills)
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // (the ring refill is unconditional -- a refill behind a branch made hipcc drain the ring at the
  // join -- while whole steps sit behind uniform guards, which keeps its register use in bounds)
  for (int sb = 0; sb < nsb; sb += U) {
    step(I0{}, I0{}, sb);
    if (sb + 1 < nsb) step(I1{}, I1{}, sb + 1);
    if constexpr (U == 4) {
      if (sb + 2 < nsb) step(I0{}, I2{}, sb + 2);
      if (sb + 3 < nsb) step(I1{}, I3{}, sb + 3);
    }
  }

  // epilogue from registers: this wave owns its tile over the whole K
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const f32x4 s = acc[0][n];
    f32x4 up = s;
    if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(s[i], 32);
    }
    const int col = n * 16 + (lane & 15);
    if (col >= a.M || (EPI == EPI_SWIGLU && lane >= 32)) continue;
    if constexpr (EPI == EPI_SLAB)  // partial over this K range: slab blockIdx.y [token][N]
      *reinterpret_cast<f32x4*>(a.out + blockIdx.y * a.slab_stride + (size_t)col * a.ldo + tile * 16 + (lane >> 4) * 4) = s;
    else
      epi_store<EPI>(a, tile, lane, col, s, up);
  }
}

template <int T, int W, int NB, int EPI, int U>
__global__ __launch_bounds__(64 * W) void mkq_wide_kernel(MMArgs a) {
  const int tile = blockIdx.x * W + (threadIdx.x >> 6);
  mkq_wide_body<T, W, NB, EPI, U>(a, tile, reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[0], tile);
}

// A matrix of up to 3 row segments of different types (q|k Q4_K + v Q6_K): every segment boundary is
// a multiple of W, so a work-group's W tiles share one type, dispatched at run time (the kernel's
// registers are those of its largest body, Q6_K)
template <int W, int NB, int EPI>
__global__ __launch_bounds__(64 * W) void mkq_wide_seg_kernel(MMArgs a) {
  const int t0 = blockIdx.x * W;
  int seg = 0;
  while (seg < a.kq_n - 1 && t0 >= a.kq_tile_end[seg]) ++seg;
  const int tb = seg ? a.kq_tile_end[seg - 1] : 0;
  const int tile = t0 + (threadIdx.x >> 6);
  const uint8_t* Ws = reinterpret_cast<const uint8_t*>(a.W) + a.kq_off[seg];
  switch (a.kq_type[seg]) {
    case 12: mkq_wide_body<12, W, NB, EPI, 4>(a, tile, Ws, tile - tb); break;
    case 13: mkq_wide_body<13, W, NB, EPI, 4>(a, tile, Ws, tile - tb); break;
    case 14: mkq_wide_body<14, W, NB, EPI, 2>(a, tile, Ws, tile - tb); break;
  }
}

// two column tiles (17..32 tokens); ring 4 deep for Q4_K / Q5_K, 2 for Q6_K (its 4-deep ring spills)
template <int T, int W, int EPI>
static void launch_kq_wide_t(const MMArgs& a, int ntiles, hipStream_t s, int ksplit = 1) {
  mkq_wide_kernel<T, W, 2, EPI, T == 14 ? 2 : 4><<<dim3(ntiles / W, ksplit), 64 * W, 0, s>>>(a);
}

template <int EPI>
static int launch_kq_wide_epi(const MMArgs& a, int ntiles, hipStream_t s) {
  const int t = a.kq_type[0];
  auto by_w = [&](auto wc) {
    constexpr int W = decltype(wc)::value;
    if (t == 12) launch_kq_wide_t<12, W, EPI>(a, ntiles, s);
    else if (t == 13) launch_kq_wide_t<13, W, EPI>(a, ntiles, s);
    else launch_kq_wide_t<14, W, EPI>(a, ntiles, s);
    return 0;
  };
  // waves per work-group sized so the grid covers the 256 CUs (Llama-3-8B gate/up: 1792 = 7 x 256)
  if (ntiles % 7 == 0 && ntiles / 7 >= 200) return by_w(std::integral_constant<int, 7>{});
  if (ntiles % 8 == 0 && ntiles / 8 >= 200) return by_w(std::integral_constant<int, 8>{});
  if (ntiles % 4 == 0) return by_w(std::integral_constant<int, 4>{});
  return -1;
}

// 17..32 tokens, one-type matrix, gate/up or lm_head: the LDS-shared form (MX_NO_KQ_WIDE=1: mkq_kernel)
static int launch_kq_wide(int epi, const MMArgs& a, int ntiles, hipStream_t s) {
  static const bool off = getenv("MX_NO_KQ_WIDE") != nullptr;
  if (off || a.M <= 16 || a.M > 32 || a.kq_n != 1 || !a.xq || !a.xd || !a.xb || (a.K / 256) % 4) return -1;
  if (epi == EPI_SWIGLU) return launch_kq_wide_epi<EPI_SWIGLU>(a, ntiles, s);
  if (epi == EPI_F32) return launch_kq_wide_epi<EPI_F32>(a, ntiles, s);
  return -1;
}

// work-groups the 17..32-row split-K launches aim at (MX_SLAB_TARGET, A/B)
static int kq_slab_target() {
  static const int t = getenv("MX_SLAB_TARGET") ? atoi(getenv("MX_SLAB_TARGET")) : 256;
  return t;
}

// 17..32 tokens, attn_output / ffn_down of a K-quant file (256 tiles for h 4096): 4-wave groups with K
// split over grid.y until ~256 work-groups, partials into slabs [ksplit][token][N] that the next
// RMS_NORM + Q8_K launch (launch_rmsnorm_q8k with slabs) folds into the residual stream in slab
// order.  Returns the split, or -1 (the caller runs mkq_kernel's in-place EPI_RESID instead).
int launch_mkq_slab(const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s) {
  static const bool off = getenv("MX_NO_KQ_WIDE") != nullptr;
  if (off || a.M <= 16 || a.M > 32 || a.kq_n != 1 || !a.xq || !a.xd || !a.xb || a.K % 256 || a.N % 64) return -1;
  const int ntiles = a.N / TILE_N, SB = a.K / 256;
  int ks = 1;
  while (ks < 8 && (ntiles / 4) * ks * 2 <= kq_slab_target() && SB / (ks * 2) >= 4) ks *= 2;
  if (ks < 2) return -1;
  MMArgs p = a;
  p.out = slabs;
  p.ldo = a.N;
  p.slab_stride = slab_stride;
  const int t = a.kq_type[0];
  if (t == 12) launch_kq_wide_t<12, 4, EPI_SLAB>(p, ntiles, s, ks);
  else if (t == 13) launch_kq_wide_t<13, 4, EPI_SLAB>(p, ntiles, s, ks);
  else if (t == 14) launch_kq_wide_t<14, 4, EPI_SLAB>(p, ntiles, s, ks);
  else return -1;
  return ks;
}

// 17..32 tokens, q|k|v of a K-quant file (segments of different types): 4-wave groups, K split in two,
// partial slabs [2][token][N] that the decode attention (FIN) or launch_qkv_finish completes.
// Returns the split or -1 (the caller runs mkq_kernel's EPI_QKV instead).
int launch_mkq_qkv_slab(const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s) {
  static const bool off = getenv("MX_NO_KQ_WIDE") != nullptr;
  if (off || a.M <= 16 || a.M > 32 || !a.xq || !a.xd || !a.xb || a.K % 256 || a.N % 64) return -1;
  for (int i = 0; i < a.kq_n; ++i)
    if (a.kq_tile_end[i] % 4) return -1;
  const int ntiles = a.N / TILE_N, SB = a.K / 256;
  int ks = 1;
  while (ks < 8 && (ntiles / 4) * ks * 2 <= kq_slab_target() && SB / (ks * 2) >= 4) ks *= 2;
  MMArgs p = a;
  p.out = slabs;
  p.ldo = a.N;
  p.slab_stride = slab_stride;
  mkq_wide_seg_kernel<4, 2, EPI_SLAB><<<dim3(ntiles / 4, ks), 256, 0, s>>>(p);
  return ks;
}

bool mkq_can_quantize_on_load(int M, int K, bool norm) {
  return M == 1 && K % 256 == 0 && (K / 256 + 7) / 8 <= QL_SB_MAX && (!norm || K / 16 <= 512);
}

int launch_mkq(int epi, const MMArgs& a, hipStream_t s) {
  if (a.M < 1 || a.K % 256 || a.N % TILE_N) return -1;
  if (a.xq == nullptr) {  // quantise on load
    if (!a.xf || !mkq_can_quantize_on_load(a.M, a.K, a.norm_w != nullptr) ||
        (a.norm_w && (!a.ssq || a.np * 16 != a.K)))
      return -1;
  } else if (!a.xd || !a.xb) {
    return -1;
  }
  if (a.kq_n < 1 || a.kq_n > 3 || a.kq_tile_end[a.kq_n - 1] * TILE_N != a.N) return -1;
  for (int i = 0; i < a.kq_n; ++i)
    if (!kq_tile_bytes(a.kq_type[i]) || (i && a.kq_tile_end[i] <= a.kq_tile_end[i - 1])) return -1;
  if (epi == EPI_SWIGLU && !a.actf) return -1;
  const int ntiles = a.N / TILE_N;
  if (epi == EPI_QKV && launch_kq_qkv_pers(a, s) == 0) return 0;
  if (launch_kq_pers(epi, a, ntiles, s) == 0) return 0;
  if (launch_kq_wide(epi, a, ntiles, s) == 0) return 0;
  switch (epi) {
    case EPI_F32: launch_mkq_epi<EPI_F32>(a, ntiles, s); return 0;
    case EPI_RESID: launch_mkq_epi<EPI_RESID>(a, ntiles, s); return 0;
    case EPI_QKV: launch_mkq_epi<EPI_QKV>(a, ntiles, s); return 0;
    case EPI_SWIGLU: launch_mkq_epi<EPI_SWIGLU>(a, ntiles, s); return 0;
  }
  return -1;
}

}  // namespace mx
