// device_common.h -- device helpers shared by the gfx950 kernel files (kernels.hip, kquant.hip):
// vector types, bf16/f16 rounding, the synthetic-weight hash, packed-row mapping, the KV-cache tile
// layout and the GEMV epilogues.  Everything here is inline; include only from .hip sources.
#pragma once
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

// Destination row of logical row `row` in a packed matrix (see kernels.h):
//   PACK_ROWS:     row + offset           (q|k|v stacked into one QKV matrix, or plain)
//   PACK_GATE/UP:  16*(row/8) + (0|8) + row%8   -- ffn_gate and ffn_up rows interleaved by
//                  halves of each 16-row tile, so one tile yields 8 SwiGLU outputs
__device__ __forceinline__ int packed_row(int row, int mode, int offset) {
  if (mode == PACK_GATE) return 16 * (row >> 3) + (row & 7);
  if (mode == PACK_UP) return 16 * (row >> 3) + 8 + (row & 7);
  return row + offset;
}
__device__ __forceinline__ size_t packed_index(int P, int col, int KT) {
  const size_t tile = (size_t)(P >> 4) * KT + (col >> 5);
  const int lane = (P & 15) + 16 * ((col & 31) >> 3);
  return tile * TILE_ELEMS + lane * 8 + (col & 7);
}

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

static int fill_grid(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g == 0 ? 1 : g));
}

// KV cache layout.  Each (slot, kv head) owns ctx_stride * D f16 of K and as many of V, stored as
// 1 KiB tiles in the lane order of the MFMA B operand that reads them, so every wave-instruction
// of the attention kernels loads one contiguous 1 KiB (llama.cpp keeps K [pos][d] and V transposed
// [d][pos] for the same reason on the CPU):
//   K: tile (pos/16, d/32) = 16 positions x 32 dims, lane = pos%16 + 16*((d%32)/8), element d%8
//      (the B operand of QK^T, v_mfma_f32_16x16x32_f16: k = dims, n = positions)
//   V: tile (pos/32, d/16) = 32 positions x 16 dims, lane = d%16 + 16*((pos%32)/8), element pos%8
//      (the B operand of P.V: k = positions, n = dims)
__device__ __forceinline__ size_t kv_k_off(int pos, int d, int D) {
  return (((size_t)(pos >> 4) * (D >> 5) + (d >> 5)) * 64 + (pos & 15) + 16 * ((d & 31) >> 3)) * 8 + (d & 7);
}
__device__ __forceinline__ size_t kv_v_off(int pos, int d, int D) {
  return (((size_t)(pos >> 5) * (D >> 4) + (d >> 4)) * 64 + (d & 15) + 16 * ((pos & 31) >> 3)) * 8 + (pos & 7);
}

// The RoPE (cos, sin) pairs of rows [row, row+4) at `pos` (clamped into the table: rows that take
// no RoPE, or positions that are not stored, load a valid entry and ignore it).  Callers that can
// issue it early (the persistent GEMVs, with pos / slot loaded once per kernel) pass it to
// qkv_store_pre: qkv_store's own chain pos -> (cs, slot) is two dependent round trips at the tail.
__device__ __forceinline__ f32x4 qkv_cs(const MMArgs& a, int row, int pos) {
  const int d = a.head_dim;
  const int rl = row < a.n_q ? row : row - a.n_q;
  const int p = min(max(pos, 0), a.n_ctx - 1);
  return *reinterpret_cast<const f32x4*>(a.rope_cs + ((size_t)p * (d / 2) + (rl % d) / 2) * 2);
}

// ---------------------------------------------------------------------------
// RMS_NORM sums of squares, one definition for every kernel that forms them (batch invariance:
// a row's scale must not depend on which kernel -- RMS_NORM on load at <= 4 rows, norm_kernel at
// more -- computed it, DESIGN.md §1 "batch invariance").
//   tile partial (16 consecutive values, f32): g_i = sequential double sums of the squares of
//     values 4i..4i+3 (each square rounded to f32, as ggml forms x*x), ((g0 + g1) + (g2 + g3))
//     rounded to f32 -- the shape the EPI_RESID epilogues produce with their C layout (lanes
//     l, l^16, l^32, l^48 hold the tile's 4 groups);
//   row sum (double): lane l of a wave sums partials 4l..4l+3, then 256+4l..256+4l+3, ...
//     sequentially, then a xor butterfly over the 64 lanes (o = 1, 2, ..., 32).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double ssq4(f32x4 v) {
#pragma clang fp contract(off)
  double q = (double)(v[0] * v[0]);
  q += (double)(v[1] * v[1]);
  q += (double)(v[2] * v[2]);
  q += (double)(v[3] * v[3]);
  return q;
}
// the tile partial from its four groups (a, b, c, d = values 0-3, 4-7, 8-11, 12-15)
__device__ __forceinline__ float ssq16(f32x4 a, f32x4 b, f32x4 c, f32x4 d) {
#pragma clang fp contract(off)
  return (float)((ssq4(a) + ssq4(b)) + (ssq4(c) + ssq4(d)));
}
// lane part of the row sum: partials 4l+256p .. +3 for p = 0, 1, ... (np % 4 == 0); q[p] holds them
template <int P>
__device__ __forceinline__ double ssq_lane(const f32x4 (&q)[P], int lane, int np) {
#pragma clang fp contract(off)
  double acc = 0.0;
#pragma unroll
  for (int p = 0; p < P; ++p)
    if (lane * 4 + 256 * p < np)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc += (double)q[p][j];
  return acc;
}
__device__ __forceinline__ double ssq_wave(double acc) {
#pragma clang fp contract(off)
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
  return acc;
}
__device__ __forceinline__ float rms_scale(double sum, int n, float eps) {
  return 1.0f / sqrtf((float)(sum / n) + eps);
}

// RoPE (mode NORM) of two adjacent pairs (s0, s1), (s2, s3) by their (cos, sin) in c: o0 = s0 c0 - s1 c1,
// ... as four scalar fmas.  Every operand passes through an empty asm so that the SLP vectorizer
// cannot turn them into v_pk_mul_f32 / v_pk_fma_f32 chains: compiled packed, the result's third
// element came out wrong in lanes 32-63 of a wave, run to run, whenever another queue's waves shared
// the CU (profiles/round5_rope_packed_hazard.txt; qkv_finish_kernel under a second process).
__device__ __forceinline__ float opq(float v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ f32x4 rope4(f32x4 s, f32x4 c) {
  const float s0 = opq(s[0]), s1 = opq(s[1]), s2 = opq(s[2]), s3 = opq(s[3]);
  const float c0 = opq(c[0]), c1 = opq(c[1]), c2 = opq(c[2]), c3 = opq(c[3]);
  f32x4 o;
  o[0] = opq(__builtin_fmaf(s0, c0, -(s1 * c1)));
  o[1] = opq(__builtin_fmaf(s0, c1, s1 * c0));
  o[2] = opq(__builtin_fmaf(s2, c2, -(s3 * c3)));
  o[3] = opq(__builtin_fmaf(s2, c3, s3 * c2));
  return o;
}

// q/k/v rows [row, row+4) of token column `col`: RoPE (mode NORM, adjacent pairs) on q and k,
// q -> f32 buffer, k / v -> the f16 K / V caches (layout above).
__device__ __forceinline__ void qkv_store_pre(const MMArgs& a, int row, int col, f32x4 s, int pos, int slot,
                                              f32x4 csv) {
  const int d = a.head_dim;
  if (pos < 0 || pos >= a.n_ctx) return;  // never write outside the slot's KV rows
  if (row < a.n_q + a.n_kv) {
    const bool is_q = row < a.n_q;
    const int rl = is_q ? row : row - a.n_q;
    const int dd = rl % d;  // multiple of 4
    const f32x4 o = rope4(s, csv);
    if (is_q) {
      *reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row) = o;
    } else {
      _Float16* kp = a.kc + (size_t)slot * a.slot_stride + (size_t)(rl / d) * a.ctx_stride * d + kv_k_off(pos, dd, d);
      *reinterpret_cast<f16x4*>(kp) = f16x4{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
    }
  } else {
    const int rl = row - a.n_q - a.n_kv;
    _Float16* vh = a.vc + (size_t)slot * a.slot_stride + (size_t)(rl / d) * a.ctx_stride * d;
#pragma unroll
    for (int i = 0; i < 4; ++i) vh[kv_v_off(pos, rl % d + i, d)] = (_Float16)s[i];
  }
}
__device__ __forceinline__ void qkv_store(const MMArgs& a, int row, int col, f32x4 s) {
  const int pos = a.pos[col], slot = a.slot[col];
  qkv_store_pre(a, row, col, s, pos, slot, qkv_cs(a, row, pos));
}

// One C-layout unit of a finished 16-row tile: rows 16*tile + 4*(l>>4) + i (i < 4) of token
// column `col`.  SWIGLU tiles hold 8 gate rows (lanes 0-31) and the matching up rows (lanes l+32).
template <int EPI>
__device__ __forceinline__ void epi_store(const MMArgs& a, int tile, int l, int col, f32x4 s, f32x4 up) {
  if constexpr (EPI == EPI_F32 || EPI == EPI_SLAB) {
    const int row = tile * 16 + (l >> 4) * 4;
    *reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row) = s;
  } else if constexpr (EPI == EPI_RESID) {
    const int row = tile * 16 + (l >> 4) * 4;
    f32x4* px = reinterpret_cast<f32x4*>(a.out + (size_t)col * a.ldo + row);
    *px = *px + s;
  } else if constexpr (EPI == EPI_SWIGLU) {
    const int row = tile * 8 + (l >> 4) * 4;  // ffn row of gate lane l / up lane l+32
    f32x4 f;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = (s[i] / (1.0f + expf(-s[i]))) * up[i];
    if (a.actf) {
      *reinterpret_cast<f32x4*>(a.actf + (size_t)col * a.lda + row) = f;
    } else {
      u32x2 o;
      o[0] = f2bf(f[0]) | (f2bf(f[1]) << 16);
      o[1] = f2bf(f[2]) | (f2bf(f[3]) << 16);
      *reinterpret_cast<u32x2*>(a.act + (size_t)col * a.lda + row) = o;
    }
  } else {  // EPI_QKV
    qkv_store(a, tile * 16 + (l >> 4) * 4, col, s);
  }
}

__device__ __forceinline__ float f16b(const uint8_t* p) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(p[0] | (p[1] << 8)));
}
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t* q, int& sc, int& m) {
  if (j < 4) {
    sc = q[j] & 63;
    m = q[j + 4] & 63;
  } else {
    sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

// Reductions over the 16 lanes of a DPP row (the 16 positions of one C-layout row): rotations
// within the row, so every lane ends with the result.  One VOP2-DPP instruction per step (the
// builtin route adds a move and an fmax canonicalisation per step, and __shfl_xor is a chain of
// ds_bpermute round trips); "s_nop 1" covers the VALU-write -> DPP-read hazard of the previous step.
#define MX_ROW_STEP(op, v, n)                                                                        \
  asm volatile("s_nop 1\n\t" op "_dpp %0, %1, %1 row_ror:" #n " row_mask:0xf bank_mask:0xf" : "=v"(v) \
               : "v"(v))
__device__ __forceinline__ float row16_max(float v) {
  MX_ROW_STEP("v_max_f32", v, 8);
  MX_ROW_STEP("v_max_f32", v, 4);
  MX_ROW_STEP("v_max_f32", v, 2);
  MX_ROW_STEP("v_max_f32", v, 1);
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  MX_ROW_STEP("v_add_f32", v, 8);
  MX_ROW_STEP("v_add_f32", v, 4);
  MX_ROW_STEP("v_add_f32", v, 2);
  MX_ROW_STEP("v_add_f32", v, 1);
  return v;
}
#undef MX_ROW_STEP
}  // namespace mx
