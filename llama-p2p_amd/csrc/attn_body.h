// attn_body.h -- the decode attention body (one kv head x one row) of attn_decode_kernel (kernels.hip).
// (Round 4's persistent one-token decode ran it on 3 waves of its own work-groups; that engine was
// measured slower than the per-op kernels and is archived under tools/archive/.)
#pragma once
#include "device_common.h"

namespace mx {

constexpr float LOG2E = 1.4426950408889634f;

// One (kv head, row) of decode attention, by the NW waves of the calling work-group.  Wave w takes
// chunks w, w + NW, ... and issues each later chunk's K/V loads when it reaches it (issuing two chunks
// ahead measured slower: 18.6 vs 11.1 us at 32 rows, profiles/round2_attention.txt).  FIN: q/k/v
// still as the wide path's split-K slabs (finished here, see below).  Everything that only the
// chunk holding `pos` (FIN) or the partial last chunk needs sits behind a wave-uniform branch, so
// the full chunks run the bare MFMA + softmax stream.
constexpr int ATTN_FIN_MAXSLAB = 8;  // split-K slabs the FIN path can sum (the wide launchers split K at most 8 ways)

// MS: slabs the FIN path loads (>= a.nslab; the ones past a.nslab re-read the last and add zero)
template <int D, int G, int NW, bool FIN, int MS = ATTN_FIN_MAXSLAB>
__device__ __forceinline__ void attn_decode_body(const AttnArgs& a, int kvh, int c) {
  constexpr int CH = ATTN_CHUNK;
  constexpr int QK = D / 32;  // k-steps of QK^T
  constexpr int DT = D / 16;  // d tiles of P.V
  const int t_ = threadIdx.x;
  const int lane = t_ & 63, w = __builtin_amdgcn_readfirstlane(t_ >> 6);
  const int r16 = lane & 15, q4 = lane >> 4;
  unsigned long long* tr = a.trace ? a.trace + (((size_t)c * a.n_head_kv + kvh) * NW + w) * 8 : nullptr;
  auto stamp = [&](int k) {
    if (tr && lane == 0) tr[k] = __builtin_amdgcn_s_memrealtime();
  };
  const int pos = a.pos[c];
  const int slot = a.slot[c];
  stamp(0);
  const int ctx = min(pos + 1, a.n_ctx);

  __shared__ __attribute__((aligned(16))) _Float16 Ps[NW][16][CH + 8];
  __shared__ float Om[NW][G][D];
  __shared__ float Mm[NW][G], Ll[NW][G];
  __shared__ __attribute__((aligned(16))) float qs[G * D + 2 * D];  // finished q rows, then this position's K, V

  const _Float16* Kb = a.kc + (size_t)slot * a.slot_stride + (size_t)kvh * a.ctx_stride * D;
  const _Float16* Vb = a.vc + (size_t)slot * a.slot_stride + (size_t)kvh * a.ctx_stride * D;
  struct KV {
    f16x8 k[2][QK], v[DT];
  };
  auto load = [&](KV& f, int ch) {
    const int p0 = ch * CH;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int kk = 0; kk < QK; ++kk)
        f.k[t][kk] = *reinterpret_cast<const f16x8*>(Kb + (((size_t)(p0 / 16 + t) * QK + kk) * 64 + lane) * 8);
#pragma unroll
    for (int t = 0; t < DT; ++t)
      f.v[t] = *reinterpret_cast<const f16x8*>(Vb + (((size_t)(p0 / 32) * DT + t) * 64 + lane) * 8);
  };
  // the wave's first chunk is loaded before anything else: its latency overlaps the q load (and the
  // FIN slab sums) instead of following them.  FIN writes this position's K/V below; the chunk
  // holding it is patched from LDS in compute(), so a stale read of that position is harmless.
  KV A;
  if (w * CH < ctx) load(A, w);

  // wide path: q/k/v of this (kv head, token) are still split-K partial slabs -- sum them in slab
  // order (bit-identical to qkv_finish_kernel), RoPE q and k, write this position's K and V into
  // the caches for later steps, and keep all of it in LDS for this step
  constexpr bool fin = FIN;
  if constexpr (FIN) {
    const int nq = a.n_head * D, nkv = a.n_head_kv * D, N = nq + 2 * nkv;
    for (int u = t_; u < (G * D + 2 * D) / 4; u += 64 * NW) {
      const int i = u * 4;  // qs index
      const int row = i < G * D ? kvh * G * D + i : i < G * D + D ? nq + kvh * D + (i - G * D)
                                                                   : nq + nkv + kvh * D + (i - G * D - D);
      // all slab and RoPE loads issued together (clamped: extra reads repeat the last slab): a run-time
      // slab loop or a load behind the RoPE branch made each load wait for itself
      f32x4 sv[MS];
#pragma unroll
      for (int k = 0; k < MS; ++k)
        sv[k] = *reinterpret_cast<const f32x4*>(a.slabs + min(k, a.nslab - 1) * a.slab_stride + (size_t)c * N + row);
      const int dd = i % D;
      const f32x4 csv =
          *reinterpret_cast<const f32x4*>(a.rope_cs + ((size_t)max(0, min(pos, a.n_ctx - 1)) * (D / 2) + dd / 2) * 2);
      // slab order, as qkv_finish_kernel; the slabs past nslab add exact zeros (a branch per slab
      // would pull its load into the branch again)
      f32x4 v = sv[0];
#pragma unroll
      for (int k = 1; k < MS; ++k) v += sv[k] * (k < a.nslab ? 1.0f : 0.0f);
      {  // RoPE (mode NORM: adjacent pairs) on q and k, as selects (a branch would pull csv's load into it)
        const bool rope = i < G * D + D && pos < a.n_ctx;
        const f32x4 s = v;
        const f32x4 rv = rope4(s, csv);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = rope ? rv[j] : s[j];
      }
      *reinterpret_cast<f32x4*>(qs + i) = v;
      if (i >= G * D && pos < a.n_ctx) {
        const size_t sb = (size_t)slot * a.slot_stride;
        if (i < G * D + D) {
          _Float16* kp = a.kc_w + sb + (size_t)kvh * a.ctx_stride * D + kv_k_off(pos, dd, D);
          *reinterpret_cast<f16x4*>(kp) = f16x4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
          _Float16* vh = a.vc_w + sb + (size_t)kvh * a.ctx_stride * D;
#pragma unroll
          for (int j = 0; j < 4; ++j) vh[kv_v_off(pos, dd + j, D)] = (_Float16)v[j];
        }
      }
    }
    __syncthreads();
  }

  // A operand of QK^T: rows = heads of the group (rows >= G are zero)
  f16x8 qa[QK];
  {
    const float* qrow = fin ? qs + (r16 < G ? r16 : 0) * D
                            : a.q + (size_t)c * a.n_head * D + (size_t)(kvh * G + (r16 < G ? r16 : 0)) * D;
    const bool live = r16 < G;
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(qrow + kk * 32 + 8 * q4);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(qrow + kk * 32 + 8 * q4 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        qa[kk][j] = live ? (_Float16)v0[j] : (_Float16)0.f;
        qa[kk][4 + j] = live ? (_Float16)v1[j] : (_Float16)0.f;
      }
    }
  }

  float m_i[4], l_i[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m_i[i] = -INFINITY;
    l_i[i] = 0.f;
  }
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (tr) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp(1);  // q in registers
  }
  int nch = 0;
  auto compute = [&](KV& f, int ch) {
    const int p0 = ch * CH;
    const int pb = p0 + 8 * q4;  // first position of this lane's P.V B fragment
    if (FIN && pos >= p0 && pos < p0 + CH) {  // this position's K/V from LDS (its stores may be in flight)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (p0 + 16 * t + r16 == pos)
#pragma unroll
          for (int kk = 0; kk < QK; ++kk)
#pragma unroll
            for (int j = 0; j < 8; ++j) f.k[t][kk][j] = (_Float16)qs[G * D + 8 * q4 + kk * 32 + j];
      if (pos >= pb && pos < pb + 8)
#pragma unroll
        for (int t = 0; t < DT; ++t) f.v[t][pos - pb] = (_Float16)qs[G * D + D + t * 16 + r16];
    }
    if (tr && nch == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      stamp(2);  // first chunk's K/V landed
    }
    nch++;
    // S[head][pos] for two 16-position tiles
    f32x4 sc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < QK; ++kk) sc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qa[kk], f.k[t][kk], sc[t], 0, 0, 0);
    }
    // online softmax in the log2 domain (scores pre-multiplied by log2 e, v_exp_f32 = 2^x):
    // C layout rows = heads 4*q4+i, cols = positions (lane r16)
    float e[2][4];
    const float sl2 = a.scale * LOG2E;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v0 = (p0 + r16 < ctx) ? sc[0][i] * sl2 : -INFINITY;
      const float v1 = (p0 + 16 + r16 < ctx) ? sc[1][i] * sl2 : -INFINITY;
      const float m_new = fmaxf(m_i[i], row16_max(fmaxf(v0, v1)));
      const float alpha = __builtin_amdgcn_exp2f(m_i[i] - m_new);  // 0 on the first chunk (m_i = -inf)
      e[0][i] = __builtin_amdgcn_exp2f(v0 - m_new);
      e[1][i] = __builtin_amdgcn_exp2f(v1 - m_new);
      l_i[i] = l_i[i] * alpha + row16_sum(e[0][i] + e[1][i]);
      m_i[i] = m_new;
#pragma unroll
      for (int t = 0; t < DT; ++t) o[t][i] *= alpha;
    }
    // P (f16) -> LDS as [head][pos], re-read as the A operand of P.V
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) Ps[w][4 * q4 + i][16 * t + r16] = (4 * q4 + i < G) ? (_Float16)e[t][i] : (_Float16)0.f;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    const f16x8 pa = *reinterpret_cast<const f16x8*>(&Ps[w][r16][8 * q4]);
    if (p0 + CH > ctx) {  // the partial last chunk: never-written positions must not reach P.V
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) f.v[t][j] = (pb + j < ctx) ? f.v[t][j] : (_Float16)0.f;
    }
#pragma unroll
    for (int t = 0; t < DT; ++t) o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa, f.v[t], o[t], 0, 0, 0);
    __builtin_amdgcn_wave_barrier();  // Ps[w] is rewritten next chunk only after every lane read it
  };
  for (int ch = w; ch * CH < ctx; ch += NW) {
    if (ch != w) load(A, ch);
    compute(A, ch);
  }
  stamp(3);  // chunk loop done
  if (tr && lane == 0) tr[7] = nch;

  // merge the NW wave partials
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = 4 * q4 + i;
    if (h < G) {
#pragma unroll
      for (int t = 0; t < DT; ++t) Om[w][h][t * 16 + r16] = o[t][i];
      if (r16 == 0) {
        Mm[w][h] = m_i[i];
        Ll[w][h] = l_i[i];
      }
    }
  }
  __syncthreads();
  stamp(4);  // partials in LDS
  for (int idx = t_; idx < G * D; idx += 64 * NW) {
    const int h = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, Mm[ww][h]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) {
      const float f = (Mm[ww][h] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(Mm[ww][h] - M);
      L += f * Ll[ww][h];
      acc += f * Om[ww][h][d];
    }
    if (a.outf) {
      a.outf[(size_t)c * a.ldo + (kvh * G + h) * D + d] = acc / L;
    } else {
      a.out[(size_t)c * a.ldo + (kvh * G + h) * D + d] = (uint16_t)f2bf(acc / L);
    }
  }
  if (tr) {
    __builtin_amdgcn_s_waitcnt(0);
    stamp(5);  // outputs stored
  }
}


}  // namespace mx
