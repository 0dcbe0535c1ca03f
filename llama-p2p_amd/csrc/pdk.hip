// pdk.hip -- persistent decode kernel: one launch per decode step of <= PDK_MAX_M tokens.
//
// Replaces, for batch-1-class decode, the per-op launches of kernels.hip (the same ggml ops of
// llm_build_llama behind /root/reference/llama_p2p_network.py:125).
// Why: at one token every projection is a short weight stream (qkv 50 MB = 7 us at HBM rate)
// and each separate launch pays a ramp-in (first loads), a tail (last work-group) and, for
// attention and RMS_NORM, a pure-latency kernel -- together ~30% of a layer
// (profiles/round1_bench_kernel_stats.txt).  Here one grid of resident work-groups (one per CU,
// 16 waves) walks every layer's phases
//     qkv (RMS_NORM on load, RoPE, KV) | attention | attn_output (+resid) | gate/up (norm on
//     load, SwiGLU) | down (+resid) | ... | lm_head (output norm on load)
// separated by grid barriers, and every wave keeps its weight-load ring running ACROSS phase
// boundaries: weights never depend on activations, so the loads of the next phase's first tile
// are issued before the barrier wait and the HBM stream does not stop at phase seams.
//
// Cross-work-group data (q, the current position's K/V, attn_out, x, ssq, act) is handed over
// with the sc1 (write-through) store + sc1 load protocol of cdna_hip_programming.md §6
// Guideline 16 (table row 1): ONE wave (wave 0) of each work-group does every publishing store,
// drains them (s_waitcnt vmcnt(0)) and adds to the arrival counter (agent-scope atomic); waiters
// poll the counter with relaxed agent loads and read handed-over bytes only with sc1 loads.
// Every wait is bounded (PDK_TIMEOUT): a grid that is not co-resident ends with sync[1] set
// instead of hanging, and the host reports it.
#include <hip/hip_runtime.h>
#include <math.h>

#include "kernels.h"

namespace mx {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((address_space(1))) const u32x4 gu32x4;  // global: no flat loads

constexpr int NW = PDK_WAVES;  // waves per work-group; also the K split of every GEMV tile
constexpr int U = 8;           // weight ring depth per wave (K-tiles of 1 KiB): 64 KiB in flight per CU
constexpr long long PDK_TIMEOUT = 200000000;  // 2 s of the 100 MHz wall clock per barrier wait

__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// sc1 (write-through / L1-bypassing) accesses through a buffer descriptor on a uniform base
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ u32x4 ld16(const void* base, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st16(void* base, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st8(void* base, unsigned off, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, rsrc(base), off, 0, 16);
}
__device__ __forceinline__ void st4(void* base, unsigned off, unsigned v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, rsrc(base), off, 0, 16);
}
// weight tile loads: non-temporal (aux 2 = nt), voffset = lane*16 (constant), K-tile offset uniform
__device__ __forceinline__ u32x4 ldw(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned tile_k) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, tile_k * 1024u, 2);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wrsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0xfffffff0, 0x00020000);
}
__device__ __forceinline__ f32x4 as_f4(u32x4 v) { return __builtin_bit_cast(f32x4, v); }
__device__ __forceinline__ u32x4 as_u4(f32x4 v) { return __builtin_bit_cast(u32x4, v); }

// K assignment inside a work-group: wave w owns K-tiles w, w+NW, w+2NW, ... (interleaved), so at
// any moment the work-group's waves read adjacent 1 KiB pieces of a tile; image index i of wave w
// holds k = kmap(w, i).
__device__ __forceinline__ int kmap(int w, int i) { return ((i >> 5) * NW + w) * TILE_K + (i & 31); }

struct Gemv {
  const uint16_t* W;  // packed tiles (kernels.h)
  int K, ntiles;
};

struct Ring {
  u32x4 r[U];
  bool primed;  // r holds items 0..U-1 of this wave's first tile of the coming phase
};

// LDS map (bytes): [0, 32K) red[2][NW][64] f32x4 | 64 B flag | 4 KiB xk[PDK_MAX_XT][64] f32x4 |
// union: per-wave B images, or attention scratch
constexpr int LDS_RED = 0;
constexpr int LDS_FLAG = 2 * NW * 64 * 16;
constexpr int LDS_XK = LDS_FLAG + 64;
constexpr int LDS_UNION = LDS_XK + PDK_MAX_XT * 64 * 16;

struct Ctx {
  const PdkArgs& a;
  unsigned char* smem;
  int lane, w, g, G;
  unsigned nbar;
  int tcount;  // GEMV tiles finished by this work-group (selects the red[] buffer)
};

// ---------------------------------------------------------------- grid barrier
// Wave 0 published everything: drain its stores, count this work-group in, prefill its own ring
// for the next phase (its loads would otherwise delay the drain), then wave 1 polls.
__device__ __forceinline__ void prefill(Ctx& c, Ring& ring, const Gemv* nx) {
  if (!nx || ring.primed || nx->ntiles <= c.g) return;
  const int KT = nx->K / TILE_K;
  const gu32x4* p = ((const gu32x4*)(nx->W)) + ((size_t)c.g * KT + c.w) * 64 + c.lane;
#pragma unroll
  for (int u = 0; u < U; ++u) ring.r[u] = __builtin_nontemporal_load(p + (size_t)u * NW * 64);
  ring.primed = true;
}

// Arrival is a two-level counter tree (contended atomics on one word serialise: 256 arrivals on
// one counter cost ~8 us): work-group g counts into group g % SYNC_GROUPS; the last arriver of
// a group (told by the value its add returns) counts the group into the root; the root's last
// arriver publishes the barrier number to SYNC_GROUPS flag replicas, each polled by its group
// only.  Every word sits on its own 128-B line.  Counters only grow (barrier b completes at
// n*b), so nothing is reset inside the launch; launch_pdk zeroes them before it.
constexpr int SYNC_GROUPS = 16;
constexpr int SYNC_STRIDE = 32;  // uints between words (128 B)
__device__ __forceinline__ unsigned* sync_root(const PdkArgs& a) { return a.sync; }
__device__ __forceinline__ unsigned* sync_group(const PdkArgs& a, int j) { return a.sync + SYNC_STRIDE * (1 + j); }
__device__ __forceinline__ unsigned* sync_flag(const PdkArgs& a, int j) {
  return a.sync + SYNC_STRIDE * (1 + SYNC_GROUPS + j);
}
__device__ __forceinline__ unsigned* sync_err(const PdkArgs& a) { return a.sync + SYNC_STRIDE * (1 + 2 * SYNC_GROUPS); }

// arrive: wave 0 (the only publisher) drains its stores and counts the work-group in
__device__ __forceinline__ void grid_arrive(Ctx& c) {
  c.nbar++;
  const int ng = c.G < SYNC_GROUPS ? c.G : SYNC_GROUPS;
  const int grp = c.g % ng;
  if (c.w == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (c.lane == 0) {
      const unsigned n_in_grp = (unsigned)((c.G - grp + ng - 1) / ng);
      const unsigned old = __hip_atomic_fetch_add(sync_group(c.a, grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == n_in_grp * c.nbar - 1) {
        const unsigned r = __hip_atomic_fetch_add(sync_root(c.a), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (r == (unsigned)ng * c.nbar - 1)
          for (int j = 0; j < ng; ++j)
            __hip_atomic_store(sync_flag(c.a, j), c.nbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// wait: wave 1 polls its group's flag replica (bounded); false = abort the launch
__device__ __forceinline__ bool grid_wait(Ctx& c) {
  unsigned* flag = reinterpret_cast<unsigned*>(c.smem + LDS_FLAG);
  const int ng = c.G < SYNC_GROUPS ? c.G : SYNC_GROUPS;
  if (c.w == 1 && c.lane == 0) {
    const long long t0 = wall_clock64();
    unsigned ok = 1;
    unsigned* f = sync_flag(c.a, c.g % ng);
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < c.nbar) {
      if (__hip_atomic_load(sync_err(c.a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
      if (wall_clock64() - t0 > PDK_TIMEOUT) {
        __hip_atomic_store(sync_err(c.a), 1u + c.nbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    flag[0] = ok;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no handed-over load moves above the poll
  const bool ok = flag[0] != 0;
  __syncthreads();  // flag[] is rewritten only after every wave read it
  return ok;
}

// ---------------------------------------------------------------- B images (per wave, LDS)
// RMS_NORM on load: img[c][i] = bf16((x[c][kbase+i] * scale_c) * w[kbase+i]), scale_c from the
// per-16-row-tile partials ssq[c][*] (fixed-order lane sums + xor tree: every lane agrees).
__device__ __forceinline__ void build_xs(Ctx& c, const float* nw, uint16_t* img, int pitch, int nkk) {
  const PdkArgs& a = c.a;
  const int np = a.h / 16;
  for (int col = 0; col < a.M; ++col) {
    f32x4 q[2], xv[2], g[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int i = c.lane * 4 + 256 * p;
      if (i < np) q[p] = as_f4(ld16(a.ssq, (unsigned)((col * np + i) * 4)));
      if (i < nkk) {
        const int k = kmap(c.w, i);
        xv[p] = as_f4(ld16(a.x, (unsigned)((col * a.h + k) * 4)));
        g[p] = *reinterpret_cast<const f32x4*>(nw + k);
      }
    }
    double acc = 0.0;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      if (c.lane * 4 + 256 * p < np)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += (double)q[p][j];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    const float sc = 1.0f / sqrtf((float)(acc / a.h) + a.eps);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int i = c.lane * 4 + 256 * p;
      if (i < nkk) {
        u32x2 o;
        o[0] = f2bf((xv[p][0] * sc) * g[p][0]) | (f2bf((xv[p][1] * sc) * g[p][1]) << 16);
        o[1] = f2bf((xv[p][2] * sc) * g[p][2]) | (f2bf((xv[p][3] * sc) * g[p][3]) << 16);
        *reinterpret_cast<u32x2*>(img + col * pitch + i) = o;
      }
    }
  }
}

// bf16 activation handed over by another phase ([M][K], sc1 loads)
__device__ __forceinline__ void build_act(Ctx& c, const uint16_t* src, int K, uint16_t* img, int pitch, int nkk) {
  for (int col = 0; col < c.a.M; ++col)
    for (int i = c.lane * 8; i < nkk; i += 512)
      *reinterpret_cast<u32x4*>(img + col * pitch + i) = ld16(src, (unsigned)((col * K + kmap(c.w, i)) * 2));
}

// ---------------------------------------------------------------- GEMV epilogues (wave 0)
// C layout of tile t: lane l holds rows 16t + 4(l>>4) + i (i < 4) of token column l & 15.
__device__ __forceinline__ void epi_qkv(Ctx& c, int layer, int t, f32x4 s) {
  const PdkArgs& a = c.a;
  const int l = c.lane, col = l & 15, row = t * 16 + (l >> 4) * 4;
  if (col >= a.M) return;
  const int D = a.head_dim, nq = a.h, nkv = a.kv;
  const int pos = a.pos[col];
  if (pos < 0 || pos >= a.n_ctx) return;
  const PdkLayer& L = a.layers[layer];
  f32x4 o = s;
  if (row < nq + nkv) {  // RoPE (mode NORM: adjacent pairs) on q and k
    const int dd = (row < nq ? row : row - nq) % D;
    const f32x4 csv = *reinterpret_cast<const f32x4*>(a.rope_cs + ((size_t)pos * (D / 2) + dd / 2) * 2);
    o[0] = s[0] * csv[0] - s[1] * csv[1];
    o[1] = s[0] * csv[1] + s[1] * csv[0];
    o[2] = s[2] * csv[2] - s[3] * csv[3];
    o[3] = s[2] * csv[3] + s[3] * csv[2];
  }
  const size_t sb = (size_t)a.slot[col] * a.slot_stride;
  if (row < nq) {
    st16(a.q, (unsigned)((col * nq + row) * 4), as_u4(o));
  } else if (row < nq + nkv) {
    const int rl = row - nq;
    st16(a.kvs, (unsigned)((col * 2 * nkv + rl) * 4), as_u4(o));  // this step's attention reads it here
    _Float16* kp = L.kc + sb + ((size_t)(rl / D) * a.ctx_stride + pos) * D + rl % D;  // later steps: cache
    *reinterpret_cast<f16x4*>(kp) = f16x4{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
  } else {
    const int rl = row - nq - nkv;
    st16(a.kvs, (unsigned)((col * 2 * nkv + nkv + rl) * 4), as_u4(s));
    _Float16* vt = L.vc + sb + ((size_t)(rl / D) * D + rl % D) * a.ctx_stride + pos;
#pragma unroll
    for (int i = 0; i < 4; ++i) vt[(size_t)i * a.ctx_stride] = (_Float16)s[i];
  }
}

// residual add (x rows of this tile live in LDS xk: only this work-group ever writes them) and
// the tile's share of the next RMS_NORM's sum of squares
__device__ __forceinline__ void epi_resid(Ctx& c, int t, int task, f32x4 s) {
  const PdkArgs& a = c.a;
  const int l = c.lane, col = l & 15, row = t * 16 + (l >> 4) * 4;
  f32x4* xk = reinterpret_cast<f32x4*>(c.smem + LDS_XK) + task * 64 + l;
  double q = 0.0;
  if (col < a.M) {
    const f32x4 xv = *xk + s;
    *xk = xv;
    st16(a.x, (unsigned)((col * a.h + row) * 4), as_u4(xv));
#pragma unroll
    for (int i = 0; i < 4; ++i) q += (double)(xv[i] * xv[i]);
  }
  q += __shfl_xor(q, 16);
  q += __shfl_xor(q, 32);
  if (l < 16 && col < a.M) st4(a.ssq, (unsigned)((col * (a.h / 16) + t) * 4), __float_as_uint((float)q));
}

// tile = 8 gate rows (lanes 0-31) + the matching 8 up rows (lanes 32-63)
__device__ __forceinline__ void epi_swiglu(Ctx& c, int t, f32x4 s) {
  const PdkArgs& a = c.a;
  f32x4 up;
#pragma unroll
  for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(s[i], 32);
  const int l = c.lane, col = l & 15;
  if (l >= 32 || col >= a.M) return;
  const int row = t * 8 + (l >> 4) * 4;
  uint32_t hh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) hh[i] = f2bf((s[i] / (1.0f + expf(-s[i]))) * up[i]);
  st8(a.act, (unsigned)((col * a.ff + row) * 2), u32x2{hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16)});
}

__device__ __forceinline__ void epi_logits(Ctx& c, int t, f32x4 s) {
  const PdkArgs& a = c.a;
  const int l = c.lane, col = l & 15;
  if (col >= a.M) return;
  *reinterpret_cast<f32x4*>(a.logits + (size_t)col * a.n_vocab + t * 16 + (l >> 4) * 4) = s;
}

enum { E_QKV, E_RESID, E_SWIGLU, E_LOGITS };

// one tile's K-slice for this wave: NK K-tiles, ring refills from this tile, then the last group's
// refills from the continuation (next tile / next phase / dummy)
template <int NK>
__device__ __forceinline__ void tile_k(Ring& ring, f32x4& acc, const uint16_t* bp, const gu32x4* Wt, const gu32x4* Wn,
                                       int nstep) {
  static_assert(NK % U == 0, "K-slice must be whole ring groups");
#pragma unroll
  for (int j = 0; j < NK; j += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4 b = *reinterpret_cast<const u32x4*>(bp + (j + u) * TILE_K);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ring.r[u]),
                                                    __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
      ring.r[u] = __builtin_nontemporal_load(j + U < NK ? Wt + (size_t)(j + u + U) * NW * 64 : Wn + u * nstep);
      __builtin_amdgcn_sched_barrier(0);  // keep each refill right behind its MFMA (ring stays U deep)
    }
  }
}

// ---------------------------------------------------------------- one GEMV phase
// Work-group g takes tiles g, g+G, ...; its 16 waves split K (wave w: K-tiles [w*nk, (w+1)*nk)).
// Each wave's loads form one stream: this tile, then the next tile, then (waves 1-15) the next
// phase's first tile; partial tiles meet in LDS and wave 0 runs the epilogue.
__device__ __forceinline__ void gemv_phase(Ctx& c, int EP, int layer, const Gemv& ph, const Gemv* nx, Ring& ring,
                                           const uint16_t* img, int pitch) {
  const int KT = ph.K / TILE_K, nk = KT / NW;
  const int ntask = ph.ntiles > c.g ? (ph.ntiles - c.g + c.G - 1) / c.G : 0;
  // every load is a global (address space 1) load of uniform base + lane*16, and every ring slot is
  // refilled unconditionally (a slot with nothing left re-reads a small L2-resident buffer):
  // straight-line code keeps the compiler's vmcnt waits at "oldest slot" depth
  const gu32x4* Wl = ((const gu32x4*)(ph.W)) + c.lane;
  if (ntask > 0 && !ring.primed) {
#pragma unroll
    for (int u = 0; u < U; ++u) ring.r[u] = __builtin_nontemporal_load(Wl + ((size_t)c.g * KT + c.w + u * NW) * 64);
  }
  ring.primed = false;
  const bool xp = nx && c.w != 0 && nx->ntiles > c.g;
  const int nKT = nx ? nx->K / TILE_K : 0;
  const gu32x4* Wx = xp ? ((const gu32x4*)(nx->W)) + ((size_t)c.g * nKT + c.w) * 64 + c.lane
                        : ((const gu32x4*)(c.a.out_norm)) + c.lane;
  const int xstep = xp ? NW * 64 : 0;
  const int bcol = min(c.lane & 15, c.a.M - 1);
  const uint16_t* bp = img + bcol * pitch + (c.lane >> 4) * 8;
  for (int i = 0; i < ntask; ++i) {
    const int t = c.g + i * c.G;
    const bool last = i + 1 == ntask;
    const gu32x4* Wt = Wl + ((size_t)t * KT + c.w) * 64;
    // continuation after this tile: the next tile, or the next phase's first tile (or the dummy)
    const gu32x4* Wn = last ? Wx : Wl + ((size_t)(t + c.G) * KT + c.w) * 64;
    const int nstep = last ? xstep : NW * 64;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // fully unrolled for the K-slices of the supported shapes (no loop header inside a tile: a loop
    // header made the compiler drain the whole ring, vmcnt(0), once per group)
    if (nk == 16) tile_k<16>(ring, acc, bp, Wt, Wn, nstep);
    else if (nk == 56) tile_k<56>(ring, acc, bp, Wt, Wn, nstep);
    else tile_k<8>(ring, acc, bp, Wt, Wn, nstep);  // pdk_supported admits only these K-slices
    if (last && xp) ring.primed = true;
    f32x4* rb = reinterpret_cast<f32x4*>(c.smem + LDS_RED) + (c.tcount & 1) * NW * 64;
    rb[c.w * 64 + c.lane] = acc;
    __syncthreads();
    if (c.w == 0) {
      f32x4 s = rb[c.lane];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) s += rb[ww * 64 + c.lane];
      if (EP == E_QKV) epi_qkv(c, layer, t, s);
      else if (EP == E_RESID) epi_resid(c, t, i, s);
      else if (EP == E_SWIGLU) epi_swiglu(c, t, s);
      else epi_logits(c, t, s);
    }
    c.tcount++;
  }
}

// ---------------------------------------------------------------- attention task
// One (kv head, token) per work-group: KQ = f16(q).K -> softmax(scale, causal) -> f16(P).V with
// the G query heads of the GQA group as the rows of f16 MFMA tiles (as kernels.hip's
// attn_decode_kernel).  The KV cache of earlier positions does not depend on this step, so the
// work-group loads its first chunk per wave BEFORE the qkv barrier (attn_prefetch); after it,
// only q and this position's K/V (sc1 staging rows written by the qkv phase) are read.
template <int D>
struct AttnRegs {
  f16x8 kf[2][D / 32];
  f16x8 vf[D / 16];
};

template <int D>
__device__ __forceinline__ void attn_load_chunk(AttnRegs<D>& r, const _Float16* Kb, const _Float16* Vb, int p0,
                                                int ctx_stride, int lane) {
  const int r16 = lane & 15, q4 = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk)
      r.kf[t][kk] = *reinterpret_cast<const f16x8*>(Kb + (size_t)(p0 + 16 * t + r16) * D + 8 * q4 + kk * 32);
#pragma unroll
  for (int t = 0; t < D / 16; ++t)
    r.vf[t] = *reinterpret_cast<const f16x8*>(Vb + (size_t)(t * 16 + r16) * ctx_stride + p0 + 8 * q4);
}

__device__ __forceinline__ int attn_wg(const Ctx& c, int task) { return c.G - 1 - task; }  // fewest qkv tiles

template <int D>
__device__ __forceinline__ void attn_prefetch(Ctx& c, int layer, AttnRegs<D>& r) {
  const PdkArgs& a = c.a;
  const int task = c.G - 1 - c.g;
  if (task >= a.n_head_kv * a.M) return;
  const int kvh = task % a.n_head_kv, tok = task / a.n_head_kv;
  const int ctx = min(a.pos[tok] + 1, a.n_ctx);
  if (c.w * ATTN_CHUNK >= ctx) return;
  const PdkLayer& L = a.layers[layer];
  const size_t sb = (size_t)a.slot[tok] * a.slot_stride;
  attn_load_chunk<D>(r, L.kc + sb + (size_t)kvh * a.ctx_stride * D, L.vc + sb + (size_t)kvh * D * a.ctx_stride,
                     c.w * ATTN_CHUNK, a.ctx_stride, c.lane);
}

template <int D, int G>
__device__ __forceinline__ void attention(Ctx& c, int layer, AttnRegs<D>& r) {
  constexpr int CH = ATTN_CHUNK;
  constexpr int QK = D / 32, DT = D / 16;
  const PdkArgs& a = c.a;
  const int task = c.G - 1 - c.g;
  if (task >= a.n_head_kv * a.M) return;
  const int kvh = task % a.n_head_kv, tok = task / a.n_head_kv;
  const PdkLayer& L = a.layers[layer];
  const int lane = c.lane, w = c.w, r16 = lane & 15, q4 = lane >> 4;
  const int pos = a.pos[tok];
  const int ctx = min(pos + 1, a.n_ctx);
  const int slot = a.slot[tok];
  unsigned char* sm = c.smem + LDS_UNION;
  _Float16(*Ps)[16][CH + 8] = reinterpret_cast<_Float16(*)[16][CH + 8]>(sm);
  float(*Om)[G][D] = reinterpret_cast<float(*)[G][D]>(sm + NW * 16 * (CH + 8) * 2);
  float(*Mm)[G] = reinterpret_cast<float(*)[G]>(sm + NW * 16 * (CH + 8) * 2 + NW * G * D * 4);
  float(*Ll)[G] = reinterpret_cast<float(*)[G]>(sm + NW * 16 * (CH + 8) * 2 + NW * G * D * 4 + NW * G * 4);
  float* stKV = reinterpret_cast<float*>(sm + NW * 16 * (CH + 8) * 2 + NW * G * D * 4 + 2 * NW * G * 4);

  // this position's K and V of head kvh -> LDS (f32)
  if (w == 0) {
    const int nkv = a.kv;
    for (int i = lane * 4; i < 2 * D; i += 256) {
      const int kvsel = i / D, d = i % D;
      *reinterpret_cast<u32x4*>(stKV + i) = ld16(a.kvs, (unsigned)((tok * 2 * nkv + kvsel * nkv + kvh * D + d) * 4));
    }
  }
  f16x8 qa[QK];
  {
    const int hq = kvh * G + (r16 < G ? r16 : 0);
#pragma unroll
    for (int kk = 0; kk < QK; ++kk) {
      const unsigned off = (unsigned)(((size_t)tok * a.h + (size_t)hq * D + kk * 32 + 8 * q4) * 4);
      const f32x4 v0 = as_f4(ld16(a.q, off)), v1 = as_f4(ld16(a.q, off + 16));
      const bool live = r16 < G;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        qa[kk][j] = live ? (_Float16)v0[j] : (_Float16)0.f;
        qa[kk][4 + j] = live ? (_Float16)v1[j] : (_Float16)0.f;
      }
    }
  }
  __syncthreads();  // stKV ready

  const _Float16* Kb = L.kc + (size_t)slot * a.slot_stride + (size_t)kvh * a.ctx_stride * D;
  const _Float16* Vb = L.vc + (size_t)slot * a.slot_stride + (size_t)kvh * D * a.ctx_stride;
  float m_i[4], l_i[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m_i[i] = -INFINITY;
    l_i[i] = 0.f;
  }
  f32x4 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = w; ch * CH < ctx; ch += NW) {
    const int p0 = ch * CH;
    if (ch != w) attn_load_chunk<D>(r, Kb, Vb, p0, a.ctx_stride, lane);  // the first chunk was prefetched
    // this position's row is not in the cache yet (or stale): take it from the staging copy
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (p0 + 16 * t + r16 == pos)
#pragma unroll
        for (int kk = 0; kk < QK; ++kk)
#pragma unroll
          for (int j = 0; j < 8; ++j) r.kf[t][kk][j] = (_Float16)stKV[8 * q4 + kk * 32 + j];
    f32x4 s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < QK; ++kk)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qa[kk], r.kf[t][kk], s[t], 0, 0, 0);
    }
    float e[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v0 = (p0 + r16 < ctx) ? s[0][i] * a.attn_scale : -INFINITY;
      const float v1 = (p0 + 16 + r16 < ctx) ? s[1][i] * a.attn_scale : -INFINITY;
      float mx = fmaxf(v0, v1);
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
      const float m_new = fmaxf(m_i[i], mx);
      const float alpha = expf(m_i[i] - m_new);
      e[0][i] = expf(v0 - m_new);
      e[1][i] = expf(v1 - m_new);
      float ls = e[0][i] + e[1][i];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) ls += __shfl_xor(ls, off);
      l_i[i] = l_i[i] * alpha + ls;
      m_i[i] = m_new;
#pragma unroll
      for (int t = 0; t < DT; ++t) o[t][i] *= alpha;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) Ps[w][4 * q4 + i][16 * t + r16] = (4 * q4 + i < G) ? (_Float16)e[t][i] : (_Float16)0.f;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const f16x8 pa = *reinterpret_cast<const f16x8*>(&Ps[w][r16][8 * q4]);
    const int pb = p0 + 8 * q4;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      f16x8 vb = r.vf[t];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (pb + j == pos) vb[j] = (_Float16)stKV[D + t * 16 + r16];
        vb[j] = (pb + j < ctx) ? vb[j] : (_Float16)0.f;
      }
      o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa, vb, o[t], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int hh = 4 * q4 + i;
    if (hh < G) {
#pragma unroll
      for (int t = 0; t < DT; ++t) Om[w][hh][t * 16 + r16] = o[t][i];
      if (r16 == 0) {
        Mm[w][hh] = m_i[i];
        Ll[w][hh] = l_i[i];
      }
    }
  }
  __syncthreads();
  if (w == 0) {  // wave 0 publishes: 8 consecutive outputs (16 B of bf16) per lane and step
    for (int u = lane; u < G * D / 8; u += 64) {
      const int hh = u / (D / 8), d0 = (u % (D / 8)) * 8;
      float M = -INFINITY;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, Mm[ww][hh]);
      float Lsum = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        const float f = (Mm[ww][hh] == -INFINITY) ? 0.f : expf(Mm[ww][hh] - M);
        Lsum += f * Ll[ww][hh];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f * Om[ww][hh][d0 + j];
      }
      u32x4 ov;
#pragma unroll
      for (int j = 0; j < 4; ++j) ov[j] = f2bf(acc[2 * j] / Lsum) | (f2bf(acc[2 * j + 1] / Lsum) << 16);
      st16(a.attn_out, (unsigned)(((size_t)tok * a.h + (size_t)(kvh * G + hh) * D + d0) * 2), ov);
    }
  }
  __syncthreads();  // scratch (union) is reused by the next phase's images
}

enum { PH_NONE, PH_GEMV, PH_ATTN };
struct Phase {
  int kind = PH_NONE, epi = 0, layer = 0;
  Gemv g{nullptr, 0, 0};
  const float* norm_w = nullptr;  // B = RMS_NORM(x) * norm_w on load, or
  const uint16_t* act = nullptr;  // B = this bf16 activation [M][K]
};

// phase p of a step: layer p/5, {qkv, attention, attn_output, gate/up, down}; then lm_head
__device__ __forceinline__ Phase phase_of(const PdkArgs& a, int p) {
  Phase ph;
  const int h = a.h, ff = a.ff;
  if (p >= 5 * a.n_layer) {
    if (a.head) {
      ph.kind = PH_GEMV; ph.epi = E_LOGITS; ph.g = Gemv{a.output, h, a.n_vocab / 16}; ph.norm_w = a.out_norm;
    }
    return ph;
  }
  const int layer = p / 5, k = p % 5;
  const PdkLayer& L = a.layers[layer];
  ph.layer = layer;
  ph.kind = PH_GEMV;
  switch (k) {
    case 0: ph.epi = E_QKV; ph.g = Gemv{L.qkv, h, (h + 2 * a.kv) / 16}; ph.norm_w = L.attn_norm; break;
    case 1: ph.kind = PH_ATTN; break;
    case 2: ph.epi = E_RESID; ph.g = Gemv{L.o, h, h / 16}; ph.act = a.attn_out; break;
    case 3: ph.epi = E_SWIGLU; ph.g = Gemv{L.gu, h, 2 * ff / 16}; ph.norm_w = L.ffn_norm; break;
    default: ph.epi = E_RESID; ph.g = Gemv{L.down, ff, h / 16}; ph.act = a.act; break;
  }
  return ph;
}

template <int D, int G>
__global__ __launch_bounds__(PDK_WAVES * 64, 1) void pdk_kernel(PdkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // the wave index is wave-uniform: readfirstlane makes the compiler keep everything derived from it in SGPRs
  Ctx c{a, smem, (int)(threadIdx.x & 63), __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), (int)blockIdx.x,
        (int)gridDim.x, 0u, 0};
  Ring ring;
  ring.primed = false;
  const int h = a.h;
  // this work-group's residual rows (attn_output / ffn_down tiles g, g+G, ...: only it writes them)
  const int ntx = (h / 16 > c.g) ? (h / 16 - c.g + c.G - 1) / c.G : 0;
  if (c.w == 0) {
    for (int i = 0; i < ntx; ++i) {
      const int t = c.g + i * c.G, col = c.lane & 15;
      if (col < a.M)
        reinterpret_cast<f32x4*>(smem + LDS_XK)[i * 64 + c.lane] =
            *reinterpret_cast<const f32x4*>(a.x + (size_t)col * h + t * 16 + (c.lane >> 4) * 4);
    }
  }
  uint16_t* img = reinterpret_cast<uint16_t*>(smem + LDS_UNION) + (size_t)c.w * a.M * a.img_pitch;
  // one flat loop over the step's phases keeps a single copy of each phase's code (register
  // allocation sees one GEMV loop, one image builder, one attention)
  const int nphase = 5 * a.n_layer + (a.head ? 1 : 0);
  AttnRegs<D> ar;
  for (int p = 0; p < nphase; ++p) {
    if (a.trace && threadIdx.x == 64) a.trace[((size_t)c.g * nphase + p) * 3] = wall_clock64();
    const Phase ph = phase_of(a, p);
    int q = p + 1;  // next GEMV phase (weights to prefetch): attention has none, skip it
    if (q < 5 * a.n_layer && q % 5 == 1) ++q;
    const Phase nx = q < nphase ? phase_of(a, q) : Phase{};
    const Gemv* nxg = nx.kind == PH_GEMV ? &nx.g : nullptr;
    if (ph.kind == PH_ATTN) {
      attention<D, G>(c, ph.layer, ar);
    } else {
      const int KS = ph.g.K / NW;
      if (ph.norm_w) build_xs(c, ph.norm_w, img, a.img_pitch, KS);
      else build_act(c, ph.act, ph.g.K, img, a.img_pitch, KS);
      if (a.trace && threadIdx.x == 64) {
        __builtin_amdgcn_s_waitcnt(0);
        a.trace[((size_t)c.g * nphase + p) * 3 + 1] = wall_clock64();
      }
      gemv_phase(c, ph.epi, ph.layer, ph.g, nxg, ring, img, a.img_pitch);
    }
    if (a.trace && threadIdx.x == 64) a.trace[((size_t)c.g * nphase + p) * 3 + 2] = wall_clock64();
    if (p + 1 < nphase) {
      grid_arrive(c);
      prefill(c, ring, nxg);  // after the drain: these loads must not delay the arrival
      if (ph.kind == PH_GEMV && ph.epi == E_QKV) attn_prefetch<D>(c, ph.layer, ar);  // KV cache chunk
      if (!grid_wait(c)) return;
    }
  }
}

template <int D, int G>
int launch_pdk_dg(const PdkArgs& a, int grid, size_t lds, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&pdk_kernel<D, G>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -1;
    attr_set = true;
  }
  pdk_kernel<D, G><<<grid, PDK_WAVES * 64, lds, s>>>(a);
  return 0;
}

template <int D, int G>
int occupancy_dg(size_t lds) {
  int n = 0;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&pdk_kernel<D, G>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)lds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, pdk_kernel<D, G>, PDK_WAVES * 64, lds) != hipSuccess) return 0;
  return n;
}

}  // namespace

size_t pdk_lds_bytes(int M, int h, int ff, int n_head, int n_head_kv, int head_dim) {
  const int G = n_head / n_head_kv;
  const size_t img = (size_t)NW * M * pdk_pitch(h, ff) * 2;
  const size_t att = (size_t)NW * 16 * (ATTN_CHUNK + 8) * 2 + (size_t)NW * G * head_dim * 4 + 2 * NW * G * 4 +
                     2 * head_dim * 4;
  return LDS_UNION + (img > att ? img : att);
}

int pdk_pitch(int h, int ff) { return (h > ff ? h : ff) / NW + 8; }

// Shapes the kernel handles: every GEMV K-slice a whole number of ring groups, residual tiles
// within the LDS keep, head_dim 64/128 with GQA group 1..8, M <= PDK_MAX_M.
bool pdk_supported(int M, int h, int ff, int n_head, int n_head_kv, int head_dim, int n_vocab, int grid) {
  if (M < 1 || M > PDK_MAX_M || grid < 1) return false;
  const int G = n_head / n_head_kv;
  if ((head_dim != 64 && head_dim != 128) || (G != 1 && G != 2 && G != 4 && G != 8)) return false;
  auto slice_ok = [](int K) { const int nk = K / TILE_K / NW; return K % (TILE_K * NW) == 0 && (nk == 8 || nk == 16 || nk == 56); };
  if (!slice_ok(h) || !slice_ok(ff)) return false;  // gemv_phase's unrolled K-slices
  if (h / NW > 512 || h / 16 > 512) return false;  // build_xs: two 256-element pieces per lane
  if ((h / 16 + grid - 1) / grid > PDK_MAX_XT) return false;
  if (n_head_kv * M > grid || n_vocab % 16) return false;
  return pdk_lds_bytes(M, h, ff, n_head, n_head_kv, head_dim) <= 160 * 1024;
}

int pdk_occupancy(int head_dim, int G, size_t lds) {
  if (head_dim == 64) {
    switch (G) {
      case 1: return occupancy_dg<64, 1>(lds);
      case 2: return occupancy_dg<64, 2>(lds);
      case 4: return occupancy_dg<64, 4>(lds);
      case 8: return occupancy_dg<64, 8>(lds);
    }
  } else {
    switch (G) {
      case 1: return occupancy_dg<128, 1>(lds);
      case 2: return occupancy_dg<128, 2>(lds);
      case 4: return occupancy_dg<128, 4>(lds);
      case 8: return occupancy_dg<128, 8>(lds);
    }
  }
  return 0;
}

int launch_pdk(const PdkArgs& a, int grid, hipStream_t s) {
  const int G = a.n_head / a.n_head_kv;
  const size_t lds = pdk_lds_bytes(a.M, a.h, a.ff, a.n_head, a.n_head_kv, a.head_dim);
  if (hipMemsetAsync(a.sync, 0, PDK_SYNC_BYTES, s) != hipSuccess) return -1;
  if (a.head_dim == 64) {
    switch (G) {
      case 1: return launch_pdk_dg<64, 1>(a, grid, lds, s);
      case 2: return launch_pdk_dg<64, 2>(a, grid, lds, s);
      case 4: return launch_pdk_dg<64, 4>(a, grid, lds, s);
      case 8: return launch_pdk_dg<64, 8>(a, grid, lds, s);
    }
  } else {
    switch (G) {
      case 1: return launch_pdk_dg<128, 1>(a, grid, lds, s);
      case 2: return launch_pdk_dg<128, 2>(a, grid, lds, s);
      case 4: return launch_pdk_dg<128, 4>(a, grid, lds, s);
      case 8: return launch_pdk_dg<128, 8>(a, grid, lds, s);
    }
  }
  return -1;
}

}  // namespace mx
