// decode1.hip -- the one-token decode step of a bf16 model as ONE persistent launch (gfx950).
//
// Batch-1 decode streams every weight byte once per token; as one kernel per op (qkv, attention,
// attn_output, gate/up, down) each launch pays its ramp (first loads in flight) and drain, and the
// next op's weights start only after the previous op's last work-group: ~16 us of an 82 us Llama-3-8B
// layer.  Here every layer of the token runs in one launch of one 256-thread work-group
// per CU, and the weight stream never stops:
//
//   wave 0 (loader)      streams this CU's share of every matrix, layer after layer, through an LDS
//                        ring of NS 16 KiB slots by LDS-DMA (global_load_lds, nt), up to 3 slots in
//                        flight; a slot = 16 consecutive k-tiles of one 16-row tile (the packed tile
//                        layout makes it 16 KiB contiguous).  It never waits for a hand-off: only for
//                        a free slot.  So while the consumers wait for the previous op's outputs, the
//                        ring fills with the next op's weights (what a kernel boundary cannot do).
//   waves 1-3 (consumers) per op: gather the op's input vector written by other CUs (write-through
//                        loads), RMS_NORM it where ggml does, then for each of this CU's items (row
//                        tile x k-range) multiply the ring's slots on the MFMA (v_mfma_f32_16x16x32_bf16,
//                        the token in B column 0; the three waves split each slot's 16 k-tiles and
//                        their partial tiles meet in LDS), and publish the op's outputs write-through.
//
// Hand-offs between CUs (every op needs all of the previous op's outputs) are 8-byte granules
// {value, tag}: the producer writes each with ONE write-through (sc1) 8-byte store, the consumer
// re-reads its granules with sc1 loads until every tag is the expected one -- the data is the flag,
// no drain, counter or fence (cdna_hip_programming.md Guideline 16, R2).  tag = (calls << 9) + 5 layer
// + op + 1, with `calls` a device counter the last work-group of each call bumps, so buffers are never
// reset.  Every spin is bounded (200 ms): a timeout sets D1Args.err and the launch ends early (the
// engine reports it and falls back to the per-op kernels).
//
// Per layer: QKV (q|k|v tiles, split-K ks ways, partials) -> ATT (work-groups 0..n_head_kv-1: the
// decode attention body of kernels.hip on the three consumer waves, finishing q/k/v from the
// partials: sum, RoPE, K/V store) -> WO (x += attn.Wo) -> GU (SwiGLU of the ffn-normed x) -> DOWN
// (x += h.Wd).  The last layer also writes x and its per-16 sums of squares for the head kernels.
// Arithmetic = the per-op kernels': bf16 weights and activations, f32 accumulation, RMS_NORM with a
// double sum, the same attention body.
#include <hip/hip_runtime.h>

#include "attn_body.h"

namespace mx {

namespace {

typedef __attribute__((address_space(1))) const void d1_gvoid;
typedef __attribute__((address_space(3))) void d1_lvoid;

// consumer waves (1..3): k-tiles c, c+3, ... of each 16-k-tile slot.  Four waves per work-group =
// one per SIMD, so a wave may hold 512 VGPRs (the attention body needs ~250); a fifth wave halves that
// budget and spilled 120 B per lane
constexpr int D1_CONS = 3;
static_assert(D1_CONS == D1_TRACE_CONS, "trace rows hold the attention stamps of D1_CONS waves");
constexpr int D1_KPW = (16 + D1_CONS - 1) / D1_CONS;  // k-tiles per consumer wave and slot (6, 5, 5)
constexpr int SLOT_BYTES = 16384;   // 16 k-tiles of one 16-row tile
constexpr int SLOT_KT = 16;
constexpr int MAX_INFLIGHT = 3;     // slots issued and not yet landed (vmcnt <= 48 < 63)
constexpr unsigned long long D1_TIMEOUT = 20000000ull;  // 200 ms of s_memrealtime (100 MHz)
enum { PH_QKV = 0, PH_ATT = 1, PH_WO = 2, PH_GU = 3, PH_DOWN = 4, NPH = 5 };

struct PhaseDesc {
  const uint8_t* W;
  int T, KT, ks;  // row tiles, k-tiles of a whole row, k-split ways
};

// the matrices with weights, in stream order: 0 QKV, 1 WO, 2 GU, 3 DOWN.  Their base pointers come
// from an LDS copy of the layer table (wtab[4 l + p]): a global load there would be counted by the
// loader's vmcnt behind its LDS-DMA stream, and waiting for it (in-order counter) drains the ring.
__device__ __forceinline__ PhaseDesc phase_desc(const D1Args& a, const uint64_t* wtab, int l, int p) {
  const uint8_t* W = reinterpret_cast<const uint8_t*>(wtab[4 * l + p]);
  switch (p) {
    case 0: return {W, (a.h + 2 * a.kv) / 16, a.h / 32, a.ks_qkv};
    case 1: return {W, a.h / 16, a.h / 32, a.ks_o};
    case 2: return {W, 2 * a.ff / 16, a.h / 32, 1};
    default: return {W, a.h / 16, a.ff / 32, a.ks_d};
  }
}

// items (row tile x k-part) of one phase owned by work-group g of G: a contiguous range
__device__ __forceinline__ void item_range(int n_items, int g, int G, int& i0, int& i1) {
  i0 = (int)((long long)n_items * g / G);
  i1 = (int)((long long)n_items * (g + 1) / G);
}
// the slots [s0, s1) of a whole row's KT/16 that k-part kp of ks covers (parts differ by <= 1 slot)
__device__ __forceinline__ void part_slots(const PhaseDesc& d, int kp, int& s0, int& s1) {
  const int ns = d.KT / SLOT_KT;
  s0 = kp * ns / d.ks;
  s1 = (kp + 1) * ns / d.ks;
}

struct Ctl {  // LDS control words
  unsigned full[8];   // slot s holds stream slot (value - 1)
  unsigned freed[8];  // consumer releases of slot s (D1_CONS per fill)
  unsigned cbar;      // consumer-wave barrier
  unsigned abort;
  double dpart[D1_CONS];
};

__device__ __forceinline__ bool timed_out(unsigned long long deadline) {
  return __builtin_amdgcn_s_memrealtime() > deadline;
}

// one 1 KiB wave-load into LDS (global_load_lds_dwordx4, nt) as inline asm: hipcc does not model it,
// so it neither counts it (the loader's own vm_wait_slots does) nor fences every LDS access of the wave
// behind it with vmcnt(0) -- which it does for the builtin (it cannot tell the DMA's LDS bytes from
// the ring's control words) and which drained the ring after every slot
__device__ __forceinline__ void glds16_nt(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

__device__ __forceinline__ void vm_wait_slots(int n) {  // vmcnt <= 16 n (n slots of 16 loads still in flight)
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
}

// ---------------------------------------------------------------------------------------- loader
// NL loader waves; wave k streams the slots k, k + NL, k + 2 NL, ... of the work-group's stream, up to
// MAX_INFLIGHT of them in flight (vmcnt counts at most 63 loads per wave: NL waves put NL x 48 KiB in
// flight per CU)
template <int NS, int NL>
__device__ void d1_loader(const D1Args& a, const uint64_t* wtab, uint8_t* ring, Ctl* ctl, unsigned long long deadline) {
  const int lane = threadIdx.x & 63, k = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int g = blockIdx.x, G = gridDim.x;
  // slots of one layer for this work-group (the same every layer)
  int per_layer = 0;
  for (int p = 0; p < 4; ++p) {
    const PhaseDesc d = phase_desc(a, wtab, 0, p);
    int i0, i1;
    item_range(d.T * d.ks, g, G, i0, i1);
    for (int it = i0; it < i1; ++it) {
      int s0, s1;
      part_slots(d, it % d.ks, s0, s1);
      per_layer += s1 - s0;
    }
  }
  const int total = per_layer * a.n_layer;
  // stream cursor (at slot `cur`)
  int l = 0, p = 0, it = 0, it1 = 0, j = 0, s0 = 0, s1 = 1, cur = 0;
  PhaseDesc d{};
  auto open_phase = [&]() {
    for (;;) {
      d = phase_desc(a, wtab, l, p);
      item_range(d.T * d.ks, g, G, it, it1);
      j = 0;
      if (it < it1) {
        part_slots(d, it % d.ks, s0, s1);
        return;
      }
      if (++p == 4) {
        p = 0;
        if (++l == a.n_layer) return;
      }
    }
  };
  auto advance = [&]() {  // cursor to the next slot of the stream
    ++cur;
    if (++j == s1 - s0) {  // next item / phase / layer
      j = 0;
      if (++it == it1) {
        if (++p == 4) {
          p = 0;
          ++l;
        }
        if (l < a.n_layer) open_phase();
      } else {
        part_slots(d, it % d.ks, s0, s1);
      }
    }
  };
  if (total > 0) open_phase();
  for (int i = 0; i < k && cur < total; ++i) advance();
  int issued = k, published = k, inflight = 0;  // this wave's next slot to issue / to publish
  unsigned long long t_vm = 0, t_idle = 0;
  unsigned long long* tr =
      a.trace && k == 0 ? a.trace + (size_t)g * d1_trace_stride(a.n_layer) + a.n_layer * 10 : nullptr;
  while (published < total) {
    if (issued < total && inflight < MAX_INFLIGHT) {
      const int s = issued % NS;
      const unsigned need = (unsigned)(D1_CONS * (issued / NS));
      if (__hip_atomic_load(&ctl->freed[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) {
        const int tile = it / d.ks, kt0 = (s0 + j) * SLOT_KT;
        const uint8_t* src = d.W + ((size_t)tile * d.KT + kt0) * 1024 + lane * 16;
        const unsigned dst = __builtin_amdgcn_readfirstlane(
            (unsigned)reinterpret_cast<uintptr_t>(ring) + (unsigned)(s * SLOT_BYTES));
#pragma unroll
        for (int c = 0; c < SLOT_KT; ++c) glds16_nt(src + c * 1024, dst + c * 1024);
        issued += NL;
        ++inflight;
        for (int i = 0; i < NL && cur < total; ++i) advance();
        continue;
      }
    }
    if (inflight > 0) {  // this wave's oldest slot in flight: wait for it, publish it
      const unsigned long long t0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
      vm_wait_slots(inflight - 1);
      if (tr) t_vm += __builtin_amdgcn_s_memrealtime() - t0;
      asm volatile("" ::: "memory");
      __hip_atomic_store(&ctl->full[published % NS], (unsigned)(published + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
      published += NL;
      --inflight;
      continue;
    }
    // nothing in flight and the next slot still in use: the consumers wait for a hand-off
    const unsigned long long t1 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    __builtin_amdgcn_s_sleep(1);
    if (tr) t_idle += __builtin_amdgcn_s_memrealtime() - t1;
    if (__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) || timed_out(deadline)) {
      __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tr && lane == 0) {
    tr[2] = t_idle;
    tr[3] = t_vm;
    tr[4] = __builtin_amdgcn_s_memrealtime();
  }
}

// ------------------------------------------------------------------------------------- consumers
struct Cons {
  const D1Args& a;
  Ctl* ctl;
  unsigned long long deadline;
  int cw, lane, tid;  // consumer wave 0..2, lane, thread 0..191
  unsigned long long* tr = nullptr;  // this work-group's trace row (consumer wave 0, lane 0 writes)
  unsigned long long t_full = 0;
  __device__ void stamp(int k) {
    if (tr && cw == 0 && lane == 0) tr[k] = __builtin_amdgcn_s_memrealtime();
  }
  unsigned gen = 0;   // consumer-barrier generation
  bool dead = false;

  __device__ Cons(const D1Args& a_, Ctl* c, unsigned long long dl, int nl)
      : a(a_), ctl(c), deadline(dl) {
    tid = (int)threadIdx.x - 64 * nl;
    cw = __builtin_amdgcn_readfirstlane(tid >> 6);
    lane = tid & 63;
  }
  __device__ bool check() {
    if (__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) || timed_out(deadline)) {
      __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      dead = true;
    }
    return dead;
  }
  // barrier of the consumer waves (LDS counter; the loader never joins)
  __device__ void sync() {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    ++gen;
    if (lane == 0) __hip_atomic_fetch_add(&ctl->cbar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&ctl->cbar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < D1_CONS * gen) {
      __builtin_amdgcn_s_sleep(0);
      if (check()) return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // wait until counter c reaches target (consumer wave 0 polls; the others meet it at the barrier)
  __device__ void wait_ctr(const unsigned* c, unsigned target) {
    if (cw == 0) {
      if (lane == 0) {
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (check()) {
            atomicOr(a.err, 1u);
            break;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    sync();
  }
  // this work-group's stores of the op are done: every consumer wave drains, then one arrival
  __device__ void arrive(unsigned* c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sync();
    if (cw == 0 && lane == 0 && !dead) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

template <int D, int G>
struct AttnSync {
  Cons* c;
  __device__ void operator()() const { c->sync(); }
};
struct AttnGive {  // the attention body's granule sweep asks whether to give up
  Cons* c;
  __device__ void operator()() const {}
  __device__ bool dead(int spin) const { return (spin & 63) == 63 && c->check(); }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Gathers: granule sweeps.  Each thread issues all its 16-byte sc1 loads (2 granules each) before it
// looks at any (a load-use loop waits one round trip per iteration), and re-reads a batch until every
// tag is the expected one.  GS 16-byte loads per thread and batch: 192 threads x GS x 16 B, so a
// Llama-3-8B x hand-off (32 KiB, GS 12) is ONE batch -- one round trip after the last producer's
// stores land -- and its SwiGLU product (56 KiB, GS 18) two, where batches of 8 loads took 2-3
// (profiles/round4_decode1_trace.txt).  Loads past the end are not issued (their tags count as
// matching).
constexpr int GU_ = 8;   // norm-weight prefetch per thread (f32x4)
template <int GS, bool TWO, class Put>
__device__ __forceinline__ void sweep(Cons& C, const unsigned long long* gran, int n, unsigned tag, Put put) {
  // two arrays (of ceil and floor GS/2; more than ~18 u32x4 in all were demoted to scratch).  TWO: the
  // granules of two K-parts of n each, the same indices of both in one thread (v0: part 0, v1: part 1)
  constexpr int H0 = TWO ? GS / 2 : (GS + 1) / 2, H1 = GS / 2;
  static_assert(GS <= 18, "gather batch");
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(gran, (size_t)n * (TWO ? 16 : 8));
  const int nv = n / 2;  // 16-byte pairs (of one part)
  constexpr int ST = 64 * D1_CONS, STEP = TWO ? ST * H0 : ST * GS;
  for (int b = C.tid; b < nv && !C.dead; b += STEP) {
    u32x4 v0[H0], v1[H1];
    for (int spin = 0;; ++spin) {
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int i = b + u * ST;
        v0[u] = i < nv ? __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(i * 16), 0, 16 /* sc1 */))
                       : u32x4{0u, tag, 0u, tag};
      }
#pragma unroll
      for (int u = 0; u < H1; ++u) {
        const int j = TWO ? b + u * ST : b + (H0 + u) * ST;
        const unsigned off = (unsigned)((TWO ? j + nv : j) * 16);
        v1[u] = j < nv ? __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /* sc1 */))
                       : u32x4{0u, tag, 0u, tag};
      }
      bool ok = true;
#pragma unroll
      for (int u = 0; u < H0; ++u) ok &= v0[u][1] == tag && v0[u][3] == tag;
#pragma unroll
      for (int u = 0; u < H1; ++u) ok &= v1[u][1] == tag && v1[u][3] == tag;
      if (ok) break;
      __builtin_amdgcn_s_sleep(1);
      if ((spin & 63) == 63 && C.check()) return;
    }
    if constexpr (TWO) {
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int i = b + u * ST;
        if (i < nv) put(i, v0[u][0], v0[u][2], v1[u][0], v1[u][2]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int i = b + u * ST;
        if (i < nv) put(i, v0[u][0], v0[u][2], 0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < H1; ++u) {
        const int j = b + (H0 + u) * ST;
        if (j < nv) put(j, v1[u][0], v1[u][2], 0u, 0u);
      }
    }
  }
}
// xf = the residual stream (f32 granules; `parts` = 2: the two K-parts summed, part 0 + part 1, in
// one sweep); returns this thread's share of sum(x^2) in double
__device__ __forceinline__ double gather_x(Cons& C, float* xf, const unsigned long long* gran, int n, unsigned tag,
                                           int parts = 1) {
  double q = 0.0;
  if (parts == 1) {
    sweep<12, false>(C, gran, n, tag, [&](int i, unsigned a0, unsigned a1, unsigned, unsigned) {
      const float x0 = __uint_as_float(a0), x1 = __uint_as_float(a1);
      *reinterpret_cast<float2*>(xf + 2 * i) = float2{x0, x1};
      q += (double)(x0 * x0) + (double)(x1 * x1);
    });
  } else {
    sweep<12, true>(C, gran, n, tag, [&](int i, unsigned a0, unsigned a1, unsigned b0, unsigned b1) {
      const float x0 = __uint_as_float(a0) + __uint_as_float(b0), x1 = __uint_as_float(a1) + __uint_as_float(b1);
      *reinterpret_cast<float2*>(xf + 2 * i) = float2{x0, x1};
      q += (double)(x0 * x0) + (double)(x1 * x1);
    });
  }
  return q;
}
// dst[0..2n) = bf16 pairs from n granules
__device__ __forceinline__ void gather_pairs(Cons& C, uint16_t* dst, const unsigned long long* gran, int n,
                                             unsigned tag) {
  sweep<18, false>(C, gran, n, tag, [&](int i, unsigned a0, unsigned a1, unsigned, unsigned) {
    *reinterpret_cast<u32x2*>(dst + 4 * i) = u32x2{a0, a1};
  });
}
__device__ __forceinline__ void put_gran(unsigned long long* g, unsigned tag, unsigned bits) {
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// act = bf16((x * 1/sqrt(mean(x^2) + eps)) * w) -- ggml's RMS_NORM + MUL, then the bf16 rounding
// of src1 for the bf16 MUL_MAT; q = this thread's share of sum(x^2) (double), reduced here in a fixed
// order (waves, then consumer waves 0, 1, 2)
// this thread's norm weights (issued before the hand-off sweep, so their round trip overlaps it)
struct NormW {
  f32x4 v[GU_];
};
__device__ __forceinline__ NormW norm_w_load(Cons& C, const float* w, int n) {
  NormW r;
  const int nv = n / 4;
#pragma unroll
  for (int u = 0; u < GU_; ++u) r.v[u] = *reinterpret_cast<const f32x4*>(w + 4 * min(C.tid + u * 64 * D1_CONS, nv - 1));
  return r;
}
__device__ __forceinline__ void rms_norm_act(Cons& C, double q, const float* xf, const float* w, uint16_t* act,
                                             int n, float eps, const NormW* pre = nullptr) {
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  if (C.lane == 0) C.ctl->dpart[C.cw] = q;
  C.sync();
  double tot = C.ctl->dpart[0];
#pragma unroll
  for (int w = 1; w < D1_CONS; ++w) tot += C.ctl->dpart[w];
  const float scale = 1.0f / sqrtf((float)(tot / n) + eps);
  const int nv = n / 4;
  for (int b = C.tid; b < nv; b += 64 * D1_CONS * GU_) {
    f32x4 wv[GU_];
    if (pre && b == C.tid) {
#pragma unroll
      for (int u = 0; u < GU_; ++u) wv[u] = pre->v[u];
    } else {
#pragma unroll
      for (int u = 0; u < GU_; ++u) wv[u] = *reinterpret_cast<const f32x4*>(w + 4 * min(b + u * 64 * D1_CONS, nv - 1));
    }
#pragma unroll
    for (int u = 0; u < GU_; ++u) {
      const int i = b + u * 64 * D1_CONS;
      if (i < nv) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(xf + 4 * i);
        u32x2 o;
        o[0] = f2bf((xv[0] * scale) * wv[u][0]) | (f2bf((xv[1] * scale) * wv[u][1]) << 16);
        o[1] = f2bf((xv[2] * scale) * wv[u][2]) | (f2bf((xv[3] * scale) * wv[u][3]) << 16);
        *reinterpret_cast<u32x2*>(act + 4 * i) = o;
      }
    }
  }
}

// one phase's items on the MFMA: acc over this wave's k-tiles of every slot, the consumer waves'
// partial tiles summed (wave order) in LDS, then epi(tile, kpart, lane q of 0..3, rows 4q..4q+3)
template <int NS, class Epi>
__device__ __forceinline__ void run_items(Cons& C, const PhaseDesc& d, const uint8_t* ring, const uint16_t* act,
                                          float (*red)[D1_CONS][16], int& seq, int& item_par, Epi epi) {
  int i0, i1;
  item_range(d.T * d.ks, blockIdx.x, gridDim.x, i0, i1);
  const int lane = C.lane;
  for (int it = i0; it < i1; ++it) {
    const int tile = it / d.ks, kp = it % d.ks;
    int s0, s1;
    part_slots(d, kp, s0, s1);
    const int nsl = s1 - s0, ktb = s0 * SLOT_KT;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f}, acc2 = acc;
    for (int j = 0; j < nsl; ++j) {
      const int s = seq % NS;
      const unsigned long long tw = C.tr ? __builtin_amdgcn_s_memrealtime() : 0;
      while (__hip_atomic_load(&C.ctl->full[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (unsigned)(seq + 1)) {
        __builtin_amdgcn_s_sleep(0);
        if (C.check()) return;
      }
      if (C.tr) C.t_full += __builtin_amdgcn_s_memrealtime() - tw;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const uint8_t* base = ring + s * SLOT_BYTES;
      // this wave's k-tiles cw, cw+4, cw+8, cw+12 of the slot: all LDS reads first, then the MFMAs
      // into two accumulators (no MFMA waits for the one before it)
      u32x4 av[D1_KPW], bv[D1_KPW];
#pragma unroll
      for (int k = 0; k < D1_KPW; ++k) {
        const int c = min(C.cw + k * D1_CONS, SLOT_KT - 1);  // the last one of waves 1, 2 is a repeat
        av[k] = *reinterpret_cast<const u32x4*>(base + c * 1024 + lane * 16);
        bv[k] = *reinterpret_cast<const u32x4*>(act + (ktb + j * SLOT_KT + c) * 32 + 8 * (lane >> 4));
      }
#pragma unroll
      for (int k = 0; k < D1_KPW; ++k) {
        const bool live = C.cw + k * D1_CONS < SLOT_KT && (lane & 15) == 0;
        const u32x4 b = live ? bv[k] : u32x4{0u, 0u, 0u, 0u};  // the token is B column 0
        if (k & 1)
          acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[k]), __builtin_bit_cast(bf16x8, b),
                                                         acc2, 0, 0, 0);
        else
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[k]), __builtin_bit_cast(bf16x8, b),
                                                        acc, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of the slot are done
      if (lane == 0) __hip_atomic_fetch_add(&C.ctl->freed[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      ++seq;
    }
    acc += acc2;
    // C column 0: lanes 0, 16, 32, 48 hold rows 4(l>>4)..+3
    float (*rb)[16] = red[item_par & 1];
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) rb[C.cw][4 * (lane >> 4) + i] = acc[i];
    }
    C.sync();
    if (C.dead) return;
    if (C.cw == 0 && lane < 4) {
      f32x4 s = *reinterpret_cast<const f32x4*>(&rb[0][4 * lane]);
#pragma unroll
      for (int w = 1; w < D1_CONS; ++w) s += *reinterpret_cast<const f32x4*>(&rb[w][4 * lane]);
      epi(tile, kp, lane, s, rb);
    }
    ++item_par;
  }
}

template <int D, int G, int NS, int NL>
__global__ __launch_bounds__(64 * (NL + D1_CONS), 1) void decode1_kernel(D1Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t d1_lds[];
  uint8_t* ring = d1_lds;
  float* xf = reinterpret_cast<float*>(d1_lds + NS * SLOT_BYTES);
  uint16_t* act = reinterpret_cast<uint16_t*>(xf + a.h);
  const int amax = a.h > a.ff ? a.h : a.ff;
  float (*red)[D1_CONS][16] = reinterpret_cast<float (*)[D1_CONS][16]>(act + amax);
  Ctl* ctl = reinterpret_cast<Ctl*>(reinterpret_cast<uint8_t*>(red) + 2 * D1_CONS * 16 * 4);
  uint64_t* wtab = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(ctl) + sizeof(Ctl));
  for (int i = threadIdx.x; i < 4 * a.n_layer; i += 64 * (NL + D1_CONS)) {
    const D1Layer& L = a.layers[i >> 2];
    const uint16_t* w = (i & 3) == 0 ? L.qkv : (i & 3) == 1 ? L.o : (i & 3) == 2 ? L.gu : L.down;
    wtab[i] = reinterpret_cast<uint64_t>(w);
  }

  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + D1_TIMEOUT;
  if (threadIdx.x < 18) reinterpret_cast<unsigned*>(ctl)[threadIdx.x] = 0u;  // full, freed, cbar, abort
  __syncthreads();  // the only full-work-group barrier: before the roles split

  if (threadIdx.x < 64 * NL) {
    d1_loader<NS, NL>(a, wtab, ring, ctl, deadline);
    return;
  }
  Cons C(a, ctl, deadline, NL);
  const int g = blockIdx.x, Gn = gridDim.x;
  if (a.trace) C.tr = a.trace + (size_t)g * d1_trace_stride(a.n_layer);
  C.stamp(a.n_layer * 10 + 0);
  const unsigned calls = __hip_atomic_load(a.ctr + a.n_layer * NPH + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto tag = [&](int l, int p) { return (calls << 9) + (unsigned)(l * NPH + p + 1); };
  const int h = a.h, ff = a.ff, Nq = a.h + 2 * a.kv;
  int seq = 0, item_par = 0;

  for (int l = 0; l < a.n_layer && !C.dead; ++l) {
    const D1Layer& L = a.layers[l];
    double q = 0.0;
    // ---------------- QKV: x -> attn_norm -> q|k|v partials
    if (l == 0) {
      if (a.tok_embd) {
        const int id = a.ids[0];
        const uint16_t* er = a.tok_embd + (size_t)id * h;
        for (int i = C.tid; i < h / 2; i += 64 * D1_CONS) {
          const uint32_t v = *reinterpret_cast<const uint32_t*>(er + 2 * i);
          const float x0 = bf2f(v & 0xffffu), x1 = bf2f(v >> 16);
          xf[2 * i] = x0;
          xf[2 * i + 1] = x1;
          q += (double)(x0 * x0) + (double)(x1 * x1);
        }
      } else {
        for (int i = C.tid; i < h / 4; i += 64 * D1_CONS) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(a.x_in + 4 * i);
          *reinterpret_cast<f32x4*>(xf + 4 * i) = v;
#pragma unroll
          for (int j = 0; j < 4; ++j) q += (double)(v[j] * v[j]);
        }
      }
      rms_norm_act(C, q, xf, L.attn_norm, act, h, a.eps);
    } else {
      const NormW nw = norm_w_load(C, L.attn_norm, h);
      q = gather_x(C, xf, a.xs, h, tag(l - 1, PH_DOWN), a.ks_d);
      rms_norm_act(C, q, xf, L.attn_norm, act, h, a.eps, &nw);
    }
    C.sync();
    if (C.dead) break;
    C.stamp(l * 10 + 0);
    const unsigned t_qkv = tag(l, PH_QKV);
    run_items<NS>(C, phase_desc(a, wtab, l, 0), ring, act, red, seq, item_par,
                  [&](int tile, int kp, int qd, f32x4 s, float (*)[16]) {
                    unsigned long long* gp = a.qkvp + (size_t)kp * Nq + tile * 16 + 4 * qd;
#pragma unroll
                    for (int i = 0; i < 4; ++i) put_gran(gp + i, t_qkv, __float_as_uint(s[i]));
                  });
    C.sync();  // wave 0's epilogue done with red / xf before anyone overwrites LDS
    C.stamp(l * 10 + 1);
    // ---------------- ATT: work-groups 0..n_head_kv-1, one kv head each
    if (g < a.n_head_kv) {
      C.stamp(l * 10 + 2);
      AttnArgs at{};
      at.kc = L.kc; at.vc = L.vc; at.kc_w = L.kc; at.vc_w = L.vc;
      at.pos = a.pos; at.slot = a.slot;
      at.ldo = h; at.M = 1;
      at.n_head = a.n_head; at.n_head_kv = a.n_head_kv; at.head_dim = D;
      at.n_ctx = a.n_ctx; at.ctx_stride = a.ctx_stride; at.slot_stride = a.slot_stride;
      at.scale = a.scale;
      at.nslab = a.ks_qkv; at.slab_stride = (size_t)Nq; at.rope_cs = a.rope_cs;
      at.gslab = a.qkvp; at.gtag_in = t_qkv; at.gout = a.attn; at.gtag_out = tag(l, PH_ATT);
      at.slabs = reinterpret_cast<const float*>(a.qkvp);  // FIN path marker (granules are read)
      if (C.tr)  // the body's stamps of wave w land in this row's words n_layer * 10 + 8 + 8 w
        at.trace = C.tr + a.n_layer * 10 + 8 - (size_t)g * D1_CONS * 8;
      attn_decode_body<D, G, D1_CONS, true, true>(at, g, 0, C.tid, AttnSync<D, G>{&C}, AttnGive{&C});
      C.sync();
      if (C.dead) break;
      C.stamp(l * 10 + 3);
    }
    // ---------------- WO: x += attn . Wo
    gather_pairs(C, act, a.attn, h / 2, tag(l, PH_ATT));
    C.sync();
    if (C.dead) break;
    C.stamp(l * 10 + 4);
    const unsigned t_wo = tag(l, PH_WO);
    run_items<NS>(C, phase_desc(a, wtab, l, 1), ring, act, red, seq, item_par,
                  [&](int tile, int kp, int qd, f32x4 s, float (*)[16]) {
                    const int row = tile * 16 + 4 * qd;
                    const f32x4 xn = kp ? s : *reinterpret_cast<const f32x4*>(xf + row) + s;  // part 0 + residual
#pragma unroll
                    for (int i = 0; i < 4; ++i) put_gran(a.xs + kp * h + row + i, t_wo, __float_as_uint(xn[i]));
                  });
    C.sync();
    C.stamp(l * 10 + 5);
    // ---------------- GU: h = silu(x_n . Wg) * (x_n . Wu)
    const NormW nw2 = norm_w_load(C, L.ffn_norm, h);
    q = gather_x(C, xf, a.xs, h, t_wo, a.ks_o);
    rms_norm_act(C, q, xf, L.ffn_norm, act, h, a.eps, &nw2);
    C.sync();
    if (C.dead) break;
    C.stamp(l * 10 + 6);
    const unsigned t_gu = tag(l, PH_GU);
    run_items<NS>(C, phase_desc(a, wtab, l, 2), ring, act, red, seq, item_par,
                  [&](int tile, int, int qd, f32x4 s, float (*rb)[16]) {
                    if (qd >= 2) return;  // lanes 0, 1: gate rows 4qd..4qd+3 with up rows 8+4qd..
                    f32x4 u = *reinterpret_cast<const f32x4*>(&rb[0][8 + 4 * qd]);
#pragma unroll
                    for (int w = 1; w < D1_CONS; ++w) u += *reinterpret_cast<const f32x4*>(&rb[w][8 + 4 * qd]);
                    float f[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) f[i] = (s[i] / (1.0f + expf(-s[i]))) * u[i];
                    unsigned long long* gp = a.hb + (tile * 8 + 4 * qd) / 2;
                    put_gran(gp, t_gu, f2bf(f[0]) | (f2bf(f[1]) << 16));
                    put_gran(gp + 1, t_gu, f2bf(f[2]) | (f2bf(f[3]) << 16));
                  });
    C.sync();
    C.stamp(l * 10 + 7);
    // ---------------- DOWN: x += h . Wd
    gather_pairs(C, act, a.hb, ff / 2, t_gu);
    C.sync();
    if (C.dead) break;
    C.stamp(l * 10 + 8);
    const unsigned t_dn = tag(l, PH_DOWN);
    const bool last = l == a.n_layer - 1;
    run_items<NS>(C, phase_desc(a, wtab, l, 3), ring, act, red, seq, item_par,
                  [&](int tile, int kp, int qd, f32x4 s, float (*)[16]) {
                    const int row = tile * 16 + 4 * qd;
                    const f32x4 xn = kp ? s : *reinterpret_cast<const f32x4*>(xf + row) + s;  // part 0 + residual
#pragma unroll
                    for (int i = 0; i < 4; ++i) put_gran(a.xs + kp * h + row + i, t_dn, __float_as_uint(xn[i]));
                    if (last && a.ks_d == 1) {  // the head's inputs: x and the per-16 sums of squares
                      *reinterpret_cast<f32x4*>(a.x_out + row) = xn;
                      double qq = 0.0;
#pragma unroll
                      for (int i = 0; i < 4; ++i) qq += (double)(xn[i] * xn[i]);
                      qq += __shfl_xor(qq, 1);
                      qq += __shfl_xor(qq, 2);
                      if (qd == 0 && a.ssq) a.ssq[tile] = (float)qq;
                    }
                  });
    C.sync();
    C.stamp(l * 10 + 9);
  }
  if (!C.dead && a.ks_d > 1 && g < h / 16 && C.cw == 0 && C.lane < 16) {
    // the last layer's x in two K-parts: tile g's 16 rows summed (part order, as the gathers do) for
    // the head kernels, with their sum of squares
    const int row = g * 16 + C.lane;
    const unsigned t_last = tag(a.n_layer - 1, PH_DOWN);
    unsigned long long v0, v1;
    for (int spin = 0;; ++spin) {
      v0 = __hip_atomic_load(a.xs + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v1 = __hip_atomic_load(a.xs + h + row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(v0 >> 32) == t_last && (unsigned)(v1 >> 32) == t_last) break;
      __builtin_amdgcn_s_sleep(1);
      if ((spin & 63) == 63 && timed_out(deadline)) {
        atomicOr(a.err, 4u);
        break;
      }
    }
    const float x = __uint_as_float((unsigned)v0) + __uint_as_float((unsigned)v1);
    a.x_out[row] = x;
    double qq = (double)(x * x);
    for (int o = 8; o > 0; o >>= 1) qq += __shfl_xor(qq, o);
    if (C.lane == 0 && a.ssq) a.ssq[g] = (float)qq;
  }
  C.stamp(a.n_layer * 10 + 1);
  if (C.tr && C.cw == 0 && C.lane == 0) C.tr[a.n_layer * 10 + 5] = C.t_full;
  if (C.dead) {
    if (C.lane == 0) atomicOr(a.err, 2u);
    return;
  }
  if (C.cw == 0 && C.lane == 0) {  // the last work-group of the call bumps `calls` (the next call's tags)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(a.ctr + a.n_layer * NPH, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (calls + 1u) * (unsigned)Gn - 1u)
      __hip_atomic_fetch_add(a.ctr + a.n_layer * NPH + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// static LDS of the attention body (its arrays) + our dynamic carve: ring, xf, act, red, ctl
template <int D, int G>
constexpr size_t attn_static_lds() {
  return (size_t)D1_CONS * 16 * (ATTN_CHUNK + 8) * 2 + (size_t)D1_CONS * G * D * 4 + 2 * D1_CONS * G * 4 +
         (size_t)(G * D + 2 * D) * 4;
}

size_t dyn_lds(int ns, int h, int ff, int n_layer) {
  return (size_t)ns * SLOT_BYTES + (size_t)h * 4 + (size_t)(h > ff ? h : ff) * 2 + 2 * D1_CONS * 16 * 4 + sizeof(Ctl) +
         (size_t)n_layer * 4 * 8;
}

template <int D, int G, int NS, int NL>
int launch_nsl(const D1Args& a, int n_cu, hipStream_t s, bool prepare) {
  const size_t lds = dyn_lds(NS, a.h, a.ff, a.n_layer);
  if (prepare)  // once, outside any stream capture: the dynamic LDS above 64 KiB
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&decode1_kernel<D, G, NS, NL>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess ? 0 : -1;
  decode1_kernel<D, G, NS, NL><<<n_cu, 64 * (NL + D1_CONS), lds, s>>>(a);
  return 0;
}
template <int D, int G, int NS>
int launch_ns(const D1Args& a, int n_cu, hipStream_t s, bool prepare) {
  // loader waves: one puts 48 KiB in flight per CU; MX_D1_LOADERS=2 puts 96 KiB, but its fifth wave
  // halves the VGPR budget (20 B/lane spilled at G 4) and measured slower in the steady state (8B 2.93
  // vs 2.88 ms per launch, TinyLlama 0.810 vs 0.804: profiles/round4_decode1_trace.txt)
  static const int nl = getenv("MX_D1_LOADERS") ? atoi(getenv("MX_D1_LOADERS")) : 1;
  if (nl != 2 || NS < 6) return launch_nsl<D, G, NS, 1>(a, n_cu, s, prepare);
  return launch_nsl<D, G, NS, 2>(a, n_cu, s, prepare);
}

template <int D, int G>
int launch_dg(const D1Args& a, int n_cu, hipStream_t s, bool prepare) {
  // as many ring slots as the 160 KiB of LDS leave (3..8)
  const size_t budget = 160 * 1024 - attn_static_lds<D, G>() - 256;
  int ns = 8;
  while (ns > 3 && dyn_lds(ns, a.h, a.ff, a.n_layer) > budget) --ns;
  if (dyn_lds(ns, a.h, a.ff, a.n_layer) > budget) return -1;
  if (ns >= 8) return launch_ns<D, G, 8>(a, n_cu, s, prepare);
  if (ns >= 6) return launch_ns<D, G, 6>(a, n_cu, s, prepare);
  return launch_ns<D, G, 3>(a, n_cu, s, prepare);
}

}  // namespace

size_t decode1_ctr_words(int n_layer) { return (size_t)n_layer * NPH + 2; }

bool decode1_supported(int h, int kv, int ff, int n_head, int n_head_kv, int head_dim) {
  if (h % 512 || ff % 512 || kv % 16 || n_head % n_head_kv) return false;  // whole 16-k-tile slots
  const int G = n_head / n_head_kv;
  if (!((head_dim == 128 && G == 4) || (head_dim == 64 && G == 8) || (head_dim == 128 && G == 8))) return false;
  return true;
}

int launch_decode1(const D1Args& a, int n_cu, hipStream_t s, bool prepare) {
  if (!decode1_supported(a.h, a.kv, a.ff, a.n_head, a.n_head_kv, a.head_dim) || a.ks_qkv < 1 ||
      a.ks_qkv > ATTN_MEGA_MAXSLAB || (a.h / 32 / a.ks_qkv) % SLOT_KT || n_cu < a.n_head_kv)
    return -1;
  const int G = a.n_head / a.n_head_kv;
  if (a.head_dim == 128 && G == 4) return launch_dg<128, 4>(a, n_cu, s, prepare);
  if (a.head_dim == 128 && G == 8) return launch_dg<128, 8>(a, n_cu, s, prepare);
  return launch_dg<64, 8>(a, n_cu, s, prepare);
}

}  // namespace mx
