// kernels.h -- launch interface of the gfx950 kernels (kernels.hip).
//
// Every kernel here replaces one ggml CPU op of llama.cpp's llm_build_llama
// (the forward pass behind /root/reference/llama_p2p_network.py:125; see
// SURVEY.md §3.3 and §8a rows a5-a14).  Host code calls only these wrappers.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mx {

// Weight matrices live in HBM as bf16 "MFMA tiles": tile (nt, kt) holds rows
// [16nt, 16nt+16) x cols [32kt, 32kt+32) of W[N][K] (GGUF order) in exactly the
// lane order of the A operand of v_mfma_f32_16x16x32_bf16, 1 KiB per tile,
// tiles ordered nt-major so a wave streaming along K reads contiguous 1 KiB
// pieces: element (lane, j) of tile = W[16nt + (lane&15)][32kt + 8(lane>>4) + j].
constexpr int TILE_N = 16;
constexpr int TILE_K = 32;
constexpr int TILE_ELEMS = TILE_N * TILE_K;
constexpr int MAX_ROWS = 64;       // tokens per decode / logits forward (4 column tiles of 16)
constexpr int PREFILL_ROWS = 4096;  // tokens per prefill forward (GEMM path, no logits): ~0.3 GB of activations for 8B
constexpr int ATTN_CHUNK = 32;     // positions per attention wave-iteration
constexpr int KV_POS_ALIGN = 64;   // KV rows per slot are allocated in multiples of this

enum Epilogue : int {
  EPI_F32 = 0,     // out[col][row] = acc                         (lm_head logits)
  EPI_RESID = 1,   // x[col][row] += acc                          (attn_output, ffn_down)
  EPI_QKV = 2,     // rope(q,k); q -> f32 buffer, k/v -> f16 KV cache (attn_q/k/v)
  EPI_SWIGLU = 3,  // act = bf16(silu(gate) * up); tile = 8 gate + 8 up rows (ffn_gate/ffn_up)
  EPI_SLAB = 4,    // split-K partial: out = slab[ksplit][col][row] (reduced by resid_norm / qkv_finish)
};

struct AttnArgs {
  const float* q;        // [M][n_head*head_dim] f32 (post-RoPE)
  const _Float16* kc;    // [slots][n_head_kv][ctx_stride * head_dim], 1 KiB B-operand tiles (kernels.hip)
  const _Float16* vc;    // [slots][n_head_kv][ctx_stride * head_dim], 1 KiB B-operand tiles
  const int* pos;        // [M]  query position; attends to [0, pos]
  const int* slot;       // [M]
  uint16_t* out;         // bf16 [M][ldo] (src1 of attn_output)
  int ldo;
  float* outf;           // f32 [M][ldo] instead of out (Q8_0 models quantise it next)
  int M, n_head, n_head_kv, head_dim, n_ctx, ctx_stride;
  size_t slot_stride;
  float scale;
  // qkv still as split-K partial slabs (wide path): the kernel sums them in slab order, applies
  // RoPE, stores this position's K/V into the caches and keeps q and the new K/V in LDS
  const float* slabs;    // [nslab][M][n_q + 2*n_kv] or nullptr (q / caches already final)
  int nslab;
  size_t slab_stride;
  const float* rope_cs;  // [n_ctx][head_dim/2][2]
  _Float16 *kc_w, *vc_w; // writable views of kc / vc
  // diagnosis only (mx_profile_kernel with MX_ATTN_TRACE): per (row, kv head, wave) 8 wall-clock
  // stamps (100 MHz) at the kernel's phases; nullptr normally
  unsigned long long* trace;
};

struct MMArgs {
  const uint16_t* W;   // packed tiles
  int N, K;            // logical W[N][K]; for SWIGLU N = 2*n_ff (interleaved tiles)
  const uint16_t* X;   // activations bf16 [>=16*NB rows][ldx]
  int ldx;
  int M;               // valid columns (tokens)
  // RMS_NORM on load (X == nullptr, M <= 16): B = bf16((xf * scale) * norm_w), scale from ssq
  const float* xf;
  const float* norm_w;
  float eps;
  // per-16-row-tile sums of squares of the residual stream, [M][np]: read by RMS_NORM-on-load
  // consumers (np = K/16), written by EPI_RESID producers when non-null (np = N/16)
  float* ssq;
  int np;
  // epilogue operands
  float* out;          // EPI_F32: [M][ldo]; EPI_RESID: residual x [M][ldo]; EPI_QKV: q [M][ldo]
  int ldo;
  uint16_t* act;       // EPI_SWIGLU: bf16 [M][lda]
  int lda;
  float* actf;         // EPI_SWIGLU: f32 [M][lda] instead of act (Q8_0 models quantise it next)
  // Q8_0 weights (mq8_kernel): activations as Q8_0 rows, xq int8 [M][K] (k permuted within
  // 64-k groups, see q8_perm) and xd f32 [M][K/32] (the f16-rounded block scales)
  const int8_t* xq;
  const float* xd;
  // EPI_QKV
  int n_q, n_kv, head_dim;     // rows [0,n_q) q, [n_q,n_q+n_kv) k, rest v
  const int* pos;              // [M]
  const int* slot;             // [M]
  const float* rope_cs;        // [n_ctx][head_dim/2][2]
  _Float16* kc;                // K cache of this layer: [slots][n_head_kv][ctx_stride * head_dim] (tiled)
  _Float16* vc;                // V cache of this layer: [slots][n_head_kv][ctx_stride * head_dim] (tiled)
  int n_ctx, ctx_stride, n_head_kv;
  size_t slot_stride;          // elements per slot in kc/vc = n_head_kv*ctx_stride*head_dim
  size_t slab_stride;          // EPI_SLAB: floats between consecutive K-split partial slabs
  // K-quant weights (mkq_kernel): activations as Q8_K rows -- xq int8 [M][K] (permuted within each
  // super-block, kquant.hip), xd f32 [M][K/256], xb f32 [M][K/32] (sub-block sums of q) -- and W
  // as up to 3 row segments of one ggml type each (e.g. q|k Q4_K, v Q6_K): segment i holds packed
  // tiles [kq_tile_end[i-1], kq_tile_end[i]) at byte offset kq_off[i] from W
  const float* xb;
  int wq4;             // Q8_0-path GEMVs: W holds Q4_0 tiles (Q4_TILE_BYTES) instead of Q8 tiles
  int kq_n;
  int kq_type[3];
  int kq_tile_end[3];
  size_t kq_off[3];
  // bf16 GEMVs, batch invariance: K is cut into 16 canonical slices
  // [KT*j/16, KT*(j+1)/16) and a row's sum is ((slices of group 0) + (slices of group 1)) + ...
  // over kgrp groups of 16/kgrp consecutive slices -- set by the launchers from the shape alone
  // (canon_kgroups), never by the row count.  mm_wide_kernel: kgrp < 0 = one MFMA chain over the
  // whole K range (no slices): the prefill GEMM's order, for prompt chunks of <= 64 rows
  int kgrp;
};



// packing / synthetic weights.  mode: PACK_ROWS (logical row r -> packed row r + offset),
// PACK_GATE / PACK_UP (ffn_gate / ffn_up rows interleaved by 8-row halves of each tile)
enum PackMode : int { PACK_ROWS = 0, PACK_GATE = 1, PACK_UP = 2 };
void launch_synth_packed(uint16_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale, int mode,
                         int row_offset, hipStream_t s);
void launch_synth_rowmajor(uint16_t* dst, size_t n, uint64_t seed, uint64_t tid, float scale, hipStream_t s);
void launch_synth_norm(float* dst, size_t n, uint64_t seed, uint64_t tid, float scale, hipStream_t s);
void launch_pack(uint16_t* dst, const uint16_t* src_rowmajor, int N, int K, int mode, int row_offset,
                 hipStream_t s);

// forward-pass ops
// ssq (optional): per-16-element-tile sums of squares of each embedded row, [M][n_embd/16]
void launch_embed(float* x, const uint16_t* tok_embd, const int* ids, int M, int n_embd, float* ssq, hipStream_t s);
void launch_ssq(const float* x, int M, int n, float* ssq, hipStream_t s);
void launch_rmsnorm(uint16_t* y, int ldy, const float* x, const float* w, const int* row_map, int M, int n,
                    float eps, hipStream_t s);
int launch_mm(int epi, const MMArgs& a, hipStream_t s);
// canonical K groups of a bf16 GEMV shape (= the K split of its 17..64-row mm_wide launch)
int canon_kgroups(int epi, int N, int K);
bool mm_can_norm_on_load(int M, int K);
// <= 16 rows, row-tile-persistent gate/up: -1 if the shape has no instantiation
bool mm_pers_supported(int epi, int M, int N, int K);
int launch_mm_pers(int epi, const MMArgs& a, hipStream_t s);
// 17..64 rows: activation chunks shared through LDS.  EPI_QKV / EPI_RESID run split-K into
// `slabs` ([ksplit][MAX_ROWS][N] floats, slab_stride apart); returns the split used (the caller
// folds RESID partials with launch_resid_norm; QKV partials are finished inside), or -1.
int launch_mm_wide(int epi, const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s,
                   bool qkv_finish = true, bool full_chain = false);  // EPI_QKV: false leaves the slabs to the attention kernel
// x[c] += sum of nslab partial slabs (fixed order); then, if y, y = bf16(rmsnorm(x) * w)
void launch_resid_norm(uint16_t* y, int ldy, float* x, const float* slabs, int nslab, size_t slab_stride,
                       const float* w, int M, int n, float eps, hipStream_t s);  // X == nullptr path (RMS_NORM fused into the GEMV) is legal
void launch_attention(const AttnArgs& a, hipStream_t s);
// rows in blocks of 16 consecutive positions of one sequence each (prefill chunks): one
// work-group per (kv head, block), the 16 queries share every K/V chunk
void launch_attention_prefill(const AttnArgs& a, hipStream_t s);
// prefill (> MAX_ROWS rows): MFMA GEMM over packed weights with the same epilogues (N % 256, K % 64)
bool gemm_supported(int N, int K);
int launch_gemm(int epi, const MMArgs& a, hipStream_t s);
// the same GEMM split over K when it has too few work-groups to fill the CUs (small prefills;
// ~target work-groups, 0 = never split): partials go to `slabs` ([S][M][N] floats, at most slab_floats); QKV / SWIGLU are finished
// inside; returns S for EPI_RESID (the caller folds the partials with launch_resid_norm, slab
// stride M*N), 0 when the epilogue ran in place, -1 on a bad shape
int launch_gemm_split(int epi, const MMArgs& a, float* slabs, size_t slab_floats, int target, hipStream_t s);
// ---- Q8_0 weights.  Packed tile = 16 rows x 64 k, Q8_TILE_BYTES:
// [0,1024): int8 A operands of two v_mfma_i32_16x16x32_i8, lane l = row l&15 holds 8 bytes of
// block 0 (k 8(l>>4)..+8) then 8 bytes of block 1 (k 32+8(l>>4)..+8); [1024,1088): f16 block
// scales, row group g = rows 4g..4g+3: [block 0 x 4 rows][block 1 x 4 rows].  Tiles nt-major.
constexpr int Q8_TILE_K = 64;
constexpr int Q8_TILE_BYTES = 1088;
inline size_t q8_matrix_bytes(int N, int K) { return (size_t)N / 16 * (K / Q8_TILE_K) * Q8_TILE_BYTES; }
void launch_pack_q8(uint8_t* dst, const uint8_t* src_blocks, int N, int K, int mode, int row_offset, hipStream_t s);
// ---- Q4_0 weights (GGUF type 2: 32 weights = f16 d + 16 bytes, q - 8) on the Q8_0
// path: a packed Q4 tile = 16 rows x 64 k in Q4_TILE_BYTES: [0,512) lane l = row l&15 holds 4 bytes of
// block 0 then 4 of block 1, its 8 values k 8(l>>4)..+8 as low nibbles (first 4) and high nibbles (last
// 4) of those bytes -- unpacked (and shifted by -8) into the int8 A operand of the same
// v_mfma_i32_16x16x32_i8 as a Q8 tile; [512,576): the f16 block scales as in a Q8 tile.  The activations
// are Q8_0 rows: ggml's ggml_vec_dot_q4_0_q8_0 (exact int32 block sums, scaled by d_w * d_x in f32).
constexpr int Q4_TILE_BYTES = 576;
inline size_t q4_matrix_bytes(int N, int K) { return (size_t)N / 16 * (K / Q8_TILE_K) * Q4_TILE_BYTES; }
void launch_pack_q4(uint8_t* dst, const uint8_t* src_blocks, int N, int K, int mode, int row_offset, hipStream_t s);
// synthetic Q4_0 matrix: ggml quantize_row_q4_0_ref of the bf16 synthetic values, packed
void launch_synth_q4_packed(uint8_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale, int mode,
                            int row_offset, hipStream_t s);
// packed Q8 tiles of a [N][K] matrix -> packed bf16 tiles (prefill GEMM operand), values d*q -> bf16
int launch_dequant_q8_tiles(uint16_t* dst, const uint8_t* W, int N, int K, hipStream_t s);
void launch_synth_q8_packed(uint8_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale, int mode,
                            int row_offset, hipStream_t s);
void launch_synth_q8_rowmajor(uint8_t* dst, int N, int K, uint64_t seed, uint64_t tid, float scale, hipStream_t s);
// any GGUF matrix type (F32 0, F16 1, Q4_0 2, Q8_0 8, Q4_K 12, Q5_K 13, Q6_K 14) -> bf16 row-major,
// n elements (ggml dequantize_row_*, then RNE to bf16); -1 for an unsupported type or ragged n
int ggml_block_elems(int type);
int launch_dequant_bf16(uint16_t* dst, const uint8_t* src, int type, size_t n, hipStream_t s);
void launch_embed_q8(float* x, const uint8_t* tok_embd_blocks, const int* ids, int M, int n_embd, float* ssq,
                     hipStream_t s);
// RMS_NORM + MUL, quantised to Q8_0 activation rows (xq [M][n], xd [M][n/32])
void launch_rmsnorm_q8(int8_t* xq, float* xd, const float* x, const float* w, const int* row_map, int M, int n,
                       float eps, hipStream_t s, const float* slabs = nullptr, int nslab = 0,
                      size_t slab_stride = 0);  // nslab: fold the producer's split-K slabs into x first
void launch_quantize_q8(int8_t* xq, float* xd, const float* src, int ld, int M, int n, hipStream_t s);
// Q8_0 x Q8_0 products for any M (column groups of <= 64 tokens on grid.y), same epilogues.
// a.xq == nullptr: quantise on load from f32 rows a.xf ([M][K]; RMS_NORM + MUL first when norm_w,
// scale from the ssq partials), for mq8_can_quantize_on_load(M, K, norm_w != nullptr).  EPI_RESID writes ssq
// partials when a.ssq.
int launch_mq8(int epi, const MMArgs& a, hipStream_t s);
// 17..32 tokens: split-K partial slabs ([ks][token][N]) for launch_rmsnorm_q8 to fold (attn_output /
// ffn_down) or the attention / launch_qkv_finish to finish (q|k|v); ks, or -1 (use launch_mq8)
int launch_mq8_slab(const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s);
bool mq8_can_quantize_on_load(int M, int K, bool norm);

// ---- K-quant weights (GGUF Q4_K 12, Q5_K 13, Q6_K 14), kquant.hip.  Packed tile =
// 16 rows x 256 k (one super-block per row) in MFMA operand lane order: kq_tile_bytes(type) bytes
// (2368 / 2880 / 3360), tiles nt-major like the bf16 tiles.
int kq_tile_bytes(int type);  // 0 for a type without a K-quant tile
int kq_block_bytes(int type);  // GGUF block bytes per 256 weights (144 / 176 / 210)
inline size_t kq_matrix_bytes(int type, int N, int K) { return (size_t)N / 16 * (K / 256) * kq_tile_bytes(type); }
// GGUF blocks [N][K/256] -> packed tiles (packed_row modes as launch_pack); -1 for a bad type/shape
int launch_pack_kq(uint8_t* dst, const uint8_t* src_blocks, int type, int N, int K, int mode, int row_offset,
                   hipStream_t s);
// the synthetic model's GGUF blocks (synth.py kq_blocks), row-major
int launch_synth_kq_blocks(uint8_t* dst, int type, size_t nblocks, uint64_t seed, uint64_t tid, hipStream_t s);
// GET_ROWS of a K-quant token_embd (dequantize_row_q{4,5,6}_K, f32)
// ssq (optional): per-16-element-tile sums of squares of each embedded row (quantise-on-load consumers)
int launch_embed_kq(float* x, const uint8_t* tok_blocks, int type, const int* ids, int M, int n, float* ssq,
                    hipStream_t s);
// one token whose K-quant GEMVs quantise their Q8_K operand on load (xq == nullptr: xf, norm_w, ssq, np)
bool mkq_can_quantize_on_load(int M, int K, bool norm);
// RMS_NORM + MUL then Q8_K (xq [M][n], xd [M][n/256], xb [M][n/32]); plain Q8_K of f32 rows
// (nslab > 0: first fold the split-K slabs of the GEMV that wrote x into x, see launch_mkq_slab)
int launch_rmsnorm_q8k(int8_t* xq, float* xd, float* xb, const float* x, const float* w, const int* row_map, int M,
                       int n, float eps, hipStream_t s, const float* slabs = nullptr, int nslab = 0,
                       size_t slab_stride = 0);
int launch_quantize_q8k(int8_t* xq, float* xd, float* xb, const float* src, int ld, int M, int n, hipStream_t s);
// K-quant x Q8_K products for any M (grid.y: groups of 32 tokens), the usual epilogues (SWIGLU: actf)
int launch_mkq(int epi, const MMArgs& a, hipStream_t s);
// 17..32 tokens, attn_output / ffn_down: split-K partials into slabs ([ks][token][N], slab_stride apart)
// for launch_rmsnorm_q8k to fold; returns ks, or -1 when the shape has no such form (use launch_mkq)
int launch_mkq_slab(const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s);
// 17..32 tokens, q|k|v: split-K partial slabs for the attention's FIN path or launch_qkv_finish
int launch_mkq_qkv_slab(const MMArgs& a, float* slabs, size_t slab_stride, hipStream_t s);
// q/k/v split-K partial slabs -> sum in slab order -> RoPE + q / KV-cache stores (EPI_QKV's epilogue)
void launch_qkv_finish(const MMArgs& a, const float* slabs, int nslab, size_t slab_stride, hipStream_t s);
// packed K-quant matrix (segments as in MMArgs) -> packed bf16 tiles [N/16][K/32] x 1 KiB (prefill GEMM)
int launch_dequant_kq(uint16_t* dst, const void* W, int K, int kq_n, const int* type, const int* tile_end,
                      const size_t* off, hipStream_t s);

// top-k (k <= TOPK_MAX) candidates per logits row, value descending, ties by lower id; ws: M*64*k
constexpr int TOPK_MAX = 64;
int launch_topk(const float* logits, int ldl, int M, int V, int K, float* ws_val, int* ws_idx, float* out_val,
                int* out_idx, hipStream_t s);
void launch_argmax(const float* logits, int ldl, int M, int V, float* ws_val, int* ws_idx, int* tok_out,
                   int* ids_next, int* pos_next, int* hist, int hist_stride, int* hist_count, int max_hist,
                   hipStream_t s);

// ---- device sampling chain (llama-cpp-python 0.3's create_completion chain as
// engine.cpp restates it): penalties over the last last_n tokens -> top_k -> top_p -> min_p ->
// temperature -> draw; temperature <= 0 = greedy (after the penalties).  One SampRow per logits row.
constexpr int SAMP_WIN = 64;
struct SampRow {
  float temp, top_p, min_p, repeat, freq, presence;
  int top_k;    // 1..TOPK_MAX on the device path
  int last_n;   // penalty window (0..SAMP_WIN); 0 = no penalties
  uint64_t seed;
  int draw0;    // index of the row's next random draw = tokens the request sampled before this run
  int n_win;    // penalty window at the start of the run: the last n_win tokens of prompt + output
  int win[SAMP_WIN];
};
// counter-based uniform draw in [0, 1) (splitmix64 of seed and draw index): host and device agree
__host__ __device__ inline double samp_u01(uint64_t seed, uint64_t draw) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (draw + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
// top_p / min_p / temperature / draw over k candidates sorted by value (descending, ties lower id
// first); p and w are scratch of k doubles.  The host sampler and sample_kernel both call this.
__host__ __device__ inline int samp_pick(const float* vals, const int* ids, int k, float temp, float top_p,
                                         float min_p, double u01, double* p, double* w) {
  if (temp <= 0.f || k <= 1) return ids[0];
  const double mx = vals[0];
  double sum = 0;
  for (int i = 0; i < k; i++) sum += (p[i] = exp((double)vals[i] - mx));
  for (int i = 0; i < k; i++) p[i] /= sum;
  int keep = k;
  if (top_p < 1.0f) {
    double cum = 0;
    for (int i = 0; i < k; i++) {
      cum += p[i];
      if (cum >= top_p) { keep = i + 1; break; }
    }
  }
  if (min_p > 0.f) {
    int kk = 1;
    for (int i = 1; i < keep; i++)
      if (p[i] >= min_p * p[0]) kk = i + 1;
    keep = kk;
  }
  const double m0 = (double)vals[0] / temp;
  double s2 = 0;
  for (int i = 0; i < keep; i++) s2 += (w[i] = exp((double)vals[i] / temp - m0));
  const double u = u01 * s2;
  double acc = 0;
  for (int i = 0; i < keep; i++) {
    acc += w[i];
    if (u < acc) return ids[i];
  }
  return ids[keep - 1];
}
// penalties (in place on the logits rows), top-k of K = max top_k of the rows, the draw, then the
// same token bookkeeping as launch_argmax (tok_out, ids_next, pos_next, history)
int launch_sample_chain(float* logits, int ldl, int M, int V, const SampRow* samp, int K, float* ws_val, int* ws_idx,
                        float* tk_val, int* tk_idx, int* tok_out, int* ids_next, int* pos_next, int* hist,
                        int hist_stride, int* hist_count, int max_hist, hipStream_t s);
// hand-off conversions of the residual stream (pipeline stages): f32 <-> bf16 rows (RNE), and the
// per-16-element sums of squares of the f32 rows made from bf16 (RMS_NORM-on-load consumers)
void launch_f32_to_bf16(uint16_t* dst, const float* src, size_t n, hipStream_t s);
void launch_copy_f32(float* dst, const float* src, size_t n, hipStream_t s);
void launch_f32_in(float* x, const float* src, int M, int n, float* ssq, hipStream_t s);  // + Σx² partials
void launch_bf16_to_f32(float* dst, const uint16_t* src, int M, int n, float* ssq, hipStream_t s);

// HBM streaming probes: variant v of probe_variants() (loads in flight, grid, non-temporal) of a
// read-only (XOR fold) or copy stream over n16 16-byte words (n16 % 4096 == 0); desc describes it
int probe_variants();
int launch_probe(int v, bool read_only, const uint4* src, uint4* dst, size_t n16, hipStream_t s, char* desc,
                 int desc_len);

}  // namespace mx
