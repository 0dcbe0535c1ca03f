// engine.cpp -- host side of the MI355X-native engine behind include/mx_engine.h.
//
// Replaces llama-cpp-python/llama.cpp as used by the reference node:
//   Llama(model_path=...)                 /root/reference/llama_p2p_network.py:19  -> mx_engine_create
//   self.model(prompt, max_tokens=100)    /root/reference/llama_p2p_network.py:125 -> mx_submit/mx_wait
// The forward pass is llama.cpp's llm_build_llama expressed as
// five fused gfx950 kernels per layer (kernels.hip).  Decode steps are captured
// once per batch shape as hipGraphs and replayed; a scheduler thread replaces
// the reference's serialising lock (p2p:121) with micro-batched decode of all
// active requests.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mx_engine.h"
#include "gguf.h"
#include "kernels.h"

using namespace mx;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPC(expr)                                                                                  \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      return fail(MX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) + " @" + __FILE__ + \
                                  ":" + std::to_string(__LINE__));                                  \
  } while (0)

struct Shape {
  const char* name;
  int n_embd, n_layer, n_head, n_head_kv, n_ff, n_vocab;
  float rope_base, eps;
  int n_ctx_train;
};
// keep in sync with llama-p2p_amd/synth.py SHAPES
const Shape kShapes[] = {
    {"tinyllama-1.1b", 2048, 22, 32, 4, 5632, 32000, 10000.f, 1e-5f, 2048},
    {"llama3-8b", 4096, 32, 32, 8, 14336, 128256, 500000.f, 1e-5f, 8192},
    {"llama3-70b", 8192, 80, 64, 8, 28672, 128256, 500000.f, 1e-5f, 8192},
    {"test-tiny", 256, 2, 4, 2, 512, 512, 10000.f, 1e-5f, 2048},
    {"test-gqa8", 512, 3, 8, 1, 1024, 1024, 500000.f, 1e-5f, 2048},
    {"test-d128", 1024, 2, 8, 2, 2816, 2048, 500000.f, 1e-5f, 2048},
    {"test-h4096", 4096, 1, 32, 8, 2048, 1024, 500000.f, 1e-5f, 2048},
    {"test-h8192", 8192, 1, 64, 8, 2048, 1024, 500000.f, 1e-5f, 2048},
    {"test-8b-ffn", 4096, 2, 32, 8, 14336, 1024, 500000.f, 1e-5f, 2048},
    {"test-70b-ffn", 8192, 1, 64, 8, 28672, 1024, 500000.f, 1e-5f, 2048},
    {"test-tiny-ffn", 2048, 1, 32, 4, 5632, 32000, 10000.f, 1e-5f, 2048},
    {"test-8b-v128k", 4096, 2, 32, 8, 14336, 128256, 500000.f, 1e-5f, 8192},
    // a non-Llama-3 geometry (Llama-2-7B: MHA, ff 11008, V 32000): the generic GEMV fallbacks' cost
    {"llama2-7b", 4096, 32, 32, 32, 11008, 32000, 10000.f, 1e-5f, 4096},
};

// decode steps the scheduler runs on the device between host syncs when every active row is greedy
constexpr int SCHED_KMAX = 8;

// synth.py tensor ids
constexpr uint64_t TID_TOK_EMBD = 1, TID_OUT_NORM = 2, TID_OUTPUT = 3;
enum { L_ATTN_NORM, L_Q, L_K, L_V, L_O, L_FFN_NORM, L_GATE, L_UP, L_DOWN };
uint64_t layer_tid(int l, int k) { return 16u + 16u * (uint64_t)l + (uint64_t)k; }
float std_scale(double std) { return (float)(std / sqrt(4294967295.0 / 3.0)); }

// Row segments of one packed K-quant matrix (MMArgs kq_*): rows appended in order, consecutive rows
// of one ggml type share a segment (q|k Q4_K + v Q6_K = two segments).
struct KqMat {
  int n = 0;
  int type[3] = {0, 0, 0}, tile_end[3] = {0, 0, 0};
  size_t off[3] = {0, 0, 0};
  size_t bytes = 0;
  int rows = 0;
  bool add(int t, int r, int K) {
    if (n && type[n - 1] == t) {
      tile_end[n - 1] += r / 16;
    } else {
      if (n == 3) return false;
      type[n] = t;
      off[n] = bytes;
      tile_end[n] = (n ? tile_end[n - 1] : 0) + r / 16;
      n++;
    }
    bytes += kq_matrix_bytes(t, r, K);
    rows += r;
    return true;
  }
  // segment holding packed row `row`, and that row's index within the segment
  int seg(int row, int* row_in_seg) const {
    int i = 0;
    while (i < n - 1 && row / 16 >= tile_end[i]) i++;
    *row_in_seg = row - 16 * (i ? tile_end[i - 1] : 0);
    return i;
  }
  void set(MMArgs& a) const {
    a.kq_n = n;
    for (int i = 0; i < 3; i++) {
      a.kq_type[i] = type[i];
      a.kq_tile_end[i] = tile_end[i];
      a.kq_off[i] = off[i];
    }
  }
};

// ggml type of a tensor in llama.cpp's Q4_K_M / Q5_K_M recipes (llama_tensor_get_type, Oct 2024;
// synth.py kq_tensor_type is the same rule): output Q6_K; attn_v and ffn_down Q6_K on the
// use_more_bits layers; attn_v of an 80-layer (70B) Q4_K_M model otherwise Q5_K; the rest `base`.
bool use_more_bits(int i, int n) { return i < n / 8 || i >= 7 * n / 8 || (i - n / 8) % 3 == 2; }
int kq_recipe_type(int base, int kind, int layer, int n_layer) {  // kind: L_* or -1 output, -2 token_embd
  if (kind == -1) return 14;
  if ((kind == 3 || kind == 8) && use_more_bits(layer, n_layer)) return 14;  // L_V, L_DOWN
  if (kind == 3 && n_layer == 80 && base == 12) return 13;
  return base;
}

struct Layer {
  uint16_t *qkv = nullptr, *o = nullptr, *gu = nullptr, *down = nullptr;
  float *attn_norm = nullptr, *ffn_norm = nullptr;
  KqMat kq_qkv, kq_o, kq_gu, kq_down;  // K-quant model: segments of the four packed matrices
};

struct Request {
  uint64_t id = 0;
  std::vector<int32_t> prompt;
  mx_sampling samp{};
  int max_tokens = 0;
  std::vector<int32_t> out;
  int finish = -1;
  bool done = false;
  bool cancel = false;  // mx_cancel: finish after the current step
  int slot = -1;
  int pos = 0;     // next position to write
  int reuse = 0;   // leading prompt positions whose K/V the slot already holds (prefix reuse)
  int32_t next_tok = 0;
  uint64_t seed = 0;  // sampler stream: the n-th sampled token draws samp_u01(seed, n) (kernels.h)
  std::string error;
};

struct GraphKey {
  int M;
  const void* xin;
  void* xout;
  hipStream_t stream;
  int ktop;  // 0: greedy argmax tail; k: the device sampling chain with top-k k
  bool operator<(const GraphKey& o) const {
    if (M != o.M) return M < o.M;
    if (xin != o.xin) return xin < o.xin;
    if (xout != o.xout) return xout < o.xout;
    if (ktop != o.ktop) return ktop < o.ktop;
    return stream < o.stream;
  }
};
}  // namespace

struct mx_batch {
  int M = 0, max_steps = 0;
  SampRow* d_samp = nullptr;  // per-row device sampler settings (mx_batch_reset); null: greedy argmax
  int ktop = 0;               // top-k of the device sampling chain, 0 = greedy argmax
  bool distinct = false;  // every row its own slot (decode); see mx_engine::rows_distinct
  int max_pos = 0;  // host mirror of the largest position, so steps never run past n_ctx
  int *d_ids = nullptr, *d_pos = nullptr, *d_slot = nullptr, *d_hist = nullptr, *d_hist_count = nullptr;
  bool ids_external = false;
  std::map<GraphKey, hipGraphExec_t> graphs;
};

struct mx_engine {
  // hyper-parameters
  int n_embd = 0, n_layer = 0, n_head = 0, n_head_kv = 0, head_dim = 0, n_embd_kv = 0, n_ff = 0, n_vocab = 0;
  int n_ctx_train = 0;
  float eps = 1e-5f, rope_base = 10000.f;
  // RoPE frequency factors (GGUF rope_freqs.weight, Llama-3.1; empty = none) and linear scaling
  std::vector<float> rope_ff;
  float rope_freq_scale = 1.0f;
  int bos = 1, eos = 2;
  int n_ctx = 512, n_seq_max = 64, lb = 0, le = 0, device = 0;
  bool has_embed = true, has_head = true, use_graphs = true;
  // <= 4 rows: RMS_NORM applied while loading the GEMV's B operand, from per-tile sums of squares
  // written by the residual-stream producer (no norm launches)
  static constexpr bool norm_on_load = true;
  // gate/up as a row-tile-persistent GEMV with RMS_NORM on load (<= 4 rows); MX_NO_PERS=1 for A/B
  bool use_pers = getenv("MX_NO_PERS") == nullptr;
  bool q8_gemm_prefill = getenv("MX_Q8_GEMM_PREFILL") != nullptr;  // see enqueue_forward
  // K-quant prefill chunks with ggml's arithmetic (Q8_K activations, the int8 K-quant GEMVs at every
  // row count) instead of bf16 GEMMs over dequantised weights; see enqueue_forward
  bool kq_ggml_prefill = getenv("MX_KQ_GGML_PREFILL") != nullptr;
  float* ssq = nullptr;  // [MAX_ROWS][n_embd/16] per-tile sums of squares of x
  // rows of the next forward belong to distinct sequences (decode): no row attends to another row's
  // new K/V, so the wide path lets the attention kernel finish q/k/v from the split-K slabs
  bool rows_distinct = false;
  // rows of the next forward come in blocks of 16 consecutive positions of one sequence (prefill):
  // attention runs as attn_prefill_kernel, 16 queries per K/V pass
  bool rows_blocked = false;
  // the next forward is a prompt chunk from the scheduler or a pipeline prefill: every row count takes
  // the GEMM path (one K range per output: the arithmetic of a prompt row does not depend on how many
  // rows share its chunk -- batch invariance)
  bool prefill_gemm = false;
  bool use_wide = getenv("MX_NO_WIDE") == nullptr;  // 17..64-row forward through mm_wide (LDS-shared activations)
  float* slabs = nullptr;                           // split-K partials [8][MAX_ROWS][n_embd + 2 n_embd_kv]
  size_t slab_stride = 0;
  float* gslabs = nullptr;  // split-K partials of small-M prefill GEMMs, [S][M][N] (launch_gemm_split)
  // K-quant model prefill: one layer's four matrices dequantised to packed bf16 for the GEMM path
  uint16_t *kqd_qkv = nullptr, *kqd_o = nullptr, *kqd_gu = nullptr, *kqd_down = nullptr;
  static constexpr size_t GSLAB_FLOATS = (size_t)32 << 20;
  // work-groups a split prefill GEMM aims at (MX_GEMM_SPLIT_TARGET; 0 = one K range per tile).  Default 0:
  // a split chosen from the chunk's row count would make a prompt's values depend on its chunk-mates
  int gemm_split_target = getenv("MX_GEMM_SPLIT_TARGET") ? atoi(getenv("MX_GEMM_SPLIT_TARGET")) : 0;
  int ctx_stride = 0;  // KV positions allocated per slot (n_ctx rounded up to KV_POS_ALIGN)
  uint64_t weight_bytes = 0;

  // device state
  hipStream_t stream = nullptr;
  uint16_t *tok_embd = nullptr, *output = nullptr;
  float* out_norm = nullptr;
  // Q8_0 model: layer matrices as packed Q8 tiles; token_embd / output may each
  // be Q8_0 (tok_embd8: GGUF blocks, row-major) or BF16
  bool wq8 = false, embd_q8 = false, out_q8 = false;
  // Q4_0 model (llama.cpp Q4_0 files): the layer matrices are Q4 tiles on the Q8_0 path (Q8_0 activation
  // rows, ggml_vec_dot_q4_0_q8_0); the head is Q8_0 / Q4_0 tiles (out_q4) or, as llama-quantize writes it,
  // a K-quant output (out_kq_head: kq_out segments, Q8_K activation rows)
  bool wq4 = false, out_q4 = false, out_kq_head = false;
  static constexpr bool q8_ql = true;  // Q8_0 GEMVs of <= 4 rows quantise their operand on load
  uint8_t* tok_embd8 = nullptr;
  // K-quant model (Q4_K / Q5_K / Q6_K matrices: llama.cpp's Q4_K_M / Q5_K_M; kquant.hip): packed
  // K-quant tiles, activations as Q8_K rows (q in xq8, d in xqd, sub-block sums in xkb)
  bool wkq = false;
  int kq_main_type = 0;          // type of ffn_gate (mx_model_info.weight_type)
  int embd_kq_type = 0;          // token_embd kept as K-quant GGUF blocks when non-zero
  uint8_t* tok_embd_kq = nullptr;
  float* xkb = nullptr;
  KqMat kq_out;
  int8_t* xq8 = nullptr;    // Q8_0 activation rows [PREFILL_ROWS][max(h, ff)]
  float* xqd = nullptr;     // their block scales
  float *attn_f = nullptr, *act_f = nullptr;  // f32 attention output / SwiGLU product (quantised next)
  std::vector<Layer> layers;  // local layers [lb, le)
  _Float16 *kcache = nullptr, *vcache = nullptr;
  size_t slot_stride = 0, layer_kv_stride = 0;
  float* rope_cs = nullptr;
  // workspaces (MAX_ROWS rows)
  float *x = nullptr, *q = nullptr, *logits = nullptr;
  uint16_t *xn = nullptr, *act = nullptr, *attn_out = nullptr;
  float* am_val = nullptr;
  bool use_dev_topk = getenv("MX_NO_DEV_TOPK") == nullptr;  // MX_NO_DEV_TOPK: all-host sampler (tests)
  float *tk_ws_val = nullptr, *tk_val = nullptr;  // device top-k for the sampler chain
  int *tk_ws_idx = nullptr, *tk_idx = nullptr;
  int *am_idx = nullptr, *d_tok = nullptr;
  int *d_ids = nullptr, *d_pos = nullptr, *d_slot = nullptr, *d_rowmap = nullptr;
  // pinned host staging of forward_rows_chunk's index arrays [4][R]: its async copies read from here
  // (engine-owned), not through the runtime's staging of pageable memory
  int32_t* h_idx = nullptr;
  std::vector<void*> allocations;

  // graphs for the scheduler's decode steps, by (M, top-k of the device sampling chain or 0 = argmax)
  std::map<std::pair<int, int>, hipGraphExec_t> sched_graphs;
  // pipeline stage hand-off dtype: x_in / x_out are bf16 [M][n_embd] instead of f32 (mx_opts.handoff_bf16)
  bool handoff_bf16 = false;
  // token pick at the end of a forward with `argmax` set: greedy argmax, or (pick_samp) the device
  // sampling chain with top-k pick_k over the rows' SampRow settings
  const SampRow* pick_samp = nullptr;
  int pick_k = 0;
  SampRow* d_samp = nullptr;  // [MAX_ROWS] the scheduler's rows
  void pick(int n_out, int* ids_next, int* pos_next, int* hist, int hist_stride, int* hist_count, int max_hist,
            hipStream_t s) {
    if (pick_samp)
      launch_sample_chain(logits, n_vocab, n_out, n_vocab, pick_samp, pick_k, tk_ws_val, tk_ws_idx, tk_val, tk_idx,
                          d_tok, ids_next, pos_next, hist, hist_stride, hist_count, max_hist, s);
    else
      launch_argmax(logits, n_vocab, n_out, n_vocab, am_val, am_idx, d_tok, ids_next, pos_next, hist, hist_stride,
                    hist_count, max_hist, s);
  }
  int copy_out(void* x_out, int M, hipStream_t s) {  // the residual stream to the next stage
    if (handoff_bf16) launch_f32_to_bf16((uint16_t*)x_out, x, (size_t)M * n_embd, s);
    else launch_copy_f32((float*)x_out, x, (size_t)M * n_embd, s);
    return 0;
  }
  // SampRow of a request for a run that starts now (draw index and penalty window at this point)
  void samp_row(const Request* r, SampRow* o) const;
  // true when the device sampling chain can serve this request (top_k 1..64, window <= 64)
  static bool device_sampleable(const mx_sampling& sp);

  // scheduler
  std::mutex gpu_mu;  // serialises all GPU work issued through the API
  std::mutex mu;
  std::condition_variable cv, cv_done;
  std::deque<Request*> pending;
  std::vector<Request*> active;
  std::map<uint64_t, std::unique_ptr<Request>> requests;
  std::vector<int> free_slots;
  // prefix-KV reuse (llama-cpp-python's Llama.generate keeps the longest common prefix of the previous
  // evaluation): tokens whose K/V each slot holds at positions 0..n-1, valid while the slot is free
  std::vector<std::vector<int32_t>> slot_tokens;
  uint64_t stat_prompt_tokens = 0, stat_reused_tokens = 0, stat_generated_tokens = 0;
  uint64_t next_id = 1;
  bool stop = false;
  std::thread worker;
  bool worker_started = false;

  ~mx_engine();
  int alloc(void** p, size_t bytes) {
    HIPC(hipMalloc(p, bytes));
    allocations.push_back(*p);
    if (poison) HIPC(hipMemset(*p, 0xFF, bytes));  // NaN in every f32 / f16 / bf16 lane
    return 0;
  }
  // diagnosis (mx_debug): MX_POISON=1 fills every allocation with 0xFF bytes and skips the zero
  // fills of init_common, so a read of a never-written element shows up as a NaN; dbg_stop ends the
  // 17..64-row forward after that many launches, dbg_sync synchronises the stream after each one
  const bool poison = getenv("MX_POISON") != nullptr;
  int dbg_stop = -1, dbg_count = 0;
  bool dbg_sync = false;
  // never while a graph is being captured: a captured forward would keep the truncation (or the capture
  // would be invalidated by the sync) for every later replay
  bool dbg_hit(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    if (dbg_sync) hipStreamSynchronize(s);
    return dbg_stop >= 0 && ++dbg_count >= dbg_stop;
  }
  int init_common();
  int load_synthetic(const Shape& s, uint64_t seed, bool q8 = false, int kq_base = 0, bool q4 = false);
  int load_gguf(const std::string& path);
  int enqueue_forward(int M, const int* ids, const int* pos, const int* slot, const void* x_in, void* x_out,
                      bool head, const int* rowmap, int n_out, bool argmax, int* ids_next, int* pos_next, int* hist,
                      int hist_stride, int* hist_count, int max_hist, hipStream_t s);
  bool q8_on_load(int M) const {
    return wq8 && q8_ql && mq8_can_quantize_on_load(M, n_embd, true) && mq8_can_quantize_on_load(M, n_ff, false);
  }
  // one-token K-quant GEMVs quantise their Q8_K operand on load (no norm / quantise launches)
  bool kq_on_load(int M) const {
    return wkq && mkq_can_quantize_on_load(M, n_embd, true) && mkq_can_quantize_on_load(M, n_ff, false);
  }
  int enqueue_forward_q8(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap, int n_out,
                         bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride, int* hist_count,
                         int max_hist, hipStream_t s);
  int enqueue_forward_kq(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap, int n_out,
                         bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride, int* hist_count,
                         int max_hist, hipStream_t s);
  int enqueue_forward_gemm(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap,
                           int n_out, hipStream_t s);
  bool gemm_shapes() const {  // the bf16 prefill GEMM takes every matrix of a layer
    return gemm_supported(n_embd + 2 * n_embd_kv, n_embd) && gemm_supported(n_embd, n_embd) &&
           gemm_supported(2 * n_ff, n_embd) && gemm_supported(n_embd, n_ff);
  }
  bool gemm_ok() const {  // chunks of PREFILL_ROWS rows can run (the Q8_0 / K-quant paths take any row count)
    return wq8 || wkq || gemm_shapes();
  }
  // rows form blocks of 16 (from row 0) of one slot each, positions consecutive within a block except
  // that a block may end in copies of its last real row (same position and token: the prompt padding
  // near n_ctx) -- what attn_prefill_kernel needs (every key position a block reads is written by it)
  bool blocked_rows(const int32_t* slots, const int32_t* pos, const int32_t* ids, int m) const {
    for (int k = 0; k < m; k++) {
      if (k % 16 == 0) continue;
      if (slots[k] != slots[k - 1]) return false;
      if (pos[k] == pos[k - 1] + 1) continue;
      if (pos[k] != pos[k - 1] || (ids && ids[k] != ids[k - 1])) return false;
    }
    return true;
  }
  int enqueue_forward_wide(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap,
                           int n_out, bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride,
                           int* hist_count, int max_hist, hipStream_t s, bool full_chain = false);
  int forward_rows_chunk(int n, const int32_t* slots, const int32_t* pos, const int32_t* ids, const void* x_in,
                         void* x_out, float* logits_host, hipStream_t s, bool last_row_only = false);
  void scheduler_loop();
  int sched_step(std::vector<Request*>& rows);
  int prefill_batch(std::vector<Request*>& reqs);
  int* sched_hist = nullptr;        // [MAX_ROWS][SCHED_KMAX] tokens of a multi-step greedy run
  int* sched_hist_count = nullptr;  // [MAX_ROWS]
  int32_t sample_host(Request* r, const float* logits);
  int32_t sample_chain(Request* r, std::vector<std::pair<float, int>>& c);  // c: top-k, sorted
  void finish(Request* r, int why);
};

mx_engine::~mx_engine() {
  {
    std::lock_guard<std::mutex> lk(mu);
    stop = true;
  }
  cv.notify_all();
  if (worker.joinable()) worker.join();
  for (auto& kv : sched_graphs) hipGraphExecDestroy(kv.second);
  if (stream) hipStreamSynchronize(stream);

  for (void* p : allocations) hipFree(p);
  if (h_idx) hipHostFree(h_idx);
  if (stream) hipStreamDestroy(stream);
}

int mx_engine::init_common() {
  head_dim = n_embd / n_head;
  n_embd_kv = head_dim * n_head_kv;
  if (n_embd % n_head || n_head % n_head_kv) return fail(MX_ERR_MODEL, "head counts do not divide n_embd/n_head");
  if (head_dim != 64 && head_dim != 128) return fail(MX_ERR_ARG, "head_dim must be 64 or 128");
  if (n_embd > 8192) return fail(MX_ERR_ARG, "n_embd > 8192 is not supported");
  if (n_embd % 64) return fail(MX_ERR_ARG, "n_embd must be a multiple of 64 (RMS_NORM tile partials)");
  const int G = n_head / n_head_kv;
  if (G != 1 && G != 2 && G != 4 && G != 8) return fail(MX_ERR_ARG, "n_head/n_head_kv must be 1,2,4 or 8");
  if (n_embd % 32 || n_ff % 32 || n_vocab % 16 || n_embd_kv % 16)
    return fail(MX_ERR_ARG, "n_embd, n_ff must be multiples of 32 and n_vocab, n_embd_kv of 16");
  if (wq8 && (n_embd % Q8_TILE_K || n_ff % Q8_TILE_K))
    return fail(MX_ERR_ARG, "Q8_0 models need n_embd and n_ff multiples of 64");
  if (wkq && (n_embd % 256 || n_ff % 256)) return fail(MX_ERR_ARG, "K-quant models need n_embd and n_ff multiples of 256");
  if (le < 0 || le > n_layer) le = n_layer;
  if (lb < 0 || lb >= le) return fail(MX_ERR_ARG, "bad layer range");
  has_embed = lb == 0;
  has_head = le == n_layer;
  ctx_stride = (n_ctx + KV_POS_ALIGN - 1) / KV_POS_ALIGN * KV_POS_ALIGN;
  const int nl = le - lb;
  layers.resize(nl);

  // KV cache per layer and slot: K and V [kv head][ctx_stride * head_dim] f16 in 1 KiB MFMA B-operand
  // tiles (kernels.hip kv_k_off / kv_v_off)
  slot_stride = (size_t)n_head_kv * ctx_stride * head_dim;
  layer_kv_stride = slot_stride * n_seq_max;
  if (int rc = alloc((void**)&kcache, layer_kv_stride * nl * sizeof(_Float16))) return rc;
  if (int rc = alloc((void**)&vcache, layer_kv_stride * nl * sizeof(_Float16))) return rc;
  if (!poison) {
    HIPC(hipMemsetAsync(kcache, 0, layer_kv_stride * nl * sizeof(_Float16), stream));
    HIPC(hipMemsetAsync(vcache, 0, layer_kv_stride * nl * sizeof(_Float16), stream));
  }

  // RoPE table, ggml_rope_cache_init + rope_yarn (ext_factor 0, mscale 1): theta *= powf(base, -2/d)
  // as an f32 running product, divided by the frequency factor, times the linear freq_scale
  if (!rope_ff.empty() && (int)rope_ff.size() != head_dim / 2) return fail(MX_ERR_MODEL, "rope_freqs.weight size");
  std::vector<float> cs((size_t)n_ctx * head_dim);
  const float theta_scale = powf(rope_base, -2.0f / (float)head_dim);
  for (int p = 0; p < n_ctx; p++) {
    float theta = (float)p;
    for (int i = 0; i < head_dim / 2; i++) {
      const float ff = rope_ff.empty() ? 1.0f : rope_ff[i];
      const float th = rope_freq_scale * (theta / ff);
      cs[((size_t)p * (head_dim / 2) + i) * 2] = cosf(th);
      cs[((size_t)p * (head_dim / 2) + i) * 2 + 1] = sinf(th);
      theta *= theta_scale;
    }
  }
  if (int rc = alloc((void**)&rope_cs, cs.size() * 4)) return rc;
  HIPC(hipMemcpy(rope_cs, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));

  const int R = PREFILL_ROWS;  // activation rows: prefill chunks (GEMM path); logits only for MAX_ROWS
  if (int rc = alloc((void**)&x, (size_t)R * n_embd * 4)) return rc;
  if (int rc = alloc((void**)&q, (size_t)R * n_embd * 4)) return rc;
  if (int rc = alloc((void**)&xn, (size_t)R * n_embd * 2)) return rc;
  if (int rc = alloc((void**)&attn_out, (size_t)R * n_embd * 2)) return rc;
  if (int rc = alloc((void**)&act, (size_t)R * n_ff * 2)) return rc;
  if (has_head) {
    if (int rc = alloc((void**)&logits, (size_t)MAX_ROWS * n_vocab * 4)) return rc;
  }
  slab_stride = (size_t)MAX_ROWS * (n_embd + 2 * n_embd_kv);
  if (int rc = alloc((void**)&slabs, slab_stride * 8 * 4)) return rc;
  if (gemm_shapes())
    if (int rc = alloc((void**)&gslabs, GSLAB_FLOATS * 4)) return rc;
  if ((wkq || (wq8 && !wq4 && q8_gemm_prefill)) && gemm_shapes()) {  // per-layer bf16 copies for the prefill GEMM
    const size_t h = n_embd, kv = n_embd_kv, ff = n_ff;
    if (int rc = alloc((void**)&kqd_qkv, (h + 2 * kv) * h * 2)) return rc;
    if (int rc = alloc((void**)&kqd_o, h * h * 2)) return rc;
    if (int rc = alloc((void**)&kqd_gu, 2 * ff * h * 2)) return rc;
    if (int rc = alloc((void**)&kqd_down, h * ff * 2)) return rc;
  }
  if (int rc = alloc((void**)&ssq, (size_t)R * (n_embd / 16) * 4)) return rc;
  if (int rc = alloc((void**)&am_val, (size_t)R * 64 * 4)) return rc;
  if (has_head) {
    if (int rc = alloc((void**)&tk_ws_val, (size_t)MAX_ROWS * 64 * TOPK_MAX * 4)) return rc;
    if (int rc = alloc((void**)&tk_ws_idx, (size_t)MAX_ROWS * 64 * TOPK_MAX * 4)) return rc;
    if (int rc = alloc((void**)&tk_val, (size_t)MAX_ROWS * TOPK_MAX * 4)) return rc;
    if (int rc = alloc((void**)&tk_idx, (size_t)MAX_ROWS * TOPK_MAX * 4)) return rc;
  }
  if (int rc = alloc((void**)&am_idx, (size_t)R * 64 * 4)) return rc;
  if (int rc = alloc((void**)&d_tok, (size_t)R * 4)) return rc;
  if (int rc = alloc((void**)&d_ids, (size_t)R * 4)) return rc;
  if (int rc = alloc((void**)&d_pos, (size_t)R * 4)) return rc;
  if (int rc = alloc((void**)&d_slot, (size_t)R * 4)) return rc;
  if (int rc = alloc((void**)&d_rowmap, (size_t)R * 4)) return rc;
  HIPC(hipHostMalloc((void**)&h_idx, (size_t)4 * R * 4, hipHostMallocDefault));
  if (int rc = alloc((void**)&sched_hist, (size_t)MAX_ROWS * SCHED_KMAX * 4)) return rc;
  if (int rc = alloc((void**)&sched_hist_count, (size_t)MAX_ROWS * 4)) return rc;
  if (int rc = alloc((void**)&d_samp, (size_t)MAX_ROWS * sizeof(SampRow))) return rc;
  if (wq8 || wkq) {
    const size_t kmax = std::max(n_embd, n_ff);
    if (int rc = alloc((void**)&xq8, (size_t)R * kmax)) return rc;
    if (int rc = alloc((void**)&xqd, (size_t)R * (kmax / 32) * 4)) return rc;
    if (int rc = alloc((void**)&attn_f, (size_t)R * n_embd * 4)) return rc;
    if (int rc = alloc((void**)&act_f, (size_t)R * n_ff * 4)) return rc;
    if (wkq || out_kq_head)
      if (int rc = alloc((void**)&xkb, (size_t)R * (kmax / 32) * 4)) return rc;
  }
  // poison-free start: zero activations so padded MFMA columns never read uninitialised memory
  if (!poison) {
    HIPC(hipMemsetAsync(xn, 0, (size_t)R * n_embd * 2, stream));
    HIPC(hipMemsetAsync(attn_out, 0, (size_t)R * n_embd * 2, stream));
    HIPC(hipMemsetAsync(act, 0, (size_t)R * n_ff * 2, stream));
  }
  for (int i = 0; i < n_seq_max; i++) free_slots.push_back(n_seq_max - 1 - i);
  slot_tokens.assign(n_seq_max, {});
  return 0;
}

static int alloc_layer(mx_engine* e, Layer& L) {
  const size_t h = e->n_embd, kv = e->n_embd_kv, ff = e->n_ff;
  if (e->wq8) {
    auto qb = e->wq4 ? q4_matrix_bytes : q8_matrix_bytes;
    const size_t bq = qb(h + 2 * kv, h), bo = qb(h, h), bg = qb(2 * ff, h), bd = qb(h, ff);
    if (int rc = e->alloc((void**)&L.qkv, bq)) return rc;
    if (int rc = e->alloc((void**)&L.o, bo)) return rc;
    if (int rc = e->alloc((void**)&L.gu, bg)) return rc;
    if (int rc = e->alloc((void**)&L.down, bd)) return rc;
    if (int rc = e->alloc((void**)&L.attn_norm, h * 4)) return rc;
    if (int rc = e->alloc((void**)&L.ffn_norm, h * 4)) return rc;
    e->weight_bytes += bq + bo + bg + bd + 2 * h * 4;
    return 0;
  }
  if (int rc = e->alloc((void**)&L.qkv, (h + 2 * kv) * h * 2)) return rc;
  if (int rc = e->alloc((void**)&L.o, h * h * 2)) return rc;
  if (int rc = e->alloc((void**)&L.gu, 2 * ff * h * 2)) return rc;
  if (int rc = e->alloc((void**)&L.down, h * ff * 2)) return rc;
  if (int rc = e->alloc((void**)&L.attn_norm, h * 4)) return rc;
  if (int rc = e->alloc((void**)&L.ffn_norm, h * 4)) return rc;
  e->weight_bytes += ((h + 2 * kv) * h + h * h + 3 * ff * h) * 2 + 2 * h * 4;
  return 0;
}

// K-quant layer: segments from the seven matrix types (L_Q, L_K, L_V, L_O, L_GATE == L_UP, L_DOWN)
static int alloc_layer_kq(mx_engine* e, Layer& L, const int t[9]) {
  const int h = e->n_embd, kv = e->n_embd_kv, ff = e->n_ff;
  L.kq_qkv = L.kq_o = L.kq_gu = L.kq_down = KqMat();
  L.kq_qkv.add(t[L_Q], h, h);
  L.kq_qkv.add(t[L_K], kv, h);
  L.kq_qkv.add(t[L_V], kv, h);
  L.kq_o.add(t[L_O], h, h);
  if (t[L_GATE] != t[L_UP]) return fail(MX_ERR_MODEL, "ffn_gate and ffn_up of different K-quant types");
  L.kq_gu.add(t[L_GATE], 2 * ff, h);
  L.kq_down.add(t[L_DOWN], h, ff);
  if (int rc = e->alloc((void**)&L.qkv, L.kq_qkv.bytes)) return rc;
  if (int rc = e->alloc((void**)&L.o, L.kq_o.bytes)) return rc;
  if (int rc = e->alloc((void**)&L.gu, L.kq_gu.bytes)) return rc;
  if (int rc = e->alloc((void**)&L.down, L.kq_down.bytes)) return rc;
  if (int rc = e->alloc((void**)&L.attn_norm, (size_t)h * 4)) return rc;
  if (int rc = e->alloc((void**)&L.ffn_norm, (size_t)h * 4)) return rc;
  e->weight_bytes += L.kq_qkv.bytes + L.kq_o.bytes + L.kq_gu.bytes + L.kq_down.bytes + 2 * (size_t)h * 4;
  return 0;
}

// pack GGUF blocks of `rows` logical rows into a K-quant matrix at packed row `row0` (mode as launch_pack)
static int pack_kq_rows(const KqMat& km, uint16_t* base, const uint8_t* blocks, int type, int rows, int K, int mode,
                        int row0, hipStream_t s) {
  int in_seg = 0;
  const int sg = km.seg(row0, &in_seg);
  if (km.type[sg] != type) return -1;
  return launch_pack_kq((uint8_t*)base + km.off[sg], blocks, type, rows, K, mode, in_seg, s);
}

int mx_engine::load_synthetic(const Shape& s, uint64_t seed, bool q8, int kq_base, bool q4) {
  n_embd = s.n_embd; n_layer = s.n_layer; n_head = s.n_head; n_head_kv = s.n_head_kv; n_ff = s.n_ff;
  n_vocab = s.n_vocab; rope_base = s.rope_base; eps = s.eps; n_ctx_train = s.n_ctx_train;
  if (le < 0 || le > n_layer) le = n_layer;
  wq8 = embd_q8 = out_q8 = q8 || q4;
  wq4 = q4;  // layer matrices Q4_0 (quantize_row_q4_0_ref of the bf16 synthetic values); embd / output Q8_0
  wkq = kq_base != 0;
  if (int rc = init_common()) return rc;
  const float ws = std_scale(0.02), ns = std_scale(0.1);
  const int h = n_embd, kv = n_embd_kv, ff = n_ff, V = n_vocab;
  if (wkq) {  // synth.py kq_tensor: the recipe's types, synthetic GGUF blocks packed like a file's
    kq_main_type = kq_base;
    const int bb_max = kq_block_bytes(14) > kq_block_bytes(kq_base) ? kq_block_bytes(14) : kq_block_bytes(kq_base);
    const size_t stage_bytes = std::max({(size_t)V * h, (size_t)ff * h, (size_t)h * h}) / 256 * bb_max;
    uint8_t* stage = nullptr;
    HIPC(hipMalloc((void**)&stage, stage_bytes));
    int rc = 0;
    auto mat = [&](const KqMat& km, uint16_t* base, int type, uint64_t tid, int rows, int K, int mode, int row0) -> int {
      if (launch_synth_kq_blocks(stage, type, (size_t)rows * K / 256, seed, tid, stream)) return fail(MX_ERR_ARG, "synth kq");
      if (pack_kq_rows(km, base, stage, type, rows, K, mode, row0, stream)) return fail(MX_ERR_ARG, "pack kq");
      return 0;
    };
    if (has_embed) {
      embd_kq_type = kq_base;
      if ((rc = alloc((void**)&tok_embd_kq, (size_t)V * (h / 256) * kq_block_bytes(kq_base)))) goto kq_out_label;
      launch_synth_kq_blocks(tok_embd_kq, kq_base, (size_t)V * h / 256, seed, TID_TOK_EMBD, stream);
      weight_bytes += (size_t)(h / 256) * kq_block_bytes(kq_base);
    }
    if (has_head) {
      kq_out = KqMat();
      kq_out.add(kq_recipe_type(kq_base, -1, 0, n_layer), V, h);
      if ((rc = alloc((void**)&output, kq_out.bytes)) || (rc = alloc((void**)&out_norm, (size_t)h * 4))) goto kq_out_label;
      if ((rc = mat(kq_out, output, kq_out.type[0], TID_OUTPUT, V, h, PACK_ROWS, 0))) goto kq_out_label;
      launch_synth_norm(out_norm, h, seed, TID_OUT_NORM, ns, stream);
      weight_bytes += kq_out.bytes + h * 4;
    }
    for (int l = lb; l < le && !rc; l++) {
      Layer& L = layers[l - lb];
      int t[9] = {0};
      for (int k : {L_Q, L_K, L_V, L_O, L_GATE, L_UP, L_DOWN}) t[k] = kq_recipe_type(kq_base, k, l, n_layer);
      if ((rc = alloc_layer_kq(this, L, t))) break;
      launch_synth_norm(L.attn_norm, h, seed, layer_tid(l, L_ATTN_NORM), ns, stream);
      launch_synth_norm(L.ffn_norm, h, seed, layer_tid(l, L_FFN_NORM), ns, stream);
      if ((rc = mat(L.kq_qkv, L.qkv, t[L_Q], layer_tid(l, L_Q), h, h, PACK_ROWS, 0)) ||
          (rc = mat(L.kq_qkv, L.qkv, t[L_K], layer_tid(l, L_K), kv, h, PACK_ROWS, h)) ||
          (rc = mat(L.kq_qkv, L.qkv, t[L_V], layer_tid(l, L_V), kv, h, PACK_ROWS, h + kv)) ||
          (rc = mat(L.kq_o, L.o, t[L_O], layer_tid(l, L_O), h, h, PACK_ROWS, 0)) ||
          (rc = mat(L.kq_gu, L.gu, t[L_GATE], layer_tid(l, L_GATE), ff, h, PACK_GATE, 0)) ||
          (rc = mat(L.kq_gu, L.gu, t[L_UP], layer_tid(l, L_UP), ff, h, PACK_UP, 0)) ||
          (rc = mat(L.kq_down, L.down, t[L_DOWN], layer_tid(l, L_DOWN), h, ff, PACK_ROWS, 0)))
        break;
    }
  kq_out_label:
    hipStreamSynchronize(stream);
    hipFree(stage);
    if (rc) return rc;
    HIPC(hipGetLastError());
    return 0;
  }
  if (wq8) {  // the Q8_0 (Q4_0) quantisation of the bf16 synthetic model (what llama-quantize makes of it)
    if (has_embed) {
      if (int rc = alloc((void**)&tok_embd8, (size_t)V * (h / 32) * 34)) return rc;
      launch_synth_q8_rowmajor(tok_embd8, V, h, seed, TID_TOK_EMBD, ws, stream);
      weight_bytes += (size_t)h / 32 * 34;
    }
    if (has_head) {
      if (int rc = alloc((void**)&output, q8_matrix_bytes(V, h))) return rc;
      if (int rc = alloc((void**)&out_norm, (size_t)h * 4)) return rc;
      launch_synth_q8_packed((uint8_t*)output, V, h, seed, TID_OUTPUT, ws, PACK_ROWS, 0, stream);
      launch_synth_norm(out_norm, h, seed, TID_OUT_NORM, ns, stream);
      weight_bytes += q8_matrix_bytes(V, h) + h * 4;
    }
    for (int l = lb; l < le; l++) {
      Layer& L = layers[l - lb];
      if (int rc = alloc_layer(this, L)) return rc;
      uint8_t *qkv = (uint8_t*)L.qkv, *o = (uint8_t*)L.o, *gu = (uint8_t*)L.gu, *dn = (uint8_t*)L.down;
      launch_synth_norm(L.attn_norm, h, seed, layer_tid(l, L_ATTN_NORM), ns, stream);
      launch_synth_norm(L.ffn_norm, h, seed, layer_tid(l, L_FFN_NORM), ns, stream);
      auto syn = q4 ? launch_synth_q4_packed : launch_synth_q8_packed;
      syn(qkv, h, h, seed, layer_tid(l, L_Q), ws, PACK_ROWS, 0, stream);
      syn(qkv, kv, h, seed, layer_tid(l, L_K), ws, PACK_ROWS, h, stream);
      syn(qkv, kv, h, seed, layer_tid(l, L_V), ws, PACK_ROWS, h + kv, stream);
      syn(o, h, h, seed, layer_tid(l, L_O), ws, PACK_ROWS, 0, stream);
      syn(gu, ff, h, seed, layer_tid(l, L_GATE), ws, PACK_GATE, 0, stream);
      syn(gu, ff, h, seed, layer_tid(l, L_UP), ws, PACK_UP, 0, stream);
      syn(dn, h, ff, seed, layer_tid(l, L_DOWN), ws, PACK_ROWS, 0, stream);
    }
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(stream));
    return 0;
  }
  if (has_embed) {
    if (int rc = alloc((void**)&tok_embd, (size_t)V * h * 2)) return rc;
    launch_synth_rowmajor(tok_embd, (size_t)V * h, seed, TID_TOK_EMBD, ws, stream);
    weight_bytes += (size_t)h * 2;  // one embedding row per token
  }
  if (has_head) {
    if (int rc = alloc((void**)&output, (size_t)V * h * 2)) return rc;
    if (int rc = alloc((void**)&out_norm, (size_t)h * 4)) return rc;
    launch_synth_packed(output, V, h, seed, TID_OUTPUT, ws, PACK_ROWS, 0, stream);
    launch_synth_norm(out_norm, h, seed, TID_OUT_NORM, ns, stream);
    weight_bytes += (size_t)V * h * 2 + h * 4;
  }
  for (int l = lb; l < le; l++) {
    Layer& L = layers[l - lb];
    if (int rc = alloc_layer(this, L)) return rc;
    launch_synth_norm(L.attn_norm, h, seed, layer_tid(l, L_ATTN_NORM), ns, stream);
    launch_synth_norm(L.ffn_norm, h, seed, layer_tid(l, L_FFN_NORM), ns, stream);
    launch_synth_packed(L.qkv, h, h, seed, layer_tid(l, L_Q), ws, PACK_ROWS, 0, stream);
    launch_synth_packed(L.qkv, kv, h, seed, layer_tid(l, L_K), ws, PACK_ROWS, h, stream);
    launch_synth_packed(L.qkv, kv, h, seed, layer_tid(l, L_V), ws, PACK_ROWS, h + kv, stream);
    launch_synth_packed(L.o, h, h, seed, layer_tid(l, L_O), ws, PACK_ROWS, 0, stream);
    launch_synth_packed(L.gu, ff, h, seed, layer_tid(l, L_GATE), ws, PACK_GATE, 0, stream);
    launch_synth_packed(L.gu, ff, h, seed, layer_tid(l, L_UP), ws, PACK_UP, 0, stream);
    launch_synth_packed(L.down, h, ff, seed, layer_tid(l, L_DOWN), ws, PACK_ROWS, 0, stream);
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(stream));
  return 0;
}

int mx_engine::load_gguf(const std::string& path) {
  GGUFFile f;
  std::string err = f.open(path);
  if (!err.empty()) return fail(MX_ERR_MODEL, err);
  const GGUFValue* arch = f.get("general.architecture");
  if (!arch || arch->str != "llama") return fail(MX_ERR_MODEL, "general.architecture must be 'llama'");
  n_embd = (int)f.get_num("llama.embedding_length", 0);
  n_layer = (int)f.get_num("llama.block_count", 0);
  n_head = (int)f.get_num("llama.attention.head_count", 0);
  n_head_kv = (int)f.get_num("llama.attention.head_count_kv", n_head);
  n_ff = (int)f.get_num("llama.feed_forward_length", 0);
  eps = (float)f.get_num("llama.attention.layer_norm_rms_epsilon", 1e-5);
  rope_base = (float)f.get_num("llama.rope.freq_base", 10000.0);
  n_ctx_train = (int)f.get_num("llama.context_length", 2048);
  bos = (int)f.get_num("tokenizer.ggml.bos_token_id", 1);
  eos = (int)f.get_num("tokenizer.ggml.eos_token_id", 2);
  const GGUFTensor* te = f.tensor("token_embd.weight");
  if (!te || te->ne.size() != 2) return fail(MX_ERR_MODEL, "missing token_embd.weight");
  n_vocab = (int)te->ne[1];
  if (!n_embd || !n_layer || !n_head || !n_ff) return fail(MX_ERR_MODEL, "missing llama.* hyper-parameters");
  if ((int)f.get_num("llama.rope.dimension_count", n_embd / n_head) != n_embd / n_head)
    return fail(MX_ERR_MODEL, "partial RoPE (rope.dimension_count != head_dim) is not supported");
  {  // RoPE scaling: llama.cpp's "linear" (freq_scale = 1/factor) and Llama-3.1 frequency factors
    const GGUFValue* st = f.get("llama.rope.scaling.type");
    const std::string stype = st ? st->str : "none";
    const double factor = f.get_num("llama.rope.scaling.factor", 0.0);
    if (stype == "linear") {
      if (!(factor > 0)) return fail(MX_ERR_MODEL, "linear RoPE scaling without a positive factor");
      rope_freq_scale = (float)(1.0 / factor);
    } else if (stype != "none" && !stype.empty()) {
      return fail(MX_ERR_MODEL, "RoPE scaling type '" + stype + "' is not supported (none, linear and rope_freqs are)");
    }
    if (const GGUFTensor* rf = f.tensor("rope_freqs.weight")) {
      const int half = n_embd / n_head / 2;
      if (rf->type != 0 || rf->ne.size() != 1 || (int)rf->ne[0] != half)
        return fail(MX_ERR_MODEL, "rope_freqs.weight must be f32 [head_dim/2]");
      rope_ff.resize(half);
      memcpy(rope_ff.data(), f.data(*rf), half * 4);
      for (float v : rope_ff)
        if (!(v > 0)) return fail(MX_ERR_MODEL, "rope_freqs.weight has a non-positive factor");
    }
  }
  if (le < 0 || le > n_layer) le = n_layer;
  // Matrix types.  All BF16 -> the bf16 path; all Q8_0 -> the Q8_0 path (int8 MFMA on the blocks);
  // all Q4_K / Q5_K / Q6_K with ffn_gate and ffn_up of one type (llama.cpp's Q4_K_M, Q5_K_M files) ->
  // the K-quant path (kquant.hip: int8 MFMA on the blocks with Q8_K activations); any other mix of
  // F32 / F16 / BF16 / Q4_0 / Q8_0 / K-quants -> every matrix is dequantised to bf16 at load
  // (ggml's dequantize_row_*) and runs on the bf16 path.
  bool deq = false;
  size_t raw_max = 0;
  {
    const int b0 = lb < 0 ? 0 : lb, e0 = (le < 0 || le > n_layer) ? n_layer : le;
    std::vector<std::string> mats;
    static const char* kinds[] = {"attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down"};
    for (int l = b0; l < e0; l++)
      for (const char* k : kinds) mats.push_back("blk." + std::to_string(l) + "." + k + ".weight");
    if (e0 == n_layer) mats.push_back(f.tensor("output.weight") ? "output.weight" : "token_embd.weight");
    int n8 = 0, n30 = 0, nkq = 0, n4 = 0;
    for (const std::string& nm : mats) {
      const GGUFTensor* t = f.tensor(nm);
      if (!t) return fail(MX_ERR_MODEL, "missing tensor " + nm);
      if (t->type != 30 && !ggml_block_elems(t->type))
        return fail(MX_ERR_MODEL, "tensor " + nm + ": ggml type " + std::to_string(t->type) +
                                      " is not supported (F32, F16, BF16, Q4_0, Q8_0, Q4_K, Q5_K, Q6_K are)");
      n8 += t->type == 8;
      n4 += t->type == 2 && nm != mats.back();  // layer matrices only (the head is checked below)
      n30 += t->type == 30;
      nkq += t->type == 12 || t->type == 13 || t->type == 14;
      raw_max = std::max(raw_max, (size_t)t->nbytes);
    }
    wq8 = out_q8 = n8 == (int)mats.size();
    if (!wq8 && n4 == (int)mats.size() - (e0 == n_layer ? 1 : 0) && n4 > 0) {
      // Q4_0 layers; the head: Q8_0 / Q4_0 tiles, or a K-quant output (llama-quantize's Q6_K) on the
      // K-quant kernels -- anything else dequantises the whole model as before
      const int ot = e0 == n_layer ? f.tensor(mats.back())->type : 8;
      if (ot == 8 || ot == 2 || ((ot == 12 || ot == 13 || ot == 14) && n_embd % 256 == 0)) {
        wq8 = wq4 = true;
        out_q8 = ot == 8 || ot == 2;
        out_q4 = ot == 2;
        out_kq_head = !out_q8;
      }
    }
    wkq = nkq == (int)mats.size() && n_embd % 256 == 0 && n_ff % 256 == 0;
    for (int l = b0; l < e0 && wkq; l++) {
      const std::string p = "blk." + std::to_string(l) + ".";
      if (f.tensor(p + "ffn_gate.weight")->type != f.tensor(p + "ffn_up.weight")->type) wkq = false;
    }
    if (wkq) kq_main_type = f.tensor("blk." + std::to_string(b0) + ".ffn_gate.weight")->type;
    deq = !wq8 && !wkq && n30 != (int)mats.size();
    if (wq8 && !out_q8) deq = false;
    embd_q8 = te->type == 8;
    if (wkq && (te->type == 12 || te->type == 13 || te->type == 14)) embd_kq_type = te->type;
    if (te->type != 30 && te->type != 8) {
      if (!ggml_block_elems(te->type))
        return fail(MX_ERR_MODEL, "token_embd.weight: ggml type " + std::to_string(te->type) + " is not supported");
      raw_max = std::max(raw_max, (size_t)te->nbytes);
    }
  }
  if (int rc = init_common()) return rc;
  const int h = n_embd, kv = n_embd_kv, ff = n_ff, V = n_vocab;
  const int mat_type = wq4 ? 2 : wq8 ? 8 : 30;

  // staging buffer for the largest matrix (bf16), and for the raw blocks of dequantised tensors
  size_t stage_bytes = std::max({(size_t)V * h * 2, (size_t)ff * h * 2, (size_t)(h + 2 * kv) * h * 2});
  uint16_t* stage = nullptr;
  uint8_t* stage_raw = nullptr;
  HIPC(hipMalloc((void**)&stage, stage_bytes));
  if (raw_max && (deq || wkq || out_kq_head || (te->type != 30 && te->type != 8))) {
    if (hipMalloc((void**)&stage_raw, raw_max) != hipSuccess) {
      hipFree(stage);
      return fail(MX_ERR_HIP, "staging buffer");
    }
  }
  // any supported type -> bf16 row-major in `stage`
  auto to_bf16 = [&](const GGUFTensor* t, size_t n) -> int {
    if (t->type == 30) {
      HIPC(hipMemcpy(stage, f.data(*t), t->nbytes, hipMemcpyHostToDevice));
      return 0;
    }
    HIPC(hipMemcpy(stage_raw, f.data(*t), t->nbytes, hipMemcpyHostToDevice));
    if (launch_dequant_bf16(stage, stage_raw, t->type, n, stream)) return fail(MX_ERR_MODEL, "dequantise " + t->name);
    return 0;
  };
  auto get_mat = [&](const std::string& name, int rows, int cols, const GGUFTensor** out, int type) -> int {
    const GGUFTensor* t = f.tensor(name);
    if (!t) return fail(MX_ERR_MODEL, "missing tensor " + name);
    if (t->ne.size() != 2 || (int)t->ne[0] != cols || (int)t->ne[1] != rows)
      return fail(MX_ERR_MODEL, "tensor " + name + " has unexpected shape");
    if (t->type != type && !(deq && type == 30))
      return fail(MX_ERR_MODEL, "tensor " + name + ": expected ggml type " + std::to_string(type) +
                                    (type == 8 ? " (Q8_0, like the other matrices)"
                                     : type == 2 ? " (Q4_0, like the other matrices)" : " (BF16, like the other matrices)") +
                                    ", got type " + std::to_string(t->type));
    *out = t;
    return 0;
  };
  auto upload_packed = [&](const std::string& name, int rows, int cols, uint16_t* dst, int mode,
                           int offset) -> int {
    const GGUFTensor* t = nullptr;
    if (int rc = get_mat(name, rows, cols, &t, mat_type)) return rc;
    if (wq8) {
      HIPC(hipMemcpy(stage, f.data(*t), t->nbytes, hipMemcpyHostToDevice));
      if (t->type == 2) launch_pack_q4((uint8_t*)dst, (const uint8_t*)stage, rows, cols, mode, offset, stream);
      else launch_pack_q8((uint8_t*)dst, (const uint8_t*)stage, rows, cols, mode, offset, stream);
    } else {
      if (int rc = to_bf16(t, (size_t)rows * cols)) return rc;
      launch_pack(dst, stage, rows, cols, mode, offset, stream);
    }
    HIPC(hipStreamSynchronize(stream));
    return 0;
  };
  auto upload_norm = [&](const std::string& name, float* dst) -> int {
    const GGUFTensor* t = f.tensor(name);
    if (!t || t->type != 0 || t->ne[0] != (uint64_t)h) return fail(MX_ERR_MODEL, "bad/missing f32 norm " + name);
    HIPC(hipMemcpy(dst, f.data(*t), (size_t)h * 4, hipMemcpyHostToDevice));
    return 0;
  };
  // K-quant matrix: raw blocks to the device, packed into the segment holding packed row row0
  auto upload_kq = [&](const std::string& name, int rows, int cols, const KqMat& km, uint16_t* dst, int mode,
                       int row0) -> int {
    const GGUFTensor* t = f.tensor(name);
    if (!t) return fail(MX_ERR_MODEL, "missing tensor " + name);
    if (t->ne.size() != 2 || (int)t->ne[0] != cols || (int)t->ne[1] != rows)
      return fail(MX_ERR_MODEL, "tensor " + name + " has unexpected shape");
    HIPC(hipMemcpy(stage_raw, f.data(*t), t->nbytes, hipMemcpyHostToDevice));
    if (pack_kq_rows(km, dst, stage_raw, t->type, rows, cols, mode, row0, stream))
      return fail(MX_ERR_MODEL, "tensor " + name + ": K-quant type does not match its matrix segment");
    HIPC(hipStreamSynchronize(stream));
    return 0;
  };
  auto kq_layer_types = [&](int l, int t[9]) {
    const std::string p = "blk." + std::to_string(l) + ".";
    static const char* nm[9] = {nullptr, "attn_q", "attn_k", "attn_v", "attn_output", nullptr, "ffn_gate", "ffn_up", "ffn_down"};
    for (int k = 0; k < 9; k++) t[k] = nm[k] ? f.tensor(p + nm[k] + ".weight")->type : 0;
  };
  int rc = 0;
  if (wkq) {
    if (has_embed) {
      const GGUFTensor* t = f.tensor("token_embd.weight");
      if (t->ne.size() != 2 || (int)t->ne[0] != h || (int)t->ne[1] != V) {
        rc = fail(MX_ERR_MODEL, "tensor token_embd.weight has unexpected shape");
        goto out;
      }
      if (embd_kq_type) {  // GET_ROWS dequantises the blocks per lookup (dequantize_row_q*_K)
        if ((rc = alloc((void**)&tok_embd_kq, t->nbytes))) goto out;
        if (hipMemcpy(tok_embd_kq, f.data(*t), t->nbytes, hipMemcpyHostToDevice) != hipSuccess) {
          rc = fail(MX_ERR_HIP, "upload token_embd");
          goto out;
        }
        weight_bytes += t->nbytes / V;
      } else if (t->type == 30 || t->type == 8) {  // BF16 rows as stored; Q8_0 rows dequantised per lookup
        void** dst = embd_q8 ? (void**)&tok_embd8 : (void**)&tok_embd;
        if ((rc = alloc(dst, t->nbytes))) goto out;
        if (hipMemcpy(*dst, f.data(*t), t->nbytes, hipMemcpyHostToDevice) != hipSuccess) {
          rc = fail(MX_ERR_HIP, "upload token_embd");
          goto out;
        }
        weight_bytes += t->nbytes / V;
      } else {  // F32 / F16 / Q4_0 / ... (llama-quantize --token-embedding-type): a bf16 table once
        if ((rc = alloc((void**)&tok_embd, (size_t)V * h * 2))) goto out;
        if ((rc = to_bf16(t, (size_t)V * h))) goto out;
        if (hipMemcpyAsync(tok_embd, stage, (size_t)V * h * 2, hipMemcpyDeviceToDevice, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess) {
          rc = fail(MX_ERR_HIP, "upload token_embd");
          goto out;
        }
        weight_bytes += (size_t)h * 2;
      }
    }
    if (has_head) {
      const char* oname = f.tensor("output.weight") ? "output.weight" : "token_embd.weight";  // tied embeddings
      kq_out = KqMat();
      kq_out.add(f.tensor(oname)->type, V, h);
      if ((rc = alloc((void**)&output, kq_out.bytes))) goto out;
      if ((rc = alloc((void**)&out_norm, (size_t)h * 4))) goto out;
      if ((rc = upload_kq(oname, V, h, kq_out, output, PACK_ROWS, 0))) goto out;
      if ((rc = upload_norm("output_norm.weight", out_norm))) goto out;
      weight_bytes += kq_out.bytes + h * 4;
    }
    for (int l = lb; l < le; l++) {
      Layer& L = layers[l - lb];
      const std::string p = "blk." + std::to_string(l) + ".";
      int t[9];
      kq_layer_types(l, t);
      if ((rc = alloc_layer_kq(this, L, t))) goto out;
      if ((rc = upload_norm(p + "attn_norm.weight", L.attn_norm))) goto out;
      if ((rc = upload_norm(p + "ffn_norm.weight", L.ffn_norm))) goto out;
      if ((rc = upload_kq(p + "attn_q.weight", h, h, L.kq_qkv, L.qkv, PACK_ROWS, 0))) goto out;
      if ((rc = upload_kq(p + "attn_k.weight", kv, h, L.kq_qkv, L.qkv, PACK_ROWS, h))) goto out;
      if ((rc = upload_kq(p + "attn_v.weight", kv, h, L.kq_qkv, L.qkv, PACK_ROWS, h + kv))) goto out;
      if ((rc = upload_kq(p + "attn_output.weight", h, h, L.kq_o, L.o, PACK_ROWS, 0))) goto out;
      if ((rc = upload_kq(p + "ffn_gate.weight", ff, h, L.kq_gu, L.gu, PACK_GATE, 0))) goto out;
      if ((rc = upload_kq(p + "ffn_up.weight", ff, h, L.kq_gu, L.gu, PACK_UP, 0))) goto out;
      if ((rc = upload_kq(p + "ffn_down.weight", h, ff, L.kq_down, L.down, PACK_ROWS, 0))) goto out;
    }
    goto out;
  }
  if (has_embed) {
    const GGUFTensor* t = f.tensor("token_embd.weight");
    if (t->ne.size() != 2 || (int)t->ne[0] != h || (int)t->ne[1] != V) {
      rc = fail(MX_ERR_MODEL, "tensor token_embd.weight has unexpected shape");
      goto out;
    }
    if (t->type == 30 || t->type == 8) {  // rows used as stored (Q8_0 rows dequantised per lookup)
      void** dst = embd_q8 ? (void**)&tok_embd8 : (void**)&tok_embd;
      if ((rc = alloc(dst, t->nbytes))) goto out;
      if (hipMemcpy(*dst, f.data(*t), t->nbytes, hipMemcpyHostToDevice) != hipSuccess) {
        rc = fail(MX_ERR_HIP, "upload token_embd");
        goto out;
      }
      weight_bytes += t->nbytes / V;
    } else {  // other block types: dequantised to a bf16 table once
      if ((rc = alloc((void**)&tok_embd, (size_t)V * h * 2))) goto out;
      if ((rc = to_bf16(t, (size_t)V * h))) goto out;
      if (hipMemcpyAsync(tok_embd, stage, (size_t)V * h * 2, hipMemcpyDeviceToDevice, stream) != hipSuccess ||
          hipStreamSynchronize(stream) != hipSuccess) {
        rc = fail(MX_ERR_HIP, "upload token_embd");
        goto out;
      }
      weight_bytes += (size_t)h * 2;
    }
  }
  if (has_head) {
    const char* oname = f.tensor("output.weight") ? "output.weight" : "token_embd.weight";  // tied embeddings
    if ((rc = alloc((void**)&out_norm, (size_t)h * 4))) goto out;
    if ((rc = upload_norm("output_norm.weight", out_norm))) goto out;
    if (out_kq_head) {  // Q4_0 model with a K-quant output: packed K-quant tiles for mkq
      kq_out = KqMat();
      kq_out.add(f.tensor(oname)->type, V, h);
      if ((rc = alloc((void**)&output, kq_out.bytes))) goto out;
      if ((rc = upload_kq(oname, V, h, kq_out, output, PACK_ROWS, 0))) goto out;
      weight_bytes += kq_out.bytes + h * 4;
    } else {
      const size_t ob = out_q4 ? q4_matrix_bytes(V, h) : wq8 ? q8_matrix_bytes(V, h) : (size_t)V * h * 2;
      if ((rc = alloc((void**)&output, ob))) goto out;
      const GGUFTensor* ot = nullptr;
      if (wq8) {  // the head keeps its own block type (Q8_0 or Q4_0 tiles)
        ot = f.tensor(oname);
        if (!ot || ot->ne.size() != 2 || (int)ot->ne[0] != h || (int)ot->ne[1] != V) {
          rc = fail(MX_ERR_MODEL, "tensor output.weight has unexpected shape");
          goto out;
        }
        if (hipMemcpy(stage, f.data(*ot), ot->nbytes, hipMemcpyHostToDevice) != hipSuccess) {
          rc = fail(MX_ERR_HIP, "upload output");
          goto out;
        }
        if (out_q4) launch_pack_q4((uint8_t*)output, (const uint8_t*)stage, V, h, PACK_ROWS, 0, stream);
        else launch_pack_q8((uint8_t*)output, (const uint8_t*)stage, V, h, PACK_ROWS, 0, stream);
        hipStreamSynchronize(stream);
      } else if ((rc = upload_packed(oname, V, h, output, PACK_ROWS, 0))) {
        goto out;
      }
      weight_bytes += ob + h * 4;
    }
  }
  for (int l = lb; l < le; l++) {
    Layer& L = layers[l - lb];
    const std::string p = "blk." + std::to_string(l) + ".";
    if ((rc = alloc_layer(this, L))) goto out;
    if ((rc = upload_norm(p + "attn_norm.weight", L.attn_norm))) goto out;
    if ((rc = upload_norm(p + "ffn_norm.weight", L.ffn_norm))) goto out;
    if ((rc = upload_packed(p + "attn_q.weight", h, h, L.qkv, PACK_ROWS, 0))) goto out;
    if ((rc = upload_packed(p + "attn_k.weight", kv, h, L.qkv, PACK_ROWS, h))) goto out;
    if ((rc = upload_packed(p + "attn_v.weight", kv, h, L.qkv, PACK_ROWS, h + kv))) goto out;
    if ((rc = upload_packed(p + "attn_output.weight", h, h, L.o, PACK_ROWS, 0))) goto out;
    if ((rc = upload_packed(p + "ffn_gate.weight", ff, h, L.gu, PACK_GATE, 0))) goto out;
    if ((rc = upload_packed(p + "ffn_up.weight", ff, h, L.gu, PACK_UP, 0))) goto out;
    if ((rc = upload_packed(p + "ffn_down.weight", h, ff, L.down, PACK_ROWS, 0))) goto out;
  }
out:
  hipStreamSynchronize(stream);
  hipFree(stage);
  if (stage_raw) hipFree(stage_raw);
  return rc;
}

// One forward of M <= MAX_ROWS rows through this stage's layers.
int mx_engine::enqueue_forward(int M, const int* ids, const int* pos, const int* slot, const void* x_in, void* x_out,
                               bool head, const int* rowmap, int n_out, bool argmax, int* ids_next, int* pos_next,
                               int* hist, int hist_stride, int* hist_count, int max_hist, hipStream_t s) {
  const int h = n_embd, kv = n_embd_kv, ff = n_ff;
  const bool wide = use_wide && M > 16;
  // RMS_NORM applied on load by the consuming GEMV (M <= 16); the residual-stream writers
  // (embedding, attn_output, ffn_down, or ssq_kernel for a stage's x_in) leave per-tile partials
  const bool nol = !wide && !wq8 && !wkq && norm_on_load && mm_can_norm_on_load(M, h);
  const bool qql = q8_on_load(M) || kq_on_load(M);  // residual-stream Σx² partials wanted
  if (x_in) {
    if (handoff_bf16) {  // bf16 hand-off from the previous stage: widen, with the Σx² partials on the way
      launch_bf16_to_f32(x, (const uint16_t*)x_in, M, h, (nol || qql) ? ssq : nullptr, s);
    } else {
      launch_f32_in(x, (const float*)x_in, M, h, (nol || qql) ? ssq : nullptr, s);
    }
  } else {
    if (!has_embed) return fail(MX_ERR_STATE, "this stage has no token embedding: x_in required");
    if (embd_kq_type) {
      if (launch_embed_kq(x, tok_embd_kq, embd_kq_type, ids, M, h, qql ? ssq : nullptr, s))
        return fail(MX_ERR_ARG, "K-quant embedding");
    } else if (embd_q8) {
      launch_embed_q8(x, tok_embd8, ids, M, h, (nol || qql) ? ssq : nullptr, s);
    } else {
      launch_embed(x, tok_embd, ids, M, h, (nol || qql) ? ssq : nullptr, s);
    }
  }
  if (wkq && !kq_ggml_prefill && M > MAX_ROWS && kqd_qkv && !argmax && !(head && n_out > MAX_ROWS))
    return enqueue_forward_gemm(M, pos, slot, x_out, head, rowmap, n_out, s);  // dequantised bf16 GEMMs
  // Q8_0 prefill chunks as dequantised bf16 GEMMs (llama.cpp's GPU-backend route for large batches):
  // ~5x the default's rate, but bf16 activations instead of ggml's Q8_0 rows, so opt-in
  // (MX_Q8_GEMM_PREFILL=1; tests/test_q8_gpu.py bounds its deviation)
  if (wq8 && !wq4 && q8_gemm_prefill && M > MAX_ROWS && kqd_qkv && !argmax && !(head && n_out > MAX_ROWS))
    return enqueue_forward_gemm(M, pos, slot, x_out, head, rowmap, n_out, s);
  if (wkq) return enqueue_forward_kq(M, pos, slot, x_out, head, rowmap, n_out, argmax, ids_next, pos_next, hist,
                                     hist_stride, hist_count, max_hist, s);
  if (wq8) return enqueue_forward_q8(M, pos, slot, x_out, head, rowmap, n_out, argmax, ids_next, pos_next, hist,
                                     hist_stride, hist_count, max_hist, s);
  if (prefill_gemm && M <= MAX_ROWS && use_wide && gemm_shapes() && !argmax)  // small prompt chunk, GEMM order
    return enqueue_forward_wide(M, pos, slot, x_out, head, rowmap, n_out, false, nullptr, nullptr, nullptr, 0,
                                nullptr, 0, s, true);
  if (M > MAX_ROWS || (prefill_gemm && gemm_shapes() && !argmax)) {
    if (!gemm_ok() || argmax || (head && n_out > MAX_ROWS))
      return fail(MX_ERR_ARG, "forward of > 64 rows: GEMM shapes only, logits for <= 64 rows");
    return enqueue_forward_gemm(M, pos, slot, x_out, head, rowmap, n_out, s);
  }
  if (wide) return enqueue_forward_wide(M, pos, slot, x_out, head, rowmap, n_out, argmax, ids_next,
                                        pos_next, hist, hist_stride, hist_count, max_hist, s);
  // on-load only for attn_norm -> qkv: qkv's 384 work-groups run 1.5 rounds, so its per-work-group
  // prologue costs less than a norm launch; gate/up (7 rounds) and lm_head (31) keep the norm kernel
  // (tools/kernel_probe.py, profiles/round1_norm_on_load.txt)
  auto norm_operand = [&](MMArgs& m, const float* w, bool on_load) {
    if (nol && on_load) {
      m.X = nullptr; m.xf = x; m.norm_w = w; m.eps = eps; m.ssq = ssq; m.np = h / 16;
    } else {
      launch_rmsnorm(xn, h, x, w, nullptr, M, h, eps, s);
      m.X = xn; m.ldx = h;
    }
  };
  for (int li = 0; li < (int)layers.size(); li++) {
    const Layer& L = layers[li];
    _Float16* kc = kcache + layer_kv_stride * li;
    _Float16* vc = vcache + layer_kv_stride * li;
    MMArgs a{};
    a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.M = M;
    norm_operand(a, L.attn_norm, true);
    a.out = q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = head_dim; a.pos = pos; a.slot = slot;
    a.rope_cs = rope_cs; a.kc = kc; a.vc = vc; a.n_ctx = n_ctx; a.ctx_stride = ctx_stride; a.n_head_kv = n_head_kv;
    a.slot_stride = slot_stride;
    AttnArgs at{};
    at.q = q; at.kc = kc; at.vc = vc; at.pos = pos; at.slot = slot;
    at.out = attn_out; at.ldo = h; at.M = M; at.n_head = n_head; at.n_head_kv = n_head_kv; at.head_dim = head_dim;
    at.n_ctx = n_ctx; at.ctx_stride = ctx_stride; at.slot_stride = slot_stride;
    at.scale = 1.0f / sqrtf((float)head_dim);
    const bool pers_qkv = use_pers && a.X == nullptr && mm_pers_supported(EPI_QKV, M, a.N, h);
    if ((pers_qkv ? launch_mm_pers(EPI_QKV, a, s) : -1) != 0 && launch_mm(EPI_QKV, a, s))
      return fail(MX_ERR_ARG, "qkv launch shape");
    MMArgs b{};
    b.W = L.o; b.N = h; b.K = h; b.X = attn_out; b.ldx = h; b.M = M; b.out = x; b.ldo = h;
    if (use_pers && nol && mm_pers_supported(EPI_SWIGLU, M, 2 * ff, h)) {  // partials for gate/up's norm on load
      b.ssq = ssq; b.np = h / 16;
    }
    launch_attention(at, s);
    if ((mm_pers_supported(EPI_RESID, M, h, h) ? launch_mm_pers(EPI_RESID, b, s) : -1) != 0 &&
        launch_mm(EPI_RESID, b, s))
      return fail(MX_ERR_ARG, "attn_output launch shape");
    MMArgs c{};
    c.W = L.gu; c.N = 2 * ff; c.K = h; c.M = M;
    const bool pers_gu = use_pers && nol && mm_pers_supported(EPI_SWIGLU, M, 2 * ff, h);
    norm_operand(c, L.ffn_norm, pers_gu);
    c.act = act; c.lda = ff;
    if ((pers_gu ? launch_mm_pers(EPI_SWIGLU, c, s) : -1) != 0 && launch_mm(EPI_SWIGLU, c, s))
      return fail(MX_ERR_ARG, "ffn gate/up launch shape");
    MMArgs d{};
    d.W = L.down; d.N = h; d.K = ff; d.X = act; d.ldx = ff; d.M = M; d.out = x; d.ldo = h;
    d.ssq = nol ? ssq : nullptr; d.np = h / 16;
    if ((mm_pers_supported(EPI_RESID, M, h, ff) ? launch_mm_pers(EPI_RESID, d, s) : -1) != 0 &&
        launch_mm(EPI_RESID, d, s))
      return fail(MX_ERR_ARG, "ffn_down launch shape");
  }
  if (x_out)
    if (int rc = copy_out(x_out, M, s)) return rc;
  if (head) {
    if (!has_head) return fail(MX_ERR_STATE, "this stage has no output head");
    MMArgs g{};
    g.W = output; g.N = n_vocab; g.K = h; g.M = n_out; g.out = logits; g.ldo = n_vocab;
    // lm_head as a row-tile-persistent GEMV with the output RMS_NORM on load (no norm launch)
    const bool pers_head = use_pers && nol && !rowmap && n_out == M && mm_pers_supported(EPI_F32, M, n_vocab, h);
    if (!rowmap && n_out == M) {
      norm_operand(g, out_norm, pers_head);
    } else {
      launch_rmsnorm(xn, h, x, out_norm, rowmap, n_out, h, eps, s);
      g.X = xn; g.ldx = h;
    }
    if ((pers_head ? launch_mm_pers(EPI_F32, g, s) : -1) != 0 && launch_mm(EPI_F32, g, s))
      return fail(MX_ERR_ARG, "lm_head launch shape");
    if (argmax)
      pick(n_out, ids_next, pos_next, hist, hist_stride,
                    hist_count, max_hist, s);
  }
  HIPC(hipGetLastError());
  return 0;
}

// 17..64 rows: wide GEMVs (activations shared through LDS); attn_output and ffn_down run split-K
// into slabs that the next resid_norm folds into the residual stream in a fixed order.
// full_chain: a prompt chunk of <= 64 rows (prefill_gemm) -- every GEMV one MFMA chain over K, the
// prefill GEMM's order, so a prompt row's values do not depend on whether its chunk had 40 rows or 4000;
// the prompt's 16-row blocks take the prefill attention as in the GEMM path
int mx_engine::enqueue_forward_wide(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap,
                                    int n_out, bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride,
                                    int* hist_count, int max_hist, hipStream_t s, bool full_chain) {
  const int h = n_embd, kv = n_embd_kv, ff = n_ff;
  int nslab = 0;  // partial slabs not yet folded into x
  dbg_count = 0;
  for (int li = 0; li < (int)layers.size(); li++) {
    const Layer& L = layers[li];
    _Float16* kc = kcache + layer_kv_stride * li;
    _Float16* vc = vcache + layer_kv_stride * li;
    launch_resid_norm(xn, h, x, slabs, nslab, slab_stride, L.attn_norm, M, h, eps, s);
    nslab = 0;
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    MMArgs a{};
    a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.M = M; a.X = xn; a.ldx = h;
    a.out = q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = head_dim; a.pos = pos; a.slot = slot;
    a.rope_cs = rope_cs; a.kc = kc; a.vc = vc; a.n_ctx = n_ctx; a.ctx_stride = ctx_stride; a.n_head_kv = n_head_kv;
    a.slot_stride = slot_stride;
    const int qsplit = launch_mm_wide(EPI_QKV, a, slabs, slab_stride, s, false, full_chain);
    if (qsplit < 0) return fail(MX_ERR_ARG, "wide qkv launch shape");
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    if (!rows_distinct) {  // rows of one sequence attend to each other's new K/V: finish them first
      launch_qkv_finish(a, slabs, qsplit, slab_stride, s);
      if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    }
    AttnArgs at{};
    if (rows_distinct) {  // the attention kernel finishes q/k/v from the split-K slabs
      at.slabs = slabs; at.nslab = qsplit; at.slab_stride = slab_stride; at.rope_cs = rope_cs; at.kc_w = kc;
      at.vc_w = vc;
    }
    at.q = q; at.kc = kc; at.vc = vc; at.pos = pos; at.slot = slot;
    at.out = attn_out; at.ldo = h; at.M = M; at.n_head = n_head; at.n_head_kv = n_head_kv; at.head_dim = head_dim;
    at.n_ctx = n_ctx; at.ctx_stride = ctx_stride; at.slot_stride = slot_stride;
    at.scale = 1.0f / sqrtf((float)head_dim);
    if (full_chain && rows_blocked) launch_attention_prefill(at, s);
    else launch_attention(at, s);
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    MMArgs b{};
    b.W = L.o; b.N = h; b.K = h; b.X = attn_out; b.ldx = h; b.M = M;
    if ((nslab = launch_mm_wide(EPI_RESID, b, slabs, slab_stride, s, true, full_chain)) < 0)
      return fail(MX_ERR_ARG, "wide attn_output launch shape");
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    launch_resid_norm(xn, h, x, slabs, nslab, slab_stride, L.ffn_norm, M, h, eps, s);
    nslab = 0;
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    MMArgs c{};
    c.W = L.gu; c.N = 2 * ff; c.K = h; c.M = M; c.X = xn; c.ldx = h; c.act = act; c.lda = ff;
    if (launch_mm_wide(EPI_SWIGLU, c, slabs, slab_stride, s, true, full_chain) < 0)
      return fail(MX_ERR_ARG, "wide gate/up launch shape");
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
    MMArgs d{};
    d.W = L.down; d.N = h; d.K = ff; d.X = act; d.ldx = ff; d.M = M;
    if ((nslab = launch_mm_wide(EPI_RESID, d, slabs, slab_stride, s, true, full_chain)) < 0)
      return fail(MX_ERR_ARG, "wide ffn_down launch shape");
    if (dbg_hit(s)) return fail(MX_DEBUG_STOPPED, "forward ended at the mx_debug stop");
  }
  if (x_out || (head && rowmap)) {
    launch_resid_norm(nullptr, 0, x, slabs, nslab, slab_stride, nullptr, M, h, eps, s);
    nslab = 0;
  }
  if (x_out)
    if (int rc = copy_out(x_out, M, s)) return rc;
  if (head) {
    if (!has_head) return fail(MX_ERR_STATE, "this stage has no output head");
    if (rowmap || n_out != M) {
      launch_rmsnorm(xn, h, x, out_norm, rowmap, n_out, h, eps, s);
    } else {
      launch_resid_norm(xn, h, x, slabs, nslab, slab_stride, out_norm, M, h, eps, s);
      nslab = 0;
    }
    MMArgs g{};
    g.W = output; g.N = n_vocab; g.K = h; g.M = n_out; g.X = xn; g.ldx = h; g.out = logits; g.ldo = n_vocab;
    const int rc = n_out > 16 ? launch_mm_wide(EPI_F32, g, slabs, slab_stride, s) : launch_mm(EPI_F32, g, s);
    if (rc < 0) return fail(MX_ERR_ARG, "lm_head launch shape");
    if (argmax)
      pick(n_out, ids_next, pos_next, hist, hist_stride,
                    hist_count, max_hist, s);
  } else if (nslab) {
    launch_resid_norm(nullptr, 0, x, slabs, nslab, slab_stride, nullptr, M, h, eps, s);
  }
  HIPC(hipGetLastError());
  return 0;
}

// Q8_0 model, any M <= PREFILL_ROWS: every MUL_MAT takes Q8_0 activation rows made by the norm
// (RMS_NORM + MUL + quantise) or by launch_quantize_q8 from the f32 attention output / SwiGLU
// product -- ggml's conversion of src1 to the weight's vec_dot_type.
int mx_engine::enqueue_forward_q8(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap,
                                  int n_out, bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride,
                                  int* hist_count, int max_hist, hipStream_t s) {
  const int h = n_embd, kv = n_embd_kv, ff = n_ff;
  if (head && n_out > MAX_ROWS) return fail(MX_ERR_ARG, "logits for at most 64 rows per forward");
  // <= 4 rows: every GEMV quantises its operand on load (RMS_NORM from the ssq partials the
  // residual writers leave); more rows: Q8_0 rows made once per GEMV by a norm / quantise launch
  const bool ql = q8_on_load(M);
  // 17..32 rows: attn_output / ffn_down as split-K slabs (launch_mq8_slab) folded by the next
  // RMS_NORM + quantise launch; nslab = partials not yet folded into x
  int nslab = 0;
  auto operand = [&](MMArgs& m, const float* src, int K, const float* norm_w, int rows, const int* rmap) {
    if (ql && !rmap) {
      m.xq = nullptr; m.xf = src; m.norm_w = norm_w; m.eps = eps; m.ssq = norm_w ? ssq : nullptr; m.np = K / 16;
    } else {
      if (norm_w && src == x && nslab) {
        launch_rmsnorm_q8(xq8, xqd, src, norm_w, rmap, rows, K, eps, s, slabs, nslab, slab_stride);
        nslab = 0;
      } else if (norm_w) {
        launch_rmsnorm_q8(xq8, xqd, src, norm_w, rmap, rows, K, eps, s);
      } else {
        launch_quantize_q8(xq8, xqd, src, K, rows, K, s);
      }
      m.xq = xq8; m.xd = xqd;
    }
  };
  auto resid = [&](MMArgs& m) -> int {
    if (!ql && M > 16 && M <= 32) {
      const int ks = launch_mq8_slab(m, slabs, slab_stride, s);
      if (ks > 0) return nslab = ks, 0;
    }
    return launch_mq8(EPI_RESID, m, s);
  };
  for (int li = 0; li < (int)layers.size(); li++) {
    const Layer& L = layers[li];
    _Float16* kc = kcache + layer_kv_stride * li;
    _Float16* vc = vcache + layer_kv_stride * li;
    MMArgs a{};
    a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.M = M; a.wq4 = wq4;
    operand(a, x, h, L.attn_norm, M, nullptr);
    a.out = q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = head_dim; a.pos = pos; a.slot = slot;
    a.rope_cs = rope_cs; a.kc = kc; a.vc = vc; a.n_ctx = n_ctx; a.ctx_stride = ctx_stride; a.n_head_kv = n_head_kv;
    a.slot_stride = slot_stride;
    AttnArgs at{};
    const int qs = (!ql && M > 16 && M <= 32) ? launch_mq8_slab(a, slabs, slab_stride, s) : -1;
    if (qs > 0 && rows_distinct) {  // the attention kernel finishes q/k/v from the split-K slabs
      at.slabs = slabs; at.nslab = qs; at.slab_stride = slab_stride; at.rope_cs = rope_cs; at.kc_w = kc;
      at.vc_w = vc;
    } else if (qs > 0) {
      launch_qkv_finish(a, slabs, qs, slab_stride, s);
    } else if (launch_mq8(EPI_QKV, a, s)) {
      return fail(MX_ERR_ARG, "q8 qkv launch shape");
    }
    at.q = q; at.kc = kc; at.vc = vc; at.pos = pos; at.slot = slot;
    at.outf = attn_f; at.ldo = h; at.M = M; at.n_head = n_head; at.n_head_kv = n_head_kv; at.head_dim = head_dim;
    at.n_ctx = n_ctx; at.ctx_stride = ctx_stride; at.slot_stride = slot_stride;
    at.scale = 1.0f / sqrtf((float)head_dim);
    if (M > MAX_ROWS && rows_blocked) launch_attention_prefill(at, s);
    else launch_attention(at, s);
    MMArgs b{};
    b.W = L.o; b.N = h; b.K = h; b.M = M; b.out = x; b.ldo = h; b.wq4 = wq4;
    operand(b, attn_f, h, nullptr, M, nullptr);
    b.ssq = ql ? ssq : nullptr; b.np = h / 16;  // partials of the new residual for gate/up's norm
    if (resid(b)) return fail(MX_ERR_ARG, "q8 attn_output launch shape");
    MMArgs c{};
    c.W = L.gu; c.N = 2 * ff; c.K = h; c.M = M; c.actf = act_f; c.lda = ff; c.wq4 = wq4;
    // (a separate RMS_NORM + quantise launch for gate/up measured slower: profiles/round5_quant_batch1_onload.txt)
    operand(c, x, h, L.ffn_norm, M, nullptr);
    if (launch_mq8(EPI_SWIGLU, c, s)) return fail(MX_ERR_ARG, "q8 gate/up launch shape");
    MMArgs d{};
    d.W = L.down; d.N = h; d.K = ff; d.M = M; d.out = x; d.ldo = h; d.wq4 = wq4;
    operand(d, act_f, ff, nullptr, M, nullptr);
    d.ssq = ql ? ssq : nullptr; d.np = h / 16;  // for the next layer's qkv (or lm_head) norm
    if (resid(d)) return fail(MX_ERR_ARG, "q8 ffn_down launch shape");
  }
  if (nslab && (x_out || !(head && !rowmap && n_out == M))) {  // x itself is read next: fold
    launch_resid_norm(nullptr, 0, x, slabs, nslab, slab_stride, nullptr, M, h, eps, s);
    nslab = 0;
  }
  if (x_out)
    if (int rc = copy_out(x_out, M, s)) return rc;
  if (head) {
    if (!has_head) return fail(MX_ERR_STATE, "this stage has no output head");
    MMArgs g{};
    g.W = output; g.N = n_vocab; g.K = h; g.M = n_out; g.out = logits; g.ldo = n_vocab;
    if (out_kq_head) {  // K-quant output (Q4_0 files): Q8_K rows of the normed rows, ggml's q6_K.q8_K
      if (nslab) {
        launch_resid_norm(nullptr, 0, x, slabs, nslab, slab_stride, nullptr, M, h, eps, s);
        nslab = 0;
      }
      kq_out.set(g);
      if (launch_rmsnorm_q8k(xq8, xqd, xkb, x, out_norm, (rowmap || n_out != M) ? rowmap : nullptr, n_out, h, eps, s))
        return fail(MX_ERR_ARG, "kq head norm");
      g.xq = xq8; g.xd = xqd; g.xb = xkb;
      if (launch_mkq(EPI_F32, g, s)) return fail(MX_ERR_ARG, "kq lm_head launch shape");
    } else {
      g.wq4 = out_q4;
      operand(g, x, h, out_norm, n_out, (rowmap || n_out != M) ? rowmap : nullptr);
      if (launch_mq8(EPI_F32, g, s)) return fail(MX_ERR_ARG, "q8 lm_head launch shape");
    }
    if (argmax)
      pick(n_out, ids_next, pos_next, hist, hist_stride,
                    hist_count, max_hist, s);
  }
  HIPC(hipGetLastError());
  return 0;
}

// K-quant model, any M <= PREFILL_ROWS: every MUL_MAT takes Q8_K activation rows made by the norm
// (RMS_NORM + MUL + quantise) or by launch_quantize_q8k from the f32 attention output / SwiGLU
// product -- ggml's conversion of src1 to the K-quants' vec_dot_type.
int mx_engine::enqueue_forward_kq(int M, const int* pos, const int* slot, void* x_out, bool head, const int* rowmap,
                                  int n_out, bool argmax, int* ids_next, int* pos_next, int* hist, int hist_stride,
                                  int* hist_count, int max_hist, hipStream_t s) {
  const int h = n_embd, kv = n_embd_kv, ff = n_ff;
  if (head && n_out > MAX_ROWS) return fail(MX_ERR_ARG, "logits for at most 64 rows per forward");
  // One token: every GEMV quantises its Q8_K operand on load (RMS_NORM from the Σx² partials the
  // residual writers leave); otherwise one norm / quantise launch per GEMV.  (A v_dot4 kernel
  // quantising on load measured slower: 3.09 vs 2.80 ms per 8B token.)
  const bool ql = kq_on_load(M);
  // 17..32 rows: attn_output / ffn_down run split-K into slabs (launch_mkq_slab) and the next
  // RMS_NORM + Q8_K launch folds them into x; nslab = partials not yet folded
  int nslab = 0;
  auto operand = [&](MMArgs& m, const KqMat& km, const float* src, int K, const float* norm_w, int rows,
                     const int* rmap) -> int {
    km.set(m);
    if (ql && !rmap) {
      m.xq = nullptr; m.xf = src; m.norm_w = norm_w; m.eps = eps; m.ssq = norm_w ? ssq : nullptr; m.np = K / 16;
      return 0;
    }
    int rc;
    if (norm_w && src == x && nslab) {
      rc = launch_rmsnorm_q8k(xq8, xqd, xkb, src, norm_w, rmap, rows, K, eps, s, slabs, nslab, slab_stride);
      nslab = 0;
    } else {
      rc = norm_w ? launch_rmsnorm_q8k(xq8, xqd, xkb, src, norm_w, rmap, rows, K, eps, s)
                  : launch_quantize_q8k(xq8, xqd, xkb, src, K, rows, K, s);
    }
    m.xq = xq8; m.xd = xqd; m.xb = xkb;
    return rc;
  };
  auto resid = [&](MMArgs& m) -> int {  // x += W . operand, in place or as slabs for the next operand()
    if (!ql && M > 16 && M <= 32) {
      const int ks = launch_mkq_slab(m, slabs, slab_stride, s);
      if (ks > 0) return nslab = ks, 0;
    }
    return launch_mkq(EPI_RESID, m, s);
  };
  for (int li = 0; li < (int)layers.size(); li++) {
    const Layer& L = layers[li];
    _Float16* kc = kcache + layer_kv_stride * li;
    _Float16* vc = vcache + layer_kv_stride * li;
    MMArgs a{};
    a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.M = M;
    if (operand(a, L.kq_qkv, x, h, L.attn_norm, M, nullptr)) return fail(MX_ERR_ARG, "kq norm shape");
    a.out = q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = head_dim; a.pos = pos; a.slot = slot;
    a.rope_cs = rope_cs; a.kc = kc; a.vc = vc; a.n_ctx = n_ctx; a.ctx_stride = ctx_stride; a.n_head_kv = n_head_kv;
    a.slot_stride = slot_stride;
    AttnArgs at{};
    // 17..32 rows: q|k|v as split-K slabs, finished by the attention kernel (distinct sequences) or
    // by launch_qkv_finish
    const int qs = (!ql && M > 16 && M <= 32) ? launch_mkq_qkv_slab(a, slabs, slab_stride, s) : -1;
    if (qs > 0 && rows_distinct) {
      at.slabs = slabs; at.nslab = qs; at.slab_stride = slab_stride; at.rope_cs = rope_cs; at.kc_w = kc;
      at.vc_w = vc;
    } else if (qs > 0) {
      launch_qkv_finish(a, slabs, qs, slab_stride, s);
    } else if (launch_mkq(EPI_QKV, a, s)) {
      return fail(MX_ERR_ARG, "kq qkv launch shape");
    }
    at.q = q; at.kc = kc; at.vc = vc; at.pos = pos; at.slot = slot;
    at.outf = attn_f; at.ldo = h; at.M = M; at.n_head = n_head; at.n_head_kv = n_head_kv; at.head_dim = head_dim;
    at.n_ctx = n_ctx; at.ctx_stride = ctx_stride; at.slot_stride = slot_stride;
    at.scale = 1.0f / sqrtf((float)head_dim);
    if (M > MAX_ROWS && rows_blocked) launch_attention_prefill(at, s);
    else launch_attention(at, s);
    MMArgs b{};
    b.W = L.o; b.N = h; b.K = h; b.M = M; b.out = x; b.ldo = h;
    if (operand(b, L.kq_o, attn_f, h, nullptr, M, nullptr)) return fail(MX_ERR_ARG, "kq quantise shape");
    b.ssq = ql ? ssq : nullptr; b.np = h / 16;  // Σx² partials of the new residual for gate/up
    if (resid(b)) return fail(MX_ERR_ARG, "kq attn_output launch shape");
    MMArgs c{};
    c.W = L.gu; c.N = 2 * ff; c.K = h; c.M = M; c.actf = act_f; c.lda = ff;
    if (operand(c, L.kq_gu, x, h, L.ffn_norm, M, nullptr) || launch_mkq(EPI_SWIGLU, c, s))
      return fail(MX_ERR_ARG, "kq gate/up launch shape");
    MMArgs d{};
    d.W = L.down; d.N = h; d.K = ff; d.M = M; d.out = x; d.ldo = h;
    if (operand(d, L.kq_down, act_f, ff, nullptr, M, nullptr)) return fail(MX_ERR_ARG, "kq quantise shape");
    d.ssq = ql ? ssq : nullptr; d.np = h / 16;  // ... for the next layer's qkv (and the head)
    if (resid(d)) return fail(MX_ERR_ARG, "kq ffn_down launch shape");
  }
  if (nslab && (x_out || !(head && !rowmap && n_out == M))) {  // x itself is read next: fold the partials
    launch_resid_norm(nullptr, 0, x, slabs, nslab, slab_stride, nullptr, M, h, eps, s);
    nslab = 0;
  }
  if (x_out)
    if (int rc = copy_out(x_out, M, s)) return rc;
  if (head) {
    if (!has_head) return fail(MX_ERR_STATE, "this stage has no output head");
    MMArgs g{};
    g.W = output; g.N = n_vocab; g.K = h; g.M = n_out; g.out = logits; g.ldo = n_vocab;
    if (operand(g, kq_out, x, h, out_norm, n_out, (rowmap || n_out != M) ? rowmap : nullptr) ||
        launch_mkq(EPI_F32, g, s))
      return fail(MX_ERR_ARG, "kq lm_head launch shape");
    if (argmax)
      pick(n_out, ids_next, pos_next, hist, hist_stride,
                    hist_count, max_hist, s);
  }
  HIPC(hipGetLastError());
  return 0;
}

// Prefill chunk of MAX_ROWS < M <= PREFILL_ROWS rows: MFMA GEMMs read each weight once per 256
// rows (not once per 64 as the wide decode kernels would); RMS_NORM as its own launch.  A K-quant
// model's layer is first dequantised to bf16 tiles (launch_dequant_kq: ~0.6 GB of HBM traffic per
// Llama-3-8B layer, a few % of a 4096-row chunk's GEMM time) -- the route llama.cpp's GPU backends
// take for large batches; decode keeps the int8-MFMA K-quant GEMVs with Q8_K activations.
int mx_engine::enqueue_forward_gemm(int M, const int* pos, const int* slot, void* x_out, bool head,
                                    const int* rowmap, int n_out, hipStream_t s) {
  const int h = n_embd, kv = n_embd_kv, ff = n_ff;
  const size_t gstride = (size_t)M * h;  // RESID partial slabs [S][M][h]
  int nslab = 0;                         // ... not yet folded into x
  auto dequant = [&](uint16_t* dst, const KqMat& km, const uint16_t* w, int K) -> int {
    return launch_dequant_kq(dst, w, K, km.n, km.type, km.tile_end, km.off, s);
  };
  for (int li = 0; li < (int)layers.size(); li++) {
    const Layer& L = layers[li];
    _Float16* kc = kcache + layer_kv_stride * li;
    _Float16* vc = vcache + layer_kv_stride * li;
    const uint16_t *Wqkv = L.qkv, *Wo = L.o, *Wgu = L.gu, *Wdown = L.down;
    if (wkq) {
      if (dequant(kqd_qkv, L.kq_qkv, L.qkv, h) || dequant(kqd_o, L.kq_o, L.o, h) || dequant(kqd_gu, L.kq_gu, L.gu, h) ||
          dequant(kqd_down, L.kq_down, L.down, ff))
        return fail(MX_ERR_ARG, "K-quant dequantisation shape");
      Wqkv = kqd_qkv, Wo = kqd_o, Wgu = kqd_gu, Wdown = kqd_down;
    } else if (wq8) {  // Q8_0: d * q per weight, rounded to bf16
      auto dq = [&](uint16_t* dst, const uint16_t* w, int N, int K) {
        return launch_dequant_q8_tiles(dst, reinterpret_cast<const uint8_t*>(w), N, K, s);
      };
      if (dq(kqd_qkv, L.qkv, h + 2 * kv, h) || dq(kqd_o, L.o, h, h) || dq(kqd_gu, L.gu, 2 * ff, h) ||
          dq(kqd_down, L.down, h, ff))
        return fail(MX_ERR_ARG, "Q8_0 dequantisation shape");
      Wqkv = kqd_qkv, Wo = kqd_o, Wgu = kqd_gu, Wdown = kqd_down;
    }
    launch_resid_norm(xn, h, x, gslabs, nslab, gstride, L.attn_norm, M, h, eps, s);
    MMArgs a{};
    a.W = Wqkv; a.N = h + 2 * kv; a.K = h; a.M = M; a.X = xn; a.ldx = h;
    a.out = q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = head_dim; a.pos = pos; a.slot = slot;
    a.rope_cs = rope_cs; a.kc = kc; a.vc = vc; a.n_ctx = n_ctx; a.ctx_stride = ctx_stride; a.n_head_kv = n_head_kv;
    a.slot_stride = slot_stride;
    if (launch_gemm_split(EPI_QKV, a, gslabs, GSLAB_FLOATS, gemm_split_target, s) < 0) return fail(MX_ERR_ARG, "prefill qkv GEMM shape");
    AttnArgs at{};
    at.q = q; at.kc = kc; at.vc = vc; at.pos = pos; at.slot = slot;
    at.out = attn_out; at.ldo = h; at.M = M; at.n_head = n_head; at.n_head_kv = n_head_kv; at.head_dim = head_dim;
    at.n_ctx = n_ctx; at.ctx_stride = ctx_stride; at.slot_stride = slot_stride;
    at.scale = 1.0f / sqrtf((float)head_dim);
    if (rows_blocked) launch_attention_prefill(at, s);
    else launch_attention(at, s);
    MMArgs b{};
    b.W = Wo; b.N = h; b.K = h; b.X = attn_out; b.ldx = h; b.M = M; b.out = x; b.ldo = h;
    if ((nslab = launch_gemm_split(EPI_RESID, b, gslabs, GSLAB_FLOATS, gemm_split_target, s)) < 0)
      return fail(MX_ERR_ARG, "prefill attn_output GEMM shape");
    launch_resid_norm(xn, h, x, gslabs, nslab, gstride, L.ffn_norm, M, h, eps, s);
    MMArgs c{};
    c.W = Wgu; c.N = 2 * ff; c.K = h; c.M = M; c.X = xn; c.ldx = h; c.act = act; c.lda = ff;
    if (launch_gemm_split(EPI_SWIGLU, c, gslabs, GSLAB_FLOATS, gemm_split_target, s) < 0)
      return fail(MX_ERR_ARG, "prefill gate/up GEMM shape");
    MMArgs d{};
    d.W = Wdown; d.N = h; d.K = ff; d.X = act; d.ldx = ff; d.M = M; d.out = x; d.ldo = h;
    if ((nslab = launch_gemm_split(EPI_RESID, d, gslabs, GSLAB_FLOATS, gemm_split_target, s)) < 0)
      return fail(MX_ERR_ARG, "prefill ffn_down GEMM shape");
  }
  if (nslab) launch_resid_norm(nullptr, 0, x, gslabs, nslab, gstride, nullptr, M, h, eps, s);
  if (x_out)
    if (int rc = copy_out(x_out, M, s)) return rc;
  if (head) {
    if (!has_head) return fail(MX_ERR_STATE, "this stage has no output head");
    if (!rowmap) return fail(MX_ERR_ARG, "prefill head needs a row map");
    MMArgs g{};
    g.W = output; g.N = n_vocab; g.K = h; g.M = n_out; g.out = logits; g.ldo = n_vocab;
    if (wkq || out_kq_head) {  // the K-quant head as at decode: Q8_K rows of the normed last rows
      kq_out.set(g);
      if (launch_rmsnorm_q8k(xq8, xqd, xkb, x, out_norm, rowmap, n_out, h, eps, s)) return fail(MX_ERR_ARG, "kq norm");
      g.xq = xq8; g.xd = xqd; g.xb = xkb;
      if (launch_mkq(EPI_F32, g, s)) return fail(MX_ERR_ARG, "kq lm_head launch shape");
    } else if (wq8) {  // the Q8_0 head as at decode
      launch_rmsnorm_q8(xq8, xqd, x, out_norm, rowmap, n_out, h, eps, s);
      g.xq = xq8; g.xd = xqd; g.wq4 = out_q4;
      if (launch_mq8(EPI_F32, g, s)) return fail(MX_ERR_ARG, "q8 lm_head launch shape");
    } else {
      launch_rmsnorm(xn, h, x, out_norm, rowmap, n_out, h, eps, s);
      g.X = xn; g.ldx = h;
      // the decode GEMVs (canonical K order at every row count), so a prompt's first token does not
      // depend on how many prompts ended in its chunk
      const int rc = (n_out > 16 && use_wide) ? (launch_mm_wide(EPI_F32, g, slabs, slab_stride, s) < 0 ? 1 : 0)
                                              : launch_mm(EPI_F32, g, s);
      if (rc) return fail(MX_ERR_ARG, "lm_head launch shape");
    }
  }
  HIPC(hipGetLastError());
  return 0;
}

__global__ void advance_pos_kernel(int* pos, int M) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) pos[i] += 1;
}

// rows forward, n <= MAX_ROWS, logits for all rows copied to host if requested
// lm_head runs only when logits are wanted: for every row, or (last_row_only, prompt chunks) for the
// last row alone -- a prefill never streams the 1 GB output matrix per 64-row chunk.
int mx_engine::forward_rows_chunk(int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                                  const void* x_in, void* x_out, float* logits_host, hipStream_t s,
                                  bool last_row_only) {
  if (n < 1 || n > PREFILL_ROWS) return fail(MX_ERR_ARG, "forward chunk of 1..PREFILL_ROWS rows");
  for (int i = 0; i < n; i++) {
    if (slots[i] < 0 || slots[i] >= n_seq_max) return fail(MX_ERR_ARG, "slot out of range");
    if (pos[i] < 0 || pos[i] >= n_ctx) return fail(MX_ERR_CTX, "position outside n_ctx");
    if (ids && has_embed && !x_in && (ids[i] < 0 || ids[i] >= n_vocab)) return fail(MX_ERR_ARG, "token id out of range");
  }
  // every call ends with a stream sync below, so the staging rows are free again at entry
  const size_t R = PREFILL_ROWS;
  auto h2d = [&](int* dst, const int32_t* src, int k, int row) -> int {
    memcpy(h_idx + row * R, src, (size_t)k * 4);
    if (hipMemcpyAsync(dst, h_idx + row * R, (size_t)k * 4, hipMemcpyHostToDevice, s) != hipSuccess) {
      hipStreamSynchronize(s);  // earlier copies of this call may still read h_idx
      return fail(MX_ERR_HIP, "index upload");
    }
    return 0;
  };
  if (ids)
    if (int rc = h2d(d_ids, ids, n, 0)) return rc;
  if (int rc = h2d(d_pos, pos, n, 1)) return rc;
  if (int rc = h2d(d_slot, slots, n, 2)) return rc;
  const bool head = has_head && !x_out && logits_host;
  const int n_out = last_row_only ? 1 : n;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < n; i++) slot_tokens[slots[i]].clear();  // direct row writes: contents unknown
  }
  std::vector<int32_t> sorted(slots, slots + n);
  std::sort(sorted.begin(), sorted.end());
  rows_distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  rows_blocked = blocked_rows(slots, pos, x_in ? nullptr : ids, n);
  if (head && last_row_only) {
    const int32_t last = n - 1;
    if (int rc = h2d(d_rowmap, &last, 1, 3)) return rc;
  }
  const int frc = enqueue_forward(n, d_ids, d_pos, d_slot, x_in, x_out, head, head && last_row_only ? d_rowmap : nullptr,
                                  n_out, false, nullptr, nullptr, nullptr, 0, nullptr, 0, s);
  rows_distinct = false;
  rows_blocked = false;
  if (frc) {  // the index copies enqueued above still read h_idx: drain them before it is reused
    hipStreamSynchronize(s);
    return frc;
  }
  if (head) HIPC(hipMemcpyAsync(logits_host, logits, (size_t)n_out * n_vocab * 4, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  return 0;
}

// ---------------------------------------------------------------- scheduler
void mx_engine::finish(Request* r, int why) {
  r->finish = why;
  r->done = true;
  if (r->slot >= 0) {
    // K/V written for: the prompt and every generated token but the last (never fed back)
    std::vector<int32_t>& st = slot_tokens[r->slot];
    st = r->prompt;
    if (!r->out.empty()) st.insert(st.end(), r->out.begin(), r->out.end() - 1);
    if ((int)st.size() > r->pos) st.resize(std::max(0, r->pos));
    free_slots.push_back(r->slot);
  }
  stat_generated_tokens += r->out.size();
  r->slot = -1;
}

// llama.cpp default sampling chain (restricted to the parameters exposed in mx_sampling):
// repetition penalty -> top_k -> top_p -> min_p -> temperature -> draw
// llama.cpp's sampler chain as llama-cpp-python 0.3 builds it for create_completion: penalties ->
// top_k -> top_p -> min_p -> temperature -> draw (greedy when temperature <= 0).  The candidates are
// ordered by logit (ties: lower id first); only the top k are ever needed, so they are selected with
// a partial sort here, or on the device (launch_topk) in the decode loop.
static bool has_penalties(const mx_sampling& sp) {
  return sp.repeat_penalty != 1.0f || sp.frequency_penalty != 0.0f || sp.presence_penalty != 0.0f;
}

int32_t mx_engine::sample_host(Request* r, const float* lg) {
  const mx_sampling& sp = r->samp;
  std::vector<std::pair<float, int>> c;
  c.reserve(n_vocab);
  for (int i = 0; i < n_vocab; i++) c.push_back({lg[i], i});
  if (has_penalties(sp) && sp.repeat_last_n != 0) {
    // llama.cpp penalties sampler over the last repeat_last_n tokens: repeat (divide positive,
    // multiply negative logits), then frequency (per occurrence) and presence (once) subtracted
    std::vector<int> hist(r->prompt);
    hist.insert(hist.end(), r->out.begin(), r->out.end());
    int n = sp.repeat_last_n < 0 ? (int)hist.size() : std::min<int>(sp.repeat_last_n, (int)hist.size());
    std::vector<int> count(n_vocab, 0);
    for (int i = (int)hist.size() - n; i < (int)hist.size(); i++) count[hist[i]]++;
    for (auto& p : c) {
      const int k = count[p.second];
      if (!k) continue;
      if (sp.repeat_penalty != 1.0f) p.first = p.first <= 0 ? p.first * sp.repeat_penalty : p.first / sp.repeat_penalty;
      p.first -= (float)k * sp.frequency_penalty + sp.presence_penalty;
    }
  }
  auto before = [](const std::pair<float, int>& a, const std::pair<float, int>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  };
  if (sp.temperature <= 0.f) return std::min_element(c.begin(), c.end(), before)->second;
  const int k = sp.top_k > 0 ? std::min<int>(sp.top_k, n_vocab) : n_vocab;
  std::partial_sort(c.begin(), c.begin() + k, c.end(), before);
  c.resize(k);
  return sample_chain(r, c);
}

int32_t mx_engine::sample_chain(Request* r, std::vector<std::pair<float, int>>& c) {
  // the device sampling chain's code (kernels.h samp_pick), over candidates of any count
  const mx_sampling& sp = r->samp;
  const int k = (int)c.size();
  std::vector<float> v(k);
  std::vector<int> id(k);
  for (int i = 0; i < k; i++) v[i] = c[i].first, id[i] = c[i].second;
  std::vector<double> p(k), w(k);
  return samp_pick(v.data(), id.data(), k, sp.temperature, sp.top_p, sp.min_p, samp_u01(r->seed, r->out.size()),
                   p.data(), w.data());
}

bool mx_engine::device_sampleable(const mx_sampling& sp) {
  if (sp.top_k < 1 || sp.top_k > TOPK_MAX) return false;
  if (has_penalties(sp) && (sp.repeat_last_n < 0 || sp.repeat_last_n > SAMP_WIN)) return false;
  return true;
}

void mx_engine::samp_row(const Request* r, SampRow* o) const {
  const mx_sampling& sp = r->samp;
  memset(o, 0, sizeof(*o));
  o->temp = sp.temperature;
  o->top_p = sp.top_p;
  o->min_p = sp.min_p;
  o->repeat = sp.repeat_penalty;
  o->freq = sp.frequency_penalty;
  o->presence = sp.presence_penalty;
  o->top_k = std::max(1, std::min(sp.top_k, TOPK_MAX));
  o->last_n = has_penalties(sp) ? std::min(sp.repeat_last_n, SAMP_WIN) : 0;
  o->seed = r->seed;
  o->draw0 = (int)r->out.size();
  const int np = (int)r->prompt.size(), no = (int)r->out.size();
  o->n_win = std::min(o->last_n, np + no);
  for (int j = 0; j < o->n_win; j++) {
    const int t = np + no - o->n_win + j;
    o->win[j] = t < np ? r->prompt[t] : r->out[t - np];
  }
}

// Prefill of every newly admitted request together (llama.cpp's eval of the prompt, SURVEY §3.2,
// for all of them in as few forwards as the GEMM chunk allows): their remaining prompt rows back
// to back, each segment padded to a multiple of 16 rows with throw-away positions past the prompt
// when that stays inside n_ctx (so the rows form 16-position blocks of one sequence and the flash
// prefill attention runs; the pad K/V is overwritten by the first decode steps before anything
// reads it), lm_head only on each request's last prompt row, and the first token by the device
// argmax (ties -> lowest id) or, for sampling requests, the device sampling chain (the host sampler
// when a request's settings are outside the device chain's range).
int mx_engine::prefill_batch(std::vector<Request*>& reqs) {
  static const bool trace = getenv("MX_SCHED_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  struct Log {
    const std::chrono::steady_clock::time_point t0;
    size_t n;
    ~Log() {
      if (trace)
        fprintf(stderr, "sched: prefill %zu requests %.3f ms\n", n,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
  } log{t0, reqs.size()};
  // every prompt's rows start a 16-row block and are padded to whole blocks (positions past the prompt,
  // overwritten by its decode later; near n_ctx copies of the last row), so each chunk is blocked
  // (attn_prefill_kernel) and a prompt's blocks are the same whatever shares its chunk
  std::vector<int32_t> slots, pos, ids;
  std::vector<int> end_row(reqs.size()), blk_end(reqs.size());
  for (size_t q = 0; q < reqs.size(); q++) {
    Request* r = reqs[q];
    const int n = (int)r->prompt.size();
    for (int p = r->reuse; p < n; p++) {
      slots.push_back(r->slot);
      pos.push_back(p);
      ids.push_back(r->prompt[p]);
    }
    end_row[q] = (int)slots.size() - 1;
    const int pad = (16 - (n - r->reuse) % 16) % 16;
    for (int k = 0; k < pad; k++) {
      slots.push_back(r->slot);
      pos.push_back(n + pad <= n_ctx ? n + k : n - 1);
      ids.push_back(r->prompt[n - 1]);
    }
    blk_end[q] = (int)slots.size();
    r->pos = n;
  }
  const int chunk = gemm_ok() ? PREFILL_ROWS : MAX_ROWS;
  const int total = (int)slots.size();
  std::vector<int32_t> tok(reqs.size());
  bool any_sampling = false, dev_pick = use_dev_topk;
  for (Request* r : reqs)
    if (r->samp.temperature > 0.f || has_penalties(r->samp)) {
      any_sampling = true;
      dev_pick &= device_sampleable(r->samp);
    }
  // every sampling request fits the device chain: first tokens are drawn on the device (the same
  // samp_pick and counter-based draw 0 as the host sampler), no logits rows cross PCIe
  dev_pick &= any_sampling;
  std::vector<float> lg;
  std::vector<SampRow> sr;
  size_t q0 = 0;  // first request whose last row is not yet evaluated
  for (int i = 0; i < total;) {
    // chunk [i, e): at most `chunk` rows and at most MAX_ROWS request ends (logits rows)
    int e = std::min(total, i + chunk);
    size_t q1 = q0;
    while (q1 < reqs.size() && end_row[q1] < e && (int)(q1 - q0) < MAX_ROWS) q1++;
    if ((int)(q1 - q0) == MAX_ROWS && q1 < reqs.size() && end_row[q1] < e) e = blk_end[q1 - 1];
    const int m = e - i, n_out = (int)(q1 - q0);
    std::vector<int32_t> rowmap(n_out);
    for (int k = 0; k < n_out; k++) rowmap[k] = end_row[q0 + k] - i;
    hipStream_t st = stream;
    HIPC(hipMemcpyAsync(d_ids, ids.data() + i, m * 4, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_pos, pos.data() + i, m * 4, hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_slot, slots.data() + i, m * 4, hipMemcpyHostToDevice, st));
    if (n_out) HIPC(hipMemcpyAsync(d_rowmap, rowmap.data(), n_out * 4, hipMemcpyHostToDevice, st));
    rows_distinct = false;
    rows_blocked = blocked_rows(slots.data() + i, pos.data() + i, ids.data() + i, m);
    prefill_gemm = true;
    const int frc = enqueue_forward(m, d_ids, d_pos, d_slot, nullptr, nullptr, n_out > 0, n_out ? d_rowmap : nullptr,
                                    n_out, false, nullptr, nullptr, nullptr, 0, nullptr, 0, st);
    rows_blocked = false;
    prefill_gemm = false;
    if (frc) return frc;
    int ktop = 0;
    if (n_out && dev_pick) {
      sr.resize(n_out);
      for (int k = 0; k < n_out; k++) {
        samp_row(reqs[q0 + k], &sr[k]);
        const mx_sampling& sp = reqs[q0 + k]->samp;
        if (sp.temperature > 0.f || has_penalties(sp)) ktop = std::max(ktop, std::min(sp.top_k, n_vocab));
      }
    }
    if (n_out && ktop > 0) {
      HIPC(hipMemcpyAsync(d_samp, sr.data(), n_out * sizeof(SampRow), hipMemcpyHostToDevice, st));
      pick_samp = d_samp;
      pick_k = ktop;
      pick(n_out, nullptr, nullptr, nullptr, 0, nullptr, 0, st);
      pick_samp = nullptr;
      pick_k = 0;
      HIPC(hipMemcpyAsync(tok.data() + q0, d_tok, n_out * 4, hipMemcpyDeviceToHost, st));
    } else if (n_out) {
      launch_argmax(logits, n_vocab, n_out, n_vocab, am_val, am_idx, d_tok, nullptr, nullptr, nullptr, 0, nullptr, 0, st);
      HIPC(hipMemcpyAsync(tok.data() + q0, d_tok, n_out * 4, hipMemcpyDeviceToHost, st));
      if (any_sampling && !dev_pick) {
        lg.resize((size_t)n_out * n_vocab);
        HIPC(hipMemcpyAsync(lg.data(), logits, lg.size() * 4, hipMemcpyDeviceToHost, st));
      }
    }
    HIPC(hipStreamSynchronize(st));
    std::lock_guard<std::mutex> lk(mu);
    for (int k = 0; k < n_out; k++) {
      Request* r = reqs[q0 + k];
      int32_t t = tok[q0 + k];
      if (!dev_pick && (r->samp.temperature > 0.f || has_penalties(r->samp)))
        t = sample_host(r, lg.data() + (size_t)k * n_vocab);
      r->out.push_back(t);
      r->next_tok = t;
    }
    q0 = q1;
    i = e;
  }
  return 0;
}

// One scheduler round over the active rows.  All greedy (no penalties): K decode steps replayed
// back to back on the device (the captured step feeds its argmax into the next step's ids and
// positions and appends it to a history), one sync, then the K tokens of every row are applied in
// order (a row that finishes early ignores the rest).  Otherwise one step, with the sampler chain
// on the host (top-k candidates from the device when possible).
int mx_engine::sched_step(std::vector<Request*>& rows) {
  const int M = (int)rows.size();
  std::vector<int32_t> ids(M), pos(M), slots(M);
  bool all_greedy = true, all_dev = true;
  int room = SCHED_KMAX, need = 1, ktop = 0;
  for (int i = 0; i < M; i++) {
    ids[i] = rows[i]->next_tok;
    pos[i] = rows[i]->pos;
    slots[i] = rows[i]->slot;
    const mx_sampling& sp = rows[i]->samp;
    if (sp.temperature > 0.f || has_penalties(sp)) {
      all_greedy = false;
      if (use_dev_topk && device_sampleable(sp)) ktop = std::max(ktop, std::min(sp.top_k, n_vocab));
      else all_dev = false;
    }
    room = std::min(room, n_ctx - rows[i]->pos);
    need = std::max(need, rows[i]->max_tokens - (int)rows[i]->out.size());
  }
  // greedy rows: argmax on the device; every row sampleable on the device: the device sampling chain
  // (penalties, top-k, top-p, min-p, temperature, draw); either way K steps run back to back on the
  // device.  Otherwise one step, sampled on the host.
  const bool dev_chain = !all_greedy && all_dev && ktop > 0;
  int K = 1;
  if (all_greedy || dev_chain) {
    K = std::max(1, std::min(room, need));
    std::lock_guard<std::mutex> lk(mu);
    if (!pending.empty() && !free_slots.empty()) K = 1;  // admit waiting requests at the next round
  }
  hipStream_t s = stream;
  HIPC(hipMemcpyAsync(d_ids, ids.data(), M * 4, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(d_pos, pos.data(), M * 4, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(d_slot, slots.data(), M * 4, hipMemcpyHostToDevice, s));
  HIPC(hipMemsetAsync(sched_hist_count, 0, M * 4, s));
  std::vector<SampRow> sr;
  if (dev_chain) {
    sr.resize(M);
    for (int i = 0; i < M; i++) samp_row(rows[i], &sr[i]);
    HIPC(hipMemcpyAsync(d_samp, sr.data(), M * sizeof(SampRow), hipMemcpyHostToDevice, s));
  }
  rows_distinct = true;  // one row per active request, each its own slot
  pick_samp = dev_chain ? d_samp : nullptr;
  pick_k = dev_chain ? ktop : 0;
  struct Reset {
    mx_engine* e;
    ~Reset() { e->rows_distinct = false; e->pick_samp = nullptr; e->pick_k = 0; }
  } reset_flags{this};
  auto step = [&]() -> int {
    return enqueue_forward(M, d_ids, d_pos, d_slot, nullptr, nullptr, true, nullptr, M, true, d_ids, d_pos,
                           sched_hist, SCHED_KMAX, sched_hist_count, SCHED_KMAX, s);
  };
  static const bool trace = getenv("MX_SCHED_TRACE") != nullptr;  // per-round timing on stderr
  const auto t0 = std::chrono::steady_clock::now();
  bool captured = false;
  const std::pair<int, int> gkey(M, pick_k);
  auto it = sched_graphs.find(gkey);
  if (use_graphs && it == sched_graphs.end()) {
    captured = true;
    hipGraph_t g;
    HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = step();
    hipError_t ce = hipStreamEndCapture(s, &g);
    if (rc) return rc;
    if (ce != hipSuccess) return fail(MX_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(ce));
    hipGraphExec_t ex;
    HIPC(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    it = sched_graphs.emplace(gkey, ex).first;
  }
  for (int k = 0; k < K; k++) {
    if (use_graphs) HIPC(hipGraphLaunch(it->second, s));
    else if (int rc = step()) return rc;
  }
  std::vector<int32_t> hist((size_t)M * SCHED_KMAX);
  std::vector<float> lg, tkv;
  std::vector<int32_t> tki;
  HIPC(hipMemcpyAsync(hist.data(), sched_hist, hist.size() * 4, hipMemcpyDeviceToHost, s));
  // sampling rows: the top-k candidates come from the device (k <= TOPK_MAX, no penalties, which
  // would reorder logits first); otherwise the whole logits rows go to the host
  int TK = 0;
  bool dev_topk = !all_greedy && !dev_chain && use_dev_topk;
  for (int i = 0; i < M && dev_topk; i++) {
    const mx_sampling& sp = rows[i]->samp;
    if (sp.temperature <= 0.f && !has_penalties(sp)) continue;
    if (has_penalties(sp) || sp.top_k < 1 || sp.top_k > TOPK_MAX) dev_topk = false;
    else TK = std::max(TK, std::min(sp.top_k, n_vocab));
  }
  if (dev_topk && TK > 0) {
    if (launch_topk(logits, n_vocab, M, n_vocab, TK, tk_ws_val, tk_ws_idx, tk_val, tk_idx, s))
      return fail(MX_ERR_HIP, "top-k launch");
    tkv.resize((size_t)M * TK);
    tki.resize((size_t)M * TK);
    HIPC(hipMemcpyAsync(tkv.data(), tk_val, (size_t)M * TK * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(tki.data(), tk_idx, (size_t)M * TK * 4, hipMemcpyDeviceToHost, s));
  } else if (!all_greedy && !dev_chain) {
    lg.resize((size_t)M * n_vocab);
    HIPC(hipMemcpyAsync(lg.data(), logits, (size_t)M * n_vocab * 4, hipMemcpyDeviceToHost, s));
  }
  HIPC(hipStreamSynchronize(s));
  if (trace) {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "sched: decode M=%d K=%d %s%s%.3f ms\n", M, K, dev_chain ? "(device sampling) " : "",
            captured ? "(graph captured) " : "", ms);
  }
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < M; i++) {
    Request* r = rows[i];
    for (int k = 0; k < K && !r->done; k++) {
      r->pos++;
      int32_t t = hist[(size_t)i * SCHED_KMAX + k];
      if (!dev_chain && (r->samp.temperature > 0.f || has_penalties(r->samp))) {
        if (!tkv.empty()) {
          std::vector<std::pair<float, int>> c(std::min(r->samp.top_k, n_vocab));
          for (size_t j = 0; j < c.size(); j++) c[j] = {tkv[(size_t)i * TK + j], tki[(size_t)i * TK + j]};
          t = sample_chain(r, c);
        } else {
          t = sample_host(r, lg.data() + (size_t)i * n_vocab);
        }
      }
      r->out.push_back(t);
      r->next_tok = t;
      if ((t == eos && !r->samp.ignore_eos) || r->cancel) finish(r, MX_FINISH_STOP);
      else if ((int)r->out.size() >= r->max_tokens || r->pos >= n_ctx) finish(r, MX_FINISH_LENGTH);
    }
  }
  return 0;
}

void mx_engine::scheduler_loop() {
  hipSetDevice(device);
  for (;;) {
    std::vector<Request*> admit;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return stop || !pending.empty() || !active.empty(); });
      if (stop) {
        for (Request* r : pending) { r->error = "engine shutting down"; finish(r, MX_FINISH_ERROR); }
        for (Request* r : active) { r->error = "engine shutting down"; finish(r, MX_FINISH_ERROR); }
        pending.clear();
        active.clear();
        cv_done.notify_all();
        return;
      }
      while (!pending.empty() && !free_slots.empty()) {
        Request* r = pending.front();
        pending.pop_front();
        if (r->cancel) {  // cancelled before admission: no tokens
          finish(r, MX_FINISH_STOP);
          continue;
        }
        // the free slot sharing the longest prefix with this prompt (ties: most recently freed)
        size_t best = free_slots.size() - 1;
        int best_lcp = -1;
        for (size_t k = free_slots.size(); k-- > 0;) {
          const std::vector<int32_t>& st = slot_tokens[free_slots[k]];
          int l = 0;
          const int lim = (int)std::min(st.size(), r->prompt.size());
          while (l < lim && st[l] == r->prompt[l]) l++;
          if (l > best_lcp) best_lcp = l, best = k;
        }
        r->slot = free_slots[best];
        free_slots.erase(free_slots.begin() + best);
        // at least the last prompt token is evaluated (its logits start generation)
        r->reuse = std::min(best_lcp, (int)r->prompt.size() - 1);
        stat_prompt_tokens += r->prompt.size();
        stat_reused_tokens += r->reuse;
        admit.push_back(r);
      }
    }
    std::lock_guard<std::mutex> glk(gpu_mu);
    if (!admit.empty()) {
      const int rc = prefill_batch(admit);
      std::lock_guard<std::mutex> lk(mu);
      for (Request* r : admit) {
        if (rc) {
          r->error = g_err;
          finish(r, MX_FINISH_ERROR);
          continue;
        }
        const int32_t t = r->out.back();
        if ((t == eos && !r->samp.ignore_eos) || r->cancel) finish(r, MX_FINISH_STOP);
        else if ((int)r->out.size() >= r->max_tokens || r->pos >= n_ctx) finish(r, MX_FINISH_LENGTH);
        else active.push_back(r);
      }
    }
    std::vector<Request*> rows;
    {
      std::lock_guard<std::mutex> lk(mu);
      active.erase(std::remove_if(active.begin(), active.end(), [](Request* r) { return r->done; }), active.end());
      for (Request* r : active)
        if ((int)rows.size() < MAX_ROWS) rows.push_back(r);
      cv_done.notify_all();
    }
    if (rows.empty()) continue;
    int rc = sched_step(rows);
    std::lock_guard<std::mutex> lk(mu);
    if (rc) {
      for (Request* r : rows) {
        r->error = g_err;
        if (!r->done) finish(r, MX_FINISH_ERROR);
      }
    }
    active.erase(std::remove_if(active.begin(), active.end(), [](Request* r) { return r->done; }), active.end());
    cv_done.notify_all();
  }
}

// ---------------------------------------------------------------- C ABI
extern "C" {

void mx_opts_default(mx_opts* o) {
  o->n_ctx = 512;
  o->n_seq_max = 64;
  o->layer_begin = 0;
  o->layer_end = -1;
  o->device = -1;
  o->use_graphs = 1;
  o->seed = 0;
  o->handoff_bf16 = 0;
}

void mx_sampling_default(mx_sampling* s) {
  s->temperature = 0.8f;
  s->top_k = 40;
  s->top_p = 0.95f;
  s->min_p = 0.05f;
  s->repeat_penalty = 1.0f;
  s->repeat_last_n = 64;
  s->seed = 0xFFFFFFFFull;
  s->ignore_eos = 0;
  s->frequency_penalty = 0.0f;
  s->presence_penalty = 0.0f;
}

const char* mx_last_error(void) { return g_err.c_str(); }

int mx_engine_create(const char* model_path, const mx_opts* opts, mx_engine** out) {
  if (!model_path || !out) return fail(MX_ERR_ARG, "null argument");
  *out = nullptr;
  mx_opts o;
  mx_opts_default(&o);
  if (opts) o = *opts;
  if (o.n_ctx < 1 || o.n_seq_max < 1) return fail(MX_ERR_ARG, "n_ctx and n_seq_max must be >= 1");
  std::unique_ptr<mx_engine> e(new mx_engine());
  e->n_ctx = o.n_ctx;
  e->n_seq_max = o.n_seq_max;
  e->lb = o.layer_begin;
  e->le = o.layer_end;
  e->use_graphs = o.use_graphs != 0 && getenv("MX_NO_GRAPHS") == nullptr;  // rocprofv3 runs set MX_NO_GRAPHS
  e->handoff_bf16 = o.handoff_bf16 != 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MX_ERR_HIP, "no HIP device visible");
  if (o.device >= 0) HIPC(hipSetDevice(o.device));
  HIPC(hipGetDevice(&e->device));
  HIPC(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  std::string path(model_path);
  int rc;
  if (path.rfind("synthetic:", 0) == 0) {
    std::string rest = path.substr(10), name = rest;
    uint64_t seed = o.seed;
    bool q8 = false, q4 = false;
    int kq = 0;
    size_t c = rest.find(':');
    if (c != std::string::npos) {
      name = rest.substr(0, c);
      std::string tail = rest.substr(c + 1);
      while (!tail.empty()) {  // ":seed=N" and/or ":q8_0"
        const size_t e2 = tail.find(':');
        const std::string part = tail.substr(0, e2);
        if (part.rfind("seed=", 0) == 0) seed = strtoull(part.c_str() + 5, nullptr, 10);
        else if (part == "q8_0") q8 = true;
        else if (part == "q4_0") q4 = true;
        else if (part == "q4_k_m") kq = 12;
        else if (part == "q5_k_m") kq = 13;
        else if (part != "bf16") return fail(MX_ERR_MODEL, "unknown synthetic option '" + part + "'");
        tail = e2 == std::string::npos ? "" : tail.substr(e2 + 1);
      }
    }
    const Shape* s = nullptr;
    for (const Shape& k : kShapes)
      if (name == k.name) s = &k;
    if (!s) return fail(MX_ERR_MODEL, "unknown synthetic shape '" + name + "'");
    rc = e->load_synthetic(*s, seed, q8, kq, q4);
  } else {
    rc = e->load_gguf(path);
  }
  if (rc) return rc;
  *out = e.release();
  return 0;
}

void mx_engine_destroy(mx_engine* e) { delete e; }

int mx_gguf_check(const char* path) {
  if (!path) return fail(MX_ERR_ARG, "null path");
  GGUFFile f;
  const std::string err = f.open(path);
  return err.empty() ? MX_OK : fail(MX_ERR_MODEL, err);
}

int mx_engine_info(const mx_engine* e, mx_model_info* o) {
  if (!e || !o) return fail(MX_ERR_ARG, "null argument");
  o->n_embd = e->n_embd; o->n_layer = e->n_layer; o->n_head = e->n_head; o->n_head_kv = e->n_head_kv;
  o->head_dim = e->head_dim; o->n_ff = e->n_ff; o->n_vocab = e->n_vocab; o->n_ctx_train = e->n_ctx_train;
  o->eps = e->eps; o->rope_base = e->rope_base; o->bos_id = e->bos; o->eos_id = e->eos;
  o->n_ctx = e->n_ctx; o->n_seq_max = e->n_seq_max; o->layer_begin = e->lb; o->layer_end = e->le;
  o->has_embed = e->has_embed; o->has_head = e->has_head; o->weight_bytes = e->weight_bytes;
  o->weight_type = e->wq4 ? 2 : e->wq8 ? 8 : e->wkq ? e->kq_main_type : 30;
  return 0;
}

int mx_forward_rows(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                    float* logits_out) {
  if (!e || n < 0 || (n && (!slots || !pos || !ids))) return fail(MX_ERR_ARG, "bad arguments");
  if (!e->has_embed || !e->has_head) return fail(MX_ERR_STATE, "mx_forward_rows needs a full-model engine");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  const int chunk = (!logits_out && e->gemm_ok()) ? PREFILL_ROWS : MAX_ROWS;  // logits: <= 64 rows per chunk
  for (int i = 0; i < n; i += chunk) {
    int m = std::min(chunk, n - i);
    if (int rc = e->forward_rows_chunk(m, slots + i, pos + i, ids + i, nullptr, nullptr,
                                       logits_out ? logits_out + (size_t)i * e->n_vocab : nullptr, e->stream))
      return rc;
  }
  return 0;
}

int mx_forward_topk(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids, int k,
                    float* vals, int32_t* idx) {
  if (!e || n < 1 || n > MAX_ROWS || !slots || !pos || !ids || !vals || !idx || k < 1 || k > TOPK_MAX)
    return fail(MX_ERR_ARG, "mx_forward_topk: 1 <= n <= 64 rows, 1 <= k <= 64");
  if (!e->has_embed || !e->has_head) return fail(MX_ERR_STATE, "mx_forward_topk needs a full-model engine");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  std::vector<float> lg((size_t)n * e->n_vocab);  // the logits stay on the device too (e->logits)
  if (int rc = e->forward_rows_chunk(n, slots, pos, ids, nullptr, nullptr, lg.data(), e->stream)) return rc;
  if (launch_topk(e->logits, e->n_vocab, n, e->n_vocab, k, e->tk_ws_val, e->tk_ws_idx, e->tk_val, e->tk_idx,
                  e->stream))
    return fail(MX_ERR_ARG, "top-k launch shape");
  HIPC(hipMemcpyAsync(vals, e->tk_val, (size_t)n * k * 4, hipMemcpyDeviceToHost, e->stream));
  HIPC(hipMemcpyAsync(idx, e->tk_idx, (size_t)n * k * 4, hipMemcpyDeviceToHost, e->stream));
  HIPC(hipStreamSynchronize(e->stream));
  return 0;
}

int mx_forward_logits(mx_engine* e, int slot, const int32_t* ids, int n, int pos0, float* logits_out) {
  if (!e || n < 0) return fail(MX_ERR_ARG, "bad arguments");
  if (pos0 < 0 || pos0 + n > e->n_ctx) return fail(MX_ERR_CTX, "tokens exceed n_ctx");
  std::vector<int32_t> slots(n, slot), pos(n);
  for (int i = 0; i < n; i++) pos[i] = pos0 + i;
  return mx_forward_rows(e, n, slots.data(), pos.data(), ids, logits_out);
}

int mx_stage_rows(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                  const void* x_in, void* x_out, float* logits_out, void* stream) {
  if (!e || n < 1 || n > MAX_ROWS) return fail(MX_ERR_ARG, "mx_stage_rows: 1 <= n <= 64 rows per call");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  return e->forward_rows_chunk(n, slots, pos, ids, x_in, x_out, logits_out, s);
}

int mx_debug(mx_engine* e, int op, long long arg, void* host, size_t bytes) {
  if (!e) return fail(MX_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  switch (op) {
    case 0: e->dbg_stop = (int)arg; return 0;
    case 1: e->dbg_sync = arg != 0; return 0;
    case 2: {
      const size_t R = PREFILL_ROWS, nl = e->layers.size();
      const void* src = nullptr;
      size_t n = 0;
      switch (arg) {
        case 0: src = e->x, n = R * e->n_embd * 4; break;
        case 1: src = e->q, n = R * e->n_embd * 4; break;
        case 2: src = e->xn, n = R * e->n_embd * 2; break;
        case 3: src = e->attn_out, n = R * e->n_embd * 2; break;
        case 4: src = e->act, n = R * e->n_ff * 2; break;
        case 5: src = e->slabs, n = e->slab_stride * 8 * 4; break;
        case 6: src = e->kcache, n = e->layer_kv_stride * nl * 2; break;
        case 7: src = e->vcache, n = e->layer_kv_stride * nl * 2; break;
        case 8: src = e->ssq, n = R * (e->n_embd / 16) * 4; break;
        case 9: src = e->d_pos, n = R * 4; break;
        case 10: src = e->d_slot, n = R * 4; break;
        case 11: src = e->rope_cs, n = (size_t)e->n_ctx * e->head_dim * 4; break;
        default: return fail(MX_ERR_ARG, "mx_debug: unknown buffer");
      }
      if (!host) return fail(MX_ERR_ARG, "mx_debug: null host buffer");
      HIPC(hipDeviceSynchronize());
      HIPC(hipMemcpy(host, src, std::min(n, bytes), hipMemcpyDeviceToHost));
      return 0;
    }
  }
  return fail(MX_ERR_ARG, "mx_debug: unknown op");
}

static int make_request(mx_engine* e, const int32_t* ids, int n, const mx_sampling* s, int max_tokens,
                        std::unique_ptr<Request>* out) {
  if (!ids || n < 1) return fail(MX_ERR_ARG, "bad arguments");
  if (n >= e->n_ctx) return fail(MX_ERR_CTX, "Requested tokens (" + std::to_string(n) + ") exceed context window of " +
                                                 std::to_string(e->n_ctx));
  for (int i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= e->n_vocab) return fail(MX_ERR_ARG, "token id out of range");
  auto r = std::make_unique<Request>();
  r->prompt.assign(ids, ids + n);
  mx_sampling_default(&r->samp);
  if (s) r->samp = *s;
  r->max_tokens = max_tokens <= 0 ? e->n_ctx - n : std::min(max_tokens, e->n_ctx - n);
  r->seed = r->samp.seed == 0xFFFFFFFFull ? ((uint64_t)std::random_device{}() << 32 | std::random_device{}())
                                           : r->samp.seed;
  *out = std::move(r);
  return 0;
}

// all-or-nothing: every request is validated first, then all are queued under one lock, so the
// scheduler admits them in the same round (one batched prefill, one decode batch)
int mx_submit_batch(mx_engine* e, int n_req, const int32_t* const* ids, const int32_t* lens, const mx_sampling* s,
                    const int32_t* max_tokens, uint64_t* reqs) {
  if (!e || n_req < 1 || !ids || !lens || !max_tokens || !reqs) return fail(MX_ERR_ARG, "bad arguments");
  if (!e->has_embed || !e->has_head) return fail(MX_ERR_STATE, "mx_submit needs a full-model engine");
  std::vector<std::unique_ptr<Request>> rs(n_req);
  for (int i = 0; i < n_req; i++)
    if (int rc = make_request(e, ids[i], lens[i], s ? s + i : nullptr, max_tokens[i], &rs[i])) return rc;
  {
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->stop) return fail(MX_ERR_STATE, "engine shutting down");
    for (int i = 0; i < n_req; i++) {
      Request* r = rs[i].get();
      r->id = e->next_id++;
      reqs[i] = r->id;
      e->pending.push_back(r);
      e->requests[r->id] = std::move(rs[i]);
    }
    if (!e->worker_started) {
      e->worker_started = true;
      e->worker = std::thread([e] { e->scheduler_loop(); });
    }
  }
  e->cv.notify_all();
  return 0;
}

int mx_submit(mx_engine* e, const int32_t* ids, int n, const mx_sampling* s, int max_tokens, uint64_t* req) {
  if (!e || !ids || n < 1 || !req) return fail(MX_ERR_ARG, "bad arguments");
  const int32_t len = n;
  return mx_submit_batch(e, 1, &ids, &len, s, &max_tokens, req);
}

int mx_wait(mx_engine* e, uint64_t req, int32_t* out_ids, int cap, int* n_out, int* finish) {
  if (!e) return fail(MX_ERR_ARG, "null engine");
  std::unique_ptr<Request> r;
  {
    std::unique_lock<std::mutex> lk(e->mu);
    auto it = e->requests.find(req);
    if (it == e->requests.end()) return fail(MX_ERR_NOTFOUND, "unknown request id");
    Request* rp = it->second.get();
    e->cv_done.wait(lk, [&] { return rp->done; });
    if (n_out) *n_out = (int)rp->out.size();
    if ((int)rp->out.size() > cap && rp->finish != MX_FINISH_ERROR)
      return fail(MX_ERR_ARG, "mx_wait: " + std::to_string(rp->out.size()) + " tokens do not fit cap " +
                                  std::to_string(cap) + " (request kept; retry with a larger buffer)");
    r = std::move(it->second);
    e->requests.erase(it);
  }
  int n = std::min<int>(cap, (int)r->out.size());
  if (out_ids && n > 0) memcpy(out_ids, r->out.data(), n * 4);
  if (n_out) *n_out = (int)r->out.size();
  if (finish) *finish = r->finish;
  if (r->finish == MX_FINISH_ERROR) return fail(MX_ERR_STATE, "request failed: " + r->error);
  return 0;
}

int mx_poll(mx_engine* e, uint64_t req, int n_have, int32_t* out_ids, int cap, int* n_out, int* done) {
  if (!e) return fail(MX_ERR_ARG, "null engine");
  std::unique_lock<std::mutex> lk(e->mu);
  auto it = e->requests.find(req);
  if (it == e->requests.end()) return fail(MX_ERR_NOTFOUND, "unknown request id");
  Request* rp = it->second.get();
  e->cv_done.wait(lk, [&] { return rp->done || (int)rp->out.size() > n_have; });
  const int n = (int)rp->out.size();
  if (out_ids && cap > 0) memcpy(out_ids, rp->out.data(), (size_t)std::min(cap, n) * 4);
  if (n_out) *n_out = n;
  if (done) *done = rp->done ? 1 : 0;
  return 0;
}

int mx_cancel(mx_engine* e, uint64_t req) {
  if (!e) return fail(MX_ERR_ARG, "null engine");
  std::lock_guard<std::mutex> lk(e->mu);
  auto it = e->requests.find(req);
  if (it == e->requests.end()) return fail(MX_ERR_NOTFOUND, "unknown request id");
  it->second->cancel = true;
  return 0;
}

int mx_batch_create(mx_engine* e, int M, const int32_t* slots, const int32_t* pos, const int32_t* ids, int max_steps,
                    mx_batch** out) {
  if (!e || !out || M < 1 || M > MAX_ROWS || !slots || !pos || max_steps < 0) return fail(MX_ERR_ARG, "bad arguments");
  int max_pos = 0;
  for (int i = 0; i < M; i++) {
    if (slots[i] < 0 || slots[i] >= e->n_seq_max) return fail(MX_ERR_ARG, "slot out of range");
    if (pos[i] < 0 || pos[i] >= e->n_ctx) return fail(MX_ERR_CTX, "position outside n_ctx");
    if (ids && (ids[i] < 0 || ids[i] >= e->n_vocab)) return fail(MX_ERR_ARG, "token id out of range");
    max_pos = std::max(max_pos, (int)pos[i]);
  }
  {
    std::lock_guard<std::mutex> lk(e->mu);
    for (int i = 0; i < M; i++) e->slot_tokens[slots[i]].clear();  // decode steps will overwrite them
  }
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  std::unique_ptr<mx_batch> b(new mx_batch());
  b->M = M;
  b->max_steps = max_steps;
  {
    std::vector<int32_t> sorted(slots, slots + M);
    std::sort(sorted.begin(), sorted.end());
    b->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  }
  b->max_pos = max_pos;
  HIPC(hipMalloc((void**)&b->d_ids, M * 4));
  HIPC(hipMalloc((void**)&b->d_pos, M * 4));
  HIPC(hipMalloc((void**)&b->d_slot, M * 4));
  HIPC(hipMalloc((void**)&b->d_hist, (size_t)M * std::max(1, max_steps) * 4));
  HIPC(hipMalloc((void**)&b->d_hist_count, M * 4));
  HIPC(hipMemcpy(b->d_pos, pos, M * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(b->d_slot, slots, M * 4, hipMemcpyHostToDevice));
  if (ids) HIPC(hipMemcpy(b->d_ids, ids, M * 4, hipMemcpyHostToDevice));
  else HIPC(hipMemset(b->d_ids, 0, M * 4));
  HIPC(hipMemset(b->d_hist_count, 0, M * 4));
  *out = b.release();
  return 0;
}

int32_t* mx_batch_ids_device(mx_batch* b) { return b ? b->d_ids : nullptr; }

int mx_batch_bind_ids(mx_engine* e, mx_batch* b, int32_t* ids_device) {
  if (!e || !b || !ids_device) return fail(MX_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  HIPC(hipDeviceSynchronize());
  HIPC(hipMemcpy(ids_device, b->d_ids, b->M * 4, hipMemcpyDeviceToDevice));
  if (!b->ids_external) hipFree(b->d_ids);
  b->d_ids = ids_device;
  b->ids_external = true;
  for (auto& kv : b->graphs) hipGraphExecDestroy(kv.second);
  b->graphs.clear();
  return 0;
}

int mx_batch_step(mx_engine* e, mx_batch* b, const void* x_in, void* x_out, void* stream) {
  if (!e || !b) return fail(MX_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  const bool head = x_out == nullptr;
  if (b->max_pos >= e->n_ctx) return fail(MX_ERR_CTX, "decode batch reached n_ctx");
  b->max_pos++;
  if (head && !e->has_head) return fail(MX_ERR_STATE, "x_out is required on a non-final pipeline stage");
  if (!x_in && !e->has_embed) return fail(MX_ERR_STATE, "x_in is required on a non-first pipeline stage");
  auto body = [&]() -> int {
    e->rows_distinct = b->distinct;
    e->pick_samp = head && b->ktop > 0 ? b->d_samp : nullptr;
    e->pick_k = head ? b->ktop : 0;
    struct Reset {
      mx_engine* e;
      ~Reset() { e->rows_distinct = false; e->pick_samp = nullptr; e->pick_k = 0; }
    } reset_flags{e};
    if (int rc = e->enqueue_forward(b->M, b->d_ids, b->d_pos, b->d_slot, x_in, x_out, head, nullptr, b->M, head,
                                    b->d_ids, b->d_pos, b->d_hist, b->max_steps, b->d_hist_count, b->max_steps, s))
      return rc;
    if (!head) advance_pos_kernel<<<(b->M + 63) / 64, 64, 0, s>>>(b->d_pos, b->M);
    return 0;
  };
  if (!e->use_graphs) return body();
  GraphKey key{b->M, x_in, x_out, s, head ? b->ktop : 0};
  auto it = b->graphs.find(key);
  if (it == b->graphs.end()) {
    hipGraph_t g;
    HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = body();
    hipError_t ce = hipStreamEndCapture(s, &g);
    if (rc) return rc;
    if (ce != hipSuccess) return fail(MX_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(ce));
    hipGraphExec_t ex;
    HIPC(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    it = b->graphs.emplace(key, ex).first;
  }
  HIPC(hipGraphLaunch(it->second, s));
  return 0;
}

int mx_batch_tokens(mx_engine* e, mx_batch* b, int32_t* out, int cap, int* n_steps) {
  if (!e || !b) return fail(MX_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  HIPC(hipDeviceSynchronize());
  std::vector<int32_t> cnt(b->M);
  HIPC(hipMemcpy(cnt.data(), b->d_hist_count, b->M * 4, hipMemcpyDeviceToHost));
  if (n_steps) *n_steps = cnt[0];
  if (out && cap > 0 && b->max_steps > 0) {
    std::vector<int32_t> h((size_t)b->M * b->max_steps);
    HIPC(hipMemcpy(h.data(), b->d_hist, h.size() * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < b->M; i++)
      for (int j = 0; j < cap && j < b->max_steps; j++) out[(size_t)i * cap + j] = h[(size_t)i * b->max_steps + j];
  }
  return 0;
}

void mx_batch_destroy(mx_engine* e, mx_batch* b) {
  if (!b) return;
  if (e) {
    std::lock_guard<std::mutex> lk(e->gpu_mu);
    hipSetDevice(e->device);
    hipDeviceSynchronize();
  }
  for (auto& kv : b->graphs) hipGraphExecDestroy(kv.second);
  if (!b->ids_external) hipFree(b->d_ids);
  hipFree(b->d_pos);
  hipFree(b->d_slot);
  hipFree(b->d_hist);
  hipFree(b->d_hist_count);
  if (b->d_samp) hipFree(b->d_samp);
  delete b;
}

static int fill_samp_rows(mx_engine* e, int n, const mx_row_sampler* rows, std::vector<SampRow>& out, int* ktop) {
  out.assign(n, SampRow{});
  *ktop = 0;
  for (int i = 0; i < n; i++) {
    const mx_sampling& sp = rows[i].s;
    const bool sampling = sp.temperature > 0.f || has_penalties(sp);
    if (sampling && !mx_engine::device_sampleable(sp))
      return fail(MX_ERR_ARG, "row " + std::to_string(i) + ": sampling settings need the host sampler "
                                  "(top_k outside 1..64 or a penalty window over 64 tokens)");
    if (rows[i].n_win < 0 || rows[i].n_win > SAMP_WIN) return fail(MX_ERR_ARG, "penalty window over 64 tokens");
    SampRow& o = out[i];
    o.temp = sp.temperature; o.top_p = sp.top_p; o.min_p = sp.min_p; o.repeat = sp.repeat_penalty;
    o.freq = sp.frequency_penalty; o.presence = sp.presence_penalty;
    o.top_k = std::max(1, std::min(sp.top_k, TOPK_MAX));
    o.last_n = has_penalties(sp) ? std::min(sp.repeat_last_n, SAMP_WIN) : 0;
    o.seed = rows[i].seed;
    o.draw0 = rows[i].n_drawn;
    o.n_win = std::min(rows[i].n_win, o.last_n);
    for (int j = 0; j < o.n_win; j++) o.win[j] = rows[i].win[rows[i].n_win - o.n_win + j];
    if (sampling) *ktop = std::max(*ktop, std::min(o.top_k, e->n_vocab));
  }
  return 0;
}

int mx_batch_reset(mx_engine* e, mx_batch* b, const int32_t* pos, const int32_t* ids, const mx_row_sampler* rows,
                   void* stream) {
  if (!e || !b || !pos) return fail(MX_ERR_ARG, "null argument");
  int max_pos = 0;
  for (int i = 0; i < b->M; i++) {
    if (pos[i] < 0 || pos[i] >= e->n_ctx) return fail(MX_ERR_CTX, "position outside n_ctx");
    if (ids && (ids[i] < 0 || ids[i] >= e->n_vocab)) return fail(MX_ERR_ARG, "token id out of range");
    max_pos = std::max(max_pos, (int)pos[i]);
  }
  std::vector<SampRow> sr;
  int ktop = 0;
  if (rows)
    if (int rc = fill_samp_rows(e, b->M, rows, sr, &ktop)) return rc;
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  HIPC(hipMemcpyAsync(b->d_pos, pos, b->M * 4, hipMemcpyHostToDevice, s));
  if (ids) HIPC(hipMemcpyAsync(b->d_ids, ids, b->M * 4, hipMemcpyHostToDevice, s));
  HIPC(hipMemsetAsync(b->d_hist_count, 0, b->M * 4, s));
  if (ktop > 0) {
    if (!b->d_samp) HIPC(hipMalloc((void**)&b->d_samp, (size_t)MAX_ROWS * sizeof(SampRow)));
    HIPC(hipMemcpyAsync(b->d_samp, sr.data(), b->M * sizeof(SampRow), hipMemcpyHostToDevice, s));
  }
  HIPC(hipStreamSynchronize(s));  // the host arrays may go away when this returns
  b->ktop = ktop;
  b->max_pos = max_pos;
  return 0;
}

int mx_stage_rows_pick(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                       const void* x_in, void* x_out, int n_out, const int32_t* rowmap, const mx_row_sampler* samp,
                       int32_t* tok_out, void* stream) {
  if (!e || n < 1 || !slots || !pos || n_out < 0 || (n_out && (!rowmap || !tok_out)))
    return fail(MX_ERR_ARG, "mx_stage_rows_pick: bad arguments");
  if (!x_in && (!e->has_embed || !ids)) return fail(MX_ERR_STATE, "x_in is required on a non-first pipeline stage");
  if (n_out && (x_out || !e->has_head)) return fail(MX_ERR_STATE, "tokens are picked on the last stage only");
  for (int k = 0; k < n_out; k++)
    if (rowmap[k] < 0 || rowmap[k] >= n || (k && rowmap[k] <= rowmap[k - 1]))
      return fail(MX_ERR_ARG, "rowmap must be increasing row indices");
  std::vector<SampRow> sr;
  int ktop = 0;
  if (samp && n_out)
    if (int rc = fill_samp_rows(e, n_out, samp, sr, &ktop)) return rc;
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  hipStream_t s = stream ? (hipStream_t)stream : e->stream;
  const size_t xb = (size_t)e->n_embd * (e->handoff_bf16 ? 2 : 4);  // hand-off bytes per row
  const int chunk = e->gemm_ok() ? PREFILL_ROWS : MAX_ROWS;
  int k0 = 0;  // first rowmap entry not yet produced
  for (int i = 0; i < n;) {
    int end = std::min(n, i + chunk), k1 = k0;
    while (k1 < n_out && rowmap[k1] < end && k1 - k0 < MAX_ROWS) k1++;
    // cut after the 64th prompt's last row, rounded up to its 16-row block (the prompts' padding)
    if (k1 - k0 == MAX_ROWS && k1 < n_out && rowmap[k1] < end) end = std::min(n, (rowmap[k1 - 1] + 16) / 16 * 16);
    const int m = end - i, no = k1 - k0;
    for (int r = i; r < end; r++) {
      if (slots[r] < 0 || slots[r] >= e->n_seq_max) return fail(MX_ERR_ARG, "slot out of range");
      if (pos[r] < 0 || pos[r] >= e->n_ctx) return fail(MX_ERR_CTX, "position outside n_ctx");
      if (!x_in && (ids[r] < 0 || ids[r] >= e->n_vocab)) return fail(MX_ERR_ARG, "token id out of range");
    }
    if (!x_in) HIPC(hipMemcpyAsync(e->d_ids, ids + i, m * 4, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(e->d_pos, pos + i, m * 4, hipMemcpyHostToDevice, s));
    HIPC(hipMemcpyAsync(e->d_slot, slots + i, m * 4, hipMemcpyHostToDevice, s));
    std::vector<int32_t> rm(no);
    for (int k = 0; k < no; k++) rm[k] = rowmap[k0 + k] - i;
    if (no) HIPC(hipMemcpyAsync(e->d_rowmap, rm.data(), no * 4, hipMemcpyHostToDevice, s));
    if (no && ktop > 0) HIPC(hipMemcpyAsync(e->d_samp, sr.data() + k0, no * sizeof(SampRow), hipMemcpyHostToDevice, s));
    {
      std::lock_guard<std::mutex> lk2(e->mu);
      for (int r = i; r < end; r++) e->slot_tokens[slots[r]].clear();
    }
    e->rows_distinct = false;
    e->rows_blocked = e->blocked_rows(slots + i, pos + i, x_in ? nullptr : ids + i, m);
    e->prefill_gemm = true;
    e->pick_samp = ktop > 0 ? e->d_samp : nullptr;
    e->pick_k = ktop;
    const char* xi = (const char*)x_in;
    char* xo = (char*)x_out;
    const int frc = e->enqueue_forward(m, e->d_ids, e->d_pos, e->d_slot, xi ? xi + i * xb : nullptr,
                                       xo ? xo + i * xb : nullptr, no > 0, no ? e->d_rowmap : nullptr, no, false,
                                       nullptr, nullptr, nullptr, 0, nullptr, 0, s);
    e->rows_blocked = false;
    e->prefill_gemm = false;
    if (!frc && no) e->pick(no, nullptr, nullptr, nullptr, 0, nullptr, 0, s);  // logits rows [no][V]
    e->pick_samp = nullptr;
    e->pick_k = 0;
    if (frc) return frc;
    if (no) HIPC(hipMemcpyAsync(tok_out + k0, e->d_tok, no * 4, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    k0 = k1;
    i = end;
  }
  return 0;
}

int mx_engine_stats(mx_engine* e, mx_stats* out) {
  if (!e || !out) return fail(MX_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(e->mu);
  out->prompt_tokens = e->stat_prompt_tokens;
  out->reused_prompt_tokens = e->stat_reused_tokens;
  out->generated_tokens = e->stat_generated_tokens;
  return 0;
}

int mx_device_count(int32_t* n) {
  if (!n) return fail(MX_ERR_ARG, "null argument");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return 0;
}

int mx_sync(mx_engine* e) {
  if (!e) return fail(MX_ERR_ARG, "null engine");
  hipSetDevice(e->device);
  HIPC(hipDeviceSynchronize());
  return 0;
}

static int probe_hbm(int device, size_t bytes, int iters, bool read_only, double* gbs, char* desc, int desc_len);

int mx_probe_copy(int device, size_t bytes, int iters, double* gbs, char* desc, int desc_len) {
  return probe_hbm(device, bytes, iters, false, gbs, desc, desc_len);
}

int mx_probe_read(int device, size_t bytes, int iters, double* gbs, char* desc, int desc_len) {
  return probe_hbm(device, bytes, iters, true, gbs, desc, desc_len);
}

}  // extern "C"

// Best of the probe variants (loads in flight x grid x non-temporal): each is warmed twice, then
// `iters` launches are timed with HIP events on a private stream.  Every HIP call is checked and
// every object created is released on all paths.
static int probe_hbm(int device, size_t bytes, int iters, bool read_only, double* gbs, char* desc, int desc_len) {
  const size_t n16 = bytes / 16 / 4096 * 4096;  // whole 4096-word chunks (the largest variant's unit)
  if (n16 == 0 || iters < 1 || !gbs) return fail(MX_ERR_ARG, "bad arguments");
  HIPC(hipSetDevice(device));
  uint4 *src = nullptr, *dst = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t t0 = nullptr, t1 = nullptr;
  hipError_t err = hipMalloc(&src, n16 * 16);
  if (err == hipSuccess) err = hipMalloc(&dst, read_only ? (size_t)4096 * 256 * 16 : n16 * 16);  // read: sink only
  if (err == hipSuccess) err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (err == hipSuccess) err = hipEventCreate(&t0);
  if (err == hipSuccess) err = hipEventCreate(&t1);
  if (err == hipSuccess) err = hipMemsetAsync(src, 1, n16 * 16, s);
  double best = 0.0;
  char d[160] = "", bestd[160] = "";
  for (int v = 0; err == hipSuccess && v < mx::probe_variants(); v++) {
    for (int i = 0; i < 2 && err == hipSuccess; i++) {
      mx::launch_probe(v, read_only, src, dst, n16, s, d, sizeof d);
      err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipEventRecord(t0, s);
    for (int i = 0; i < iters && err == hipSuccess; i++) {
      mx::launch_probe(v, read_only, src, dst, n16, s, nullptr, 0);
      err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipEventRecord(t1, s);
    if (err == hipSuccess) err = hipEventSynchronize(t1);
    float ms = 0.f;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, t0, t1);
    if (err == hipSuccess && ms > 0.f) {
      const double r = (read_only ? 1.0 : 2.0) * (double)n16 * 16 * iters / (ms * 1e-3) / 1e9;
      if (r > best) {
        best = r;
        memcpy(bestd, d, sizeof d);
      }
    }
  }
  if (t0) hipEventDestroy(t0);
  if (t1) hipEventDestroy(t1);
  if (s) hipStreamDestroy(s);
  if (src) hipFree(src);
  if (dst) hipFree(dst);
  if (err != hipSuccess) return fail(MX_ERR_HIP, std::string("HBM probe: ") + hipGetErrorString(err));
  if (best <= 0.0) return fail(MX_ERR_HIP, "HBM probe: no timing");
  *gbs = best;
  if (desc && desc_len > 0) snprintf(desc, desc_len, "%s", bestd);
  return MX_OK;
}

extern "C" {

int mx_profile_kernel(mx_engine* e, int kind, int M, int iters, double* us, double* bytes) {
  if (!e || M < 1 || M > MAX_ROWS || iters < 1) return fail(MX_ERR_ARG, "bad arguments");
  std::lock_guard<std::mutex> lk(e->gpu_mu);
  hipSetDevice(e->device);
  hipStream_t s = e->stream;
  const int h = e->n_embd, kv = e->n_embd_kv, ff = e->n_ff;
  const int prof_pos = std::min(e->n_ctx - 1, std::max(0, getenv("MX_PROF_POS") ? atoi(getenv("MX_PROF_POS")) : 0));
  const bool prof_fin = getenv("MX_PROF_FIN") != nullptr;  // kind 7: the FIN form (slabs finished in the kernel)
  const bool prof_warm = getenv("MX_PROF_WARM") != nullptr;  // diagnosis: every launch on layer 0 (Infinity-Cache warm)
  std::vector<int32_t> zero(M, prof_pos), slots(M);
  for (int i = 0; i < M; i++) slots[i] = i % e->n_seq_max;
  HIPC(hipMemcpyAsync(e->d_pos, zero.data(), M * 4, hipMemcpyHostToDevice, s));
  HIPC(hipMemcpyAsync(e->d_slot, slots.data(), M * 4, hipMemcpyHostToDevice, s));
  hipEvent_t t0, t1;
  HIPC(hipEventCreate(&t0));
  HIPC(hipEventCreate(&t1));
  const int nl = (int)e->layers.size();
  size_t per = 0;
  int launches = 0;
  auto one = [&](int li) -> int {
    const Layer& L = e->layers[li];
    MMArgs a{};
    a.M = M;
    if (e->wq8 && kind <= 4) {  // Q8_0 weights: the activations are Q8_0 rows in xq8/xqd
      a.xq = e->xq8; a.xd = e->xqd; a.wq4 = e->wq4;
      // <= 4 rows: the form the decode runs -- the GEMV quantises its operand on load (gate/up and q|k|v
      // with the RMS_NORM from the ssq partials)
      const bool pql = e->q8_on_load(M) && getenv("MX_PROF_PREQUANT") == nullptr;
      auto ql_operand = [&](const float* src, int K, const float* norm_w) {
        if (!pql) return;
        a.xq = nullptr; a.xd = nullptr; a.xf = src; a.norm_w = norm_w; a.eps = e->eps;
        a.ssq = norm_w ? e->ssq : nullptr; a.np = K / 16;
      };
      auto qb = e->wq4 ? q4_matrix_bytes : q8_matrix_bytes;
      switch (kind) {
        case 0:
          a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.out = e->q; a.ldo = h; a.n_q = h; a.n_kv = kv;
          a.head_dim = e->head_dim; a.pos = e->d_pos; a.slot = e->d_slot; a.rope_cs = e->rope_cs;
          a.kc = e->kcache + e->layer_kv_stride * li; a.vc = e->vcache + e->layer_kv_stride * li;
          a.n_ctx = e->n_ctx; a.ctx_stride = e->ctx_stride; a.n_head_kv = e->n_head_kv; a.slot_stride = e->slot_stride;
          per = qb(h + 2 * kv, h);
          ql_operand(e->x, h, L.attn_norm);
          return launch_mq8(EPI_QKV, a, s);
        case 1: case 3:
          a.W = kind == 1 ? L.o : L.down; a.N = h; a.K = kind == 1 ? h : ff; a.out = e->x; a.ldo = h;
          per = qb(h, a.K);
          ql_operand(kind == 1 ? e->attn_f : e->act_f, a.K, nullptr);
          return launch_mq8(EPI_RESID, a, s);
        case 2:
          a.W = L.gu; a.N = 2 * ff; a.K = h; a.actf = e->act_f; a.lda = ff;
          per = qb(2 * ff, h);
          ql_operand(e->x, h, L.ffn_norm);
          return launch_mq8(EPI_SWIGLU, a, s);
        case 4:
          if (!e->has_head || e->out_kq_head) return -1;
          a.wq4 = e->out_q4;
          a.W = e->output; a.N = e->n_vocab; a.K = h; a.out = e->logits; a.ldo = e->n_vocab;
          per = e->out_q4 ? q4_matrix_bytes(e->n_vocab, h) : q8_matrix_bytes(e->n_vocab, h);
          return launch_mq8(EPI_F32, a, s);
      }
    }
    if (e->wkq && kind <= 4) {  // K-quant weights: the activations are Q8_K rows in xq8/xqd/xkb
      a.xq = e->xq8; a.xd = e->xqd; a.xb = e->xkb;
      const bool pql = e->kq_on_load(M) && getenv("MX_PROF_PREQUANT") == nullptr;  // as the decode runs it
      auto ql_operand = [&](const float* src, int K, const float* norm_w) {
        if (!pql) return;
        a.xq = nullptr; a.xd = nullptr; a.xb = nullptr; a.xf = src; a.norm_w = norm_w; a.eps = e->eps;
        a.ssq = norm_w ? e->ssq : nullptr; a.np = K / 16;
      };
      switch (kind) {
        case 0:
          a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.out = e->q; a.ldo = h; a.n_q = h; a.n_kv = kv;
          a.head_dim = e->head_dim; a.pos = e->d_pos; a.slot = e->d_slot; a.rope_cs = e->rope_cs;
          a.kc = e->kcache + e->layer_kv_stride * li; a.vc = e->vcache + e->layer_kv_stride * li;
          a.n_ctx = e->n_ctx; a.ctx_stride = e->ctx_stride; a.n_head_kv = e->n_head_kv; a.slot_stride = e->slot_stride;
          L.kq_qkv.set(a);
          per = L.kq_qkv.bytes;
          ql_operand(e->x, h, L.attn_norm);
          return launch_mkq(EPI_QKV, a, s);
        case 1: case 3:
          a.W = kind == 1 ? L.o : L.down; a.N = h; a.K = kind == 1 ? h : ff; a.out = e->x; a.ldo = h;
          (kind == 1 ? L.kq_o : L.kq_down).set(a);
          per = (kind == 1 ? L.kq_o : L.kq_down).bytes;
          ql_operand(kind == 1 ? e->attn_f : e->act_f, a.K, nullptr);
          return launch_mkq(EPI_RESID, a, s);
        case 2:
          a.W = L.gu; a.N = 2 * ff; a.K = h; a.actf = e->act_f; a.lda = ff;
          L.kq_gu.set(a);
          per = L.kq_gu.bytes;
          ql_operand(e->x, h, L.ffn_norm);
          return launch_mkq(EPI_SWIGLU, a, s);
        case 4:
          if (!e->has_head) return -1;
          a.W = e->output; a.N = e->n_vocab; a.K = h; a.out = e->logits; a.ldo = e->n_vocab;
          e->kq_out.set(a);
          per = e->kq_out.bytes;
          return launch_mkq(EPI_F32, a, s);
      }
    }
    if ((e->wq8 || e->wkq) && (kind >= 5 && kind <= 6)) return -1;
    switch (kind) {
      case 0:
        a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.X = e->xn; a.ldx = h; a.out = e->q; a.ldo = h; a.n_q = h;
        a.n_kv = kv; a.head_dim = e->head_dim; a.pos = e->d_pos; a.slot = e->d_slot; a.rope_cs = e->rope_cs;
        a.kc = e->kcache + e->layer_kv_stride * li; a.vc = e->vcache + e->layer_kv_stride * li; a.n_ctx = e->n_ctx;
        a.ctx_stride = e->ctx_stride;
        a.n_head_kv = e->n_head_kv; a.slot_stride = e->slot_stride;
        per = (size_t)(h + 2 * kv) * h * 2;
        return (M > 16 && e->use_wide) ? (launch_mm_wide(EPI_QKV, a, e->slabs, e->slab_stride, s) < 0) : launch_mm(EPI_QKV, a, s);
      case 1:
        a.W = L.o; a.N = h; a.K = h; a.X = e->attn_out; a.ldx = h; a.out = e->x; a.ldo = h;
        per = (size_t)h * h * 2;
        return (M > 16 && e->use_wide) ? (launch_mm_wide(EPI_RESID, a, e->slabs, e->slab_stride, s) < 0) : launch_mm(EPI_RESID, a, s);
      case 2:
        a.W = L.gu; a.N = 2 * ff; a.K = h; a.X = e->xn; a.ldx = h; a.act = e->act; a.lda = ff;
        per = (size_t)2 * ff * h * 2;
        return (M > 16 && e->use_wide) ? (launch_mm_wide(EPI_SWIGLU, a, e->slabs, e->slab_stride, s) < 0) : launch_mm(EPI_SWIGLU, a, s);
      case 3:
        a.W = L.down; a.N = h; a.K = ff; a.X = e->act; a.ldx = ff; a.out = e->x; a.ldo = h;
        per = (size_t)h * ff * 2;
        return (M > 16 && e->use_wide) ? (launch_mm_wide(EPI_RESID, a, e->slabs, e->slab_stride, s) < 0) : launch_mm(EPI_RESID, a, s);
      case 4:
        if (!e->has_head) return -1;
        a.W = e->output; a.N = e->n_vocab; a.K = h; a.X = e->xn; a.ldx = h; a.out = e->logits; a.ldo = e->n_vocab;
        per = (size_t)e->n_vocab * h * 2;
        return (M > 16 && e->use_wide) ? (launch_mm_wide(EPI_F32, a, e->slabs, e->slab_stride, s) < 0) : launch_mm(EPI_F32, a, s);
      case 5:  // qkv with the attention RMSNorm applied on load (M <= 16)
        a.W = L.qkv; a.N = h + 2 * kv; a.K = h; a.X = nullptr; a.xf = e->x; a.norm_w = L.attn_norm; a.eps = e->eps;
        a.ssq = e->ssq; a.np = h / 16;
        a.out = e->q; a.ldo = h; a.n_q = h; a.n_kv = kv; a.head_dim = e->head_dim; a.pos = e->d_pos;
        a.slot = e->d_slot; a.rope_cs = e->rope_cs; a.kc = e->kcache + e->layer_kv_stride * li;
        a.vc = e->vcache + e->layer_kv_stride * li; a.n_ctx = e->n_ctx; a.ctx_stride = e->ctx_stride;
        a.n_head_kv = e->n_head_kv; a.slot_stride = e->slot_stride;
        per = (size_t)(h + 2 * kv) * h * 2;
        return launch_mm(EPI_QKV, a, s);
      case 6:  // gate/up with the ffn RMSNorm applied on load (M <= 16)
        a.W = L.gu; a.N = 2 * ff; a.K = h; a.X = nullptr; a.xf = e->x; a.norm_w = L.ffn_norm; a.eps = e->eps;
        a.ssq = e->ssq; a.np = h / 16;
        a.act = e->act; a.lda = ff;
        per = (size_t)2 * ff * h * 2;
        return (e->use_pers && mm_pers_supported(EPI_SWIGLU, M, a.N, a.K)) ? launch_mm_pers(EPI_SWIGLU, a, s)
                                                                            : launch_mm(EPI_SWIGLU, a, s);
      case 8: case 9: case 10: {  // RMS_NORM of M rows folding 4 (8) / 8 (9) / 0 (10) split-K slabs
        const int ns = kind == 8 ? 4 : kind == 9 ? 8 : 0;
        per = (size_t)M * h * 4 * (2 + ns) + (size_t)M * h * 2;
        launch_resid_norm(e->xn, h, e->x, e->slabs, ns, e->slab_stride, L.ffn_norm, M, h, e->eps, s);
        return 0;
      }
      case 7: {  // attention at the positions set below (ctx = pos + 1)
        AttnArgs at{};
        at.q = e->q; at.kc = e->kcache + e->layer_kv_stride * li; at.vc = e->vcache + e->layer_kv_stride * li;
        at.pos = e->d_pos; at.slot = e->d_slot; at.out = e->attn_out; at.ldo = h; at.M = M; at.n_head = e->n_head;
        at.n_head_kv = e->n_head_kv; at.head_dim = e->head_dim; at.n_ctx = e->n_ctx; at.ctx_stride = e->ctx_stride;
        at.slot_stride = e->slot_stride; at.scale = 1.0f / sqrtf((float)e->head_dim);
        if (prof_fin) {  // the 32-row decode's form: q/k/v still as 4 split-K slabs, finished here
          at.slabs = e->slabs; at.nslab = 4; at.slab_stride = e->slab_stride; at.rope_cs = e->rope_cs;
          at.kc_w = e->kcache + e->layer_kv_stride * li; at.vc_w = e->vcache + e->layer_kv_stride * li;
        }
        per = (size_t)M * (prof_pos + 1) * kv * 2 * 2;
        launch_attention(at, s);
        return 0;
      }
    }
    return -1;
  };
  // warm-up pass, then timed passes; each pass walks every local layer so no
  // launch re-reads weights that the previous one left in the caches
  for (int li = 0; li < nl; li++)
    if (one(li)) return fail(MX_ERR_ARG, "bad kernel kind");
  HIPC(hipEventRecord(t0, s));
  for (int it = 0; it < iters; it++) {
    if (kind == 4) {
      if (one(0)) return fail(MX_ERR_ARG, "bad kernel kind");
      launches++;
    } else {
      for (int li = 0; li < nl; li++) {
        one(prof_warm ? 0 : li);
        launches++;
      }
    }
  }
  HIPC(hipEventRecord(t1, s));
  HIPC(hipEventSynchronize(t1));
  float ms = 0;
  HIPC(hipEventElapsedTime(&ms, t0, t1));
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  if (kind == 7 && getenv("MX_ATTN_TRACE")) {  // diagnosis: phase stamps of one launch (layer 0)
    const size_t n = (size_t)M * e->n_head_kv * 8 * 8;
    unsigned long long* tr = nullptr;
    HIPC(hipMalloc((void**)&tr, n * 8));
    HIPC(hipMemsetAsync(tr, 0, n * 8, s));
    AttnArgs at{};
    at.q = e->q; at.kc = e->kcache; at.vc = e->vcache; at.pos = e->d_pos; at.slot = e->d_slot; at.out = e->attn_out;
    at.ldo = h; at.M = M; at.n_head = e->n_head; at.n_head_kv = e->n_head_kv; at.head_dim = e->head_dim;
    at.n_ctx = e->n_ctx; at.ctx_stride = e->ctx_stride; at.slot_stride = e->slot_stride;
    at.scale = 1.0f / sqrtf((float)e->head_dim); at.trace = tr;
    if (prof_fin) {
      at.slabs = e->slabs; at.nslab = 4; at.slab_stride = e->slab_stride; at.rope_cs = e->rope_cs;
      at.kc_w = e->kcache; at.vc_w = e->vcache;
    }
    launch_attention(at, s);
    HIPC(hipStreamSynchronize(s));
    std::vector<unsigned long long> t(n);
    HIPC(hipMemcpy(t.data(), tr, n * 8, hipMemcpyDeviceToHost));
    hipFree(tr);
    unsigned long long t0m = ~0ull, tend = 0;
    double ph[5] = {0, 0, 0, 0, 0};
    int cnt = 0;
    double chunks = 0;
    for (size_t g = 0; g < n / 8; g++) {
      const unsigned long long* p = &t[g * 8];
      if (!p[0]) continue;
      t0m = std::min(t0m, p[0]);
      tend = std::max(tend, p[5]);
      for (int k = 0; k < 5; k++)
        if (p[k + 1] >= p[k] && p[k]) ph[k] += (double)(p[k + 1] - p[k]) / 100.0;
      chunks += (double)p[7];
      cnt++;
    }
    fprintf(stderr, "attn trace M=%d pos=%d: waves %d, span %.2f us (first start -> last end); mean per wave: "
                    "q %.2f | first K/V %.2f | chunks %.2f (%.2f chunks) | merge wait %.2f | store %.2f us\n",
            M, prof_pos, cnt, (tend - t0m) / 100.0, ph[0] / cnt, ph[1] / cnt, ph[2] / cnt, chunks / cnt, ph[3] / cnt,
            ph[4] / cnt);
  }
  if (us) *us = ms * 1000.0 / launches;
  if (bytes) *bytes = (double)per;
  return 0;
}

}  // extern "C"
