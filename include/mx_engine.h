/*
 * mx_engine.h -- C ABI of the MI355X-native local-inference engine.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * node builds its model and calls it exactly twice:
 *
 *   self.model = Llama(model_path=model_path)                 llama_p2p_network.py:19
 *   result = self.model(prompt, max_tokens=100)["choices"][0]["text"]
 *                                                             llama_p2p_network.py:125
 *
 * Both calls land in llama-cpp-python (module llama_cpp, ~0.3.1), whose own
 * ctypes binding to llama.cpp is what these entry points replace:
 *   mx_engine_create   <- llama_load_model_from_file + llama_new_context_with_model
 *                         (Llama.__init__, reached from :19)
 *   mx_submit/mx_wait  <- Llama.__call__ -> create_completion -> generate():
 *                         llama_decode + sampling per token (reached from :125)
 *   mx_forward_logits  <- llama_decode + llama_get_logits (Llama.eval), parity hook
 *   mx_engine_destroy  <- llama_free / llama_free_model (Llama.__del__)
 * The Python layer (llama-p2p_amd/llama.py) mirrors the Llama class on top of
 * this ABI, so handle_requests / cached_inference / distributed_inference /
 * compute_model_hash (llama_p2p_network.py:84-182) run unchanged.
 *
 * Conventions: plain pointers and sizes only; every function returns 0 on
 * success or a negative MX_ERR_* code, with a message in mx_last_error()
 * (thread-local).  The engine owns device weights, KV cache and streams; the
 * caller owns every host buffer it passes.  mx_submit/mx_wait may be called
 * from any thread (one internal scheduler thread micro-batches all requests);
 * blocking calls are made with the GIL released when bound via ctypes.CDLL.
 */
#ifndef MX_ENGINE_H
#define MX_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MX_OK 0
#define MX_ERR_ARG (-1)      /* bad argument / unsupported shape */
#define MX_ERR_HIP (-2)      /* HIP runtime error */
#define MX_ERR_MODEL (-3)    /* model file missing / malformed / unsupported tensor type */
#define MX_ERR_CTX (-4)      /* prompt does not fit n_ctx (Llama raises ValueError) */
#define MX_ERR_NOTFOUND (-5) /* unknown request id */
#define MX_ERR_STATE (-6)    /* engine shutting down / wrong pipeline stage for this call */
#define MX_DEBUG_STOPPED 1   /* a 17..64-row forward ended at the mx_debug stop (diagnosis only) */

#define MX_FINISH_LENGTH 0 /* max_tokens or n_ctx reached  ("length") */
#define MX_FINISH_STOP 1   /* end-of-generation token       ("stop")   */
#define MX_FINISH_ERROR 2

typedef struct mx_engine mx_engine;
typedef struct mx_batch mx_batch;

typedef struct {
  int32_t n_ctx;       /* positions per sequence; llama-cpp-python default 512 */
  int32_t n_seq_max;   /* concurrent sequences (KV slots) */
  int32_t layer_begin; /* pipeline stage: first layer held here (0) */
  int32_t layer_end;   /* one past the last layer held here (-1 = all) */
  int32_t device;      /* HIP device ordinal, -1 = current device */
  int32_t use_graphs;  /* capture decode steps as hipGraphs (1) */
  uint64_t seed;       /* weights seed for "synthetic:<shape>" model paths */
  int32_t handoff_bf16;/* pipeline stage hand-off: x_in / x_out of mx_batch_step, mx_stage_rows and
                          mx_stage_rows_pick are bf16 [rows][n_embd] (1) instead of f32 (0) */
} mx_opts;

typedef struct {
  int32_t n_embd, n_layer, n_head, n_head_kv, head_dim, n_ff, n_vocab, n_ctx_train;
  float eps, rope_base;
  int32_t bos_id, eos_id;
  int32_t n_ctx, n_seq_max;
  int32_t layer_begin, layer_end, has_embed, has_head;
  uint64_t weight_bytes; /* device bytes of the weights this stage streams per decode step */
  int32_t weight_type;       /* ggml type of the layer matrices: 30 BF16, 8 Q8_0, 2 Q4_0, 12 Q4_K (Q4_K_M), 13 Q5_K (Q5_K_M) */
} mx_model_info;

typedef struct {
  float temperature;    /* <= 0 -> greedy argmax on device (ties -> lowest id) */
  int32_t top_k;        /* llama-cpp-python defaults: 40 */
  float top_p;          /* 0.95 */
  float min_p;          /* 0.05 */
  float repeat_penalty; /* 1.0 = off */
  int32_t repeat_last_n;/* 64 */
  uint64_t seed;
  int32_t ignore_eos;
  float frequency_penalty; /* 0.0 = off: logit -= count * frequency_penalty (llama.cpp penalties sampler) */
  float presence_penalty;  /* 0.0 = off: logit -= (count > 0) * presence_penalty */
} mx_sampling;

/* One row's sampler for the device sampling chain (pipeline lanes, mx_batch_reset / mx_stage_rows_pick):
 * the settings, the request's sampler stream (seed; the n-th sampled token of a request uses draw n),
 * how many tokens it sampled so far, and its penalty window -- the last n_win (<= 64) tokens of
 * prompt + output.  temperature <= 0 without penalties = greedy argmax.  Device-sampleable settings:
 * top_k in 1..64 and, with penalties, repeat_last_n in 0..64 (otherwise MX_ERR_ARG). */
typedef struct {
  mx_sampling s;
  uint64_t seed;
  int32_t n_drawn;
  int32_t n_win;
  int32_t win[64];
} mx_row_sampler;

void mx_opts_default(mx_opts* o);
void mx_sampling_default(mx_sampling* s);
const char* mx_last_error(void);

/* model_path: a GGUF file (LLaMA; all-BF16, all-Q8_0, all-Q4_0 and Q4_K_M / Q5_K_M files natively -- the
 * quantised ones on the int8 MFMA with ggml's arithmetic; any other mix of F32 / F16 / BF16 / Q4_0 / Q8_0
 * / K-quant matrices dequantised to bf16 at load) or "synthetic:<shape>[:seed=N][:q8_0|:q4_0|:q4_k_m|:q5_k_m]" */
int mx_engine_create(const char* model_path, const mx_opts* opts, mx_engine** out);
void mx_engine_destroy(mx_engine* e);
/* Parse a GGUF container without touching a GPU (header, metadata, tensor table, bounds of every
 * tensor against the file): 0, or MX_ERR_MODEL with the reason in mx_last_error(). */
int mx_gguf_check(const char* path);
int mx_engine_info(const mx_engine* e, mx_model_info* out);

/* Parity hook: evaluate n tokens of sequence `slot` at positions pos0..pos0+n-1
 * (prefill or decode, chunked internally by 64 rows) and copy the f32 logits of
 * every row to logits_out[n][n_vocab]; NULL skips lm_head entirely (prefill). */
int mx_forward_logits(mx_engine* e, int slot, const int32_t* ids, int n, int pos0, float* logits_out);

/* General rows forward: row i is token ids[i] of sequence slots[i] at pos[i]; logits_out as above. */
int mx_forward_rows(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                    float* logits_out);

/* Parity hook for the sampler: rows forward as mx_forward_rows (n <= 64), then the device top-k
 * kernel (the sampler chain's candidate selection): vals/idx [n][k], value descending, ties -> lower
 * id; k <= 64. */
int mx_forward_topk(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids, int k,
                    float* vals, int32_t* idx);

/* Request API (what Llama.__call__ uses).  Tokens are generated by the
 * scheduler thread, micro-batched with every other active request. */
int mx_submit(mx_engine* e, const int32_t* ids, int n, const mx_sampling* s, int max_tokens, uint64_t* req);
/* n_req requests submitted atomically (all validated first, then queued under one lock): the
 * scheduler admits them in one round -- one batched prefill, one decode batch.  s: n_req sampling
 * settings (NULL: defaults); reqs receives the ids. */
int mx_submit_batch(mx_engine* e, int n_req, const int32_t* const* ids, const int32_t* lens, const mx_sampling* s,
                    const int32_t* max_tokens, uint64_t* reqs);
/* Blocks until the request finishes; copies up to cap generated ids and releases the request.
 * If more than cap ids were generated, nothing is released: *n_out is set and MX_ERR_ARG returned,
 * so the caller can retry with a larger buffer. */
int mx_wait(mx_engine* e, uint64_t req, int32_t* out_ids, int cap, int* n_out, int* finish);
/* Incremental read (streaming / stop strings): blocks until the request holds more than n_have
 * generated ids or has finished; copies the first min(cap, n) ids, *n_out = n, *done = finished.
 * The request stays registered (mx_wait releases it). */
int mx_poll(mx_engine* e, uint64_t req, int n_have, int32_t* out_ids, int cap, int* n_out, int* done);
/* Ask the scheduler to end a request after its current step (finish reason STOP), e.g. when the
 * caller found a stop string.  The request still has to be released with mx_wait. */
int mx_cancel(mx_engine* e, uint64_t req);

/* Device-resident decode batch (benchmark, pipeline stages).  Rows are M
 * sequences in KV slots `slots`, next token ids[i] at position pos[i].
 * mx_batch_step runs one decode step on `stream` (NULL = engine stream):
 *   x_in  == NULL -> embed ids (stage 0), else f32 [M][n_embd] device input
 *   x_out == NULL -> final norm + lm_head + greedy argmax (last stage), tokens
 *                    written back to the batch's ids and history;
 *                    else f32 [M][n_embd] device output for the next stage.
 * Each stage advances its own positions. */
int mx_batch_create(mx_engine* e, int M, const int32_t* slots, const int32_t* pos, const int32_t* ids, int max_steps,
                    mx_batch** out);
int mx_batch_step(mx_engine* e, mx_batch* b, const void* x_in, void* x_out, void* stream);
/* Device pointer of the batch's next-token ids (int32[M]) -- the pipeline's
 * last stage sends these to stage 0, which receives into the same buffer. */
int32_t* mx_batch_ids_device(mx_batch* b);
/* Make the batch read/write its next-token ids in a caller-owned device buffer
 * (int32[M], e.g. a torch tensor that RCCL receives into); current ids are copied over. */
int mx_batch_bind_ids(mx_engine* e, mx_batch* b, int32_t* ids_device);
int mx_batch_tokens(mx_engine* e, mx_batch* b, int32_t* out, int cap, int* n_steps);
/* Re-arm a batch for its next run without re-capturing its graphs (pipeline lanes): positions of all
 * M rows, next ids (NULL: keep the device ids), per-row samplers (NULL: greedy argmax over the last
 * stage's logits), token history restarted; the copies are ordered on `stream` (NULL: engine stream). */
int mx_batch_reset(mx_engine* e, mx_batch* b, const int32_t* pos, const int32_t* ids, const mx_row_sampler* rows,
                   void* stream);
void mx_batch_destroy(mx_engine* e, mx_batch* b);

/* Stage forward of arbitrary rows (pipelined prefill): like mx_forward_rows but
 * with device x_in / x_out as in mx_batch_step; logits_out (host) only on the last stage. */
int mx_stage_rows(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                  const void* x_in, void* x_out, float* logits_out, void* stream);
/* Pipelined prefill of n rows (any count: GEMM chunks as mx_forward_rows; x_in / x_out device
 * [n][n_embd] in the hand-off dtype).  On the last stage, rows rowmap[0..n_out) (increasing) each pick
 * a token -- the device sampling chain with samp[i], or greedy argmax when samp is NULL -- copied to
 * tok_out (host int32[n_out]); the first token of each prompt in the pipeline server. */
int mx_stage_rows_pick(mx_engine* e, int n, const int32_t* slots, const int32_t* pos, const int32_t* ids,
                       const void* x_in, void* x_out, int n_out, const int32_t* rowmap, const mx_row_sampler* samp,
                       int32_t* tok_out, void* stream);

/* Time `iters` passes of one layer-kernel kind over this stage's layers with
 * HIP events on the engine stream (benchmark roofline); kind: 0 qkv, 1 attn_output,
 * 2 ffn_gate_up, 3 ffn_down, 4 lm_head, 5 qkv with fused RMSNorm, 6 ffn_gate_up with fused
 * RMSNorm (M <= 8), 7 attention (positions = env MX_PROF_POS).  Returns mean microseconds per launch. */
/* Diagnosis: op 0 sets the number of launches after which an eager 17..64-row forward stops (-1:
 * never; the forward then returns MX_DEBUG_STOPPED, never 0), op 1 synchronises the stream after every
 * such launch (arg != 0); neither acts on a forward being captured into a graph (graph replays run
 * whole).  Op 2 copies internal buffer `arg`
 * (0 x, 1 q, 2 xn, 3 attn_out, 4 act, 5 split-K slabs, 6 K cache, 7 V cache, 8 ssq partials, 9 row
 * positions, 10 row slots, 11 RoPE table) to
 * `host`, at most `bytes`.  MX_POISON=1 at creation fills every allocation with 0xFF bytes. */
int mx_debug(mx_engine* e, int op, long long arg, void* host, size_t bytes);
int mx_profile_kernel(mx_engine* e, int kind, int M, int iters, double* us_per_launch, double* bytes_per_launch);

int mx_sync(mx_engine* e);

/* HBM streaming probes on `device` (no engine): the best of a sweep of 16-byte-per-lane streaming
 * kernels (loads in flight per lane x grid x non-temporal) over `bytes`-sized buffers, `iters`
 * passes each timed with HIP events.  copy: *gbs = (read + write) bytes / s; read: bytes read / s.
 * desc (optional) receives the winning variant.  Benchmark support (SURVEY.md §8d "also report a
 * measured copy-kernel peak"), not a reference API. */
int mx_probe_copy(int device, size_t bytes, int iters, double* gbs, char* desc, int desc_len);
int mx_probe_read(int device, size_t bytes, int iters, double* gbs, char* desc, int desc_len);

/* Request-path counters (mx_submit/mx_wait).  reused_prompt_tokens: prompt positions whose K/V were
 * kept from the slot's previous request (longest common prefix, as llama-cpp-python's generate). */
typedef struct {
  uint64_t prompt_tokens, reused_prompt_tokens, generated_tokens;
} mx_stats;
int mx_engine_stats(mx_engine* e, mx_stats* out);

/* Number of visible HIP devices (serving: one engine replica per GPU). */
int mx_device_count(int32_t* n);

#ifdef __cplusplus
}
#endif
#endif /* MX_ENGINE_H */
