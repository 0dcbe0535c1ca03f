/*
 * llama_oracle.c -- CPU restatement of the reference's hot path.  TEST
 * INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker / CPU baseline.  The product
 * (llama-p2p_amd/) never links, loads or calls this file.
 *
 * What it restates.  The reference's hot path is one call,
 *   result = self.model(prompt, max_tokens=100)   /root/reference/llama_p2p_network.py:125
 * on   self.model = Llama(model_path=model_path)  /root/reference/llama_p2p_network.py:19
 * i.e. llama-cpp-python (~0.3.1, Oct 2024; module llama_cpp) -> llama.cpp
 * llm_build_llama -> ggml CPU ops.  That dependency is NOT vendored in
 * /root/reference and is absent from this machine, so this is a
 * restatement of its published algorithm:
 *   - GET_ROWS token embedding (bf16 -> f32)                     SURVEY §8a a5
 *   - RMS_NORM: sum of squares in double, scale = 1/sqrtf(mean+eps), then
 *     MUL by the f32 norm weight                                 a6
 *   - MUL_MAT with bf16 weights: activations rounded to bf16 (vec_dot_type of
 *     GGML_TYPE_BF16), products accumulated in f32                a7, a11, a12, a13
 *   - ROPE_EXT mode NORM: adjacent pairs (2i, 2i+1) rotated by theta_i, with
 *     theta built by the f32 cumulative product theta *= powf(base, -2/d)  a8
 *   - K and V stored as f16 (ggml_cpy f32->f16, round-nearest-even)          a9
 *   - KQ = f16(q) . K (f32 accumulate); SOFT_MAX_EXT with scale 1/sqrt(d),
 *     causal mask, max-subtracted expf, sum in double, probs *= (float)(1/sum);
 *     KQV = f16(probs) . V (f32 accumulate); GQA head h -> kv head h/(nh/nkv)  a10
 *   - SwiGLU: silu(g) = g/(1+expf(-g)) in f32, times up, rounded to bf16 for
 *     ffn_down                                                   a12
 *   - logits f32 for the requested rows; greedy = argmax, ties -> lowest id  a13, a14
 *   - Q8_0 weights (a GGUF quantised with llama.cpp's Q8_0): MUL_MAT
 *     quantises the f32 activation rows to Q8_0 (vec_dot_type of GGML_TYPE_Q8_0):
 *     per block of 32, d = amax/127, id = d ? 1/d : 0, q = round-half-even(x*id) (the
 *     rounding of ggml's AVX2 / NEON quantize_row_q8_0; the scalar _ref rounds ties away
 *     from zero -- a measure-zero difference), d kept as f16; then
 *     ggml_vec_dot_q8_0_q8_0: sum over blocks of (f32(d_w)*f32(d_x)) * sum_i(qw*qx).
 *     GET_ROWS of a Q8_0 token_embd dequantises: x = q * f32(d).  Weight blocks come
 *     from the caller (the bytes of the GGUF) or from orc_quantize_q8 (ggml
 *     quantize_row_q8_0_ref: ties away from zero), never from the engine.
 *   - K-quant weights (Q4_K 12, Q5_K 13, Q6_K 14: llama.cpp's Q4_K_M / Q5_K_M files, SURVEY §8a
 *     a16): MUL_MAT quantises the activation rows to Q8_K (vec_dot_type of the K-quants,
 *     ggml quantize_row_q8_K_ref: per 256, iscale = -127/max with max the signed value of
 *     largest magnitude, q = nearest_int(iscale*x), d = 1/iscale, bsums per 16), then
 *     ggml_vec_dot_q{4,5,6}_K_q8_K in their generic (scalar) form: exact int32 super-block
 *     sums, f32 scales.  GET_ROWS of a K-quant token_embd is dequantize_row_q{4,5,6}_K.
 *     Source: ggml-quants.c / ggml-common.h of llama.cpp (the version llama-cpp-python 0.3.1
 *     vendors, Oct 2024) -- restated from the published algorithm, not copied.
 * ORC_EXACT mode drops every bf16/f16 activation rounding (fp32 math over the
 * same bf16 weights): that is what tests cross-check against
 * transformers.LlamaForCausalLM (an independent implementation) to pin the
 * layout conventions (tests/golden/make_golden.py).
 *
 * Weights: bf16 for every matrix, f32 for norms, GGUF data order W[out][in].
 * Synthetic weights follow llama-p2p_amd/synth.py bit for bit (orc_synth_value).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_EXACT 1

typedef struct {
    int n_embd, n_layer, n_head, n_head_kv, n_ff, n_vocab;
    float eps, rope_base;
} orc_hparams;

typedef struct {
    uint16_t *wq, *wk, *wv, *wo, *wg, *wu, *wd; /* bf16 */
    float *attn_norm, *ffn_norm;
    uint8_t *q8[9]; /* Q8_0 blocks by L_* kind (NULL: the bf16 matrix is used) */
    uint8_t *kq[9]; /* K-quant blocks by L_* kind (NULL: not a K-quant matrix) */
    uint8_t *q4[9]; /* Q4_0 blocks by L_* kind (NULL: not a Q4_0 matrix) */
    int kq_type[9];
} orc_layer;

typedef struct {
    orc_hparams hp;
    int flags;
    int head_dim, n_embd_kv;
    uint16_t *tok_embd, *output; /* bf16 [V][h] */
    uint8_t *tok_embd_q8, *output_q8; /* Q8_0 blocks or NULL */
    uint8_t *tok_embd_kq, *output_kq; /* K-quant blocks or NULL */
    uint8_t *output_q4;               /* Q4_0 blocks or NULL */
    int tok_embd_kq_type, output_kq_type;
    float *out_norm;
    orc_layer *layers;
    float *rope_ff;         /* rope_freqs.weight [head_dim/2] (Llama-3.1 frequency factors) or NULL */
    float rope_freq_scale;  /* 1 / llama.rope.scaling.factor for "linear" scaling, else 1 */
} orc_model;

typedef struct {
    orc_model *m;
    int n_ctx;
    /* per layer: K [n_ctx][n_embd_kv], V [n_ctx][n_embd_kv]; f16 bits or f32 */
    void **k, **v;
    float *rope_cs; /* [n_ctx][head_dim/2][2] */
} orc_ctx;

/* ------------------------------------------------------------------ numerics */
static inline float bf16_to_f32(uint16_t h) {
    union { uint32_t u; float f; } v; v.u = (uint32_t)h << 16; return v.f;
}
static inline uint16_t f32_to_bf16(float f) {
    union { uint32_t u; float f; } v; v.f = f;
    if ((v.u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((v.u >> 16) | 64); /* NaN */
    return (uint16_t)((v.u + (0x7fffu + ((v.u >> 16) & 1u))) >> 16);
}
static inline float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }

/* IEEE binary16, round-nearest-even (matches F16C _cvtss_sh(x, 0)). */
static uint16_t f32_to_f16(float f) {
    union { uint32_t u; float f; } v; v.f = f;
    uint32_t x = v.u, sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* overflow -> inf */
    if (ax < 0x38800000u) { /* subnormal or zero in half */
        if (ax < 0x33000000u) return (uint16_t)sign; /* < 2^-25 rounds to 0 */
        uint32_t mant = (ax & 0x7fffffu) | 0x800000u;
        int e = (int)(ax >> 23); /* 102..112 */
        int shift = 126 - e; /* 14..24 */
        uint32_t hm = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t h = ((ax >> 13) - (112u << 10));
    uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}
static float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    union { uint32_t u; float f; } v;
    if (e == 0) {
        if (m == 0) { v.u = sign; return v.f; }
        float r = ldexpf((float)m, -24); return sign ? -r : r;
    }
    if (e == 31) { v.u = sign | 0x7f800000u | (m << 13); return v.f; }
    v.u = sign | ((e + 112u) << 23) | (m << 13);
    return v.f;
}
static inline float round_f16(float f) { return f16_to_f32(f32_to_f16(f)); }

float orc_round_f16(float f) { return round_f16(f); }
float orc_round_bf16(float f) { return round_bf16(f); }

/* --------------------------------------------------- synthetic weights (spec) */
float orc_synth_value(uint64_t seed, uint64_t tid, uint64_t idx, float scale) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + tid * 0xD1B54A32D192ED03ull + idx;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint32_t s = (uint32_t)(z & 0xffff) + (uint32_t)((z >> 16) & 0xffff) +
                 (uint32_t)((z >> 32) & 0xffff) + (uint32_t)(z >> 48);
    return (float)((int32_t)s - 131070) * scale;
}
static float std_scale(double std) { return (float)(std / sqrt(4294967295.0 / 3.0)); }

static void synth_bf16(uint16_t *dst, uint64_t seed, uint64_t tid, size_t n) {
    float sc = std_scale(0.02);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) dst[i] = f32_to_bf16(orc_synth_value(seed, tid, i, sc));
}
static void synth_norm(float *dst, uint64_t seed, uint64_t tid, size_t n) {
    float sc = std_scale(0.1);
    for (size_t i = 0; i < n; i++) dst[i] = 1.0f + orc_synth_value(seed, tid, i, sc);
}

/* ------------------------------------------------------------------ model */
orc_model *orc_create(const orc_hparams *hp, int flags) {
    orc_model *m = (orc_model *)calloc(1, sizeof(orc_model));
    m->hp = *hp;
    m->flags = flags;
    m->rope_freq_scale = 1.0f;
    m->head_dim = hp->n_embd / hp->n_head;
    m->n_embd_kv = m->head_dim * hp->n_head_kv;
    size_t h = hp->n_embd, kv = m->n_embd_kv, ff = hp->n_ff, V = hp->n_vocab;
    m->tok_embd = (uint16_t *)malloc(V * h * 2);
    m->output = (uint16_t *)malloc(V * h * 2);
    m->out_norm = (float *)malloc(h * 4);
    m->layers = (orc_layer *)calloc(hp->n_layer, sizeof(orc_layer));
    for (int l = 0; l < hp->n_layer; l++) {
        orc_layer *L = &m->layers[l];
        L->wq = (uint16_t *)malloc(h * h * 2);
        L->wk = (uint16_t *)malloc(kv * h * 2);
        L->wv = (uint16_t *)malloc(kv * h * 2);
        L->wo = (uint16_t *)malloc(h * h * 2);
        L->wg = (uint16_t *)malloc(ff * h * 2);
        L->wu = (uint16_t *)malloc(ff * h * 2);
        L->wd = (uint16_t *)malloc(h * ff * 2);
        L->attn_norm = (float *)malloc(h * 4);
        L->ffn_norm = (float *)malloc(h * 4);
    }
    return m;
}

void orc_free(orc_model *m) {
    if (!m) return;
    for (int l = 0; l < m->hp.n_layer; l++) {
        orc_layer *L = &m->layers[l];
        free(L->wq); free(L->wk); free(L->wv); free(L->wo); free(L->wg); free(L->wu); free(L->wd);
        free(L->attn_norm); free(L->ffn_norm);
        for (int k = 0; k < 9; k++) { free(L->q8[k]); free(L->kq[k]); free(L->q4[k]); }
    }
    free(m->tok_embd_q8); free(m->output_q8); free(m->tok_embd_kq); free(m->output_kq); free(m->output_q4);
    free(m->rope_ff);
    free(m->layers); free(m->tok_embd); free(m->output); free(m->out_norm); free(m);
}

/* tensor kinds, matching llama-p2p_amd/synth.py */
enum { K_TOK_EMBD = 1, K_OUT_NORM = 2, K_OUTPUT = 3 };
enum { L_ATTN_NORM, L_Q, L_K, L_V, L_O, L_FFN_NORM, L_GATE, L_UP, L_DOWN };
static uint64_t layer_tid(int l, int k) { return 16u + 16u * (uint64_t)l + (uint64_t)k; }

/* RoPE frequency factors (rope_freqs.weight, head_dim/2 floats; NULL clears) and linear
 * scaling (freq_scale = 1 / llama.rope.scaling.factor); used by contexts created afterwards. */
void orc_set_rope(orc_model *m, const float *freq_factors, float freq_scale) {
    free(m->rope_ff);
    m->rope_ff = NULL;
    if (freq_factors) {
        m->rope_ff = (float *)malloc(sizeof(float) * (size_t)(m->head_dim / 2));
        memcpy(m->rope_ff, freq_factors, sizeof(float) * (size_t)(m->head_dim / 2));
    }
    m->rope_freq_scale = freq_scale;
}

/* Synthesise layers [lb, le) and, with globals, token_embd / output / output_norm: a per-layer test of
 * a model too large to synthesise whole on the host (Llama-3-70B) fills only the layers it runs; the
 * other layers' buffers stay untouched (never committed). */
void orc_fill_synthetic_layers(orc_model *m, uint64_t seed, int lb, int le, int globals) {
    size_t h = m->hp.n_embd, kv = m->n_embd_kv, ff = m->hp.n_ff, V = m->hp.n_vocab;
    if (globals) {
        synth_bf16(m->tok_embd, seed, K_TOK_EMBD, V * h);
        synth_bf16(m->output, seed, K_OUTPUT, V * h);
        synth_norm(m->out_norm, seed, K_OUT_NORM, h);
    }
    if (lb < 0) lb = 0;
    if (le > m->hp.n_layer) le = m->hp.n_layer;
    for (int l = lb; l < le; l++) {
        orc_layer *L = &m->layers[l];
        synth_norm(L->attn_norm, seed, layer_tid(l, L_ATTN_NORM), h);
        synth_bf16(L->wq, seed, layer_tid(l, L_Q), h * h);
        synth_bf16(L->wk, seed, layer_tid(l, L_K), kv * h);
        synth_bf16(L->wv, seed, layer_tid(l, L_V), kv * h);
        synth_bf16(L->wo, seed, layer_tid(l, L_O), h * h);
        synth_norm(L->ffn_norm, seed, layer_tid(l, L_FFN_NORM), h);
        synth_bf16(L->wg, seed, layer_tid(l, L_GATE), ff * h);
        synth_bf16(L->wu, seed, layer_tid(l, L_UP), ff * h);
        synth_bf16(L->wd, seed, layer_tid(l, L_DOWN), h * ff);
    }
}

void orc_fill_synthetic(orc_model *m, uint64_t seed) { orc_fill_synthetic_layers(m, seed, 0, m->hp.n_layer, 1); }

/* Set one tensor from caller memory (bf16 bits for matrices, f32 for norms).
 * layer = -1 for global tensors; kind uses the synth.py numbering. */
int orc_set_tensor(orc_model *m, int layer, int kind, const void *src) {
    size_t h = m->hp.n_embd, kv = m->n_embd_kv, ff = m->hp.n_ff, V = m->hp.n_vocab;
    if (layer < 0) {
        switch (kind) {
        case K_TOK_EMBD: /* the table becomes bf16: drop any block representation set before */
            memcpy(m->tok_embd, src, V * h * 2);
            free(m->tok_embd_q8); m->tok_embd_q8 = NULL;
            free(m->tok_embd_kq); m->tok_embd_kq = NULL;
            return 0;
        case K_OUTPUT: memcpy(m->output, src, V * h * 2); return 0;
        case K_OUT_NORM: memcpy(m->out_norm, src, h * 4); return 0;
        }
        return -1;
    }
    if (layer >= m->hp.n_layer) return -1;
    orc_layer *L = &m->layers[layer];
    switch (kind) {
    case L_ATTN_NORM: memcpy(L->attn_norm, src, h * 4); return 0;
    case L_Q: memcpy(L->wq, src, h * h * 2); return 0;
    case L_K: memcpy(L->wk, src, kv * h * 2); return 0;
    case L_V: memcpy(L->wv, src, kv * h * 2); return 0;
    case L_O: memcpy(L->wo, src, h * h * 2); return 0;
    case L_FFN_NORM: memcpy(L->ffn_norm, src, h * 4); return 0;
    case L_GATE: memcpy(L->wg, src, ff * h * 2); return 0;
    case L_UP: memcpy(L->wu, src, ff * h * 2); return 0;
    case L_DOWN: memcpy(L->wd, src, h * ff * 2); return 0;
    }
    return -1;
}

/* ------------------------------------------------------------------ Q8_0 */
#define QK8_0 32
#define Q8_0_BLOCK 34

/* ggml quantize_row_q8_0_ref: what the quantize tool writes for weights (ties away from zero) */
static void quantize_row_q8_0_ref(const float *x, uint8_t *y, int n) {
    for (int b = 0; b < n / QK8_0; b++) {
        const float *xb = x + (size_t)b * QK8_0;
        float amax = 0.f;
        for (int j = 0; j < QK8_0; j++) amax = fmaxf(amax, fabsf(xb[j]));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.0f;
        uint8_t *yb = y + (size_t)b * Q8_0_BLOCK;
        uint16_t dh = f32_to_f16(d);
        memcpy(yb, &dh, 2);
        for (int j = 0; j < QK8_0; j++) yb[2 + j] = (uint8_t)(int8_t)roundf(xb[j] * id);
    }
}

static size_t q8_bytes(size_t rows, size_t cols) { return rows * (cols / QK8_0) * Q8_0_BLOCK; }

static uint8_t **q8_slot(orc_model *m, int layer, int kind, size_t *rows, size_t *cols, uint16_t **bf) {
    size_t h = m->hp.n_embd, kv = m->n_embd_kv, ff = m->hp.n_ff, V = m->hp.n_vocab;
    if (layer < 0) {
        if (kind == K_TOK_EMBD) { *rows = V; *cols = h; *bf = m->tok_embd; return &m->tok_embd_q8; }
        if (kind == K_OUTPUT) { *rows = V; *cols = h; *bf = m->output; return &m->output_q8; }
        return NULL;
    }
    if (layer >= m->hp.n_layer) return NULL;
    orc_layer *L = &m->layers[layer];
    switch (kind) {
    case L_Q: *rows = h; *cols = h; *bf = L->wq; break;
    case L_K: *rows = kv; *cols = h; *bf = L->wk; break;
    case L_V: *rows = kv; *cols = h; *bf = L->wv; break;
    case L_O: *rows = h; *cols = h; *bf = L->wo; break;
    case L_GATE: *rows = ff; *cols = h; *bf = L->wg; break;
    case L_UP: *rows = ff; *cols = h; *bf = L->wu; break;
    case L_DOWN: *rows = h; *cols = ff; *bf = L->wd; break;
    default: return NULL;
    }
    return &L->q8[kind];
}

/* Make one matrix Q8_0 from caller bytes (GGUF block layout, rows x cols/32 blocks of 34 B). */
int orc_set_tensor_q8(orc_model *m, int layer, int kind, const void *blocks) {
    size_t rows, cols;
    uint16_t *bf;
    uint8_t **slot = q8_slot(m, layer, kind, &rows, &cols, &bf);
    if (!slot || cols % QK8_0) return -1;
    if (!*slot) *slot = (uint8_t *)malloc(q8_bytes(rows, cols));
    memcpy(*slot, blocks, q8_bytes(rows, cols));
    if (layer < 0 && kind == K_TOK_EMBD) { free(m->tok_embd_kq); m->tok_embd_kq = NULL; } /* Q8_0 table wins */
    return 0;
}

/* Quantise every matrix (token_embd, output, and the seven per layer) from its bf16 values. */
int orc_quantize_q8(orc_model *m) {
    static const int kinds[] = {L_Q, L_K, L_V, L_O, L_GATE, L_UP, L_DOWN};
    for (int l = -1; l < m->hp.n_layer; l++) {
        int nk = l < 0 ? 2 : 7;
        for (int i = 0; i < nk; i++) {
            int kind = l < 0 ? (i ? K_OUTPUT : K_TOK_EMBD) : kinds[i];
            size_t rows, cols;
            uint16_t *bf;
            uint8_t **slot = q8_slot(m, l, kind, &rows, &cols, &bf);
            if (!slot || cols % QK8_0) return -1;
            if (!*slot) *slot = (uint8_t *)malloc(q8_bytes(rows, cols));
            uint8_t *dst = *slot;
#pragma omp parallel for schedule(static)
            for (size_t r = 0; r < rows; r++)
                for (size_t b = 0; b < cols / QK8_0; b++) {
                    float blk[QK8_0];
                    for (int j = 0; j < QK8_0; j++) blk[j] = bf16_to_f32(bf[r * cols + b * QK8_0 + j]);
                    quantize_row_q8_0_ref(blk, dst + (r * (cols / QK8_0) + b) * Q8_0_BLOCK, QK8_0);
                }
        }
    }
    return 0;
}

/* activation row -> Q8_0 (vec_dot_type of Q8_0): q int8, d = f32 of the f16 scale */
static void quantize_act_q8_0(const float *x, int n, int8_t *q, float *d) {
    for (int b = 0; b < n / QK8_0; b++) {
        const float *xb = x + (size_t)b * QK8_0;
        float amax = 0.f;
        for (int j = 0; j < QK8_0; j++) amax = fmaxf(amax, fabsf(xb[j]));
        const float dd = amax / 127.0f;
        const float id = dd != 0.f ? 1.0f / dd : 0.0f;
        d[b] = round_f16(dd);
        for (int j = 0; j < QK8_0; j++) q[(size_t)b * QK8_0 + j] = (int8_t)nearbyintf(xb[j] * id);
    }
}

/* ggml_vec_dot_q8_0_q8_0 */
static float dot_q8_0(const uint8_t *w, const int8_t *q, const float *d, int n) {
    float s = 0.f;
    for (int b = 0; b < n / QK8_0; b++) {
        const uint8_t *wb = w + (size_t)b * Q8_0_BLOCK;
        uint16_t dh;
        memcpy(&dh, wb, 2);
        int sumi = 0;
        for (int j = 0; j < QK8_0; j++) sumi += (int)(int8_t)wb[2 + j] * (int)q[(size_t)b * QK8_0 + j];
        s += (f16_to_f32(dh) * d[b]) * (float)sumi;
    }
    return s;
}

/* Sensitivity probe for tests: a relative perturbation of up to q8_jitter (deterministic hash
 * noise) on every activation before it is quantised (Q8_0 and Q8_K) or rounded to bf16 for a bf16
 * weight product.  0 = off (the restatement proper).  The
 * Q8_0 forward is discontinuous in its inputs (x*id crossing a rounding boundary moves q by one
 * step), so the tests bound the engine's deviation by the oracle's own under 1e-6 noise. */
static float q8_jitter = 0.0f;
void orc_set_q8_jitter(float eps) { q8_jitter = eps; }
static void jitter_row(const float *xr, float *xj, int n_in, int t, int n_out) {
    for (int i = 0; i < n_in; i++) {
        unsigned hsh = (unsigned)i * 2654435761u + (unsigned)t * 97u + (unsigned)n_out;
        xj[i] = q8_jitter != 0.0f ? xr[i] * (1.0f + q8_jitter * (float)((int)(hsh % 2001u) - 1000) / 1000.0f) : xr[i];
    }
}

static void matmul_q8(float *y, const uint8_t *W, const float *x, int T, int n_in, int n_out) {
    int8_t *xq = (int8_t *)malloc((size_t)T * n_in);
    float *xd = (float *)malloc(sizeof(float) * (size_t)T * (n_in / QK8_0));
    float *xj = q8_jitter != 0.0f ? (float *)malloc(sizeof(float) * n_in) : NULL;
    for (int t = 0; t < T; t++) {
        const float *xr = x + (size_t)t * n_in;
        if (xj) {
            jitter_row(xr, xj, n_in, t, n_out);
            xr = xj;
        }
        quantize_act_q8_0(xr, n_in, xq + (size_t)t * n_in, xd + (size_t)t * (n_in / QK8_0));
    }
    free(xj);
    const size_t rb = (size_t)(n_in / QK8_0) * Q8_0_BLOCK;
#pragma omp parallel for schedule(static)
    for (int o = 0; o < n_out; o++)
        for (int t = 0; t < T; t++)
            y[(size_t)t * n_out + o] = dot_q8_0(W + (size_t)o * rb, xq + (size_t)t * n_in,
                                                xd + (size_t)t * (n_in / QK8_0), n_in);
    free(xq);
    free(xd);
}


/* ------------------------------------------------------------------ Q4_0 */
/* ggml block_q4_0 {f16 d; uint8 qs[16]}: weight j = (qs[j] & 15) - 8, weight j+16 = (qs[j] >> 4) - 8 */
#define Q4_0_BLOCK 18

/* ggml quantize_row_q4_0_ref: d = (signed value of largest magnitude) / -8, q = min(15, (int8)(x*id + 8.5)) */
static void quantize_row_q4_0_ref(const float *x, uint8_t *y, int k) {
    for (int b = 0; b < k / 32; b++) {
        const float *xb = x + (size_t)b * 32;
        float amax = 0.f, max = 0.f;
        for (int j = 0; j < 32; j++)
            if (amax < fabsf(xb[j])) { amax = fabsf(xb[j]); max = xb[j]; }
        const float d = max / -8;
        const float id = d ? 1.0f / d : 0.0f;
        uint8_t *yb = y + (size_t)b * Q4_0_BLOCK;
        const uint16_t dh = f32_to_f16(d);
        memcpy(yb, &dh, 2);
        for (int j = 0; j < 16; j++) {
            const float x0 = xb[j] * id, x1 = xb[16 + j] * id;
            int xi0 = (int8_t)(x0 + 8.5f), xi1 = (int8_t)(x1 + 8.5f);
            if (xi0 > 15) xi0 = 15;
            if (xi1 > 15) xi1 = 15;
            yb[2 + j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

/* ggml_vec_dot_q4_0_q8_0 (generic): exact int block sums, scaled by d_w * d_x */
static float dot_q4_0(const uint8_t *w, const int8_t *q, const float *d, int n) {
    float s = 0.f;
    for (int b = 0; b < n / 32; b++) {
        const uint8_t *wb = w + (size_t)b * Q4_0_BLOCK;
        uint16_t dh;
        memcpy(&dh, wb, 2);
        int sumi = 0;
        for (int j = 0; j < 16; j++) {
            sumi += ((wb[2 + j] & 15) - 8) * (int)q[(size_t)b * 32 + j];
            sumi += ((wb[2 + j] >> 4) - 8) * (int)q[(size_t)b * 32 + 16 + j];
        }
        s += (f16_to_f32(dh) * d[b]) * (float)sumi;
    }
    return s;
}

static void jitter_row(const float *xr, float *xj, int n_in, int t, int n_out);

static void matmul_q4_0(float *y, const uint8_t *W, const float *x, int T, int n_in, int n_out) {
    int8_t *xq = (int8_t *)malloc((size_t)T * n_in);
    float *xd = (float *)malloc(sizeof(float) * (size_t)T * (n_in / 32));
    float *xj = (float *)malloc(sizeof(float) * n_in);
    for (int t = 0; t < T; t++) {
        jitter_row(x + (size_t)t * n_in, xj, n_in, t, n_out);
        quantize_act_q8_0(xj, n_in, xq + (size_t)t * n_in, xd + (size_t)t * (n_in / 32));
    }
    free(xj);
    const size_t rb = (size_t)(n_in / 32) * Q4_0_BLOCK;
#pragma omp parallel for schedule(static)
    for (int o = 0; o < n_out; o++)
        for (int t = 0; t < T; t++)
            y[(size_t)t * n_out + o] = dot_q4_0(W + (size_t)o * rb, xq + (size_t)t * n_in, xd + (size_t)t * (n_in / 32), n_in);
    free(xq);
    free(xd);
}

static uint8_t **q4_slot(orc_model *m, int layer, int kind, size_t *rows, size_t *cols, uint16_t **bf) {
    if (layer < 0) {
        if (kind != K_OUTPUT) return NULL;
        *rows = m->hp.n_vocab; *cols = m->hp.n_embd; *bf = m->output;
        return &m->output_q4;
    }
    uint8_t **q8 = q8_slot(m, layer, kind, rows, cols, bf);
    return q8 ? &m->layers[layer].q4[kind] : NULL;
}

/* Make one matrix Q4_0 from GGUF block bytes (rows x cols/32 blocks of 18 bytes). */
int orc_set_tensor_q4_0(orc_model *m, int layer, int kind, const void *blocks) {
    size_t rows, cols;
    uint16_t *bf;
    uint8_t **slot = q4_slot(m, layer, kind, &rows, &cols, &bf);
    if (!slot || cols % 32) return -1;
    const size_t nb = rows * (cols / 32) * Q4_0_BLOCK;
    if (!*slot) *slot = (uint8_t *)malloc(nb);
    memcpy(*slot, blocks, nb);
    return 0;
}

/* The synthetic "q4_0" model: every layer matrix -> quantize_row_q4_0_ref of its bf16 values, token_embd
 * and output -> Q8_0 (as the engine's synthetic:<shape>:q4_0). */
int orc_quantize_q4_0(orc_model *m) {
    static const int kinds[] = {L_Q, L_K, L_V, L_O, L_GATE, L_UP, L_DOWN};
    for (int l = -1; l < m->hp.n_layer; l++) {
        int nk = l < 0 ? 2 : 7;
        for (int i = 0; i < nk; i++) {
            int kind = l < 0 ? (i ? K_OUTPUT : K_TOK_EMBD) : kinds[i];
            size_t rows, cols;
            uint16_t *bf;
            uint8_t **slot = l < 0 ? q8_slot(m, l, kind, &rows, &cols, &bf) : q4_slot(m, l, kind, &rows, &cols, &bf);
            if (!slot || cols % 32) return -1;
            const size_t bb = l < 0 ? Q8_0_BLOCK : Q4_0_BLOCK;
            if (!*slot) *slot = (uint8_t *)malloc(rows * (cols / 32) * bb);
            uint8_t *dst = *slot;
#pragma omp parallel for schedule(static)
            for (size_t r = 0; r < rows; r++) {
                float *v = (float *)malloc(sizeof(float) * cols);
                for (size_t c = 0; c < cols; c++) v[c] = bf16_to_f32(bf[r * cols + c]);
                if (l < 0) {
                    quantize_row_q8_0_ref(v, dst + r * (cols / 32) * Q8_0_BLOCK, (int)cols);
                } else {
                    quantize_row_q4_0_ref(v, dst + r * (cols / 32) * Q4_0_BLOCK, (int)cols);
                }
                free(v);
            }
        }
    }
    return 0;
}

/* test hooks: one Q4_0 row of a float row, and its dot product with the Q8_0 image of x */
int orc_q4_0_quantize_row(const float *x, int k, uint8_t *out) {
    if (k % 32) return -1;
    quantize_row_q4_0_ref(x, out, k);
    return 0;
}
float orc_q4_0_vec_dot(const uint8_t *w, const float *x, int n) {
    int8_t *q = (int8_t *)malloc(n);
    float *d = (float *)malloc(sizeof(float) * (n / 32));
    quantize_act_q8_0(x, n, q, d);
    const float r = dot_q4_0(w, q, d, n);
    free(q);
    free(d);
    return r;
}

/* ------------------------------------------------------------------ K-quants */
#define QK_K 256

int orc_kq_block_bytes(int type) { return type == 12 ? 144 : type == 13 ? 176 : type == 14 ? 210 : 0; }

/* ggml get_scale_min_k4: the 6-bit (scale, min) pair j of the 12 packed bytes */
static void scale_min_k4(int j, const uint8_t *q, int *sc, int *mn) {
    if (j < 4) {
        *sc = q[j] & 63;
        *mn = q[j + 4] & 63;
    } else {
        *sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *mn = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
    }
}

/* The 256 integer values of one super-block, in k order (Q4_K 0..15, Q5_K 0..31, Q6_K -32..31),
 * and its 16-element scales (Q6_K) or 32-element (scale, min) pairs (Q4_K / Q5_K).
 * Layouts: ggml-common.h block_q4_K {d, dmin, scales[12], qs[128]}, block_q5_K {d, dmin,
 * scales[12], qh[32], qs[128]}, block_q6_K {ql[128], qh[64], scales[16], d}. */
static void kq_values(int type, const uint8_t *b, int *v) {
    if (type == 12 || type == 13) {
        const uint8_t *qh = b + 16, *qs = b + (type == 13 ? 48 : 16);
        for (int g = 0; g < 4; g++)
            for (int l = 0; l < 32; l++) {
                int lo = qs[32 * g + l] & 15, hi = qs[32 * g + l] >> 4;
                if (type == 13) {
                    lo += (qh[l] >> (2 * g)) & 1 ? 16 : 0;
                    hi += (qh[l] >> (2 * g + 1)) & 1 ? 16 : 0;
                }
                v[64 * g + l] = lo;
                v[64 * g + 32 + l] = hi;
            }
    } else {
        const uint8_t *ql = b, *qh = b + 128;
        for (int h = 0; h < 2; h++)
            for (int l = 0; l < 32; l++) {
                const int L0 = ql[64 * h + l], L1 = ql[64 * h + 32 + l], H = qh[32 * h + l];
                v[128 * h + l] = ((L0 & 15) | (((H >> 0) & 3) << 4)) - 32;
                v[128 * h + 32 + l] = ((L1 & 15) | (((H >> 2) & 3) << 4)) - 32;
                v[128 * h + 64 + l] = ((L0 >> 4) | (((H >> 4) & 3) << 4)) - 32;
                v[128 * h + 96 + l] = ((L1 >> 4) | (((H >> 6) & 3) << 4)) - 32;
            }
    }
}

/* ggml dequantize_row_q4_K / q5_K / q6_K: f32, one rounding per operation (C11, no contraction) */
int orc_kq_dequant(int type, const uint8_t *x, float *y, int64_t k) {
    const int bb = orc_kq_block_bytes(type);
    if (!bb || k % QK_K) return -1;
    int v[QK_K];
    for (int64_t i = 0; i < k / QK_K; i++) {
        const uint8_t *b = x + i * bb;
        float *yb = y + i * QK_K;
        kq_values(type, b, v);
        if (type == 14) {
            uint16_t dh;
            memcpy(&dh, b + 208, 2);
            const float d = f16_to_f32(dh);
            const int8_t *sc = (const int8_t *)(b + 192);
            for (int j = 0; j < QK_K; j++) yb[j] = d * (float)sc[j / 16] * (float)v[j];
        } else {
            uint16_t dh, mh;
            memcpy(&dh, b, 2);
            memcpy(&mh, b + 2, 2);
            const float d = f16_to_f32(dh), dmin = f16_to_f32(mh);
            for (int j = 0; j < 8; j++) {
                int sc, mn;
                scale_min_k4(j, b + 4, &sc, &mn);
                const float d1 = d * (float)sc, m1 = dmin * (float)mn;
                for (int l = 0; l < 32; l++) yb[32 * j + l] = d1 * (float)v[32 * j + l] - m1;
            }
        }
    }
    return 0;
}

/* ggml block_q8_K */
typedef struct {
    float d;
    int8_t qs[QK_K];
    int16_t bsums[QK_K / 16];
} q8k_block;

/* ggml nearest_int: round half to even through the 1.5*2^23 trick */
static inline int nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

/* ggml quantize_row_q8_K_ref (what x86 quantize_row_q8_K runs) */
static void quantize_row_q8_K(const float *x, q8k_block *y, int64_t k) {
    for (int64_t i = 0; i < k / QK_K; i++, x += QK_K) {
        float max = 0, amax = 0;
        for (int j = 0; j < QK_K; j++) {
            const float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; max = x[j]; }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; j++) {
            const int v = nearest_int(iscale * x[j]);
            y[i].qs[j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < QK_K / 16; j++) {
            int sum = 0;
            for (int ii = 0; ii < 16; ii++) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t)sum;
        }
        y[i].d = 1 / iscale;
    }
}

/* ggml_vec_dot_q4_K_q8_K / q5_K / q6_K, generic form: per super-block 8 int32 lane sums of
 * scale * (w . x) (and, for Q4_K / Q5_K, sum(bsums * mins)), scaled in f32. */
static float vec_dot_kq(int type, const uint8_t *vx, const q8k_block *y, int n) {
    const int bb = orc_kq_block_bytes(type);
    float sums[8] = {0};
    float sumf = 0;
    int v[QK_K];
    for (int i = 0; i < n / QK_K; i++) {
        const uint8_t *b = vx + (size_t)i * bb;
        kq_values(type, b, v);
        int32_t aux32[8] = {0};
        const int8_t *q8 = y[i].qs;
        if (type == 14) {
            const int8_t *sc = (const int8_t *)(b + 192);
            for (int j = 0; j < QK_K / 16; j++) {
                const int scale = sc[j];
                for (int half = 0; half < 2; half++)
                    for (int l = 0; l < 8; l++) aux32[l] += scale * (int16_t)(q8[16 * j + 8 * half + l] * v[16 * j + 8 * half + l]);
            }
            uint16_t dh;
            memcpy(&dh, b + 208, 2);
            const float d = f16_to_f32(dh) * y[i].d;
            for (int l = 0; l < 8; l++) sums[l] += d * aux32[l];
        } else {
            int scales[8], mins[8];
            for (int j = 0; j < 8; j++) scale_min_k4(j, b + 4, &scales[j], &mins[j]);
            int sumi = 0;
            for (int j = 0; j < QK_K / 16; j++) sumi += y[i].bsums[j] * mins[j / 2];
            for (int j = 0; j < QK_K / 32; j++)
                for (int quarter = 0; quarter < 4; quarter++)
                    for (int l = 0; l < 8; l++)
                        aux32[l] += scales[j] * (int16_t)(q8[32 * j + 8 * quarter + l] * v[32 * j + 8 * quarter + l]);
            uint16_t dh, mh;
            memcpy(&dh, b, 2);
            memcpy(&mh, b + 2, 2);
            const float d = f16_to_f32(dh) * y[i].d;
            for (int l = 0; l < 8; l++) sums[l] += d * aux32[l];
            const float dmin = f16_to_f32(mh) * y[i].d;
            sumf -= dmin * sumi;
        }
    }
    for (int l = 0; l < 8; l++) sumf += sums[l];
    return sumf;
}

static void jitter_row(const float *xr, float *xj, int n_in, int t, int n_out);

static void matmul_kq(float *y, int type, const uint8_t *W, const float *x, int T, int n_in, int n_out) {
    const int nb = n_in / QK_K;
    q8k_block *xq = (q8k_block *)malloc(sizeof(q8k_block) * (size_t)T * nb);
    float *xj = (float *)malloc(sizeof(float) * n_in);
    for (int t = 0; t < T; t++) {
        jitter_row(x + (size_t)t * n_in, xj, n_in, t, n_out);  /* the Q8_0 path's sensitivity probe */
        quantize_row_q8_K(xj, xq + (size_t)t * nb, n_in);
    }
    free(xj);
    const size_t rb = (size_t)nb * orc_kq_block_bytes(type);
#pragma omp parallel for schedule(static)
    for (int o = 0; o < n_out; o++)
        for (int t = 0; t < T; t++) y[(size_t)t * n_out + o] = vec_dot_kq(type, W + (size_t)o * rb, xq + (size_t)t * nb, n_in);
    free(xq);
}

/* test hooks: the Q8_K image of one row (qs [k], d [k/256], bsums [k/16]) and one dot product */
int orc_kq_quantize_q8k(const float *x, int64_t k, int8_t *qs, float *d, int16_t *bsums) {
    if (k % QK_K) return -1;
    q8k_block *y = (q8k_block *)malloc(sizeof(q8k_block) * (size_t)(k / QK_K));
    quantize_row_q8_K(x, y, k);
    for (int64_t i = 0; i < k / QK_K; i++) {
        memcpy(qs + i * QK_K, y[i].qs, QK_K);
        d[i] = y[i].d;
        memcpy(bsums + i * 16, y[i].bsums, 32);
    }
    free(y);
    return 0;
}
float orc_kq_vec_dot(int type, const uint8_t *w, const float *x, int n) {
    q8k_block *y = (q8k_block *)malloc(sizeof(q8k_block) * (size_t)(n / QK_K));
    quantize_row_q8_K(x, y, n);
    const float r = vec_dot_kq(type, w, y, n);
    free(y);
    return r;
}

/* Synthetic K-quant blocks (llama-p2p_amd/synth.py kq_blocks is the spec; the engine's
 * synth_kq_kernel is bit-identical): every byte from the synthetic hash, then the f16 scale
 * fields set to fixed-exponent bit patterns with a random mantissa byte (no float conversion),
 * and Q6_K's int8 scales folded into [-24, 23]. */
static uint64_t synth_hash(uint64_t seed, uint64_t tid, uint64_t idx) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + tid * 0xD1B54A32D192ED03ull + idx;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
int orc_kq_synth_blocks(int type, int64_t nblocks, uint64_t seed, uint64_t tid, uint8_t *out) {
    const int bb = orc_kq_block_bytes(type);
    if (!bb) return -1;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblocks; b++) {
        uint8_t *p = out + b * bb;
        for (int i = 0; i < bb; i++) {
            const uint64_t gi = (uint64_t)b * bb + i;
            p[i] = (uint8_t)(synth_hash(seed, tid, gi >> 3) >> (8 * (gi & 7)));
        }
        if (type == 14) {
            for (int j = 0; j < 16; j++) p[192 + j] = (uint8_t)(int8_t)((int)(p[192 + j] % 48) - 24);
            const uint16_t d = (uint16_t)(0x0500 + p[208]);
            p[208] = (uint8_t)d; p[209] = (uint8_t)(d >> 8);
        } else {
            const uint16_t d = (uint16_t)(0x0500 + p[0]), mn = (uint16_t)((type == 13 ? 0x1500 : 0x1100) + p[1]);
            p[0] = (uint8_t)d; p[1] = (uint8_t)(d >> 8);
            p[2] = (uint8_t)mn; p[3] = (uint8_t)(mn >> 8);
        }
    }
    return 0;
}

/* Make one matrix a K-quant from caller bytes (GGUF blocks, rows x cols/256 blocks). */
int orc_set_tensor_kq(orc_model *m, int layer, int kind, int type, const void *blocks) {
    size_t h = m->hp.n_embd, kv = m->n_embd_kv, ff = m->hp.n_ff, V = m->hp.n_vocab;
    size_t rows = 0, cols = 0;
    uint8_t **slot = NULL;
    int *tslot = NULL;
    const int bb = orc_kq_block_bytes(type);
    if (!bb) return -1;
    if (layer < 0) {
        if (kind == K_TOK_EMBD) { rows = V; cols = h; slot = &m->tok_embd_kq; tslot = &m->tok_embd_kq_type; }
        else if (kind == K_OUTPUT) { rows = V; cols = h; slot = &m->output_kq; tslot = &m->output_kq_type; }
        else return -1;
    } else {
        if (layer >= m->hp.n_layer) return -1;
        orc_layer *L = &m->layers[layer];
        switch (kind) {
        case L_Q: rows = h; cols = h; break;
        case L_K: case L_V: rows = kv; cols = h; break;
        case L_O: rows = h; cols = h; break;
        case L_GATE: case L_UP: rows = ff; cols = h; break;
        case L_DOWN: rows = h; cols = ff; break;
        default: return -1;
        }
        slot = &L->kq[kind];
        tslot = &L->kq_type[kind];
    }
    if (cols % QK_K) return -1;
    const size_t nbytes = rows * (cols / QK_K) * bb;
    free(*slot);
    *slot = (uint8_t *)malloc(nbytes);
    memcpy(*slot, blocks, nbytes);
    *tslot = type;
    return 0;
}

/* ------------------------------------------------------------------ context */
orc_ctx *orc_ctx_create(orc_model *m, int n_ctx) {
    orc_ctx *c = (orc_ctx *)calloc(1, sizeof(orc_ctx));
    c->m = m;
    c->n_ctx = n_ctx;
    int L = m->hp.n_layer;
    size_t esz = (m->flags & ORC_EXACT) ? 4 : 2;
    c->k = (void **)calloc(L, sizeof(void *));
    c->v = (void **)calloc(L, sizeof(void *));
    for (int l = 0; l < L; l++) {
        c->k[l] = calloc((size_t)n_ctx * m->n_embd_kv, esz);
        c->v[l] = calloc((size_t)n_ctx * m->n_embd_kv, esz);
    }
    /* rope cache, ggml_rope_cache_init + rope_yarn with ext_factor 0 and mscale 1:
     * theta_i = freq_scale * ((p * theta_scale^i, an f32 running product) / freq_factor_i) */
    int half = m->head_dim / 2;
    c->rope_cs = (float *)malloc((size_t)n_ctx * half * 2 * sizeof(float));
    float theta_scale = powf(m->hp.rope_base, -2.0f / (float)m->head_dim);
    for (int p = 0; p < n_ctx; p++) {
        float theta = (float)p;
        for (int i = 0; i < half; i++) {
            const float ff = m->rope_ff ? m->rope_ff[i] : 1.0f;
            const float th = m->rope_freq_scale * (theta / ff);
            c->rope_cs[((size_t)p * half + i) * 2 + 0] = cosf(th);
            c->rope_cs[((size_t)p * half + i) * 2 + 1] = sinf(th);
            theta *= theta_scale;
        }
    }
    return c;
}

void orc_ctx_free(orc_ctx *c) {
    if (!c) return;
    for (int l = 0; l < c->m->hp.n_layer; l++) { free(c->k[l]); free(c->v[l]); }
    free(c->k); free(c->v); free(c->rope_cs); free(c);
}

/* --------------------------------------------------------------- kernels */
static void rmsnorm(float *y, const float *x, const float *w, int n, float eps) {
    double sum = 0.0;
    for (int i = 0; i < n; i++) sum += (double)(x[i] * x[i]);
    float mean = (float)(sum / n);
    float scale = 1.0f / sqrtf(mean + eps);
    for (int i = 0; i < n; i++) y[i] = (x[i] * scale) * w[i];
}

static float dot_bf16(const uint16_t *w, const uint16_t *x, int n) {
    float acc[16] = {0};
    int i = 0;
    for (; i + 16 <= n; i += 16)
        for (int j = 0; j < 16; j++) acc[j] += bf16_to_f32(w[i + j]) * bf16_to_f32(x[i + j]);
    float s = 0.f;
    for (int j = 0; j < 16; j++) s += acc[j];
    for (; i < n; i++) s += bf16_to_f32(w[i]) * bf16_to_f32(x[i]);
    return s;
}
static float dot_bf16_f32(const uint16_t *w, const float *x, int n) {
    float acc[16] = {0};
    int i = 0;
    for (; i + 16 <= n; i += 16)
        for (int j = 0; j < 16; j++) acc[j] += bf16_to_f32(w[i + j]) * x[i + j];
    float s = 0.f;
    for (int j = 0; j < 16; j++) s += acc[j];
    for (; i < n; i++) s += bf16_to_f32(w[i]) * x[i];
    return s;
}

/* y[t][o] = W[o] . x[t] for T rows; ggml converts x to bf16 first (unless exact). */
static void matmul_bf16(float *y, const uint16_t *W, const float *x, int T, int n_in, int n_out, int exact,
                        uint16_t *scratch /* T*n_in */) {
    if (!exact) {
        if (q8_jitter != 0.0f) { /* sensitivity probe (tests): noise before the bf16 rounding too */
            float *xj = (float *)malloc(sizeof(float) * n_in);
            for (int t = 0; t < T; t++) {
                jitter_row(x + (size_t)t * n_in, xj, n_in, t, n_out);
                for (int i = 0; i < n_in; i++) scratch[(size_t)t * n_in + i] = f32_to_bf16(xj[i]);
            }
            free(xj);
        } else {
            for (size_t i = 0; i < (size_t)T * n_in; i++) scratch[i] = f32_to_bf16(x[i]);
        }
#pragma omp parallel for schedule(static)
        for (int o = 0; o < n_out; o++)
            for (int t = 0; t < T; t++)
                y[(size_t)t * n_out + o] = dot_bf16(W + (size_t)o * n_in, scratch + (size_t)t * n_in, n_in);
    } else {
#pragma omp parallel for schedule(static)
        for (int o = 0; o < n_out; o++)
            for (int t = 0; t < T; t++)
                y[(size_t)t * n_out + o] = dot_bf16_f32(W + (size_t)o * n_in, x + (size_t)t * n_in, n_in);
    }
}

static void matmul(float *y, const uint16_t *W, const uint8_t *Wq8, const uint8_t *Wkq, int kq_type, const float *x,
                   int T, int n_in, int n_out, int exact, uint16_t *scratch, const uint8_t *Wq4) {
    if (Wq4) matmul_q4_0(y, Wq4, x, T, n_in, n_out);
    else if (Wkq) matmul_kq(y, kq_type, Wkq, x, T, n_in, n_out);
    else if (Wq8) matmul_q8(y, Wq8, x, T, n_in, n_out);
    else matmul_bf16(y, W, x, T, n_in, n_out, exact, scratch);
}

static void rope_rows(float *v, int n_heads, int d, const float *cs /* [d/2][2] at pos */) {
    for (int hh = 0; hh < n_heads; hh++) {
        float *r = v + (size_t)hh * d;
        for (int i = 0; i < d / 2; i++) {
            float c = cs[2 * i], s = cs[2 * i + 1];
            float x0 = r[2 * i], x1 = r[2 * i + 1];
            r[2 * i] = x0 * c - x1 * s;
            r[2 * i + 1] = x0 * s + x1 * c;
        }
    }
}

/* GET_ROWS of the token embedding (bf16, Q8_0 or K-quant rows) into x[T][h] (f32). */
static void embed_rows(const orc_model *m, const int32_t *ids, int T, float *x) {
    const int h = m->hp.n_embd;
    for (int t = 0; t < T; t++) {
        if (m->tok_embd_kq) { /* GET_ROWS of a K-quant: dequantize_row_q{4,5,6}_K */
            const size_t rb = (size_t)(h / QK_K) * orc_kq_block_bytes(m->tok_embd_kq_type);
            orc_kq_dequant(m->tok_embd_kq_type, m->tok_embd_kq + (size_t)ids[t] * rb, x + (size_t)t * h, h);
        } else if (m->tok_embd_q8) { /* GET_ROWS of Q8_0: dequantize_row_q8_0 */
            const uint8_t *rw = m->tok_embd_q8 + (size_t)ids[t] * (h / QK8_0) * Q8_0_BLOCK;
            for (int i = 0; i < h; i++) {
                uint16_t dh;
                memcpy(&dh, rw + (size_t)(i / QK8_0) * Q8_0_BLOCK, 2);
                x[(size_t)t * h + i] = (float)(int8_t)rw[(size_t)(i / QK8_0) * Q8_0_BLOCK + 2 + i % QK8_0] * f16_to_f32(dh);
            }
        } else {
            for (int i = 0; i < h; i++) x[(size_t)t * h + i] = bf16_to_f32(m->tok_embd[(size_t)ids[t] * h + i]);
        }
    }
}

/*
 * Layers [lb, le) of llm_build_llama on the residual stream x[T][h] (in place) for T tokens of this
 * context at positions pos0..pos0+T-1 (their K/V go into the context's cache of those layers).
 */
static void layers_fwd(orc_ctx *c, float *x, int T, int pos0, int lb, int le) {
    orc_model *m = c->m;
    const orc_hparams *hp = &m->hp;
    int exact = m->flags & ORC_EXACT;
    int h = hp->n_embd, kvd = m->n_embd_kv, ff = hp->n_ff;
    int nh = hp->n_head, nkv = hp->n_head_kv, d = m->head_dim, gq = nh / nkv;
    int mx = ff > h ? ff : h;
    float *cur = (float *)malloc(sizeof(float) * T * mx);
    float *q = (float *)malloc(sizeof(float) * T * h);
    float *k = (float *)malloc(sizeof(float) * T * kvd);
    float *v = (float *)malloc(sizeof(float) * T * kvd);
    float *att = (float *)malloc(sizeof(float) * T * h);
    float *g = (float *)malloc(sizeof(float) * T * ff);
    float *u = (float *)malloc(sizeof(float) * T * ff);
    float *tmp = (float *)malloc(sizeof(float) * T * h);
    uint16_t *scratch = (uint16_t *)malloc(sizeof(uint16_t) * T * mx);
    const float kq_scale = 1.0f / sqrtf((float)d);
    for (int l = lb; l < le; l++) {
        orc_layer *L = &m->layers[l];
        for (int t = 0; t < T; t++) rmsnorm(cur + (size_t)t * h, x + (size_t)t * h, L->attn_norm, h, hp->eps);
        matmul(q, L->wq, L->q8[L_Q], L->kq[L_Q], L->kq_type[L_Q], cur, T, h, h, exact, scratch, L->q4[L_Q]);
        matmul(k, L->wk, L->q8[L_K], L->kq[L_K], L->kq_type[L_K], cur, T, h, kvd, exact, scratch, L->q4[L_K]);
        matmul(v, L->wv, L->q8[L_V], L->kq[L_V], L->kq_type[L_V], cur, T, h, kvd, exact, scratch, L->q4[L_V]);
        for (int t = 0; t < T; t++) {
            const float *cs = c->rope_cs + (size_t)(pos0 + t) * (d / 2) * 2;
            rope_rows(q + (size_t)t * h, nh, d, cs);
            rope_rows(k + (size_t)t * kvd, nkv, d, cs);
            size_t off = (size_t)(pos0 + t) * kvd;
            if (exact) {
                memcpy((float *)c->k[l] + off, k + (size_t)t * kvd, kvd * 4);
                memcpy((float *)c->v[l] + off, v + (size_t)t * kvd, kvd * 4);
            } else {
                for (int i = 0; i < kvd; i++) {
                    ((uint16_t *)c->k[l])[off + i] = f32_to_f16(k[(size_t)t * kvd + i]);
                    ((uint16_t *)c->v[l])[off + i] = f32_to_f16(v[(size_t)t * kvd + i]);
                }
            }
        }
        /* attention */
#pragma omp parallel for collapse(2) schedule(static)
        for (int t = 0; t < T; t++) {
            for (int hh = 0; hh < nh; hh++) {
                int n_kv = pos0 + t + 1; /* causal */
                int kh = hh / gq;
                float qv[256];
                double *dummy = NULL; (void)dummy;
                for (int i = 0; i < d; i++) {
                    float qq = q[(size_t)t * h + hh * d + i];
                    qv[i] = exact ? qq : round_f16(qq);
                }
                float *s = (float *)malloc(sizeof(float) * n_kv);
                float smax = -INFINITY;
                for (int p = 0; p < n_kv; p++) {
                    float acc = 0.f;
                    size_t off = (size_t)p * kvd + (size_t)kh * d;
                    if (exact) {
                        const float *kr = (const float *)c->k[l] + off;
                        for (int i = 0; i < d; i++) acc += qv[i] * kr[i];
                    } else {
                        const uint16_t *kr = (const uint16_t *)c->k[l] + off;
                        for (int i = 0; i < d; i++) acc += qv[i] * f16_to_f32(kr[i]);
                    }
                    s[p] = acc * kq_scale;
                    if (s[p] > smax) smax = s[p];
                }
                double sum = 0.0;
                for (int p = 0; p < n_kv; p++) {
                    float e = expf(s[p] - smax);
                    sum += (double)e;
                    s[p] = e;
                }
                float inv = (float)(1.0 / sum);
                for (int p = 0; p < n_kv; p++) {
                    s[p] *= inv;
                    if (!exact) s[p] = round_f16(s[p]);
                }
                float o[256];
                for (int i = 0; i < d; i++) o[i] = 0.f;
                for (int p = 0; p < n_kv; p++) {
                    size_t off = (size_t)p * kvd + (size_t)kh * d;
                    if (exact) {
                        const float *vr = (const float *)c->v[l] + off;
                        for (int i = 0; i < d; i++) o[i] += s[p] * vr[i];
                    } else {
                        const uint16_t *vr = (const uint16_t *)c->v[l] + off;
                        for (int i = 0; i < d; i++) o[i] += s[p] * f16_to_f32(vr[i]);
                    }
                }
                for (int i = 0; i < d; i++) att[(size_t)t * h + hh * d + i] = o[i];
                free(s);
            }
        }
        matmul(tmp, L->wo, L->q8[L_O], L->kq[L_O], L->kq_type[L_O], att, T, h, h, exact, scratch, L->q4[L_O]);
        for (size_t i = 0; i < (size_t)T * h; i++) x[i] += tmp[i];
        /* ffn */
        for (int t = 0; t < T; t++) rmsnorm(cur + (size_t)t * h, x + (size_t)t * h, L->ffn_norm, h, hp->eps);
        matmul(u, L->wu, L->q8[L_UP], L->kq[L_UP], L->kq_type[L_UP], cur, T, h, ff, exact, scratch, L->q4[L_UP]);
        matmul(g, L->wg, L->q8[L_GATE], L->kq[L_GATE], L->kq_type[L_GATE], cur, T, h, ff, exact, scratch, L->q4[L_GATE]);
        for (size_t i = 0; i < (size_t)T * ff; i++) {
            float gg = g[i];
            g[i] = (gg / (1.0f + expf(-gg))) * u[i];
        }
        matmul(tmp, L->wd, L->q8[L_DOWN], L->kq[L_DOWN], L->kq_type[L_DOWN], g, T, ff, h, exact, scratch, L->q4[L_DOWN]);
        for (size_t i = 0; i < (size_t)T * h; i++) x[i] += tmp[i];
    }
    free(cur); free(q); free(k); free(v); free(att); free(g); free(u); free(tmp); free(scratch);
}

/* Final RMS_NORM + lm_head of nt rows of x[.][h] -> logits[nt][V]. */
static void head_rows(const orc_model *m, const float *x, int nt, float *logits) {
    const orc_hparams *hp = &m->hp;
    int h = hp->n_embd, V = hp->n_vocab;
    float *cur = (float *)malloc(sizeof(float) * (size_t)nt * h);
    uint16_t *scratch = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)nt * h);
    for (int t = 0; t < nt; t++) rmsnorm(cur + (size_t)t * h, x + (size_t)t * h, m->out_norm, h, hp->eps);
    matmul(logits, m->output, m->output_q8, m->output_kq, m->output_kq_type, cur, nt, h, V, m->flags & ORC_EXACT,
           scratch, m->output_q4);
    free(cur); free(scratch);
}

/*
 * Evaluate n tokens at positions pos0..pos0+n-1 of this context (one llama_decode
 * of a ubatch).  logits: if all_logits, [n][V]; else [V] for the last token.
 * Returns 0 on success.
 */
int orc_eval(orc_ctx *c, const int32_t *ids, int n, int pos0, float *logits, int all_logits) {
    orc_model *m = c->m;
    const orc_hparams *hp = &m->hp;
    int h = hp->n_embd, V = hp->n_vocab;
    if (n <= 0 || pos0 < 0 || pos0 + n > c->n_ctx) return -1;
    for (int t = 0; t < n; t++)
        if (ids[t] < 0 || ids[t] >= V) return -2;
    float *x = (float *)malloc(sizeof(float) * (size_t)n * h);
    embed_rows(m, ids, n, x);
    layers_fwd(c, x, n, pos0, 0, hp->n_layer);
    int t0 = all_logits ? 0 : n - 1;
    head_rows(m, x + (size_t)t0 * h, n - t0, logits);
    free(x);
    return 0;
}

/*
 * Per-layer parity hook (a pipeline stage of the oracle): x_out[n][h] = layers [lb, le) applied to
 * the residual stream x_in[n][h] of n tokens at positions pos0.. (K/V of those layers are written).
 * With ids != NULL the stream starts from their embedding (x_in ignored), with logits != NULL the
 * final norm + lm_head of every row follow (x_out may then be NULL).  0 on success.
 */
int orc_layers(orc_ctx *c, const int32_t *ids, const float *x_in, int n, int pos0, int lb, int le, float *x_out,
               float *logits) {
    orc_model *m = c->m;
    int h = m->hp.n_embd;
    if (n <= 0 || pos0 < 0 || pos0 + n > c->n_ctx || lb < 0 || le > m->hp.n_layer || lb > le) return -1;
    float *x = (float *)malloc(sizeof(float) * (size_t)n * h);
    if (ids) {
        for (int t = 0; t < n; t++)
            if (ids[t] < 0 || ids[t] >= m->hp.n_vocab) { free(x); return -2; }
        embed_rows(m, ids, n, x);
    } else {
        memcpy(x, x_in, sizeof(float) * (size_t)n * h);
    }
    layers_fwd(c, x, n, pos0, lb, le);
    if (x_out) memcpy(x_out, x, sizeof(float) * (size_t)n * h);
    if (logits) head_rows(m, x, n, logits);
    free(x);
    return 0;
}

int orc_argmax(const float *logits, int n) {
    int best = 0;
    for (int i = 1; i < n; i++)
        if (logits[i] > logits[best]) best = i; /* strict: ties keep the lowest id */
    return best;
}

/* Greedy generation: prefill prompt in chunks of n_batch, then decode one token
 * at a time (llama_cpp generate/eval loop at temperature 0).  out[n_gen]. */
int orc_generate_greedy(orc_ctx *c, const int32_t *prompt, int n_prompt, int n_gen, int n_batch, int32_t *out) {
    int V = c->m->hp.n_vocab;
    float *logits = (float *)malloc(sizeof(float) * V);
    int pos = 0, rc = 0;
    for (int i = 0; i < n_prompt; i += n_batch) {
        int nb = n_prompt - i < n_batch ? n_prompt - i : n_batch;
        if ((rc = orc_eval(c, prompt + i, nb, pos, logits, 0))) goto done;
        pos += nb;
    }
    for (int g = 0; g < n_gen; g++) {
        int32_t tok = orc_argmax(logits, V);
        out[g] = tok;
        if (g + 1 == n_gen) break;
        if ((rc = orc_eval(c, &tok, 1, pos, logits, 0))) goto done;
        pos++;
    }
done:
    free(logits);
    return rc;
}

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
void orc_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
