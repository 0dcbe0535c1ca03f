"""Model shapes and the deterministic synthetic-weight definition.

The reference loads a GGUF through ``Llama(model_path=model_path)``
(/root/reference/llama_p2p_network.py:19).  No GGUF checkpoint exists on this
machine or on the GPU box and there is no network, so every benchmark and test
uses *synthetic* weights of the exact LLaMA shapes.  The generator below is the
single definition of those weights.  It is integer-only up to one float32
multiply, so the numpy version here, the engine's HIP kernel
(csrc/kernels.hip: ``synth_value``) and the CPU oracle
(oracle/llama_oracle.c: ``orc_synth_value``) produce bit-identical bf16 values.

    z  = seed*0x9E3779B97F4A7C15 + tensor_id*0xD1B54A32D192ED03 + index   (mod 2^64)
    z  = splitmix64_finalize(z)
    s  = sum of the four 16-bit fields of z          (Irwin-Hall, n=4)
    v  = float32(s - 131070) * float32(std / sqrt((2^32-1)/3))
    weight = bf16_rne(v)            norm weight = float32(1 + v)   (std 0.1)

``index`` is the element's position in GGUF data order (row-major, ``ne0``
fastest), i.e. ``row * n_in + col`` for a 2-D weight W[out][in].
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

WEIGHT_STD = 0.02
NORM_STD = 0.1

# tensor ids (stable across host / device / oracle)
TID_TOK_EMBD = 1
TID_OUT_NORM = 2
TID_OUTPUT = 3
TID_LAYER_BASE = 16
TID_LAYER_STRIDE = 16
L_ATTN_NORM, L_Q, L_K, L_V, L_O, L_FFN_NORM, L_GATE, L_UP, L_DOWN = range(9)


def layer_tid(layer: int, kind: int) -> int:
    return TID_LAYER_BASE + TID_LAYER_STRIDE * layer + kind


@dataclasses.dataclass(frozen=True)
class LlamaShape:
    name: str
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    n_ff: int
    n_vocab: int
    rope_base: float = 10000.0
    eps: float = 1e-5
    n_ctx_train: int = 2048

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    @property
    def n_embd_kv(self) -> int:
        return self.head_dim * self.n_head_kv

    def weight_bytes_per_token(self) -> int:
        """bf16 bytes streamed per decode step at batch 1."""
        h, kv, ff, L, V = self.n_embd, self.n_embd_kv, self.n_ff, self.n_layer, self.n_vocab
        lin = L * (h * h + 2 * h * kv + h * h + 3 * h * ff)
        norms = (2 * L + 1) * h * 4  # f32 norm weights
        return 2 * lin + 2 * V * h + norms + 2 * h  # + one embedding row

    def kv_bytes_per_pos(self) -> int:
        return self.n_layer * 2 * self.n_embd_kv * 2  # f16 K and V

    def n_params(self) -> int:
        h, kv, ff, L, V = self.n_embd, self.n_embd_kv, self.n_ff, self.n_layer, self.n_vocab
        return L * (2 * h * h + 2 * h * kv + 3 * h * ff + 2 * h) + 2 * V * h + h


SHAPES = {
    "tinyllama-1.1b": LlamaShape("tinyllama-1.1b", 2048, 22, 32, 4, 5632, 32000, 10000.0, 1e-5),
    "llama3-8b": LlamaShape("llama3-8b", 4096, 32, 32, 8, 14336, 128256, 500000.0, 1e-5, 8192),
    "llama3-70b": LlamaShape("llama3-70b", 8192, 80, 64, 8, 28672, 128256, 500000.0, 1e-5, 8192),
    # small shapes for parity tests (oracle finishes in well under a second)
    "test-tiny": LlamaShape("test-tiny", 256, 2, 4, 2, 512, 512, 10000.0, 1e-5),
    "test-gqa8": LlamaShape("test-gqa8", 512, 3, 8, 1, 1024, 1024, 500000.0, 1e-5),
    "test-d128": LlamaShape("test-d128", 1024, 2, 8, 2, 2816, 2048, 500000.0, 1e-5),
    # Llama-3-8B hidden geometry (n_embd 4096, 32 q / 8 kv heads of 128), one layer, small FFN/vocab
    "test-h4096": LlamaShape("test-h4096", 4096, 1, 32, 8, 2048, 1024, 500000.0, 1e-5),
    # Llama-3-70B hidden geometry (h 8192, 64 q / 8 kv heads: GQA group 8), one layer
    "test-h8192": LlamaShape("test-h8192", 8192, 1, 64, 8, 2048, 1024, 500000.0, 1e-5),
    # full Llama-3-8B / -70B FFN width (the row-tile-persistent gate/up instantiations), small vocab
    "test-8b-ffn": LlamaShape("test-8b-ffn", 4096, 2, 32, 8, 14336, 1024, 500000.0, 1e-5),
    "test-70b-ffn": LlamaShape("test-70b-ffn", 8192, 1, 64, 8, 28672, 1024, 500000.0, 1e-5),
    # TinyLlama-1.1B hidden/FFN/vocab geometry, one layer (gate/up 704 tiles: 235 groups x <= 3)
    "test-tiny-ffn": LlamaShape("test-tiny-ffn", 2048, 1, 32, 4, 5632, 32000, 10000.0, 1e-5),
    # Llama-3-8B layers (2 of 32) with the full 128256-token vocabulary: the bench's lm_head / argmax /
    # top-k instantiations at the real width
    "test-8b-v128k": LlamaShape("test-8b-v128k", 4096, 2, 32, 8, 14336, 128256, 500000.0, 1e-5, 8192),
    # a non-Llama-3 geometry (Llama-2-7B: multi-head attention, ff 11008): the generic GEMV paths
    "llama2-7b": LlamaShape("llama2-7b", 4096, 32, 32, 32, 11008, 32000, 10000.0, 1e-5, 4096),
}

_M64 = (1 << 64) - 1


def _std_scale(std: float) -> np.float32:
    return np.float32(std / math.sqrt(4294967295.0 / 3.0))


def synth_values(seed: int, tid: int, start: int, count: int, std: float) -> np.ndarray:
    """float32 values of elements [start, start+count) of tensor ``tid``."""
    base = (seed * 0x9E3779B97F4A7C15 + tid * 0xD1B54A32D192ED03) & _M64
    with np.errstate(over="ignore"):
        z = np.arange(start, start + count, dtype=np.uint64) + np.uint64(base)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    m = np.uint64(0xFFFF)
    s = (z & m) + ((z >> np.uint64(16)) & m) + ((z >> np.uint64(32)) & m) + (z >> np.uint64(48))
    v = (s.astype(np.int64) - 131070).astype(np.float32)
    return v * _std_scale(std)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even float32 -> bf16 bit pattern (uint16). No NaNs expected."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = (u + np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1))) >> np.uint32(16)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def synth_weight_bf16(seed: int, tid: int, n_out: int, n_in: int) -> np.ndarray:
    """bf16 bits of W[n_out][n_in] (GGUF data order)."""
    return f32_to_bf16_bits(synth_values(seed, tid, 0, n_out * n_in, WEIGHT_STD)).reshape(n_out, n_in)


def synth_norm_f32(seed: int, tid: int, n: int) -> np.ndarray:
    return (np.float32(1.0) + synth_values(seed, tid, 0, n, NORM_STD)).astype(np.float32)


def synth_tensors(shape: LlamaShape, seed: int):
    """Yield (gguf_name, kind, array) for every tensor of the model in GGUF order.

    kind: 'bf16' (uint16 bits, 2-D [out][in]) or 'f32' (1-D).
    """
    h, kv, ff, V = shape.n_embd, shape.n_embd_kv, shape.n_ff, shape.n_vocab
    yield "token_embd.weight", "bf16", synth_weight_bf16(seed, TID_TOK_EMBD, V, h)
    for l in range(shape.n_layer):
        p = f"blk.{l}."
        yield p + "attn_norm.weight", "f32", synth_norm_f32(seed, layer_tid(l, L_ATTN_NORM), h)
        yield p + "attn_q.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_Q), h, h)
        yield p + "attn_k.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_K), kv, h)
        yield p + "attn_v.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_V), kv, h)
        yield p + "attn_output.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_O), h, h)
        yield p + "ffn_norm.weight", "f32", synth_norm_f32(seed, layer_tid(l, L_FFN_NORM), h)
        yield p + "ffn_gate.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_GATE), ff, h)
        yield p + "ffn_up.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_UP), ff, h)
        yield p + "ffn_down.weight", "bf16", synth_weight_bf16(seed, layer_tid(l, L_DOWN), h, ff)
    yield "output_norm.weight", "f32", synth_norm_f32(seed, TID_OUT_NORM, h)
    yield "output.weight", "bf16", synth_weight_bf16(seed, TID_OUTPUT, V, h)


# ---------------------------------------------------------------------------------------------
# K-quant synthetic models ("synthetic:<shape>:q4_k_m" / ":q5_k_m"): the per-tensor ggml types of
# llama.cpp's Q4_K_M / Q5_K_M recipes (llama_tensor_get_type, Oct 2024) with synthetic blocks.
# ---------------------------------------------------------------------------------------------
GGML_Q4_K, GGML_Q5_K, GGML_Q6_K = 12, 13, 14
KQ_BLOCK_BYTES = {GGML_Q4_K: 144, GGML_Q5_K: 176, GGML_Q6_K: 210}
KQ_FTYPES = {"q4_k_m": GGML_Q4_K, "q5_k_m": GGML_Q5_K}


def use_more_bits(i_layer: int, n_layers: int) -> bool:
    """llama.cpp use_more_bits: the first and last eighth of the layers and every third in between."""
    return i_layer < n_layers // 8 or i_layer >= 7 * n_layers // 8 or (i_layer - n_layers // 8) % 3 == 2


def kq_tensor_type(ftype: str, kind: str, layer: int, n_layer: int) -> int:
    """ggml type of one tensor of a Q4_K_M / Q5_K_M model.  kind: 'token_embd', 'output' or a layer
    kind ('attn_q', 'attn_k', 'attn_v', 'attn_output', 'ffn_gate', 'ffn_up', 'ffn_down').
    output -> Q6_K; attn_v and ffn_down -> Q6_K on use_more_bits layers; attn_v of an 80-layer
    (70B) Q4_K_M model otherwise Q5_K; everything else the ftype's base type."""
    base = KQ_FTYPES[ftype]
    if kind == "output":
        return GGML_Q6_K
    if kind in ("attn_v", "ffn_down") and use_more_bits(layer, n_layer):
        return GGML_Q6_K
    if kind == "attn_v" and n_layer == 80 and base == GGML_Q4_K:
        return GGML_Q5_K
    return base


def _hash64(seed: int, tid: int, idx: np.ndarray) -> np.ndarray:
    base = (seed * 0x9E3779B97F4A7C15 + tid * 0xD1B54A32D192ED03) & _M64
    with np.errstate(over="ignore"):
        z = idx.astype(np.uint64) + np.uint64(base)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def kq_blocks(ggml_type: int, nblocks: int, seed: int, tid: int) -> np.ndarray:
    """Synthetic GGUF blocks of a K-quant tensor, uint8 [nblocks][block bytes].  Byte i of the tensor's
    block stream is byte i%8 of hash(seed, tid, i//8); then the f16 scales are set without any float
    conversion: d = 0x0500 + (its first random byte) (7.6e-5 .. 9.5e-5), dmin = 0x1100 (Q4_K) /
    0x1500 (Q5_K) + the next byte, and Q6_K's int8 scales are folded into [-24, 23] (byte % 48 - 24),
    so weights come out roughly zero-mean with std ~0.02-0.05.  The engine (csrc/kquant.hip
    synth_kq_kernel) and the oracle (orc_kq_synth_blocks) compute the same bytes."""
    bb = KQ_BLOCK_BYTES[ggml_type]
    n = nblocks * bb
    z = _hash64(seed, tid, np.arange((n + 7) // 8, dtype=np.uint64))
    b = z.view(np.uint8)[:n].reshape(nblocks, bb).copy()  # little-endian: byte k of word = bits 8k..
    if ggml_type == GGML_Q6_K:
        b[:, 192:208] = ((b[:, 192:208].astype(np.int32) % 48) - 24).astype(np.int8).view(np.uint8)
        d = 0x0500 + b[:, 208].astype(np.uint16)
        b[:, 208], b[:, 209] = (d & 0xFF).astype(np.uint8), (d >> 8).astype(np.uint8)
    else:
        d = 0x0500 + b[:, 0].astype(np.uint16)
        m = (0x1500 if ggml_type == GGML_Q5_K else 0x1100) + b[:, 1].astype(np.uint16)
        b[:, 0], b[:, 1] = (d & 0xFF).astype(np.uint8), (d >> 8).astype(np.uint8)
        b[:, 2], b[:, 3] = (m & 0xFF).astype(np.uint8), (m >> 8).astype(np.uint8)
    return b


def kq_tensor(ftype: str, kind: str, layer: int, shape: "LlamaShape", seed: int):
    """(ggml type, uint8 blocks [rows][row bytes]) of one K-quant synthetic matrix (GGUF order)."""
    h, kv, ff, V = shape.n_embd, shape.n_embd_kv, shape.n_ff, shape.n_vocab
    rows, cols = {"token_embd": (V, h), "output": (V, h), "attn_q": (h, h), "attn_k": (kv, h),
                  "attn_v": (kv, h), "attn_output": (h, h), "ffn_gate": (ff, h), "ffn_up": (ff, h),
                  "ffn_down": (h, ff)}[kind]
    kidx = {"attn_q": L_Q, "attn_k": L_K, "attn_v": L_V, "attn_output": L_O, "ffn_gate": L_GATE,
            "ffn_up": L_UP, "ffn_down": L_DOWN}
    tid = TID_TOK_EMBD if kind == "token_embd" else TID_OUTPUT if kind == "output" else layer_tid(layer, kidx[kind])
    t = kq_tensor_type(ftype, kind, layer, shape.n_layer)
    blocks = kq_blocks(t, rows * cols // 256, seed, tid)
    return t, blocks.reshape(rows, cols // 256 * KQ_BLOCK_BYTES[t])


def kq_weight_bytes_per_token(shape: "LlamaShape", ftype: str) -> int:
    """Bytes a batch-1 decode step streams for a K-quant model: every layer matrix and the output
    head at their GGUF block sizes, the f32 norms and one token_embd row."""
    h, kv, ff, V, L = shape.n_embd, shape.n_embd_kv, shape.n_ff, shape.n_vocab, shape.n_layer
    tot = V * h // 256 * KQ_BLOCK_BYTES[kq_tensor_type(ftype, "output", 0, L)]
    tot += h // 256 * KQ_BLOCK_BYTES[kq_tensor_type(ftype, "token_embd", 0, L)]
    for l in range(L):
        for kind, n in (("attn_q", h * h), ("attn_k", kv * h), ("attn_v", kv * h), ("attn_output", h * h),
                        ("ffn_gate", ff * h), ("ffn_up", ff * h), ("ffn_down", h * ff)):
            tot += n // 256 * KQ_BLOCK_BYTES[kq_tensor_type(ftype, kind, l, L)]
    return tot + (2 * L + 1) * h * 4


def parse_synthetic_path(path: str):
    """``synthetic:<shape>[:seed=N]`` -> (LlamaShape, seed) or None."""
    if not isinstance(path, str) or not path.startswith("synthetic:"):
        return None
    parts = path.split(":")[1:]
    name = parts[0]
    seed = 0
    for p in parts[1:]:
        if p.startswith("seed="):
            seed = int(p[5:])
    if name not in SHAPES:
        raise ValueError(f"unknown synthetic shape {name!r}; known: {sorted(SHAPES)}")
    return SHAPES[name], seed
