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
