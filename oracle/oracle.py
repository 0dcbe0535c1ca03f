"""ctypes wrapper of the CPU oracle (llama_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See the header of
llama_oracle.c for what it restates (llama.cpp llm_build_llama on CPU, the
hot path behind /root/reference/llama_p2p_network.py:125).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc.so")

ORC_EXACT = 1


class _HP(ctypes.Structure):
    _fields_ = [("n_embd", ctypes.c_int), ("n_layer", ctypes.c_int), ("n_head", ctypes.c_int),
                ("n_head_kv", ctypes.c_int), ("n_ff", ctypes.c_int), ("n_vocab", ctypes.c_int),
                ("eps", ctypes.c_float), ("rope_base", ctypes.c_float)]


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "llama_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liborc.so"])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.orc_create.restype = vp
        L.orc_create.argtypes = [ctypes.POINTER(_HP), i32]
        L.orc_free.argtypes = [vp]
        L.orc_fill_synthetic.argtypes = [vp, u64]
        L.orc_fill_synthetic_layers.argtypes = [vp, u64, i32, i32, i32]
        L.orc_set_tensor.argtypes = [vp, i32, i32, vp]
        L.orc_set_tensor.restype = i32
        L.orc_set_tensor_q8.argtypes = [vp, i32, i32, vp]
        L.orc_set_tensor_q8.restype = i32
        L.orc_quantize_q8.argtypes = [vp]
        L.orc_quantize_q8.restype = i32
        L.orc_set_q8_jitter.argtypes = [ctypes.c_float]
        L.orc_set_tensor_q4_0.argtypes = [vp, i32, i32, vp]
        L.orc_set_tensor_q4_0.restype = i32
        L.orc_quantize_q4_0.argtypes = [vp]
        L.orc_quantize_q4_0.restype = i32
        L.orc_q4_0_quantize_row.argtypes = [vp, i32, vp]
        L.orc_q4_0_quantize_row.restype = i32
        L.orc_q4_0_vec_dot.argtypes = [vp, vp, i32]
        L.orc_q4_0_vec_dot.restype = ctypes.c_float
        L.orc_set_tensor_kq.argtypes = [vp, i32, i32, i32, vp]
        L.orc_set_tensor_kq.restype = i32
        L.orc_kq_synth_blocks.argtypes = [i32, ctypes.c_int64, u64, u64, vp]
        L.orc_kq_synth_blocks.restype = i32
        L.orc_kq_dequant.argtypes = [i32, vp, vp, ctypes.c_int64]
        L.orc_kq_dequant.restype = i32
        L.orc_kq_quantize_q8k.argtypes = [vp, ctypes.c_int64, vp, vp, vp]
        L.orc_kq_quantize_q8k.restype = i32
        L.orc_kq_vec_dot.argtypes = [i32, vp, vp, i32]
        L.orc_kq_vec_dot.restype = ctypes.c_float
        L.orc_kq_block_bytes.argtypes = [i32]
        L.orc_kq_block_bytes.restype = i32
        L.orc_set_rope.argtypes = [vp, vp, ctypes.c_float]
        L.orc_ctx_create.restype = vp
        L.orc_ctx_create.argtypes = [vp, i32]
        L.orc_ctx_free.argtypes = [vp]
        L.orc_eval.argtypes = [vp, vp, i32, i32, vp, i32]
        L.orc_eval.restype = i32
        L.orc_layers.argtypes = [vp, vp, vp, i32, i32, i32, i32, vp, vp]
        L.orc_layers.restype = i32
        L.orc_generate_greedy.argtypes = [vp, vp, i32, i32, i32, vp]
        L.orc_generate_greedy.restype = i32
        L.orc_num_threads.restype = i32
        L.orc_set_num_threads.argtypes = [i32]
        L.orc_synth_value.restype = ctypes.c_float
        L.orc_synth_value.argtypes = [u64, u64, u64, ctypes.c_float]
        L.orc_round_f16.restype = ctypes.c_float
        L.orc_round_f16.argtypes = [ctypes.c_float]
        L.orc_round_bf16.restype = ctypes.c_float
        L.orc_round_bf16.argtypes = [ctypes.c_float]
        _lib = L
    return _lib


class OracleModel:
    """A LLaMA model on the CPU oracle.  ``shape`` is a synth.LlamaShape."""

    def __init__(self, shape, seed: int | None = 0, exact: bool = False):
        self.shape = shape
        hp = _HP(shape.n_embd, shape.n_layer, shape.n_head, shape.n_head_kv, shape.n_ff, shape.n_vocab,
                 shape.eps, shape.rope_base)
        self._m = lib().orc_create(ctypes.byref(hp), ORC_EXACT if exact else 0)
        if seed is not None:
            lib().orc_fill_synthetic(self._m, seed)

    def fill_synthetic_layers(self, seed: int, layer_begin: int, layer_end: int, globals_: bool = True):
        """Synthesise only layers [layer_begin, layer_end) (+ embedding / head with globals_): for
        per-layer checks of a model too large to synthesise whole (create with seed=None)."""
        lib().orc_fill_synthetic_layers(self._m, seed, layer_begin, layer_end, 1 if globals_ else 0)

    def set_tensor(self, layer: int, kind: int, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        rc = lib().orc_set_tensor(self._m, layer, kind, arr.ctypes.data)
        if rc:
            raise ValueError(f"orc_set_tensor({layer},{kind}) failed")

    def set_tensor_q8(self, layer: int, kind: int, blocks: np.ndarray):
        """Make one matrix Q8_0 from GGUF block bytes (uint8 [rows][cols/32*34])."""
        blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
        if lib().orc_set_tensor_q8(self._m, layer, kind, blocks.ctypes.data):
            raise ValueError(f"orc_set_tensor_q8({layer},{kind}) failed")

    def set_tensor_q4_0(self, layer: int, kind: int, blocks: np.ndarray):
        """Make one matrix Q4_0 from GGUF block bytes (uint8 [rows][cols/32*18]); output: layer -1 kind 3."""
        blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
        if lib().orc_set_tensor_q4_0(self._m, layer, kind, blocks.ctypes.data):
            raise ValueError(f"orc_set_tensor_q4_0({layer},{kind}) failed")

    def quantize_q4_0(self):
        """Layer matrices -> Q4_0 of their bf16 values (ggml quantize_row_q4_0_ref), token_embd and
        output -> Q8_0: the engine's synthetic:<shape>:q4_0 model."""
        if lib().orc_quantize_q4_0(self._m):
            raise ValueError("orc_quantize_q4_0 failed")

    def set_tensor_kq(self, layer: int, kind: int, ggml_type: int, blocks: np.ndarray):
        """Make one matrix a K-quant (Q4_K 12, Q5_K 13, Q6_K 14) from GGUF block bytes."""
        blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
        if lib().orc_set_tensor_kq(self._m, layer, kind, ggml_type, blocks.ctypes.data):
            raise ValueError(f"orc_set_tensor_kq({layer},{kind},{ggml_type}) failed")

    def kq_synthetic(self, ftype: str, seed: int):
        """Every matrix -> the K-quant synthetic blocks of ``synthetic:<shape>:<ftype>`` (synth.kq_tensor
        types; blocks from the oracle's own generator, orc_kq_synth_blocks)."""
        import sys
        sys.path.insert(0, os.path.dirname(HERE))
        from llama_p2p_amd import synth

        sh = self.shape
        h, kv, ff, V = sh.n_embd, sh.n_embd_kv, sh.n_ff, sh.n_vocab
        mats = [(-1, 1, "token_embd", V * h, synth.TID_TOK_EMBD), (-1, 3, "output", V * h, synth.TID_OUTPUT)]
        for l in range(sh.n_layer):
            for kind, k, n in (("attn_q", synth.L_Q, h * h), ("attn_k", synth.L_K, kv * h), ("attn_v", synth.L_V, kv * h),
                               ("attn_output", synth.L_O, h * h), ("ffn_gate", synth.L_GATE, ff * h),
                               ("ffn_up", synth.L_UP, ff * h), ("ffn_down", synth.L_DOWN, h * ff)):
                mats.append((l, k, kind, n, synth.layer_tid(l, k)))
        for layer, k, kind, n, tid in mats:
            t = synth.kq_tensor_type(ftype, kind, layer, sh.n_layer)
            self.set_tensor_kq(layer, k, t, kq_synth_blocks(t, n // 256, seed, tid))

    def set_rope(self, freq_factors=None, freq_scale: float = 1.0):
        """Llama-3.1 RoPE frequency factors (head_dim/2 floats) and linear scaling (1/factor)."""
        self._ff = None if freq_factors is None else np.ascontiguousarray(freq_factors, dtype=np.float32)
        lib().orc_set_rope(self._m, self._ff.ctypes.data if self._ff is not None else None, freq_scale)

    def quantize_q8(self):
        """Every matrix -> Q8_0 of its bf16 values (ggml quantize_row_q8_0_ref)."""
        if lib().orc_quantize_q8(self._m):
            raise ValueError("orc_quantize_q8 failed")

    def context(self, n_ctx: int = 512) -> "OracleContext":
        return OracleContext(self, n_ctx)

    def close(self):
        if self._m:
            lib().orc_free(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OracleContext:
    def __init__(self, model: OracleModel, n_ctx: int):
        self.model = model
        self.n_ctx = n_ctx
        self._c = lib().orc_ctx_create(model._m, n_ctx)

    def eval(self, ids, pos0: int, all_logits: bool = False) -> np.ndarray:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        n = len(ids)
        V = self.model.shape.n_vocab
        out = np.zeros((n if all_logits else 1, V), dtype=np.float32)
        rc = lib().orc_eval(self._c, ids.ctypes.data, n, pos0, out.ctypes.data, 1 if all_logits else 0)
        if rc:
            raise ValueError(f"orc_eval rc={rc}")
        return out

    def layers(self, x_in, pos0: int, layer_begin: int, layer_end: int, ids=None, logits: bool = False):
        """Per-layer hook (orc_layers): the residual stream after layers [layer_begin, layer_end) of
        x_in [n][n_embd] f32 (or of the embedding of ``ids``) for n tokens at positions pos0..; their
        K/V enter this context's cache.  Returns x_out [n][n_embd], or (x_out, logits [n][V])."""
        h = self.model.shape.n_embd
        ids_a = None if ids is None else np.ascontiguousarray(ids, dtype=np.int32)
        xin = None if ids_a is not None else np.ascontiguousarray(x_in, dtype=np.float32).reshape(-1, h)
        n = len(ids_a) if ids_a is not None else xin.shape[0]
        out = np.zeros((n, h), dtype=np.float32)
        lg = np.zeros((n, self.model.shape.n_vocab), dtype=np.float32) if logits else None
        rc = lib().orc_layers(self._c, ids_a.ctypes.data if ids_a is not None else None,
                              xin.ctypes.data if xin is not None else None, n, pos0, layer_begin, layer_end,
                              out.ctypes.data, lg.ctypes.data if lg is not None else None)
        if rc:
            raise ValueError(f"orc_layers rc={rc}")
        return (out, lg) if logits else out

    def generate_greedy(self, prompt, n_gen: int, n_batch: int = 512) -> np.ndarray:
        prompt = np.ascontiguousarray(prompt, dtype=np.int32)
        out = np.zeros(n_gen, dtype=np.int32)
        rc = lib().orc_generate_greedy(self._c, prompt.ctypes.data, len(prompt), n_gen, n_batch, out.ctypes.data)
        if rc:
            raise ValueError(f"orc_generate_greedy rc={rc}")
        return out

    def close(self):
        if self._c:
            lib().orc_ctx_free(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def q8_jitter(eps: float):
    """Relative activation noise before every Q8_0 quantisation (sensitivity probe; 0 = off)."""
    lib().orc_set_q8_jitter(eps)


def q4_0_quantize_row(x: np.ndarray) -> np.ndarray:
    """ggml quantize_row_q4_0_ref of one f32 row -> block_q4_0 bytes (uint8 [n/32*18])."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size // 32 * 18, np.uint8)
    if lib().orc_q4_0_quantize_row(x.ctypes.data, x.size, out.ctypes.data):
        raise ValueError("orc_q4_0_quantize_row failed")
    return out


def q4_0_vec_dot(blocks: np.ndarray, x: np.ndarray) -> float:
    """ggml_vec_dot_q4_0_q8_0 of one Q4_0 row with the Q8_0 image of x."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.float32)
    return float(lib().orc_q4_0_vec_dot(blocks.ctypes.data, x.ctypes.data, x.size))


def kq_synth_blocks(ggml_type: int, nblocks: int, seed: int, tid: int) -> np.ndarray:
    """The oracle's synthetic K-quant blocks (uint8 [nblocks][block bytes])."""
    bb = lib().orc_kq_block_bytes(ggml_type)
    out = np.empty((nblocks, bb), np.uint8)
    if lib().orc_kq_synth_blocks(ggml_type, nblocks, seed, tid, out.ctypes.data):
        raise ValueError("orc_kq_synth_blocks failed")
    return out


def kq_dequant(ggml_type: int, blocks: np.ndarray, n: int) -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    out = np.empty(n, np.float32)
    if lib().orc_kq_dequant(ggml_type, blocks.ctypes.data, out.ctypes.data, n):
        raise ValueError("orc_kq_dequant failed")
    return out


def kq_quantize_q8k(x: np.ndarray):
    """Q8_K image of one activation row: (qs int8 [n], d f32 [n/256], bsums int16 [n/16])."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = x.size
    qs, d, bs = np.empty(n, np.int8), np.empty(n // 256, np.float32), np.empty(n // 16, np.int16)
    if lib().orc_kq_quantize_q8k(x.ctypes.data, n, qs.ctypes.data, d.ctypes.data, bs.ctypes.data):
        raise ValueError("orc_kq_quantize_q8k failed")
    return qs, d, bs


def kq_vec_dot(ggml_type: int, blocks: np.ndarray, x: np.ndarray) -> float:
    """ggml_vec_dot_q{4,5,6}_K_q8_K of one weight row with the Q8_K image of x."""
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.float32)
    return float(lib().orc_kq_vec_dot(ggml_type, blocks.ctypes.data, x.ctypes.data, x.size))


def argmax_lowest(logits: np.ndarray) -> int:
    """Greedy pick with ties -> lowest id (llama.cpp greedy sampler)."""
    return int(np.argmax(logits))  # numpy argmax returns the first maximum
