"""GGUF v3 reader/writer (pure Python + numpy).

The reference hands a GGUF path to ``Llama(model_path=...)``
(/root/reference/llama_p2p_network.py:19, ``--model`` help text at :194).  The
``gguf`` package is not installed here, so this module restates the container
format (GGUF v3, little-endian): header, typed key/value metadata, tensor
infos, and a data section aligned to ``general.alignment`` (default 32).  The
engine's C++ loader (csrc/gguf.cpp) parses the same format independently; this
module is used to *write* synthetic models and by tests.
"""
from __future__ import annotations

import os
import struct
from typing import Any, Dict, List, Tuple

import numpy as np

GGUF_MAGIC = b"GGUF"
GGUF_VERSION = 3

# metadata value types
T_UINT8, T_INT8, T_UINT16, T_INT16, T_UINT32, T_INT32, T_FLOAT32, T_BOOL, T_STRING, T_ARRAY, T_UINT64, T_INT64, T_FLOAT64 = range(13)
_SCALAR = {
    T_UINT8: "<B", T_INT8: "<b", T_UINT16: "<H", T_INT16: "<h", T_UINT32: "<I", T_INT32: "<i",
    T_FLOAT32: "<f", T_BOOL: "<?", T_UINT64: "<Q", T_INT64: "<q", T_FLOAT64: "<d",
}

# ggml tensor types used here
GGML_F32, GGML_F16, GGML_Q4_0, GGML_Q8_0, GGML_Q4_K, GGML_Q6_K, GGML_BF16 = 0, 1, 2, 8, 12, 14, 30
_TYPE_ELEM_BYTES = {GGML_F32: 4, GGML_F16: 2, GGML_BF16: 2}
QK8_0 = 32          # ggml block_q8_0: f16 d + 32 x int8 (ggml-common.h)
Q8_0_BLOCK = 34


def type_nbytes(ggml_type: int, n: int) -> int:
    if ggml_type == GGML_Q8_0:
        if n % QK8_0:
            raise ValueError("Q8_0 rows must be a multiple of 32")
        return n // QK8_0 * Q8_0_BLOCK
    return n * _TYPE_ELEM_BYTES[ggml_type]


def _round_half_away(v: np.ndarray) -> np.ndarray:
    """C roundf(): ties away from zero (numpy's round is ties-to-even).  v is f32; the
    +-0.5 is added in f64, where it is exact, so no second rounding can creep in."""
    v = v.astype(np.float64)
    return np.trunc(v + np.copysign(0.5, v))


def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    """ggml quantize_row_q8_0_ref (ggml-quants.c), row-wise over the last axis: per block of
    32, d = amax/127 (f32), id = d ? 1/d : 0, q = roundf(x*id), d stored as f16.  This is what
    llama.cpp's convert/quantize tools write for weights.  Returns uint8 [..., K/32*34]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    K = x.shape[-1]
    if K % QK8_0:
        raise ValueError("Q8_0 rows must be a multiple of 32")
    b = x.reshape(-1, K // QK8_0, QK8_0)
    amax = np.abs(b).max(axis=-1)
    d = (amax / np.float32(127)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1) / d, np.float32(0)).astype(np.float32)
    q = _round_half_away(b * idv[..., None]).astype(np.int8)
    out = np.empty(b.shape[:2] + (Q8_0_BLOCK,), dtype=np.uint8)
    out[..., :2] = d.astype(np.float16).view(np.uint8).reshape(b.shape[:2] + (2,))
    out[..., 2:] = q.view(np.uint8)
    return out.reshape(x.shape[:-1] + (K // QK8_0 * Q8_0_BLOCK,))


def dequantize_q8_0(blocks: np.ndarray, K: int) -> np.ndarray:
    """ggml dequantize_row_q8_0: y = q * f32(d)."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, K // QK8_0, Q8_0_BLOCK)
    d = b[..., :2].copy().view(np.float16).astype(np.float32)
    q = b[..., 2:].view(np.int8).astype(np.float32)
    return (q * d).reshape(blocks.shape[:-1] + (K,))


class GGUFWriter:
    """Streaming writer: add metadata + tensor *infos* first, then data in order."""

    def __init__(self, path: str, alignment: int = 32):
        self.path = path
        self.alignment = alignment
        self.kv: List[Tuple[str, int, Any, int]] = []  # (key, type, value, array elem type)
        self.tensors: List[Tuple[str, Tuple[int, ...], int, int]] = []  # name, ne, type, nbytes
        self.add_uint32("general.alignment", alignment)

    # -- metadata -------------------------------------------------------
    def add(self, key: str, vtype: int, value: Any, atype: int = -1):
        self.kv.append((key, vtype, value, atype))

    def add_string(self, key, v): self.add(key, T_STRING, v)
    def add_uint32(self, key, v): self.add(key, T_UINT32, int(v))
    def add_int32(self, key, v): self.add(key, T_INT32, int(v))
    def add_float32(self, key, v): self.add(key, T_FLOAT32, float(v))
    def add_bool(self, key, v): self.add(key, T_BOOL, bool(v))
    def add_array(self, key, atype, values): self.add(key, T_ARRAY, list(values), atype)

    # -- tensors ---------------------------------------------------------
    def add_tensor_info(self, name: str, shape_rowmajor: Tuple[int, ...], ggml_type: int):
        """shape_rowmajor is numpy order ([out, in]); GGUF stores ne reversed ([in, out])."""
        ne = tuple(int(x) for x in reversed(shape_rowmajor))
        n = int(np.prod(ne))
        nbytes = type_nbytes(ggml_type, n)
        self.tensors.append((name, ne, ggml_type, nbytes))

    @staticmethod
    def _str(s: str) -> bytes:
        b = s.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    def _val(self, vtype: int, v: Any, atype: int) -> bytes:
        if vtype == T_STRING:
            return self._str(v)
        if vtype == T_ARRAY:
            out = struct.pack("<IQ", atype, len(v))
            if atype == T_STRING:
                return out + b"".join(self._str(x) for x in v)
            return out + b"".join(struct.pack(_SCALAR[atype], x) for x in v)
        return struct.pack(_SCALAR[vtype], v)

    def write(self, data_iter):
        """data_iter yields numpy arrays in the order of add_tensor_info."""
        al = self.alignment
        with open(self.path, "wb") as f:
            f.write(GGUF_MAGIC + struct.pack("<IQQ", GGUF_VERSION, len(self.tensors), len(self.kv)))
            for key, vtype, v, atype in self.kv:
                f.write(self._str(key) + struct.pack("<I", vtype) + self._val(vtype, v, atype))
            off = 0
            for name, ne, t, nbytes in self.tensors:
                f.write(self._str(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", x) for x in ne))
                f.write(struct.pack("<IQ", t, off))
                off += (nbytes + al - 1) // al * al
            pad = (-f.tell()) % al
            f.write(b"\0" * pad)
            for (name, ne, t, nbytes), arr in zip(self.tensors, data_iter):
                b = np.ascontiguousarray(arr).tobytes()
                if len(b) != nbytes:
                    raise ValueError(f"tensor {name}: got {len(b)} bytes, expected {nbytes}")
                f.write(b)
                f.write(b"\0" * ((-nbytes) % al))


class GGUFReader:
    def __init__(self, path: str):
        self.path = path
        self.metadata: Dict[str, Any] = {}
        self.tensors: Dict[str, Dict[str, Any]] = {}
        with open(path, "rb") as f:
            data = f.read(min(os.path.getsize(path), 1 << 26))
        self._parse(data)

    def _parse(self, b: bytes):
        if b[:4] != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file")
        version, n_t, n_kv = struct.unpack_from("<IQQ", b, 4)
        if version not in (2, 3):
            raise ValueError(f"unsupported GGUF version {version}")
        p = 24

        def rstr(p):
            (n,) = struct.unpack_from("<Q", b, p)
            return b[p + 8:p + 8 + n].decode("utf-8", errors="replace"), p + 8 + n

        def rval(t, p):
            if t == T_STRING:
                return rstr(p)
            if t == T_ARRAY:
                at, n = struct.unpack_from("<IQ", b, p)
                p += 12
                if at == T_STRING:
                    out = []
                    for _ in range(n):
                        s, p = rstr(p)
                        out.append(s)
                    return out, p
                fmt = _SCALAR[at]
                sz = struct.calcsize(fmt)
                arr = np.frombuffer(b, dtype=np.dtype(fmt), count=n, offset=p)
                return arr.tolist(), p + sz * n
            fmt = _SCALAR[t]
            return struct.unpack_from(fmt, b, p)[0], p + struct.calcsize(fmt)

        for _ in range(n_kv):
            k, p = rstr(p)
            (t,) = struct.unpack_from("<I", b, p)
            v, p = rval(t, p + 4)
            self.metadata[k] = v
        infos = []
        for _ in range(n_t):
            name, p = rstr(p)
            (nd,) = struct.unpack_from("<I", b, p)
            ne = struct.unpack_from("<" + "Q" * nd, b, p + 4)
            p += 4 + 8 * nd
            t, off = struct.unpack_from("<IQ", b, p)
            p += 12
            infos.append((name, ne, t, off))
        al = int(self.metadata.get("general.alignment", 32))
        data_start = (p + al - 1) // al * al
        for name, ne, t, off in infos:
            self.tensors[name] = {"ne": ne, "type": t, "offset": data_start + off}

    def tensor(self, name: str) -> np.ndarray:
        info = self.tensors[name]
        t = info["type"]
        shape = tuple(reversed(info["ne"]))
        n = int(np.prod(shape))
        if t == GGML_Q8_0:  # raw blocks, [rows][K/32*34] uint8
            nb = type_nbytes(t, n)
            return np.memmap(self.path, dtype=np.uint8, mode="r", offset=info["offset"],
                             shape=(nb,)).reshape(shape[:-1] + (shape[-1] // QK8_0 * Q8_0_BLOCK,))
        dt = {GGML_F32: np.float32, GGML_F16: np.float16, GGML_BF16: np.uint16}[t]
        return np.memmap(self.path, dtype=dt, mode="r", offset=info["offset"], shape=(n,)).reshape(shape)


# ---------------------------------------------------------------------------
# synthetic tokenizer vocabulary (SentencePiece-style, byte fallback) so that a
# synthetic GGUF carries the same tokenizer metadata keys a real one does.
# ---------------------------------------------------------------------------
TOKEN_NORMAL, TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_USER, TOKEN_UNUSED, TOKEN_BYTE = 1, 2, 3, 4, 5, 6


def synthetic_spm_vocab(n_vocab: int):
    toks = ["<unk>", "<s>", "</s>"]
    types = [TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_CONTROL]
    for i in range(256):
        toks.append(f"<0x{i:02X}>")
        types.append(TOKEN_BYTE)
    base = [chr(c) for c in range(ord("a"), ord("z") + 1)] + [chr(c) for c in range(ord("A"), ord("Z") + 1)]
    base += list("0123456789.,!?'-:;()")
    pieces: List[str] = []
    seen = set()
    for c in base:
        for p in (c, "▁" + c):
            if p not in seen:
                seen.add(p); pieces.append(p)
    pieces.insert(0, "▁")
    common = ["the", "and", "of", "to", "in", "is", "it", "that", "for", "on", "with", "as", "was", "he", "be",
              "at", "by", "this", "had", "not", "are", "but", "from", "or", "have", "an", "they", "which", "one",
              "you", "were", "her", "all", "she", "there", "would", "their", "we", "him", "been", "has", "when",
              "who", "will", "more", "no", "if", "out", "so", "said", "what", "up", "its", "about", "into", "than",
              "them", "can", "only", "other", "new", "some", "could", "time", "these", "two", "may", "then", "do",
              "first", "any", "my", "now", "such", "like", "our", "over", "man", "me", "even", "most", "made",
              "after", "also", "did", "many", "before", "must", "through", "back", "years", "where", "much",
              "your", "way", "well", "down", "should", "because", "each", "just", "those", "people", "how",
              "too", "little", "state", "good", "very", "make", "world", "still", "own", "see", "men", "work",
              "long", "get", "here", "between", "both", "life", "being", "under", "never", "day", "same",
              "another", "know", "while", "last", "might", "us", "great", "old", "year", "off", "come",
              "since", "against", "go", "came", "right", "used", "take", "three", "hello", "model", "peer", "node"]
    for w in common:
        for p in ("▁" + w, w):
            if p not in seen:
                seen.add(p); pieces.append(p)
    # fill the rest with letter pairs / triples
    letters = "etaoinshrdlcumwfgypbvkjxqz"
    i = 0
    while len(toks) + len(pieces) < n_vocab:
        a = letters[i % 26]; b_ = letters[(i // 26) % 26]; c = letters[(i // 676) % 26]
        cand = a + b_ if i < 676 else a + b_ + c
        for p in (cand, "▁" + cand):
            if p not in seen and len(toks) + len(pieces) < n_vocab:
                seen.add(p); pieces.append(p)
        i += 1
        if i > 26 ** 3 * 2:
            break
    pieces = pieces[: max(0, n_vocab - len(toks))]
    # scores: longer pieces merge first (higher score), ties by order
    scores = [0.0] * len(toks)
    for j, p in enumerate(pieces):
        scores.append(-float(j) * 0.01 + 0.5 * len(p))
    toks += pieces
    types += [TOKEN_NORMAL] * len(pieces)
    while len(toks) < n_vocab:  # tiny vocab: pad with unused
        toks.append(f"<unused{len(toks)}>"); types.append(TOKEN_UNUSED); scores.append(-1e9)
    return toks[:n_vocab], scores[:n_vocab], types[:n_vocab]


def synth_q8_0_tensor(arr_bf16: np.ndarray) -> np.ndarray:
    """Q8_0 blocks of a synthetic bf16 matrix: what llama.cpp's quantize tool makes of a bf16
    checkpoint (bf16 -> f32 -> quantize_row_q8_0_ref)."""
    from . import synth
    return quantize_q8_0(synth.bf16_bits_to_f32(arr_bf16))


def write_synthetic_gguf(path: str, shape, seed: int = 0, n_ctx_train: int = None, wtype: str = "bf16"):
    """Write a LLaMA GGUF with the synthetic weights of synth.py: every matrix bf16, or (wtype
    "q8_0") the Q8_0 quantisation of those bf16 matrices; norms f32 either way."""
    from . import synth

    if wtype not in ("bf16", "q8_0"):
        raise ValueError("wtype must be 'bf16' or 'q8_0'")

    w = GGUFWriter(path)
    w.add_string("general.architecture", "llama")
    w.add_string("general.name", f"synthetic-{shape.name}-seed{seed}")
    w.add_uint32("general.file_type", 32 if wtype == "bf16" else 7)  # MOSTLY_BF16 / MOSTLY_Q8_0
    w.add_uint32("llama.context_length", n_ctx_train or shape.n_ctx_train)
    w.add_uint32("llama.embedding_length", shape.n_embd)
    w.add_uint32("llama.block_count", shape.n_layer)
    w.add_uint32("llama.feed_forward_length", shape.n_ff)
    w.add_uint32("llama.rope.dimension_count", shape.head_dim)
    w.add_uint32("llama.attention.head_count", shape.n_head)
    w.add_uint32("llama.attention.head_count_kv", shape.n_head_kv)
    w.add_float32("llama.attention.layer_norm_rms_epsilon", shape.eps)
    w.add_float32("llama.rope.freq_base", shape.rope_base)
    w.add_uint32("llama.vocab_size", shape.n_vocab)
    toks, scores, types = synthetic_spm_vocab(shape.n_vocab)
    w.add_string("tokenizer.ggml.model", "llama")
    w.add_array("tokenizer.ggml.tokens", T_STRING, toks)
    w.add_array("tokenizer.ggml.scores", T_FLOAT32, scores)
    w.add_array("tokenizer.ggml.token_type", T_INT32, types)
    w.add_uint32("tokenizer.ggml.bos_token_id", 1)
    w.add_uint32("tokenizer.ggml.eos_token_id", 2)
    w.add_uint32("tokenizer.ggml.unknown_token_id", 0)
    w.add_bool("tokenizer.ggml.add_bos_token", True)
    arrays = []
    for name, kind, arr in synth.synth_tensors(shape, seed):
        if kind == "bf16" and wtype == "q8_0":
            w.add_tensor_info(name, arr.shape, GGML_Q8_0)
            arrays.append(synth_q8_0_tensor(arr))
        else:
            w.add_tensor_info(name, arr.shape, GGML_BF16 if kind == "bf16" else GGML_F32)
            arrays.append(arr)
    w.write(arrays)
    return path
