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
GGML_F32, GGML_F16, GGML_Q4_0, GGML_Q8_0, GGML_Q4_K, GGML_Q5_K, GGML_Q6_K, GGML_BF16 = 0, 1, 2, 8, 12, 13, 14, 30
# block (elements, bytes) of the quantised types (ggml-common.h block_q4_0, block_q8_0, block_q4_K,
# block_q5_K, block_q6_K; QK_K = 256)
BLOCKS = {GGML_Q4_0: (32, 18), GGML_Q8_0: (32, 34), GGML_Q4_K: (256, 144), GGML_Q5_K: (256, 176),
          GGML_Q6_K: (256, 210)}
_TYPE_ELEM_BYTES = {GGML_F32: 4, GGML_F16: 2, GGML_BF16: 2}
QK8_0 = 32          # ggml block_q8_0: f16 d + 32 x int8 (ggml-common.h)
Q8_0_BLOCK = 34


def type_nbytes(ggml_type: int, n: int) -> int:
    if ggml_type in BLOCKS:
        be, bb = BLOCKS[ggml_type]
        if n % be:
            raise ValueError(f"ggml type {ggml_type}: rows must be a multiple of {be}")
        return n // be * bb
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


def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    """ggml quantize_row_q4_0_ref over rows of f32 [rows][K] -> block_q4_0 bytes [rows][K/32*18]:
    d = (first value of largest magnitude) / -8, id = 1/d, q = min(15, (int8)(x*id + 8.5)), f32 steps."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    rows, K = x.shape
    xb = x.reshape(rows, K // 32, 32)
    idx = np.abs(xb).argmax(axis=2)
    mx = np.take_along_axis(xb, idx[..., None], axis=2)[..., 0]
    d = (mx / np.float32(-8)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1) / d, np.float32(0)).astype(np.float32)
    v = ((xb * idv[..., None]).astype(np.float32) + np.float32(8.5)).astype(np.float32)
    q = np.minimum(15, np.trunc(v).astype(np.int32)).astype(np.uint8)
    out = np.empty((rows, K // 32, 18), np.uint8)
    out[..., :2] = d.astype(np.float16).view(np.uint8).reshape(rows, K // 32, 2)
    out[..., 2:] = q[..., :16] | (q[..., 16:] << 4)
    return out.reshape(rows, K // 32 * 18)


def dequantize_q8_0(blocks: np.ndarray, K: int) -> np.ndarray:
    """ggml dequantize_row_q8_0: y = q * f32(d)."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, K // QK8_0, Q8_0_BLOCK)
    d = b[..., :2].copy().view(np.float16).astype(np.float32)
    q = b[..., 2:].view(np.int8).astype(np.float32)
    return (q * d).reshape(blocks.shape[:-1] + (K,))


# --- the other block formats, restated from ggml-quants.c dequantize_row_* (all arithmetic in f32,
# one rounding per operation, as the C code: products are NOT fused with the following subtraction)
def _f16(b: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(b).view(np.float16).astype(np.float32)[..., 0]


def dequantize_q4_0(blocks: np.ndarray, K: int) -> np.ndarray:
    """block_q4_0 {f16 d; u8 qs[16]}: y[j] = ((qs[j] & 15) - 8) * d, y[j+16] = ((qs[j] >> 4) - 8) * d."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 18)
    d = _f16(b[:, 0:2])[:, None]
    qs = b[:, 2:18].astype(np.int32)
    q = np.concatenate([(qs & 15) - 8, (qs >> 4) - 8], axis=1).astype(np.float32)
    return (q * d).astype(np.float32).reshape(blocks.shape[:-1] + (K,))


def _scale_min_k4(sc: np.ndarray):
    """get_scale_min_k4 for j = 0..7 over the 12 packed 6-bit scale/min bytes -> (scale, min) [nb][8]."""
    sc = sc.astype(np.int32)
    s = np.empty(sc.shape[:-1] + (8,), np.int32)
    m = np.empty_like(s)
    s[..., :4] = sc[..., 0:4] & 63
    m[..., :4] = sc[..., 4:8] & 63
    s[..., 4:] = (sc[..., 8:12] & 0xF) | ((sc[..., 0:4] >> 6) << 4)
    m[..., 4:] = (sc[..., 8:12] >> 4) | ((sc[..., 4:8] >> 6) << 4)
    return s, m


def dequantize_q4_k(blocks: np.ndarray, K: int) -> np.ndarray:
    """block_q4_K {f16 d; f16 dmin; u8 scales[12]; u8 qs[128]}: per 64 values j, sub-blocks 2j/2j+1 with
    (sc, m) from get_scale_min_k4: y = (d*sc) * q - (dmin*m), low nibbles then high nibbles."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 144)
    d, dmin = _f16(b[:, 0:2])[:, None], _f16(b[:, 2:4])[:, None]
    sc, mn = _scale_min_k4(b[:, 4:16])
    dl = (d * sc.astype(np.float32)).astype(np.float32)     # [nb][8]
    ml = (dmin * mn.astype(np.float32)).astype(np.float32)
    qs = b[:, 16:144].reshape(-1, 4, 32).astype(np.int32)   # 4 groups of 32 bytes (64 values each)
    q = np.stack([qs & 15, qs >> 4], axis=2).reshape(-1, 8, 32).astype(np.float32)  # sub-block 2g, 2g+1
    y = (dl[:, :, None] * q).astype(np.float32) - ml[:, :, None]
    return y.astype(np.float32).reshape(blocks.shape[:-1] + (K,))


def dequantize_q5_k(blocks: np.ndarray, K: int) -> np.ndarray:
    """block_q5_K {f16 d; f16 dmin; u8 scales[12]; u8 qh[32]; u8 qs[128]}: as Q4_K with the 5th bit of
    sub-block 2g from bit 2g of qh and of 2g+1 from bit 2g+1."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 176)
    d, dmin = _f16(b[:, 0:2])[:, None], _f16(b[:, 2:4])[:, None]
    sc, mn = _scale_min_k4(b[:, 4:16])
    dl = (d * sc.astype(np.float32)).astype(np.float32)
    ml = (dmin * mn.astype(np.float32)).astype(np.float32)
    qh = b[:, 16:48].astype(np.int32)                       # [nb][32]
    qs = b[:, 48:176].reshape(-1, 4, 32).astype(np.int32)
    q = np.empty((b.shape[0], 8, 32), np.float32)
    for g in range(4):
        q[:, 2 * g] = (qs[:, g] & 15) + np.where(qh & (1 << (2 * g)), 16, 0)
        q[:, 2 * g + 1] = (qs[:, g] >> 4) + np.where(qh & (2 << (2 * g)), 16, 0)
    y = (dl[:, :, None] * q).astype(np.float32) - ml[:, :, None]
    return y.astype(np.float32).reshape(blocks.shape[:-1] + (K,))


def dequantize_q6_k(blocks: np.ndarray, K: int) -> np.ndarray:
    """block_q6_K {u8 ql[128]; u8 qh[64]; i8 scales[16]; f16 d}: two halves of 128 values; in half h,
    for l < 32: q1..q4 from ql[64h+l], ql[64h+l+32] nibbles and the 2-bit pairs of qh[32h+l], minus 32;
    y[128h + 32i + l] = d * sc[8h + l/16 + 2i] * q_(i+1)."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 210)
    ql = b[:, 0:128].astype(np.int32)
    qh = b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = _f16(b[:, 208:210])[:, None]
    y = np.empty((b.shape[0], 256), np.float32)
    l = np.arange(32)
    for h in range(2):
        L0, L1, H = ql[:, 64 * h + l], ql[:, 64 * h + 32 + l], qh[:, 32 * h + l]
        qv = [(L0 & 15) | (((H >> 0) & 3) << 4), (L1 & 15) | (((H >> 2) & 3) << 4),
              (L0 >> 4) | (((H >> 4) & 3) << 4), (L1 >> 4) | (((H >> 6) & 3) << 4)]
        for i in range(4):
            s = sc[:, 8 * h + l // 16 + 2 * i]
            y[:, 128 * h + 32 * i + l] = ((d * s).astype(np.float32) * (qv[i] - 32).astype(np.float32)).astype(np.float32)
    return y.reshape(blocks.shape[:-1] + (K,))


def dequantize(ggml_type: int, data: np.ndarray, shape) -> np.ndarray:
    """Any supported tensor -> f32 [rows][K] (GGUF order), as ggml's to_float does."""
    K = shape[-1]
    if ggml_type == GGML_F32:
        return np.asarray(data, dtype=np.float32).reshape(shape)
    if ggml_type == GGML_F16:
        return np.asarray(data, dtype=np.float16).astype(np.float32).reshape(shape)
    if ggml_type == GGML_BF16:
        return (np.asarray(data, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32).reshape(shape)
    fn = {GGML_Q4_0: dequantize_q4_0, GGML_Q8_0: dequantize_q8_0, GGML_Q4_K: dequantize_q4_k,
          GGML_Q5_K: dequantize_q5_k, GGML_Q6_K: dequantize_q6_k}[ggml_type]
    return fn(np.asarray(data), K).reshape(shape)


def random_blocks(ggml_type: int, rows: int, K: int, rng, amp: float = 0.03) -> np.ndarray:
    """Valid random blocks of a quantised type whose values are roughly zero-mean within +-amp (test
    models: no quantiser needed to exercise a decoder)."""
    be, bb = BLOCKS[ggml_type]
    nb = rows * K // be
    b = rng.integers(0, 256, size=(nb, bb), dtype=np.uint8)
    if ggml_type == GGML_Q4_0:
        b[:, 0:2] = np.full((nb, 1), amp / 8, np.float16).view(np.uint8)
    elif ggml_type == GGML_Q8_0:
        b[:, 0:2] = np.full((nb, 1), amp / 127, np.float16).view(np.uint8)
    elif ggml_type in (GGML_Q4_K, GGML_Q5_K):
        top = 15 if ggml_type == GGML_Q4_K else 31
        # scales 32..63, mins ~ scale * (top/2) * d / dmin so every sub-block is centred
        d = amp / (63 * top / 2)
        dmin = 8 * d
        s = rng.integers(32, 64, size=(nb, 8))
        m = np.clip(np.rint(s * (top / 2) * d / dmin), 0, 63).astype(np.int64)
        sc = np.zeros((nb, 12), np.int64)
        sc[:, 0:4] = (s[:, 0:4] & 63) | ((s[:, 4:8] >> 4) << 6)
        sc[:, 4:8] = (m[:, 0:4] & 63) | ((m[:, 4:8] >> 4) << 6)
        sc[:, 8:12] = (s[:, 4:8] & 15) | ((m[:, 4:8] & 15) << 4)
        b[:, 0:2] = np.full((nb, 1), d, np.float16).view(np.uint8)
        b[:, 2:4] = np.full((nb, 1), dmin, np.float16).view(np.uint8)
        b[:, 4:16] = sc.astype(np.uint8)
    elif ggml_type == GGML_Q6_K:
        b[:, 192:208] = rng.integers(8, 16, size=(nb, 16)).astype(np.int8).view(np.uint8)
        b[:, 208:210] = np.full((nb, 1), amp / (16 * 32), np.float16).view(np.uint8)
    return b.reshape(rows, K // be * bb)


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
        if t in BLOCKS:  # raw blocks, [rows][K/block*bytes] uint8
            be, bb = BLOCKS[t]
            nb = type_nbytes(t, n)
            return np.memmap(self.path, dtype=np.uint8, mode="r", offset=info["offset"],
                             shape=(nb,)).reshape(shape[:-1] + (shape[-1] // be * bb,))
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


# per-tensor types of the mixed test files (Q4_0: Q6_K output) -- the weights of these are random
# valid blocks, not quantisations of the synthetic model.  "q4_k_m" / "q5_k_m" files follow
# synth.kq_tensor_type (llama.cpp's per-layer recipe) instead of these entries.
MIXED = {
    "q4_k_m": {"token_embd": GGML_Q4_K, "output": GGML_Q6_K, "attn_v": GGML_Q6_K, "ffn_down": GGML_Q6_K,
               "*": GGML_Q4_K},
    "q5_k_m": {"token_embd": GGML_Q5_K, "output": GGML_Q6_K, "attn_v": GGML_Q6_K, "ffn_down": GGML_Q6_K,
               "*": GGML_Q5_K},
    "q4_0": {"token_embd": GGML_Q4_0, "output": GGML_Q6_K, "*": GGML_Q4_0},
    "f16": {"*": GGML_F16},
}


def _mixed_type(wtype: str, name: str) -> int:
    m = MIXED[wtype]
    for key, t in m.items():
        if key != "*" and (name.startswith(key + ".") or f".{key}." in name):
            return t
    return m["*"]


def write_synthetic_gguf(path: str, shape, seed: int = 0, n_ctx_train: int = None, wtype: str = "bf16",
                         dequant_from: str = None, rope_freqs=None, rope_scaling=None, embd_type: int = None):
    """Write a LLaMA GGUF with the synthetic weights of synth.py: every matrix bf16, or (wtype
    "q8_0") the Q8_0 quantisation of those bf16 matrices; norms f32 either way.  wtype "q4_k_m",
    "q5_k_m", "q4_0", "f16": matrices in those per-tensor types (MIXED), with random valid blocks
    (seeded) for the quantised ones and the synthetic values for f16 -- except "q4_k_m" / "q5_k_m", whose
    tensors take llama.cpp's per-layer recipe types with synth.kq_tensor's blocks.  dequant_from: a GGUF of the
    same shape whose matrices are written here dequantised (dequantize(), then bf16 RNE) as BF16.
    rope_freqs: a rope_freqs.weight tensor (head_dim/2 f32, Llama-3.1 style); rope_scaling:
    (type, factor) written as llama.rope.scaling.type / .factor.  embd_type: token_embd.weight as this
    type instead (GGML_Q8_0 or GGML_F16 of the synthetic bf16 table; llama-quantize
    --token-embedding-type)."""
    from . import synth

    if wtype not in ("bf16", "q8_0", "q4_0_synth") and wtype not in MIXED:
        raise ValueError(f"unknown wtype {wtype!r}")
    rng = np.random.default_rng(1000 + seed)

    w = GGUFWriter(path)
    w.add_string("general.architecture", "llama")
    w.add_string("general.name", f"synthetic-{shape.name}-seed{seed}")
    w.add_uint32("general.file_type", {"bf16": 32, "q8_0": 7, "q4_k_m": 15, "q5_k_m": 17, "q4_0": 2,
                                        "q4_0_synth": 2, "f16": 1}[wtype])  # llama_ftype
    w.add_uint32("llama.context_length", n_ctx_train or shape.n_ctx_train)
    w.add_uint32("llama.embedding_length", shape.n_embd)
    w.add_uint32("llama.block_count", shape.n_layer)
    w.add_uint32("llama.feed_forward_length", shape.n_ff)
    w.add_uint32("llama.rope.dimension_count", shape.head_dim)
    w.add_uint32("llama.attention.head_count", shape.n_head)
    w.add_uint32("llama.attention.head_count_kv", shape.n_head_kv)
    w.add_float32("llama.attention.layer_norm_rms_epsilon", shape.eps)
    w.add_float32("llama.rope.freq_base", shape.rope_base)
    if rope_scaling is not None:
        w.add_string("llama.rope.scaling.type", rope_scaling[0])
        w.add_float32("llama.rope.scaling.factor", rope_scaling[1])
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
    src = GGUFReader(dequant_from) if dequant_from else None
    for name, kind, arr in synth.synth_tensors(shape, seed):
        if name == "token_embd.weight" and embd_type is not None:
            w.add_tensor_info(name, arr.shape, embd_type)
            arrays.append(synth_q8_0_tensor(arr) if embd_type == GGML_Q8_0
                          else synth.bf16_bits_to_f32(arr).astype(np.float16))
            continue
        if kind == "bf16" and src is not None:
            info = src.tensors[name]
            y = dequantize(info["type"], src.tensor(name), arr.shape)
            w.add_tensor_info(name, arr.shape, GGML_BF16)
            arrays.append(synth.f32_to_bf16_bits(y))
        elif kind == "bf16" and (wtype == "q8_0" or (wtype == "q4_0_synth" and name.count(".") == 1)):
            w.add_tensor_info(name, arr.shape, GGML_Q8_0)
            arrays.append(synth_q8_0_tensor(arr))
        elif kind == "bf16" and wtype == "q4_0_synth":  # the engine's synthetic:<shape>:q4_0 model
            w.add_tensor_info(name, arr.shape, GGML_Q4_0)
            arrays.append(quantize_q4_0(synth.bf16_bits_to_f32(arr)))
        elif kind == "bf16" and wtype in synth.KQ_FTYPES:
            # llama.cpp's recipe types per tensor, the synthetic K-quant blocks of synth.kq_tensor
            # (the same bytes the engine's "synthetic:<shape>:<wtype>" model packs)
            if name in ("token_embd.weight", "output.weight"):
                k, layer = name.split(".")[0], 0
            else:
                _, layer, k, _ = name.split(".")
            t, blocks = synth.kq_tensor(wtype, k, int(layer), shape, seed)
            w.add_tensor_info(name, arr.shape, t)
            arrays.append(blocks)
        elif kind == "bf16" and wtype in MIXED:
            t = _mixed_type(wtype, name)
            w.add_tensor_info(name, arr.shape, t)
            if t == GGML_F16:
                arrays.append(synth.bf16_bits_to_f32(arr).astype(np.float16))
            else:
                arrays.append(random_blocks(t, arr.shape[0], arr.shape[1], rng))
        else:
            w.add_tensor_info(name, arr.shape, GGML_BF16 if kind == "bf16" else GGML_F32)
            arrays.append(arr)
    if rope_freqs is not None:
        rf = np.ascontiguousarray(rope_freqs, dtype=np.float32)
        assert rf.shape == (shape.head_dim // 2,)
        w.add_tensor_info("rope_freqs.weight", rf.shape, GGML_F32)
        arrays.append(rf)
    w.write(arrays)
    return path
