"""GGUF container round trip and the C ABI surface (CPU-only: no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gguf_roundtrip_synthetic(tmp_path):
    from llama_p2p_amd import gguf, synth

    sh = synth.SHAPES["test-tiny"]
    p = str(tmp_path / "t.gguf")
    gguf.write_synthetic_gguf(p, sh, seed=5)
    r = gguf.GGUFReader(p)
    md = r.metadata
    assert md["general.architecture"] == "llama"
    assert md["llama.embedding_length"] == sh.n_embd and md["llama.block_count"] == sh.n_layer
    assert md["llama.attention.head_count_kv"] == sh.n_head_kv
    assert abs(md["llama.rope.freq_base"] - sh.rope_base) < 1e-3
    assert len(md["tokenizer.ggml.tokens"]) == sh.n_vocab
    for name, kind, arr in synth.synth_tensors(sh, 5):
        t = r.tensor(name)
        assert t.shape == arr.shape, name
        assert np.array_equal(np.asarray(t), arr), name
        info = r.tensors[name]
        assert info["offset"] % 32 == 0
        assert info["type"] == (gguf.GGML_BF16 if kind == "bf16" else gguf.GGML_F32)


def test_gguf_rejects_garbage(tmp_path):
    from llama_p2p_amd import gguf

    p = tmp_path / "bad.gguf"
    p.write_bytes(b"NOTGGUF" + b"\0" * 64)
    with pytest.raises(ValueError):
        gguf.GGUFReader(str(p))


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "mx_engine.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(mx_[a-z_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    from llama_p2p_amd import engine

    L = engine.lib()
    declared = _declared_symbols()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), f"{name} declared in include/mx_engine.h but not exported"
    assert sorted(engine.EXPORTS) == declared


def test_defaults_match_llama_cpp_python():
    from llama_p2p_amd import engine

    L = engine.lib()
    o = engine.MxOpts()
    L.mx_opts_default(ctypes.byref(o))
    assert o.n_ctx == 512 and o.layer_begin == 0 and o.layer_end == -1
    s = engine.MxSampling()
    L.mx_sampling_default(ctypes.byref(s))
    assert (round(s.temperature, 3), s.top_k, round(s.top_p, 3), round(s.min_p, 3)) == (0.8, 40, 0.95, 0.05)


def test_engine_fails_loudly_without_gpu_or_model():
    """No CPU fallback: a missing device or model is an error, never a silent CPU path."""
    import torch

    from llama_p2p_amd import engine

    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    with pytest.raises(engine.MxError):
        engine.Engine("synthetic:test-tiny")


# ---- crafted headers: the C parser must reject them with MX_ERR_MODEL, never crash or over-read
def _gguf_bytes(kvs, tensors, data=b"", pad_to=32):
    """kvs: [(key, type, payload_bytes)]; tensors: [(name, ne, ggml_type, offset)]."""
    import struct

    def s(x):
        b = x.encode()
        return struct.pack("<Q", len(b)) + b

    out = b"GGUF" + struct.pack("<IQQ", 3, len(tensors), len(kvs))
    for k, t, payload in kvs:
        out += s(k) + struct.pack("<I", t) + payload
    for name, ne, typ, off in tensors:
        out += s(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", n) for n in ne)
        out += struct.pack("<IQ", typ, off)
    out += b"\0" * ((-len(out)) % pad_to)
    return out + data


def _check_rejects(tmp_path, blob, what):
    from llama_p2p_amd import engine

    p = tmp_path / "crafted.gguf"
    p.write_bytes(blob)
    with pytest.raises(engine.MxError) as ei:
        engine.gguf_check(str(p))
    assert ei.value.code == engine.MX_ERR_MODEL, what
    return str(ei.value)


def test_gguf_check_accepts_valid_file(tmp_path):
    import struct

    from llama_p2p_amd import engine

    p = tmp_path / "ok.gguf"
    p.write_bytes(_gguf_bytes([("general.alignment", 4, struct.pack("<I", 32))], [("w", [32, 2], 0, 0)],
                              data=b"\0" * 256))
    engine.gguf_check(str(p))  # no exception


def test_gguf_check_rejects_crafted_headers(tmp_path):
    import struct

    u32 = lambda v: struct.pack("<I", v)  # noqa: E731
    data = b"\0" * 256
    # general.alignment = 0 (was a division by zero) and a non-power-of-two alignment
    msg = _check_rejects(tmp_path, _gguf_bytes([("general.alignment", 4, u32(0))], [("w", [32], 0, 0)], data), "al 0")
    assert "alignment" in msg
    _check_rejects(tmp_path, _gguf_bytes([("general.alignment", 4, u32(24))], [("w", [32], 0, 0)], data), "al 24")
    # an offset that wraps offset + size past 2^64 (passed the old bounds check)
    _check_rejects(tmp_path, _gguf_bytes([], [("w", [32], 0, 2 ** 64 - 16)], data), "wrapping offset")
    # tensor past the end of the file
    _check_rejects(tmp_path, _gguf_bytes([], [("w", [1024], 0, 0)], data), "past end")
    # element count overflowing 64 bits
    _check_rejects(tmp_path, _gguf_bytes([], [("w", [2 ** 40, 2 ** 40], 0, 0)], data), "ne overflow")
    # ragged block count for a block type (Q8_0 rows of 33 elements)
    _check_rejects(tmp_path, _gguf_bytes([], [("w", [33], 8, 0)], data), "ragged q8_0")
    # unknown ggml type
    _check_rejects(tmp_path, _gguf_bytes([], [("w", [32], 99, 0)], data), "unknown type")
    # array whose count exceeds the bytes left (would have reserved 2^60 elements)
    arr = u32(4) + struct.pack("<Q", 2 ** 60)
    _check_rejects(tmp_path, _gguf_bytes([("a", 9, arr)], [], data), "huge array")
    # string longer than the file
    _check_rejects(tmp_path, b"GGUF" + struct.pack("<IQQ", 3, 0, 1) + struct.pack("<Q", 2 ** 62), "huge string")


def test_gguf_check_survives_truncation_fuzz(tmp_path):
    """Every prefix of a valid file and random byte flips: an error or success, never a crash."""
    from llama_p2p_amd import engine, gguf, synth

    p = str(tmp_path / "t.gguf")
    gguf.write_synthetic_gguf(p, synth.SHAPES["test-tiny"], seed=1)
    blob = open(p, "rb").read()
    hdr_end = 4096
    q = tmp_path / "f.gguf"
    for cut in list(range(0, 200, 7)) + [hdr_end // 2, hdr_end]:
        q.write_bytes(blob[:cut])
        with pytest.raises(engine.MxError):
            engine.gguf_check(str(q))
    rng = np.random.default_rng(0)
    head = bytearray(blob[:hdr_end])
    for _ in range(200):
        b = bytearray(head)
        for i in rng.integers(8, hdr_end, 4):
            b[i] = int(rng.integers(0, 256))
        q.write_bytes(bytes(b) + blob[hdr_end:hdr_end + 1024])
        try:
            engine.gguf_check(str(q))
        except engine.MxError as ex:
            assert ex.code == engine.MX_ERR_MODEL
