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
