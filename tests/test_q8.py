"""Q8_0 weights on the CPU side: the block format and quantiser that
write the GGUF files, and the oracle's Q8_0 MUL_MAT.

Parity anchor.  Q8_0 lives in ggml (a dependency of llama-cpp-python ~0.3.1, not vendored in
/root/reference and not installed here; no `gguf` package either), so these tests pin the
restatement to ggml's published definitions: block_q8_0 = {f16 d; int8 qs[32]} (ggml-common.h),
quantize_row_q8_0_ref (d = amax/127, id = 1/d, q = roundf(x*id)), dequantize_row_q8_0
(y = q*d) -- known-answer blocks below -- and check that the numpy quantiser (GGUF writer)
and the C oracle's quantiser agree bit for bit.  The reference holds no Q8_0 fixtures:
beyond the format, parity of the Q8_0 forward is against this oracle ("parity pinned to the
published format")."""
import struct

import numpy as np
import pytest

from llama_p2p_amd import gguf, synth


def _block(d16: float, qs):
    return np.frombuffer(struct.pack("<e32b", d16, *qs), dtype=np.uint8)


def test_q8_0_known_answers():
    # amax 12.7 -> d = 0.1 (f32 12.7/127), values are exact multiples -> q = 10*x
    x = np.array([(-1) ** j * 0.1 * j for j in range(32)], dtype=np.float32)
    x[31] = 12.7
    b = gguf.quantize_q8_0(x[None])[0]
    d = np.float32(np.float32(12.7) / np.float32(127))
    q = [int(v) for v in np.trunc(x * (np.float32(1) / d) + np.copysign(0.5, x))]
    assert np.array_equal(b, _block(float(np.float16(d)), q))
    assert q[31] == 127 and q[1] == -1 and q[2] == 2
    # zero block: d = 0, id = 0, q = 0
    z = gguf.quantize_q8_0(np.zeros((1, 32), np.float32))[0]
    assert np.array_equal(z, np.zeros(34, np.uint8))
    # ties round away from zero (roundf), not to even: x*id = +-2.5 -> +-3, 0.5 -> 1
    t = np.zeros(32, np.float32)
    t[0], t[1], t[2], t[3] = 127.0, 2.5, -2.5, 0.5   # amax 127 -> d = 1, id = 1
    tq = gguf.quantize_q8_0(t[None])[0][2:].view(np.int8)
    assert tq[:4].tolist() == [127, 3, -3, 1]
    # dequantize_row_q8_0: q * f32(d)
    y = gguf.dequantize_q8_0(b[None], 32)[0]
    assert np.array_equal(y, np.array(q, np.float32) * np.float32(np.float16(d)))


def test_q8_0_quantisation_error_bound():
    rng = np.random.default_rng(0)
    w = (rng.standard_normal((64, 256)) * 0.02).astype(np.float32)
    back = gguf.dequantize_q8_0(gguf.quantize_q8_0(w), 256)
    d = np.abs(w).reshape(64, 8, 32).max(-1) / 127
    err = np.abs(back - w).reshape(64, 8, 32).max(-1)
    # half a step, plus 127 * the f16 rounding of d (relative 2^-11) on the largest q
    assert (err <= d * (0.5 + 127 * 2.0 ** -11) * 1.001).all()


def test_q8_gguf_roundtrip(tmp_path):
    shape = synth.SHAPES["test-tiny"]
    path = str(tmp_path / "q8.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype="q8_0")
    r = gguf.GGUFReader(path)
    assert r.metadata["general.file_type"] == 7
    t = r.tensors["blk.1.ffn_down.weight"]
    assert t["type"] == gguf.GGML_Q8_0 and list(t["ne"]) == [shape.n_ff, shape.n_embd]
    blocks = r.tensor("blk.1.ffn_down.weight")
    assert blocks.shape == (shape.n_embd, shape.n_ff // 32 * 34)
    bf = synth.synth_weight_bf16(3, synth.layer_tid(1, synth.L_DOWN), shape.n_embd, shape.n_ff)
    assert np.array_equal(blocks, gguf.synth_q8_0_tensor(bf))
    assert r.tensors["blk.0.attn_norm.weight"]["type"] == gguf.GGML_F32


def test_oracle_q8_quantiser_matches_numpy(oracle_mod):
    """orc_quantize_q8 (C) and quantize_q8_0 (numpy, the GGUF writer) give identical blocks:
    a model fed the numpy blocks through orc_set_tensor_q8 evaluates bit-identically."""
    shape = synth.SHAPES["test-tiny"]
    a = oracle_mod.OracleModel(shape, seed=5)
    a.quantize_q8()
    b = oracle_mod.OracleModel(shape, seed=5)
    kinds = {"token_embd.weight": (-1, 1), "output.weight": (-1, 3)}
    for l in range(shape.n_layer):
        for nm, k in (("attn_q", synth.L_Q), ("attn_k", synth.L_K), ("attn_v", synth.L_V),
                      ("attn_output", synth.L_O), ("ffn_gate", synth.L_GATE), ("ffn_up", synth.L_UP),
                      ("ffn_down", synth.L_DOWN)):
            kinds[f"blk.{l}.{nm}.weight"] = (l, k)
    n = 0
    for name, kind, arr in synth.synth_tensors(shape, 5):
        if name in kinds:
            b.set_tensor_q8(*kinds[name], gguf.synth_q8_0_tensor(arr))
            n += 1
    assert n == 2 + 7 * shape.n_layer
    ids = [1, 17, 300, 42, 9, 255]
    la = a.context(32).eval(ids, 0, all_logits=True)
    lb = b.context(32).eval(ids, 0, all_logits=True)
    assert np.array_equal(la, lb)
    # and the Q8_0 model is a close quantisation of the bf16 one
    l0 = oracle_mod.OracleModel(shape, seed=5).context(32).eval(ids, 0, all_logits=True)
    assert np.abs(la - l0).max() < 0.05 * np.abs(l0).max()
