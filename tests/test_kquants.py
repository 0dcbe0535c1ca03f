"""GGUF block formats beyond BF16 / Q8_0: Q4_0, Q4_K, Q5_K, Q6_K, F16.

A file whose matrices mix these types (llama.cpp's Q4_K_M, Q5_K_M, Q4_0 ... recipes) loads by
dequantising every matrix to bf16 (the engine's dequant_bf16_kernel; numpy gguf.dequantize here)
and runs on the bf16 path.  Parity anchor: ggml is not available offline, so the vectorised numpy
decoders are checked against literal scalar transcriptions of ggml-quants.c's dequantize_row_*
loops below (same statement order, f32 arithmetic), over random valid blocks and the edge values of
every packed field.  Against llama.cpp's own K-quant arithmetic (Q8_K activations) parity is
unpinned: this path deliberately computes with the dequantised weights in bf16."""
import struct

import numpy as np
import pytest

from llama_p2p_amd import gguf, synth

f32 = np.float32


def _h(b, o):
    return f32(np.frombuffer(bytes(b[o:o + 2]), dtype=np.float16)[0])


def ref_q4_0(b):
    d = _h(b, 0)
    y = [f32(0)] * 32
    for j in range(16):
        y[j] = f32(f32((b[2 + j] & 0x0F) - 8) * d)
        y[j + 16] = f32(f32((b[2 + j] >> 4) - 8) * d)
    return y


def get_scale_min_k4(j, q):
    if j < 4:
        return q[j] & 63, q[j + 4] & 63
    return (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4), (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4)


def ref_q4_k(b):
    d, mn = _h(b, 0), _h(b, 2)
    scales, q = b[4:16], b[16:144]
    y, qo, is_ = [], 0, 0
    for _ in range(0, 256, 64):
        sc, m = get_scale_min_k4(is_ + 0, scales)
        d1, m1 = f32(d * f32(sc)), f32(mn * f32(m))
        sc, m = get_scale_min_k4(is_ + 1, scales)
        d2, m2 = f32(d * f32(sc)), f32(mn * f32(m))
        y += [f32(f32(d1 * f32(q[qo + l] & 0xF)) - m1) for l in range(32)]
        y += [f32(f32(d2 * f32(q[qo + l] >> 4)) - m2) for l in range(32)]
        qo += 32
        is_ += 2
    return y


def ref_q5_k(b):
    d, mn = _h(b, 0), _h(b, 2)
    scales, qh, ql = b[4:16], b[16:48], b[48:176]
    y, qo, is_, u1, u2 = [], 0, 0, 1, 2
    for _ in range(0, 256, 64):
        sc, m = get_scale_min_k4(is_ + 0, scales)
        d1, m1 = f32(d * f32(sc)), f32(mn * f32(m))
        sc, m = get_scale_min_k4(is_ + 1, scales)
        d2, m2 = f32(d * f32(sc)), f32(mn * f32(m))
        y += [f32(f32(d1 * f32((ql[qo + l] & 0xF) + (16 if qh[l] & u1 else 0))) - m1) for l in range(32)]
        y += [f32(f32(d2 * f32((ql[qo + l] >> 4) + (16 if qh[l] & u2 else 0))) - m2) for l in range(32)]
        qo += 32
        is_ += 2
        u1 <<= 2
        u2 <<= 2
    return y


def ref_q6_k(b):
    d = _h(b, 208)
    ql, qh = list(b[0:128]), list(b[128:192])
    sc = list(np.frombuffer(bytes(b[192:208]), dtype=np.int8))
    y = [f32(0)] * 256
    yo, qlo, qho, sco = 0, 0, 0, 0
    for _ in range(0, 256, 128):
        for l in range(32):
            is_ = l // 16
            q1 = ((ql[qlo + l] & 0xF) | (((qh[qho + l] >> 0) & 3) << 4)) - 32
            q2 = ((ql[qlo + l + 32] & 0xF) | (((qh[qho + l] >> 2) & 3) << 4)) - 32
            q3 = ((ql[qlo + l] >> 4) | (((qh[qho + l] >> 4) & 3) << 4)) - 32
            q4 = ((ql[qlo + l + 32] >> 4) | (((qh[qho + l] >> 6) & 3) << 4)) - 32
            y[yo + l + 0] = f32(f32(d * f32(sc[sco + is_ + 0])) * f32(q1))
            y[yo + l + 32] = f32(f32(d * f32(sc[sco + is_ + 2])) * f32(q2))
            y[yo + l + 64] = f32(f32(d * f32(sc[sco + is_ + 4])) * f32(q3))
            y[yo + l + 96] = f32(f32(d * f32(sc[sco + is_ + 6])) * f32(q4))
        yo += 128
        qlo += 64
        qho += 32
        sco += 8
    return y


REFS = {gguf.GGML_Q4_0: ref_q4_0, gguf.GGML_Q4_K: ref_q4_k, gguf.GGML_Q5_K: ref_q5_k,
        gguf.GGML_Q6_K: ref_q6_k}


@pytest.mark.parametrize("t", sorted(REFS))
def test_vectorised_decoder_matches_ggml_loop(t):
    rng = np.random.default_rng(t)
    be, bb = gguf.BLOCKS[t]
    blocks = rng.integers(0, 256, size=(6, bb), dtype=np.uint8)   # every bit pattern of every field
    # finite scales: replace the f16 fields by random finite values, one block with extreme ones
    fields = {gguf.GGML_Q4_0: [0], gguf.GGML_Q4_K: [0, 2], gguf.GGML_Q5_K: [0, 2], gguf.GGML_Q6_K: [208]}[t]
    for o in fields:
        vals = rng.uniform(-2, 2, size=6).astype(np.float16)
        vals[0] = np.float16(65504.0) if o == fields[0] else np.float16(6e-8)
        blocks[:, o:o + 2] = vals.view(np.uint8).reshape(6, 2)
    blocks[1, :] = 0xFF  # all-ones fields (scales 63, 6-bit top bits set) with a finite scale below
    for o in fields:
        blocks[1, o:o + 2] = np.array([0.5], np.float16).view(np.uint8)
    got = gguf.dequantize(t, blocks.reshape(1, -1), (1, 6 * be))[0]
    want = np.array([v for b in blocks for v in REFS[t]([int(x) for x in b])], dtype=np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_q4_k_known_block():
    # d = 1, dmin = 0.5, sub-block j: scale j+1, min j (j < 4 stored directly; j >= 4 split fields)
    s, m = list(range(1, 9)), list(range(8))
    sc = [0] * 12
    for j in range(4):
        sc[j] = s[j] | ((s[j + 4] >> 4) << 6)
        sc[j + 4] = m[j] | ((m[j + 4] >> 4) << 6)
        sc[j + 8] = (s[j + 4] & 15) | ((m[j + 4] & 15) << 4)
    qs = [(l % 16) | ((15 - l % 16) << 4) for l in range(128)]
    b = np.frombuffer(struct.pack("<ee", 1.0, 0.5) + bytes(sc) + bytes(qs), dtype=np.uint8)
    y = gguf.dequantize_q4_k(b[None], 256)[0]
    for j in range(8):
        g, hi = j // 2, j % 2
        for l in (0, 7, 31):
            q = qs[32 * g + l] >> 4 if hi else qs[32 * g + l] & 15
            assert y[32 * j + l] == np.float32(s[j] * q - 0.5 * m[j])


@pytest.mark.parametrize("wtype", ["q4_k_m", "q5_k_m", "q4_0", "f16"])
def test_mixed_files_roundtrip(tmp_path, wtype):
    shape = synth.SHAPES["test-tiny"]
    p = str(tmp_path / f"{wtype}.gguf")
    gguf.write_synthetic_gguf(p, shape, seed=2, wtype=wtype)
    r = gguf.GGUFReader(p)
    for name in ("token_embd.weight", "output.weight", "blk.1.attn_v.weight", "blk.0.ffn_up.weight"):
        t = r.tensors[name]["type"]
        y = gguf.dequantize(t, r.tensor(name), tuple(reversed(r.tensors[name]["ne"])))
        assert y.dtype == np.float32 and np.isfinite(y).all() and 0.001 < float(np.abs(y).mean()) < 0.1
    q = str(tmp_path / f"{wtype}_bf16.gguf")
    gguf.write_synthetic_gguf(q, shape, seed=2, dequant_from=p)
    rb = gguf.GGUFReader(q)
    a = gguf.dequantize(r.tensors["blk.0.attn_q.weight"]["type"], r.tensor("blk.0.attn_q.weight"),
                        (shape.n_embd, shape.n_embd))
    assert np.array_equal(rb.tensor("blk.0.attn_q.weight"), synth.f32_to_bf16_bits(a))
