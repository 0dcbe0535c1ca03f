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


# ------------------------------------------------------------------------------------------------
# Native K-quant arithmetic (the engine's kquant.hip path, oracle/llama_oracle.c vec_dot_kq):
# literal scalar transcriptions of ggml-quants.c's quantize_row_q8_K_ref and the generic
# ggml_vec_dot_q{4,5,6}_K_q8_K loops, checked bit for bit against the C oracle.  (ggml itself is
# absent offline, so these transcriptions -- not golden outputs of llama.cpp -- pin the restatement.)
# ------------------------------------------------------------------------------------------------
def ref_nearest_int(fval):
    val = f32(f32(fval) + f32(12582912.0))
    i = int(np.array([val], np.float32).view(np.int32)[0])
    return (i & 0x007FFFFF) - 0x00400000


def ref_quantize_q8_k(x):
    """quantize_row_q8_K_ref: blocks of (d, qs[256], bsums[16])"""
    out = []
    for i in range(0, len(x), 256):
        xb = [f32(v) for v in x[i:i + 256]]
        mx, amax = f32(0), f32(0)
        for v in xb:
            if abs(v) > amax:
                amax, mx = f32(abs(v)), v
        if not amax:
            out.append((f32(0), [0] * 256, [0] * 16))
            continue
        iscale = f32(f32(-127.0) / mx)
        qs = [min(127, ref_nearest_int(f32(iscale * v))) for v in xb]
        bs = [sum(qs[16 * j:16 * j + 16]) for j in range(16)]
        out.append((f32(f32(1) / iscale), qs, bs))
    return out


def _kq_ints(t, b):
    """integer values (Q6_K: minus 32) of one block in k order, via the dequantisers' own loops"""
    if t == gguf.GGML_Q6_K:
        ql, qh, v = b[0:128], b[128:192], [0] * 256
        for h in range(2):
            for l in range(32):
                L0, L1, H = ql[64 * h + l], ql[64 * h + 32 + l], qh[32 * h + l]
                v[128 * h + l] = ((L0 & 15) | (((H >> 0) & 3) << 4)) - 32
                v[128 * h + 32 + l] = ((L1 & 15) | (((H >> 2) & 3) << 4)) - 32
                v[128 * h + 64 + l] = ((L0 >> 4) | (((H >> 4) & 3) << 4)) - 32
                v[128 * h + 96 + l] = ((L1 >> 4) | (((H >> 6) & 3) << 4)) - 32
        return v
    q5 = t == gguf.GGML_Q5_K
    qh, qs, v = b[16:48], b[48:176] if q5 else b[16:144], [0] * 256
    for g in range(4):
        for l in range(32):
            v[64 * g + l] = (qs[32 * g + l] & 15) + (16 if q5 and qh[l] & (1 << (2 * g)) else 0)
            v[64 * g + 32 + l] = (qs[32 * g + l] >> 4) + (16 if q5 and qh[l] & (2 << (2 * g)) else 0)
    return v


def ref_vec_dot(t, blocks, x):
    """ggml_vec_dot_q{4,5,6}_K_q8_K, generic (scalar) form"""
    y = ref_quantize_q8_k(x)
    sums, sumf = [f32(0)] * 8, f32(0)
    bb = gguf.BLOCKS[t][1]
    for i, (yd, q8, bsums) in enumerate(y):
        b = [int(c) for c in blocks[i * bb:(i + 1) * bb]]
        a = _kq_ints(t, b)
        aux32 = [0] * 8
        if t == gguf.GGML_Q6_K:
            sc = list(np.frombuffer(bytes(b[192:208]), dtype=np.int8))
            for j in range(16):
                for half in range(2):
                    for l in range(8):
                        aux32[l] += int(sc[j]) * (q8[16 * j + 8 * half + l] * a[16 * j + 8 * half + l])
            d = f32(_h(b, 208) * yd)
            sums = [f32(sums[l] + f32(d * f32(aux32[l]))) for l in range(8)]
        else:
            scm = [get_scale_min_k4(j, b[4:16]) for j in range(8)]
            sumi = sum(bsums[j] * scm[j // 2][1] for j in range(16))
            for j in range(8):
                for quarter in range(4):
                    for l in range(8):
                        aux32[l] += scm[j][0] * (q8[32 * j + 8 * quarter + l] * a[32 * j + 8 * quarter + l])
            d = f32(_h(b, 0) * yd)
            sums = [f32(sums[l] + f32(d * f32(aux32[l]))) for l in range(8)]
            dmin = f32(_h(b, 2) * yd)
            sumf = f32(sumf - f32(dmin * f32(sumi)))
    for l in range(8):
        sumf = f32(sumf + sums[l])
    return sumf


KQ_TYPES = [gguf.GGML_Q4_K, gguf.GGML_Q5_K, gguf.GGML_Q6_K]


def test_q8_k_quantisation_matches_ggml_loop(oracle_mod):
    rng = np.random.default_rng(7)
    x = rng.normal(0, 1.3, 768).astype(np.float32)
    x[256:512] = 0.0                        # an all-zero super-block (d = 0)
    x[600] = -np.abs(x[512:768]).max() * 2  # the signed max is negative in the last block
    x[700] = -x[600]                        # ... and tied in magnitude by a later positive value
    qs, d, bs = oracle_mod.kq_quantize_q8k(x)
    for i, (rd, rq, rb) in enumerate(ref_quantize_q8_k(x)):
        assert np.float32(d[i]).view(np.uint32) == np.float32(rd).view(np.uint32)
        assert qs[256 * i:256 * i + 256].tolist() == rq
        assert bs[16 * i:16 * i + 16].tolist() == rb
    assert d[2] > 0  # first max is the negative one: iscale = -127/max > 0, so d > 0


@pytest.mark.parametrize("t", KQ_TYPES)
def test_vec_dot_matches_ggml_loop(oracle_mod, t):
    rng = np.random.default_rng(t)
    blocks = synth.kq_blocks(t, 3, seed=4, tid=77).reshape(-1)
    x = rng.normal(0, 1.0, 768).astype(np.float32)
    got = oracle_mod.kq_vec_dot(t, blocks, x)
    want = ref_vec_dot(t, blocks, x)
    assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (got, want)
    # and it approximates the real-valued product (Q8_K rounds x to ~1/254 of each block's max)
    w = oracle_mod.kq_dequant(t, blocks, 768)
    exact = float(np.dot(w.astype(np.float64), x.astype(np.float64)))
    assert abs(got - exact) <= 0.02 * np.abs(w).sum() * np.abs(x).max() / 127 + 1e-6


@pytest.mark.parametrize("t", KQ_TYPES)
def test_kq_dequant_matches_ggml_loop(oracle_mod, t):
    blocks = synth.kq_blocks(t, 4, seed=1, tid=5)
    got = oracle_mod.kq_dequant(t, blocks.reshape(-1), 1024)
    want = np.array([v for b in blocks for v in REFS[t]([int(c) for c in b])], np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("t", KQ_TYPES)
def test_synthetic_blocks_host_equals_oracle(oracle_mod, t):
    a = synth.kq_blocks(t, 101, seed=3, tid=synth.layer_tid(5, synth.L_DOWN))
    b = oracle_mod.kq_synth_blocks(t, 101, 3, synth.layer_tid(5, synth.L_DOWN))
    assert np.array_equal(a, b)
    w = gguf.dequantize(t, a.reshape(1, -1), (1, 101 * 256))
    assert np.isfinite(w).all() and 0.005 < float(w.std()) < 0.08


def test_q4_k_m_recipe_types():
    # llama.cpp Q4_K_M: output Q6_K, attn_v / ffn_down Q6_K on use_more_bits layers, 70B attn_v Q5_K
    more = [l for l in range(32) if synth.use_more_bits(l, 32)]
    assert more == [0, 1, 2, 3, 6, 9, 12, 15, 18, 21, 24, 27, 28, 29, 30, 31]
    assert synth.kq_tensor_type("q4_k_m", "output", 0, 32) == gguf.GGML_Q6_K
    assert synth.kq_tensor_type("q4_k_m", "attn_v", 4, 32) == gguf.GGML_Q4_K
    assert synth.kq_tensor_type("q4_k_m", "attn_v", 6, 32) == gguf.GGML_Q6_K
    assert synth.kq_tensor_type("q4_k_m", "ffn_down", 31, 32) == gguf.GGML_Q6_K
    assert synth.kq_tensor_type("q4_k_m", "attn_v", 40, 80) == gguf.GGML_Q5_K
    assert synth.kq_tensor_type("q5_k_m", "ffn_gate", 40, 80) == gguf.GGML_Q5_K
    # Llama-3-8B Q4_K_M streams ~4.6 GB per token (SURVEY §8d bytes: 15.0 GB in bf16)
    assert 4.5e9 < synth.kq_weight_bytes_per_token(synth.SHAPES["llama3-8b"], "q4_k_m") < 4.8e9


@pytest.mark.parametrize("wtype", ["q4_k_m", "q5_k_m"])
def test_kq_gguf_file_holds_synthetic_blocks(tmp_path, wtype):
    shape = synth.SHAPES["test-tiny"]
    p = str(tmp_path / f"{wtype}.gguf")
    gguf.write_synthetic_gguf(p, shape, seed=9, wtype=wtype)
    r = gguf.GGUFReader(p)
    for name, kind, layer in (("blk.1.attn_v.weight", "attn_v", 1), ("blk.0.ffn_down.weight", "ffn_down", 0),
                              ("output.weight", "output", 0), ("token_embd.weight", "token_embd", 0)):
        t, blocks = synth.kq_tensor(wtype, kind, layer, shape, 9)
        assert r.tensors[name]["type"] == t
        assert np.array_equal(np.frombuffer(r.tensor(name).tobytes(), np.uint8), blocks.reshape(-1))
