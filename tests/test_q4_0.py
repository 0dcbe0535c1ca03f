"""Q4_0 on CPU: the oracle's block format, quantiser and dot product pinned against
literal scalar transcriptions of ggml-quants.c (quantize_row_q4_0_ref, ggml_vec_dot_q4_0_q8_0's generic
loop) and against gguf.dequantize_q4_0; known-answer blocks included."""
import numpy as np
import pytest


def ggml_quantize_row_q4_0_ref(x):
    """ggml-quants.c quantize_row_q4_0_ref, statement by statement (f32 arithmetic)."""
    x = np.asarray(x, np.float32)
    out = bytearray()
    for b in range(x.size // 32):
        xb = x[32 * b:32 * b + 32]
        amax, mx = np.float32(0.0), np.float32(0.0)
        for v in xb:
            if amax < abs(v):
                amax, mx = np.float32(abs(v)), v
        d = np.float32(mx / np.float32(-8))
        idv = np.float32(np.float32(1.0) / d) if d != 0 else np.float32(0.0)
        out += np.float16(d).tobytes()
        for j in range(16):
            x0 = np.float32(xb[j] * idv)
            x1 = np.float32(xb[16 + j] * idv)
            xi0 = min(15, int(np.trunc(np.float32(x0 + np.float32(8.5)))))
            xi1 = min(15, int(np.trunc(np.float32(x1 + np.float32(8.5)))))
            out.append(xi0 | (xi1 << 4))
    return np.frombuffer(bytes(out), np.uint8)


def ggml_quantize_row_q8_0(x):
    """The activation side (ggml quantize_row_q8_0, AVX2/NEON rounding: round half to even)."""
    x = np.asarray(x, np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1)
    d = (amax / np.float32(127)).astype(np.float32)
    idv = np.where(d != 0, np.float32(1) / np.where(d != 0, d, 1), 0).astype(np.float32)
    q = np.rint((x * idv[:, None]).astype(np.float32)).astype(np.int8)
    return q, d.astype(np.float16).astype(np.float32)


def ggml_vec_dot_q4_0_q8_0(blocks, x):
    """ggml_vec_dot_q4_0_q8_0, generic loop: int sums per block, sumf += sumi * (d_w * d_x)."""
    q8, dx = ggml_quantize_row_q8_0(x)
    blocks = np.asarray(blocks, np.uint8).reshape(-1, 18)
    s = np.float32(0)
    for b in range(blocks.shape[0]):
        d = np.frombuffer(blocks[b, :2].tobytes(), np.float16)[0].astype(np.float32)
        qs = blocks[b, 2:]
        sumi = 0
        for j in range(16):
            sumi += (int(qs[j] & 15) - 8) * int(q8[b][j])
            sumi += (int(qs[j] >> 4) - 8) * int(q8[b][16 + j])
        s = np.float32(s + np.float32(np.float32(d * dx[b]) * np.float32(sumi)))
    return float(s)


@pytest.fixture(scope="module")
def orc(oracle_mod):
    return oracle_mod


def test_q4_0_quantiser_matches_ggml_transcription(orc):
    rng = np.random.default_rng(0)
    for scale in (0.02, 1.0, 300.0):
        x = (rng.standard_normal(32 * 24) * scale).astype(np.float32)
        x[5] = -np.abs(x).max() * 1.5  # a negative maximum: d = max / -8 > 0
        assert np.array_equal(orc.q4_0_quantize_row(x), ggml_quantize_row_q4_0_ref(x))
    z = np.zeros(64, np.float32)  # all-zero blocks: d = 0, every nibble 8
    b = orc.q4_0_quantize_row(z)
    assert np.array_equal(b, ggml_quantize_row_q4_0_ref(z))
    assert np.all(b.reshape(2, 18)[:, 2:] == 0x88)


def test_q4_0_known_answer_block(orc):
    # x = 0..31 - 16: max |x| = 16 at x[0] = -16 -> d = 2, id = 0.5, q = trunc(x/2 + 8.5)
    x = np.arange(32, dtype=np.float32) - 16
    b = orc.q4_0_quantize_row(x)
    assert np.frombuffer(b[:2].tobytes(), np.float16)[0] == 2.0
    q = [min(15, int(v / 2 + 8.5)) for v in x]
    assert list(b[2:]) == [q[j] | (q[16 + j] << 4) for j in range(16)]


def test_q4_0_dot_and_dequant(orc):
    from llama_p2p_amd.gguf import dequantize_q4_0

    rng = np.random.default_rng(1)
    w = (rng.standard_normal(32 * 16) * 0.05).astype(np.float32)
    blocks = orc.q4_0_quantize_row(w)
    for _ in range(5):
        x = (rng.standard_normal(w.size) * rng.uniform(0.1, 10)).astype(np.float32)
        assert orc.q4_0_vec_dot(blocks, x) == ggml_vec_dot_q4_0_q8_0(blocks, x)
    deq = dequantize_q4_0(blocks.reshape(1, -1), w.size).reshape(-1)
    bl = blocks.reshape(-1, 18)
    d = np.frombuffer(bl[:, :2].tobytes(), np.float16).astype(np.float32)
    ref = np.concatenate([np.concatenate([(bl[i, 2:] & 15).astype(np.float32) - 8,
                                          (bl[i, 2:] >> 4).astype(np.float32) - 8]) * d[i] for i in range(len(bl))])
    assert np.array_equal(deq, ref)
    assert np.abs(deq - w).max() <= np.abs(w).max() / 8 + 1e-6  # within one step of the 4-bit grid


def test_numpy_q4_0_quantiser_equals_oracle(orc):
    """gguf.quantize_q4_0 (vectorised, writes the synthetic q4_0 GGUF) == the oracle's quantiser."""
    from llama_p2p_amd.gguf import quantize_q4_0

    rng = np.random.default_rng(2)
    x = (rng.standard_normal((7, 32 * 8)) * 0.03).astype(np.float32)
    x[3, 40] = -1.0
    got = quantize_q4_0(x)
    for r in range(x.shape[0]):
        assert np.array_equal(got[r], orc.q4_0_quantize_row(x[r]))
