"""Native Q4_0 on the GPU: Q4 tiles (csrc/kernels.hip q4_place / q4_operand) on the Q8_0
path -- Q8_0 activation rows and v_mfma_i32_16x16x32_i8, i.e. ggml_vec_dot_q4_0_q8_0 -- against the CPU
oracle's restatement (matmul_q4_0, pinned in tests/test_q4_0.py), for the synthetic q4_0 model
(quantize_row_q4_0_ref of the bf16 weights, Q8_0 token_embd / output) and for a Q4_0 GGUF as
llama-quantize writes it (Q4_0 matrices and token_embd, Q6_K output on the K-quant head).
Tolerance as tests/test_q8_gpu.py: the bf16 one, and 2x the oracle's own deviation under 1e-6 relative
activation noise (the Q8_0 rounding of the activations is discontinuous in its inputs)."""
import numpy as np
import pytest

from conftest import assert_logits_close, assert_tokens_match, check_chain_batched

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    from llama_p2p_amd import engine

    engine.lib()
    return engine


def _seq(shape, n, seed=7):
    rng = np.random.default_rng(seed)
    return np.concatenate([[1], rng.integers(3, shape.n_vocab, n - 1)]).astype(np.int32)


def _oracle_q4(oracle_mod, shape, seed):
    om = oracle_mod.OracleModel(shape, seed=seed)
    om.quantize_q4_0()
    return om


def _tokens_decided(got, ref, dev, what):
    """Greedy argmax identical wherever the oracle's top-1/top-2 gap exceeds twice the larger of the bf16
    tolerance and twice the oracle's own deviation under noise."""
    srt = np.sort(ref, axis=-1)
    gap = srt[:, -1] - srt[:, -2]
    bar = 2 * np.maximum(1e-2 * np.abs(srt[:, -1]) + 2e-2 * np.abs(ref).max(), 2 * dev)
    bad = (gap > bar) & (got.argmax(-1) != ref.argmax(-1))
    assert not bad.any(), f"{what}: argmax differs at decided rows {np.nonzero(bad)[0].tolist()}"


def _bounded(oracle_mod, make, ids, got, ref, what):
    err = np.abs(got - ref).max()
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = make().context(256).eval(ids, 0, all_logits=True)
    finally:
        oracle_mod.q8_jitter(0.0)
    self_dev = np.abs(jit - ref).max()
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (what, err, self_dev)
    return err, self_dev


@pytest.mark.parametrize("name", ["test-tiny", "test-d128", "test-h4096"])
def test_q4_0_prefill_and_decode_vs_oracle(mx, oracle_mod, name):
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, 112, seed=5)
    eng = mx.Engine(f"synthetic:{name}:seed=0:q4_0", n_ctx=256, n_seq_max=2)
    assert eng.info.weight_type == 2
    octx = _oracle_q4(oracle_mod, shape, 0).context(256)
    got = eng.forward_logits(ids[:100], 0, slot=1)
    ref = octx.eval(ids[:100], 0, all_logits=True)
    # the jitter bound first: Q8_0 activation rounding makes ordering-level differences discontinuous
    err, dev = _bounded(oracle_mod, lambda: _oracle_q4(oracle_mod, shape, 0), ids[:100], got, ref, name)
    _tokens_decided(got, ref, dev, f"{name} q4_0 prefill")
    gs, rs = [], []
    for p in range(100, 112):  # one-token steps: the quantise-on-load GEMVs
        gs.append(eng.forward_logits(ids[p:p + 1], p, slot=1)[0])
        rs.append(octx.eval(ids[p:p + 1], p)[0])
    gs, rs = np.stack(gs), np.stack(rs)
    _tokens_decided(gs, rs, dev, f"{name} q4_0 decode")
    inside = int((np.abs(got - ref) <= 1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max()).all(axis=1).sum())
    print(f"{name}: q4_0 prefill max|d| {err:.3g} (oracle under 1e-6 noise {dev:.3g}; {inside}/100 rows inside "
          f"the bf16 tolerance), decode max|d| {np.abs(gs - rs).max():.3g} (max|ref| {np.abs(ref).max():.3g})")
    assert np.abs(gs - rs).max() <= 2 * dev + 1e-4 * np.abs(ref).max()
    eng.close()


@pytest.mark.parametrize("P", [300, 520])
def test_q4_0_gemm_prefill_vs_oracle(mx, oracle_mod, P):
    """A >= 256-row Q4_0 prompt chunk on q8gemm_kernel's Q4 form (ggml_vec_dot_q4_0_q8_0: nibbles
    expanded to q - 8 in registers, per-block int32 products on the int8 MFMA): at 300 rows q|k|v
    only, at 520 all four matrices; the next 8 rows against the oracle under the jitter bound."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES["test-h4096"]
    ids = _seq(shape, P + 8, seed=11)
    eng = mx.Engine("synthetic:test-h4096:seed=0:q4_0", n_ctx=544, n_seq_max=2)
    assert eng.forward_rows([0] * P, list(range(P)), ids[:P], want_logits=False) is None
    got = eng.forward_logits(ids[P:], P, slot=0)
    ref = _oracle_q4(oracle_mod, shape, 0).context(544).eval(ids, 0, all_logits=True)[P:]
    err = np.abs(got - ref).max()
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = _oracle_q4(oracle_mod, shape, 0).context(544).eval(ids, 0, all_logits=True)[P:]
    finally:
        oracle_mod.q8_jitter(0.0)
    dev = np.abs(jit - ref).max()
    assert err <= 2 * dev + 1e-4 * np.abs(ref).max(), (err, dev)
    _tokens_decided(got, ref, dev, f"q4_0 gemm prefill P={P}")
    eng.close()


def test_q4_0_gguf_equals_synthetic(mx, tmp_path):
    """The synthetic q4_0 model written as a GGUF by numpy (gguf.quantize_q4_0 == the oracle's quantiser,
    tests/test_q4_0.py) and synthesised on the device (synth_q4_packed_kernel) give bit-identical logits:
    the device quantiser reproduces ggml's quantize_row_q4_0_ref bit for bit, and pack_q4_kernel places
    a file's blocks as the synthesis does."""
    from llama_p2p_amd import gguf, synth

    shape = synth.SHAPES["test-tiny"]
    path = str(tmp_path / "tiny_q4_0.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype="q4_0_synth")
    ids = _seq(shape, 24)
    a = mx.Engine(path, n_ctx=64, n_seq_max=2)
    b = mx.Engine("synthetic:test-tiny:seed=3:q4_0", n_ctx=64, n_seq_max=2)
    assert a.info.weight_type == 2 and b.info.weight_type == 2
    assert np.array_equal(a.forward_logits(ids), b.forward_logits(ids))
    a.close()
    b.close()


def test_q4_0_wide_rows_and_greedy_loop(mx, oracle_mod):
    """24 and 32 distinct sequences in one forward (the LDS-shared 17-32-row kernels and split-K slabs),
    then the device greedy loop at 32 rows, against the oracle."""
    from llama_p2p_amd import synth

    name = "test-h4096"
    shape = synth.SHAPES[name]
    eng = mx.Engine(f"synthetic:{name}:seed=0:q4_0", n_ctx=128, n_seq_max=32)
    om = _oracle_q4(oracle_mod, shape, 0)
    rng = np.random.default_rng(3)
    prompts = [_seq(shape, int(rng.integers(3, 12)), seed=100 + i) for i in range(32)]
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    got = eng.forward_rows(list(range(32)), [len(p) - 1 for p in prompts], [int(p[-1]) for p in prompts])
    refs = np.stack([om.context(128).eval(p, 0)[0] for p in prompts])
    assert_logits_close(got, refs, "q4_0 32 rows")
    assert_tokens_match(got, refs, "q4_0 32 rows")
    first = [int(np.argmax(g)) for g in got]
    b = eng.batch(list(range(32)), [len(p) for p in prompts], first, max_steps=4)
    for _ in range(4):
        b.step()
    toks = b.tokens()
    b.close()
    exact = 0
    for i, p in enumerate(prompts):
        e, _ = check_chain_batched(om.context(128), p, [first[i]] + toks[i].tolist(), f"q4_0 seq {i}")
        exact += e
    assert exact >= 0.85 * 32 * 5
    eng.close()


def test_q4_0_gguf_llama_quantize_layout(mx, oracle_mod, tmp_path):
    """A Q4_0 file as llama-quantize writes it: Q4_0 matrices and token_embd, Q6_K output.  The matrices
    run on Q4 tiles, the head on the K-quant kernels (Q8_K activations), the embedding as a bf16 table of
    the dequantised rows; the oracle gets the same blocks."""
    from llama_p2p_amd import gguf, synth

    shape = synth.SHAPES["test-d128"]
    path = str(tmp_path / "q4_0.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=6, wtype="q4_0")
    eng = mx.Engine(path, n_ctx=64, n_seq_max=2)
    assert eng.info.weight_type == 2
    ids = _seq(shape, 40, seed=11)
    got = eng.forward_logits(ids)
    eng.close()
    r = gguf.GGUFReader(path)
    kinds = {"attn_q": 1, "attn_k": 2, "attn_v": 3, "attn_output": 4, "ffn_gate": 6, "ffn_up": 7, "ffn_down": 8}
    om = oracle_mod.OracleModel(shape, seed=None)
    for name, info in r.tensors.items():
        raw = np.ascontiguousarray(r.tensor(name))
        if name == "token_embd.weight":
            emb = gguf.dequantize(info["type"], raw, (shape.n_vocab, shape.n_embd))
            om.set_tensor(-1, 1, synth.f32_to_bf16_bits(emb))
        elif name == "output_norm.weight":
            om.set_tensor(-1, 2, raw)
        elif name == "output.weight":
            assert info["type"] == gguf.GGML_Q6_K
            om.set_tensor_kq(-1, 3, gguf.GGML_Q6_K, raw)
        else:
            _, l, kind, _ = name.split(".")
            if kind in ("attn_norm", "ffn_norm"):
                om.set_tensor(int(l), {"attn_norm": 0, "ffn_norm": 5}[kind], raw)
            else:
                assert info["type"] == gguf.GGML_Q4_0
                om.set_tensor_q4_0(int(l), kinds[kind], raw)
    ref = om.context(64).eval(ids, 0, all_logits=True)
    assert_logits_close(got, ref, "q4_0 gguf")
    assert_tokens_match(got, ref, "q4_0 gguf")
