"""The CPU oracle against the golden vectors (CPU-only).

Pinning: llama.cpp (the reference's arithmetic) is absent, so the oracle is
checked against transformers' LlamaForCausalLM run over the same bf16 weights
(tests/golden/hf_*.npz, made by tests/golden/make_golden.py):
  * ORC_EXACT mode (fp32 math)      must match HF to 5e-5 of the logit scale;
  * ggml mode (bf16/f16 roundings)  must match within the bf16 tolerance.
"""
import numpy as np
import pytest

from conftest import assert_logits_close

SHAPES = ["test-tiny", "test-gqa8", "test-d128", "test-h4096"]


def _golden(name):
    import os

    return np.load(os.path.join(os.path.dirname(__file__), "golden", f"hf_{name}.npz"))


@pytest.mark.parametrize("name", SHAPES)
def test_oracle_exact_matches_transformers(oracle_mod, name):
    from llama_p2p_amd import synth

    g = _golden(name)
    m = oracle_mod.OracleModel(synth.SHAPES[name], seed=int(g["seed"]), exact=True)
    got = m.context(64).eval(g["ids"], 0, all_logits=True)
    ref = g["logits"]
    assert np.abs(got - ref).max() < 5e-5 * np.abs(ref).max()


@pytest.mark.parametrize("name", SHAPES)
def test_oracle_ggml_mode_within_bf16_tolerance(oracle_mod, name):
    from llama_p2p_amd import synth

    g = _golden(name)
    m = oracle_mod.OracleModel(synth.SHAPES[name], seed=int(g["seed"]))
    got = m.context(64).eval(g["ids"], 0, all_logits=True)
    assert_logits_close(got, g["logits"], name)


def test_oracle_incremental_equals_batched(oracle_mod):
    """KV-cache path: token-by-token evaluation == one batched prefill (same ubatch semantics)."""
    from llama_p2p_amd import synth

    sh = synth.SHAPES["test-gqa8"]
    g = _golden("test-gqa8")
    m = oracle_mod.OracleModel(sh, seed=0)
    full = m.context(64).eval(g["ids"][:12], 0, all_logits=True)
    c = m.context(64)
    inc = np.stack([c.eval(g["ids"][i:i + 1], i)[0] for i in range(12)])
    assert np.abs(full - inc).max() < 1e-5


def test_synthetic_weights_bit_identical_numpy_vs_c(oracle_mod):
    from llama_p2p_amd import synth

    L = oracle_mod.lib()
    sc = float(synth._std_scale(0.02))
    for tid in (1, 17, 12345):
        idx = np.array([0, 1, 2, 1000, 2 ** 33 + 7, 2 ** 40 + 3], dtype=np.uint64)
        ref = np.array([L.orc_synth_value(0, tid, int(i), sc) for i in idx], dtype=np.float32)
        got = np.array([synth.synth_values(0, tid, int(i), 1, 0.02)[0] for i in idx], dtype=np.float32)
        assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))


def test_synthetic_weight_statistics():
    from llama_p2p_amd import synth

    v = synth.synth_values(0, 3, 0, 1 << 20, 0.02)
    assert abs(v.mean()) < 1e-4 and abs(v.std() - 0.02) < 2e-4
    n = synth.synth_norm_f32(0, 2, 4096)
    assert abs(n.mean() - 1.0) < 0.01


def test_f16_rounding_matches_numpy(oracle_mod):
    L = oracle_mod.lib()
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.normal(0, 1, 2000), rng.normal(0, 1e-5, 500), [65504.0, 65520.0, 1e-8, -0.0, 6.1e-5]])
    for v in vals.astype(np.float32):
        assert np.float32(L.orc_round_f16(float(v))) == np.float32(np.float16(v)), v


def test_bf16_rounding_matches_spec(oracle_mod):
    from llama_p2p_amd import synth

    L = oracle_mod.lib()
    rng = np.random.default_rng(1)
    vals = rng.normal(0, 3, 1000).astype(np.float32)
    ref = synth.bf16_bits_to_f32(synth.f32_to_bf16_bits(vals))
    got = np.array([L.orc_round_bf16(float(v)) for v in vals], dtype=np.float32)
    assert np.array_equal(ref, got)


def test_greedy_tie_breaks_to_lowest_id(oracle_mod):
    assert oracle_mod.argmax_lowest(np.array([0.0, 2.0, 1.0, 2.0], dtype=np.float32)) == 1


def test_context_overflow_rejected(oracle_mod):
    from llama_p2p_amd import synth

    m = oracle_mod.OracleModel(synth.SHAPES["test-tiny"], seed=0)
    with pytest.raises(ValueError):
        m.context(8).eval(list(range(3, 12)), 0)


@pytest.mark.parametrize("case", ["llama3", "linear"])
def test_oracle_rope_scaling_matches_transformers(oracle_mod, case):
    """RoPE frequency factors (GGUF rope_freqs.weight, Llama-3.1) and linear scaling: the oracle with
    the fixture's factors / freq_scale matches transformers' "llama3" / "linear" rope types; without
    them the logits are clearly different (the scaling reaches the positions used)."""
    from llama_p2p_amd import synth

    g = _golden(f"test-tiny_rope_{case}")
    sh = synth.SHAPES["test-tiny"]
    m = oracle_mod.OracleModel(sh, seed=int(g["seed"]), exact=True)
    plain = m.context(64).eval(g["ids"], 0, all_logits=True)
    m.set_rope(g["rope_ff"] if case == "llama3" else None, float(g["freq_scale"]))
    got = m.context(64).eval(g["ids"], 0, all_logits=True)
    ref = g["logits"]
    assert np.abs(got - ref).max() < 5e-5 * np.abs(ref).max()
    assert np.abs(plain - ref).max() > 100 * np.abs(got - ref).max()
    # unit factors and scale 1 are the identity, bit for bit
    m.set_rope(np.ones(sh.head_dim // 2, np.float32), 1.0)
    assert np.array_equal(m.context(64).eval(g["ids"], 0, all_logits=True), plain)


@pytest.mark.parametrize("name", ["test-gqa8", "test-d128"])
def test_per_layer_hook_equals_eval(oracle_mod, name):
    """orc_layers (the per-layer parity hook) composes to orc_eval bit for bit: the embedding, every
    layer as its own call on the previous call's residual stream, then the head -- for a prompt and
    for a decode token that reads the K/V the per-layer calls wrote."""
    from llama_p2p_amd import synth

    sh = synth.SHAPES[name]
    m = oracle_mod.OracleModel(sh, seed=0)
    ids = np.random.default_rng(4).integers(3, sh.n_vocab, 11).astype(np.int32)
    ref = m.context(32).eval(ids, 0, all_logits=True)
    c = m.context(32)
    for a, b in ((0, 10), (10, 11)):
        x = c.layers(None, a, 0, 0, ids=ids[a:b])
        for l in range(sh.n_layer):
            x = c.layers(x, a, l, l + 1)
        _, lg = c.layers(x, a, sh.n_layer, sh.n_layer, logits=True)
        assert np.array_equal(lg, ref[a:b])
    with pytest.raises(ValueError):
        c.layers(x, 0, 0, sh.n_layer + 1)


def test_layer_range_synthesis_equals_whole_model(oracle_mod):
    """orc_fill_synthetic_layers (the 70B per-layer GPU test's oracle) fills exactly what the whole-model
    fill does for its layers: one layer on the same input gives the same bits, and the head too."""
    from llama_p2p_amd import synth

    sh = synth.SHAPES["test-tiny"]
    whole = oracle_mod.OracleModel(sh, seed=3)
    part = oracle_mod.OracleModel(sh, seed=None)
    last = sh.n_layer - 1
    part.fill_synthetic_layers(3, 1, 2, globals_=False)
    part.fill_synthetic_layers(3, last, last + 1, globals_=True)
    x = np.random.default_rng(0).normal(0, 0.5, (5, sh.n_embd)).astype(np.float32)
    for l, head in ((1, False), (last, True)):
        a, b = whole.context(16), part.context(16)
        ra, rb = a.layers(x, 0, l, l + 1, logits=head), b.layers(x, 0, l, l + 1, logits=head)
        for u, v in zip(ra if head else [ra], rb if head else [rb]):
            assert np.array_equal(u, v)
        a.close()
        b.close()
    whole.close()
    part.close()
