"""Quantised GGUF files on the GPU.

Native K-quants (Q4_K_M / Q5_K_M: Q4_K, Q5_K, Q6_K matrices; csrc/kquant.hip): int8 MFMA over packed
K-quant tiles with Q8_K activations, against the CPU oracle's restatement of ggml's
quantize_row_q8_K + ggml_vec_dot_q{4,5,6}_K_q8_K (pinned to scalar transcriptions of ggml's loops in
tests/test_kquants.py) for every row regime, the device greedy loop, the GGUF loader against on-device
synthesis, and Llama-3-8B Q4_K_M at full size.  Tolerance as tests/test_q8_gpu.py: the bf16 one, and
2x the oracle's own deviation under 1e-6 relative input noise (Q8_K rounding is discontinuous).

Other block types (F16 files, mixes without a native path): the engine dequantises every matrix at load
(dequant_bf16_kernel) and runs the bf16 path -- bit-identical to a BF16 file holding numpy's
dequantisation of the same blocks, and close to the CPU oracle built from those bf16 weights.  (Q4_0
files run natively: tests/test_q4_0_gpu.py.)"""
import os

import numpy as np
import pytest

from conftest import assert_logits_close, assert_tokens_match

pytestmark = pytest.mark.gpu

KINDS = {"attn_norm": 0, "attn_q": 1, "attn_k": 2, "attn_v": 3, "attn_output": 4, "ffn_norm": 5, "ffn_gate": 6,
         "ffn_up": 7, "ffn_down": 8}


def _oracle_from_gguf(oracle_mod, path, shape):
    from llama_p2p_amd import gguf

    r = gguf.GGUFReader(path)
    om = oracle_mod.OracleModel(shape, seed=None)
    for name in r.tensors:
        arr = np.ascontiguousarray(r.tensor(name))
        if name == "token_embd.weight":
            om.set_tensor(-1, 1, arr)
        elif name == "output_norm.weight":
            om.set_tensor(-1, 2, arr)
        elif name == "output.weight":
            om.set_tensor(-1, 3, arr)
        else:
            _, l, kind, _ = name.split(".")
            om.set_tensor(int(l), KINDS[kind], arr)
    return om


@pytest.mark.parametrize("wtype", ["f16"])
def test_dequantised_file_equals_bf16_file_and_oracle(oracle_mod, tmp_path, wtype):
    from llama_p2p_amd import engine, gguf, synth

    shape = synth.SHAPES["test-d128"]
    p = str(tmp_path / f"{wtype}.gguf")
    q = str(tmp_path / f"{wtype}_bf16.gguf")
    gguf.write_synthetic_gguf(p, shape, seed=6, wtype=wtype)
    gguf.write_synthetic_gguf(q, shape, seed=6, dequant_from=p)
    rng = np.random.default_rng(11)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, 39)]).astype(np.int32)
    a = engine.Engine(p, n_ctx=64, n_seq_max=2)
    b = engine.Engine(q, n_ctx=64, n_seq_max=2)
    assert a.info.weight_type == 30 and b.info.weight_type == 30
    la, lb = a.forward_logits(ids), b.forward_logits(ids)
    assert np.array_equal(la, lb)
    ref = _oracle_from_gguf(oracle_mod, q, shape).context(64).eval(ids, 0, all_logits=True)
    assert_logits_close(la, ref, wtype)
    assert_tokens_match(la, ref, wtype)
    a.close()
    b.close()


# ------------------------------------------------------------------------------------ native K-quants
@pytest.fixture(scope="module")
def mx():
    from llama_p2p_amd import engine

    engine.lib()
    return engine


def _seq(shape, n, seed=7):
    rng = np.random.default_rng(seed)
    return np.concatenate([[1], rng.integers(3, shape.n_vocab, n - 1)]).astype(np.int32)


def _oracle_kq(oracle_mod, shape, seed, ftype):
    om = oracle_mod.OracleModel(shape, seed=seed)
    om.kq_synthetic(ftype, seed)
    return om


@pytest.mark.parametrize("ftype", ["q4_k_m", "q5_k_m"])
def test_kq_gguf_equals_synthetic(mx, tmp_path, ftype):
    """A Q4_K_M / Q5_K_M GGUF (synth.kq_tensor blocks, C++ parser, pack_kq_kernel) and the on-device
    synthesis of the same model give bit-identical logits; the info reports the K-quant type."""
    from llama_p2p_amd import gguf, synth

    shape = synth.SHAPES["test-tiny"]
    path = str(tmp_path / f"tiny_{ftype}.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype=ftype)
    ids = _seq(shape, 24)
    a = mx.Engine(path, n_ctx=64, n_seq_max=2)
    b = mx.Engine(f"synthetic:test-tiny:seed=3:{ftype}", n_ctx=64, n_seq_max=2)
    t = synth.KQ_FTYPES[ftype]
    assert a.info.weight_type == t and b.info.weight_type == t
    la, lb = a.forward_logits(ids), b.forward_logits(ids)
    assert np.array_equal(la, lb)
    a.close()
    b.close()


@pytest.mark.parametrize("embd", ["q8_0", "f16"])
def test_kq_gguf_with_other_token_embd_type(mx, oracle_mod, tmp_path, embd):
    """A Q4_K_M file whose token_embd is Q8_0 or F16 (llama-quantize --token-embedding-type) loads on
    the native K-quant path: Q8_0 rows are dequantised per lookup (ggml GET_ROWS), other types become a
    bf16 table once.  Q8_0: logits vs the oracle with the same Q8_0 embedding; F16: vs the oracle with
    the bf16 rounding of those f16 values (the table the engine keeps)."""
    from llama_p2p_amd import gguf, synth

    shape = synth.SHAPES["test-tiny"]
    t = {"q8_0": gguf.GGML_Q8_0, "f16": gguf.GGML_F16}[embd]
    path = str(tmp_path / f"tiny_q4_k_m_embd_{embd}.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype="q4_k_m", embd_type=t)
    eng = mx.Engine(path, n_ctx=64, n_seq_max=2)
    assert eng.info.weight_type == synth.KQ_FTYPES["q4_k_m"]
    ids = _seq(shape, 20)
    got = eng.forward_logits(ids)
    eng.close()
    om = _oracle_kq(oracle_mod, shape, 3, "q4_k_m")
    emb = next(a for n, k, a in synth.synth_tensors(shape, 3) if n == "token_embd.weight")
    if embd == "q8_0":
        om.set_tensor_q8(-1, 1, gguf.synth_q8_0_tensor(emb))
    else:
        f16 = synth.bf16_bits_to_f32(emb).astype(np.float16).astype(np.float32)
        om.set_tensor(-1, 1, synth.f32_to_bf16_bits(f16))
    ref = om.context(64).eval(ids, 0, all_logits=True)
    assert_logits_close(got, ref, f"q4_k_m with {embd} token_embd")
    assert_tokens_match(got, ref, f"q4_k_m with {embd} token_embd")


@pytest.mark.parametrize("name,ftype", [("test-tiny", "q4_k_m"), ("test-d128", "q4_k_m"), ("test-d128", "q5_k_m"),
                                        ("test-h4096", "q4_k_m")])
def test_kq_prefill_and_decode_vs_oracle(mx, oracle_mod, name, ftype):
    """100-row prefill (64-row logits chunks: the 33-64-row and 17-32-row kernels), then 12 single-row
    decode steps, teacher-forced, against the oracle's K-quant forward."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, 112, seed=5)
    eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=256, n_seq_max=2)
    octx = _oracle_kq(oracle_mod, shape, 0, ftype).context(256)
    got = eng.forward_logits(ids[:100], 0, slot=1)
    ref = octx.eval(ids[:100], 0, all_logits=True)
    assert_logits_close(got, ref, f"{name} {ftype} prefill")
    assert_tokens_match(got, ref, f"{name} {ftype} prefill")
    err = np.abs(got - ref).max()
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = _oracle_kq(oracle_mod, shape, 0, ftype).context(256).eval(ids[:100], 0, all_logits=True)
    finally:
        oracle_mod.q8_jitter(0.0)
    self_dev = np.abs(jit - ref).max()
    print(f"{name} {ftype}: prefill max|d| {err:.4g}, oracle self-deviation {self_dev:.4g}, max|ref| "
          f"{np.abs(ref).max():.4g}")
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (err, self_dev)
    gs, rs = [], []
    for p in range(100, 112):
        gs.append(eng.forward_logits(ids[p:p + 1], p, slot=1))
        rs.append(octx.eval(ids[p:p + 1], p))
    g, r = np.concatenate(gs), np.concatenate(rs)
    assert_logits_close(g, r, f"{name} {ftype} decode")
    assert_tokens_match(g, r, f"{name} {ftype} decode")
    eng.close()


def test_kq_wide_rows_and_greedy_loop_vs_oracle(mx, oracle_mod):
    """24 sequences decoded together (the 17-32-row kernel) through the device greedy loop, every
    picked token checked along the oracle's teacher-forced chain."""
    from llama_p2p_amd import synth

    from conftest import check_chain_batched

    shape = synth.SHAPES["test-d128"]
    M, G = 24, 6
    rng = np.random.default_rng(12)
    prompts = [np.concatenate([[1], rng.integers(3, shape.n_vocab, int(rng.integers(3, 12)))]).astype(np.int32)
               for _ in range(M)]
    eng = mx.Engine("synthetic:test-d128:seed=0:q4_k_m", n_ctx=64, n_seq_max=M)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    b = eng.batch(slots=list(range(M)), pos=[len(p) - 1 for p in prompts], ids=[int(p[-1]) for p in prompts],
                  max_steps=G)
    for _ in range(G):
        b.step()
    toks = b.tokens()
    b.close()
    om = _oracle_kq(oracle_mod, shape, 0, "q4_k_m")
    exact = 0
    for i, p in enumerate(prompts):
        e, _ = check_chain_batched(om.context(64), p, toks[i].tolist(), f"seq {i}")
        exact += e
    assert exact >= 0.9 * M * G
    eng.close()


def test_kq_llama3_8b_q4_k_m_full_size(mx):
    """Llama-3-8B Q4_K_M at full size: the bytes a decode step streams match the recipe's GGUF
    bytes (synth.kq_weight_bytes_per_token, +<3% for byte-aligned K-quant scales), 1-row logits
    equal the same sequence's row inside a 32-row step (within twice the bf16 tolerance: the two
    column-tile kernels differ only in f32 summation order), and the greedy loop runs."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES["llama3-8b"]
    eng = mx.Engine("synthetic:llama3-8b:seed=0:q4_k_m", n_ctx=64, n_seq_max=32)
    want = synth.kq_weight_bytes_per_token(shape, "q4_k_m")
    assert want <= eng.info.weight_bytes <= 1.03 * want, (eng.info.weight_bytes, want)
    rng = np.random.default_rng(2)
    seqs = [np.concatenate([[128000], rng.integers(3, shape.n_vocab, 8)]).astype(np.int32) for _ in range(32)]
    slots, pos, ids = [], [], []
    for i, sq in enumerate(seqs):
        slots += [i] * 8
        pos += list(range(8))
        ids += [int(t) for t in sq[:8]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    wide = eng.forward_rows(list(range(32)), [8] * 32, [int(sq[8]) for sq in seqs])
    for i in (0, 17, 31):
        one = eng.forward_rows([i], [8], [int(seqs[i][8])])
        ref = wide[i]
        d = np.abs(one[0] - ref)
        tol2 = 2 * (1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max())
        print(f"8b q4_k_m row {i}: max|d| {d.max():.4f} (max|logit| {np.abs(ref).max():.3f})")
        assert (d <= tol2).all()
    b = eng.batch(slots=list(range(32)), pos=[9] * 32, ids=[int(np.argmax(w)) for w in wide], max_steps=4)
    for _ in range(4):
        b.step()
    toks = b.tokens()
    assert toks.shape == (32, 4) and (toks >= 0).all() and (toks < shape.n_vocab).all()
    b.close()
    eng.close()


@pytest.mark.parametrize("name,ftype", [("test-8b-ffn", "q4_k_m"), ("test-tiny-ffn", "q4_k_m"), ("test-tiny-ffn", "q5_k_m"),
                                        ("test-8b-v128k", "q4_k_m")])
def test_kq_persistent_gemv_vs_grouped_and_oracle(mx, oracle_mod, monkeypatch, name, ftype):
    """<= 16 rows of a single-type K-quant matrix with the Llama gate/up or lm_head geometry run the
    tile-persistent kernel (mkq_pers_kernel).  Against the one-tile-per-work-group kernel
    (MX_NO_KQ_PERS=1): same K split and per-tile summation order, but hipcc may contract the f32
    scale arithmetic differently (1-ulp differences that a Q8_K rounding step can amplify), so the
    two agree within twice the bf16 tolerance; 4 single-row decode steps and a 5-row prefill match
    the oracle's K-quant forward within the bf16 tolerance, greedy tokens equal (the 1e-6-noise
    self-deviation bound of the tests above is not used: at this shape the oracle's noise does not
    flip any Q8_K rounding, so that bound degenerates to ~1e-5)."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, 12, seed=9)

    def run():
        eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=64, n_seq_max=2)
        eng.forward_logits(ids[:8], 0, slot=0)
        steps = np.concatenate([eng.forward_logits(ids[p:p + 1], p, slot=0) for p in range(8, 12)])
        five = eng.forward_logits(ids[:5], 0, slot=1)
        eng.close()
        return steps, five

    got, five_p = run()
    monkeypatch.setenv("MX_NO_KQ_PERS", "1")
    ref, five_r = run()
    for g, r in ((got, ref), (five_p, five_r)):
        tol2 = 2 * (1e-2 * np.abs(r) + 2e-2 * np.abs(r).max(axis=-1, keepdims=True))
        assert (np.abs(g - r) <= tol2).all()

    octx = _oracle_kq(oracle_mod, shape, 0, ftype).context(64)
    o_five = octx.eval(ids[:5], 0, all_logits=True)
    octx2 = _oracle_kq(oracle_mod, shape, 0, ftype).context(64)
    octx2.eval(ids[:8], 0)
    o_steps = np.concatenate([octx2.eval(ids[p:p + 1], p) for p in range(8, 12)])
    for g, o, what in ((got, o_steps, "decode"), (five_p, o_five, "prefill")):
        assert_logits_close(g, o, f"{name} {ftype} persistent {what}")
        assert_tokens_match(g, o, f"{name} {ftype} persistent {what}")


@pytest.mark.parametrize("name,ftype,M", [("test-8b-ffn", "q4_k_m", 32), ("test-8b-ffn", "q5_k_m", 20),
                                          ("test-8b-v128k", "q4_k_m", 32), ("test-tiny-ffn", "q4_k_m", 17)])
def test_kq_wide_lds_gemv_vs_grouped_and_oracle(mx, oracle_mod, monkeypatch, name, ftype, M):
    """17-32 rows of a single-type K-quant gate/up or lm_head (Llama-3-8B: 1792 gate/up tiles on 7-wave
    groups, 8016 Q6_K lm_head tiles on 8-wave groups) run mkq_wide_kernel, the Q8_K activations of a
    super-block shared by the group's waves through LDS.  Against mkq_kernel (MX_NO_KQ_WIDE=1): the
    same integer super-block sums, the f32 sum over K in one wave instead of 8 K-slices, so within
    twice the bf16 tolerance; against the oracle's K-quant forward within the bf16 tolerance."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    rng = np.random.default_rng(M)
    prompts = [np.concatenate([[1], rng.integers(3, shape.n_vocab, int(rng.integers(3, 8)))]).astype(np.int32)
               for _ in range(M)]

    def run():
        eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=64, n_seq_max=M)
        for i, p in enumerate(prompts):
            eng.forward_logits(p[:-1], 0, slot=i)
        out = eng.forward_rows(list(range(M)), [len(p) - 1 for p in prompts], [int(p[-1]) for p in prompts])
        eng.close()
        return out

    got = run()
    monkeypatch.setenv("MX_NO_KQ_WIDE", "1")
    ref = run()
    monkeypatch.delenv("MX_NO_KQ_WIDE")
    tol2 = 2 * (1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max(axis=-1, keepdims=True))
    assert (np.abs(got - ref) <= tol2).all()
    om = _oracle_kq(oracle_mod, shape, 0, ftype)
    o = np.stack([om.context(64).eval(p, 0)[0] for p in prompts])
    assert_logits_close(got, o, f"{name} {ftype} wide M={M}")
    assert_tokens_match(got, o, f"{name} {ftype} wide M={M}")
    # M rows of ONE sequence (a prompt chunk): the q|k|v slabs are finished by launch_qkv_finish
    # before the attention (rows attend to each other's new K/V)
    seq = np.concatenate([[1], rng.integers(3, shape.n_vocab, M - 1)]).astype(np.int32)
    eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=64, n_seq_max=2)
    g1 = eng.forward_logits(seq, 0, slot=0)
    eng.close()
    o1 = om.context(64).eval(seq, 0, all_logits=True)
    assert_logits_close(g1, o1, f"{name} {ftype} one-sequence chunk M={M}")


@pytest.mark.parametrize("name,ftype,n_prompt", [("test-d128", "q4_k_m", 300), ("test-h4096", "q5_k_m", 200),
                                                 ("test-8b-ffn", "q4_k_m", 150)])
def test_kq_prefill_gemm_vs_oracle(mx, oracle_mod, name, ftype, n_prompt):
    """A K-quant prompt of > 64 rows without logits runs as dequantised bf16 GEMMs (launch_dequant_kq
    + the prefill GEMM; the oracle keeps ggml's Q8_K activations there): the next decode step, which
    attends to the K/V the GEMM path stored, matches the oracle within the bf16 tolerance."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, n_prompt + 1, seed=31)
    eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=512, n_seq_max=2)
    assert eng.forward_rows([0] * n_prompt, list(range(n_prompt)), ids[:n_prompt], want_logits=False) is None
    got = eng.forward_logits(ids[n_prompt:], n_prompt, slot=0)
    ref = _oracle_kq(oracle_mod, shape, 0, ftype).context(512).eval(ids, 0)
    assert_logits_close(got, ref, f"{name} {ftype} after K-quant GEMM prefill")
    assert_tokens_match(got, ref, f"{name} {ftype} after K-quant GEMM prefill")
    eng.close()


@pytest.mark.parametrize("name,ftype,n_prompt", [("test-8b-ffn", "q4_k_m", 150), ("test-d128", "q5_k_m", 120)])
def test_kq_prefill_ggml_arithmetic_vs_oracle(mx, oracle_mod, name, ftype, n_prompt):
    """MX_KQ_GGML_PREFILL=1: prompt chunks of > 64 rows run with ggml's arithmetic (every row quantised
    to Q8_K, the int8 K-quant GEMVs, no dequantised bf16 GEMM): the prompt's logits of every row and the
    next decode step against the oracle under the Q8 jitter bound (2x the oracle's own deviation under
    1e-6 relative activation noise), as test_kq_prefill_and_decode_vs_oracle."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, n_prompt + 1, seed=37)
    os.environ["MX_KQ_GGML_PREFILL"] = "1"
    try:
        eng = mx.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=512, n_seq_max=2)
    finally:
        del os.environ["MX_KQ_GGML_PREFILL"]
    # rows 64.. of the prompt: one chunk of > 64 rows without logits (the path under test), then the
    # next token attends to the K/V it stored
    got = eng.forward_logits(ids[:64], 0, slot=0)
    assert eng.forward_rows([0] * (n_prompt - 64), list(range(64, n_prompt)), ids[64:n_prompt], want_logits=False) is None
    nxt = eng.forward_logits(ids[n_prompt:], n_prompt, slot=0)
    eng.close()
    rows = list(range(64)) + [n_prompt]
    ref = _oracle_kq(oracle_mod, shape, 0, ftype).context(512).eval(ids, 0, all_logits=True)[rows]
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = _oracle_kq(oracle_mod, shape, 0, ftype).context(512).eval(ids, 0, all_logits=True)[rows]
    finally:
        oracle_mod.q8_jitter(0.0)
    self_dev = float(np.abs(jit - ref).max())
    allg = np.concatenate([got, nxt])
    err = float(np.abs(allg - ref).max())
    print(f"{name} {ftype} ggml-arithmetic prefill: max|d| {err:.4g}, oracle self-deviation {self_dev:.4g}, "
          f"max|ref| {np.abs(ref).max():.4g}")
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (err, self_dev)
    assert_tokens_match(allg, ref, f"{name} {ftype} ggml-arithmetic prefill")
