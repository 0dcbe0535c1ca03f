"""Q8_0 GGUF models on the GPU: mq8_kernel (v_mfma_i32_16x16x32_i8 over
packed Q8 tiles, activations quantised to Q8_0 rows as ggml's vec_dot_type) against the CPU
oracle's Q8_0 MUL_MAT, for every row regime (1, 17-32, 33-64 and > 64 rows), the device greedy
loop, and the GGUF loader (C++ parser + pack_q8_kernel) against on-device synthesis.

Tolerance: the bf16 one of tests/conftest.py, and a sharper one.  Both sides quantise the same
f32 activations with the same arithmetic, but Q8_0 is discontinuous: an activation whose x/d sits
near a rounding boundary moves a whole step under any f32 reordering, and on these random-weight
models that reaches ~1% of max|logit| (the oracle alone moves 0.075 of 5.4 on test-h4096 under
1e-6 relative input noise).  So the engine's deviation is bounded by 2x the oracle's own deviation
under 1e-6 noise (oracle.q8_jitter), the same-arithmetic-up-to-ordering claim made measurable."""
import numpy as np
import pytest

from conftest import assert_logits_close, assert_tokens_match, check_greedy_chain

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mx():
    from llama_p2p_amd import engine

    engine.lib()
    return engine


def _seq(shape, n, seed=7):
    rng = np.random.default_rng(seed)
    return np.concatenate([[1], rng.integers(3, shape.n_vocab, n - 1)]).astype(np.int32)


def _oracle_q8(oracle_mod, shape, seed):
    om = oracle_mod.OracleModel(shape, seed=seed)
    om.quantize_q8()
    return om


def test_q8_gguf_equals_synthetic(mx, tmp_path):
    """A Q8_0 GGUF (numpy quantiser + C++ parser + pack_q8_kernel) and the on-device Q8_0 synthesis
    of the same model give bit-identical logits; the info reports the weight type."""
    from llama_p2p_amd import gguf, synth

    shape = synth.SHAPES["test-tiny"]
    path = str(tmp_path / "tiny_q8.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype="q8_0")
    ids = _seq(shape, 24)
    a = mx.Engine(path, n_ctx=64, n_seq_max=2)
    b = mx.Engine("synthetic:test-tiny:seed=3:q8_0", n_ctx=64, n_seq_max=2)
    assert a.info.weight_type == 8 and b.info.weight_type == 8
    la, lb = a.forward_logits(ids), b.forward_logits(ids)
    assert np.array_equal(la, lb)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["test-tiny", "test-d128", "test-h4096"])
def test_q8_prefill_and_decode_vs_oracle(mx, oracle_mod, name):
    """100-row prefill (64-row logits chunks: NB=4 and NB=2 kernels), then 12 single-row decode
    steps (NB=1), teacher-forced, against the oracle's Q8_0 forward."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, 112, seed=5)
    eng = mx.Engine(f"synthetic:{name}:seed=0:q8_0", n_ctx=256, n_seq_max=2)
    octx = _oracle_q8(oracle_mod, shape, 0).context(256)
    got = eng.forward_logits(ids[:100], 0, slot=1)
    ref = octx.eval(ids[:100], 0, all_logits=True)
    assert_logits_close(got, ref, f"{name} q8 prefill")
    assert_tokens_match(got, ref, f"{name} q8 prefill")
    err = np.abs(got - ref).max()
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = _oracle_q8(oracle_mod, shape, 0).context(256).eval(ids[:100], 0, all_logits=True)
    finally:
        oracle_mod.q8_jitter(0.0)
    self_dev = np.abs(jit - ref).max()
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (err, self_dev)
    gs, rs = [], []
    for p in range(100, 112):
        gs.append(eng.forward_logits(ids[p:p + 1], p, slot=1)[0])
        rs.append(octx.eval(ids[p:p + 1], p)[0])
    gs, rs = np.stack(gs), np.stack(rs)
    assert_logits_close(gs, rs, f"{name} q8 decode")
    assert_tokens_match(gs, rs, f"{name} q8 decode")
    print(f"{name}: q8 prefill max|d| {err:.3g} (oracle under 1e-6 noise: {self_dev:.3g}), "
          f"decode max|d| {np.abs(gs - rs).max():.3g} (max|ref| {np.abs(ref).max():.3g})")
    eng.close()


def test_q8_large_prefill_then_wide_rows(mx, oracle_mod):
    """A 600-row prompt as ONE forward (grid.y = 10 column groups, no logits), then rows of 24
    and 40 different sequences in one forward each."""
    from llama_p2p_amd import synth

    name = "test-d128"
    shape = synth.SHAPES[name]
    om = _oracle_q8(oracle_mod, shape, 0)
    eng = mx.Engine(f"synthetic:{name}:seed=0:q8_0", n_ctx=640, n_seq_max=40)
    ids = _seq(shape, 610, seed=9)
    assert eng.forward_rows([0] * 600, list(range(600)), ids[:600], want_logits=False) is None
    got = eng.forward_logits(ids[600:610], 600, slot=0)
    ref = om.context(640).eval(ids, 0, all_logits=True)[600:]
    assert_logits_close(got, ref, "q8 600-row prefill")
    for M in (24, 40):
        seqs = [_seq(shape, 7, seed=100 + M + i) for i in range(M)]
        for i, sq in enumerate(seqs):
            eng.forward_rows([i] * 6, list(range(6)), sq[:6], want_logits=False)
        gw = eng.forward_rows(list(range(M)), [6] * M, [int(sq[6]) for sq in seqs])
        for i, sq in enumerate(seqs):
            assert_logits_close(gw[i:i + 1], om.context(16).eval(sq, 0), f"q8 M={M} row {i}")
    eng.close()


@pytest.mark.parametrize("name,P", [("test-h4096", 300), ("test-h4096", 520)])
def test_q8_gemm_prefill_vs_oracle(mx, oracle_mod, name, P):
    """A >= 256-row Q8_0 prompt chunk runs q8gemm_kernel (ggml_vec_dot_q8_0_q8_0's per-block int32
    products on the int8 MFMA, times d_w * d_x, in 256-row x 128-token blocks) wherever its grid has
    >= 64 blocks: at 300 rows q|k|v only (attn_output / gate-up / ffn_down stay on the GEMVs), at 520
    all four, with a ragged last token block; the next 8 rows' logits, which attend to the K/V it
    stored and read the residual it wrote, against the oracle's Q8_0 forward, within twice the
    oracle's own deviation under 1e-6 noise."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    ids = _seq(shape, P + 8, seed=11)
    eng = mx.Engine(f"synthetic:{name}:seed=0:q8_0", n_ctx=544, n_seq_max=2)
    assert eng.forward_rows([0] * P, list(range(P)), ids[:P], want_logits=False) is None
    got = eng.forward_logits(ids[P:], P, slot=0)
    ref = _oracle_q8(oracle_mod, shape, 0).context(544).eval(ids, 0, all_logits=True)[P:]
    assert_logits_close(got, ref, f"{name} q8 gemm prefill")
    assert_tokens_match(got, ref, f"{name} q8 gemm prefill")
    oracle_mod.q8_jitter(1e-6)
    try:
        jit = _oracle_q8(oracle_mod, shape, 0).context(544).eval(ids, 0, all_logits=True)[P:]
    finally:
        oracle_mod.q8_jitter(0.0)
    err, self_dev = np.abs(got - ref).max(), np.abs(jit - ref).max()
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (err, self_dev)
    eng.close()


def test_q8_batch_greedy_loop_vs_oracle(mx, oracle_mod):
    """device-resident greedy loop (graph replay + on-device argmax) on a Q8_0 model."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES["test-h4096"]
    eng = mx.Engine("synthetic:test-h4096:seed=0:q8_0", n_ctx=128, n_seq_max=4)
    M, P, G = 3, 10, 16
    prompts = [_seq(shape, P, seed=30 + i) for i in range(M)]
    first = [int(np.argmax(eng.forward_logits(p, 0, slot=i)[-1])) for i, p in enumerate(prompts)]
    b = eng.batch(slots=list(range(M)), pos=[P] * M, ids=first, max_steps=G)
    for _ in range(G):
        b.step()
    toks = b.tokens()
    om = _oracle_q8(oracle_mod, shape, 0)
    for i, p in enumerate(prompts):
        assert check_greedy_chain(om.context(128), p, [first[i]] + toks[i].tolist(), f"q8 seq {i}") >= G
    b.close()
    eng.close()


@pytest.mark.parametrize("name,M", [("test-8b-ffn", 32), ("test-8b-v128k", 24), ("test-d128", 17)])
def test_q8_wide_lds_gemv_vs_grouped_and_oracle(mx, oracle_mod, monkeypatch, name, M):
    """17-32 rows of a Q8_0 gate/up or lm_head (Llama-3-8B: 1792 gate/up tiles on 7-wave groups, 8016
    lm_head tiles on 8-wave groups) run mq8_wide_kernel, a 256-k chunk of Q8_0 activation rows shared
    by the group's waves through LDS.  Against mq8_kernel (MX_NO_Q8_WIDE=1): the same exact block
    products and scales, summed over K in one wave instead of several K-slices -- within twice the
    bf16 tolerance; against the oracle's Q8_0 forward within the bf16 tolerance."""
    from llama_p2p_amd import synth

    shape = synth.SHAPES[name]
    rng = np.random.default_rng(M)
    prompts = [np.concatenate([[1], rng.integers(3, shape.n_vocab, int(rng.integers(3, 8)))]).astype(np.int32)
               for _ in range(M)]

    def run():
        eng = mx.Engine(f"synthetic:{name}:seed=0:q8_0", n_ctx=64, n_seq_max=M)
        for i, p in enumerate(prompts):
            eng.forward_logits(p[:-1], 0, slot=i)
        out = eng.forward_rows(list(range(M)), [len(p) - 1 for p in prompts], [int(p[-1]) for p in prompts])
        eng.close()
        return out

    got = run()
    monkeypatch.setenv("MX_NO_Q8_WIDE", "1")
    ref = run()
    monkeypatch.delenv("MX_NO_Q8_WIDE")
    tol2 = 2 * (1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max(axis=-1, keepdims=True))
    assert (np.abs(got - ref) <= tol2).all()
    om = _oracle_q8(oracle_mod, shape, 0)
    o = np.stack([om.context(64).eval(p, 0)[0] for p in prompts])
    # Q8_0 rounding is discontinuous (module docstring): the engine's deviation is bounded by twice the
    # oracle's own deviation under 1e-6 input noise, on top of twice the bf16 tolerance
    oracle_mod.q8_jitter(1e-6)
    try:
        oj = _oracle_q8(oracle_mod, shape, 0)
        jit = np.stack([oj.context(64).eval(p, 0)[0] for p in prompts])
    finally:
        oracle_mod.q8_jitter(0.0)
    self_dev = np.abs(jit - o).max()
    err = np.abs(got - o).max()
    assert err <= 2 * self_dev + 1e-4 * np.abs(o).max(), (err, self_dev)
    tol2o = 2 * (1e-2 * np.abs(o) + 2e-2 * np.abs(o).max(axis=-1, keepdims=True))
    assert (np.abs(got - o) <= tol2o).all()
    assert_tokens_match(got, o, f"{name} q8_0 wide M={M}")


def test_q8_dequantised_gemm_prefill_opt_in(mx, oracle_mod, monkeypatch):
    """MX_Q8_GEMM_PREFILL=1: a > 64-row Q8_0 prompt chunk runs as bf16 GEMMs over weights dequantised
    per layer (dequant_q8_tiles_kernel: d*q rounded to bf16).  Its activations are bf16, not ggml's
    Q8_0 rows, so the next decode rows (attending to the K/V the GEMM path stored) are held to twice
    the bf16 tolerance against the oracle, and the dequantised tiles are checked against the packed
    Q8 tiles through the default path's logits on the same prompt."""
    from llama_p2p_amd import synth

    monkeypatch.setenv("MX_Q8_GEMM_PREFILL", "1")
    name = "test-d128"
    shape = synth.SHAPES[name]
    om = _oracle_q8(oracle_mod, shape, 0)
    eng = mx.Engine(f"synthetic:{name}:seed=0:q8_0", n_ctx=640, n_seq_max=2)
    ids = _seq(shape, 610, seed=9)
    assert eng.forward_rows([0] * 600, list(range(600)), ids[:600], want_logits=False) is None
    got = eng.forward_logits(ids[600:610], 600, slot=0)
    eng.close()
    ref = om.context(640).eval(ids, 0, all_logits=True)[600:]
    tol2 = 2 * (1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max(axis=-1, keepdims=True))
    assert (np.abs(got - ref) <= tol2).all(), np.abs(got - ref).max()
    assert_tokens_match(got, ref, "q8 dequantised GEMM prefill")


_PQL_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, {root!r})
from llama_p2p_amd.engine import Engine
eng = Engine("synthetic:test-8b-ffn:seed=0:{w}", n_ctx=64, n_seq_max=1)
ids = np.asarray({ids!r}, dtype=np.int32)
eng.forward_rows([0] * 16, list(range(16)), ids[:16], want_logits=False)
rows = [eng.forward_rows([0], [p], ids[p:p + 1])[0] for p in range(16, len(ids))]
np.save({out!r}, np.stack(rows))
eng.close()
"""


@pytest.mark.parametrize("w", ["q8_0", "q4_0"])
def test_one_token_gate_up_persistent_form(oracle_mod, tmp_path, w):
    """The one-token Q8_0 / Q4_0 gate/up as 256 work-groups walking 7 tiles with one quantise-on-load
    image (mq8_pers_ql_kernel: K 4096, 1792 tiles -- test-8b-ffn has Llama-3-8B's FFN) against the
    one-tile-per-group form (MX_NO_Q8_PERS_QL=1, read once per process: a child process each) bit for
    bit, and against the oracle within the Q8 jitter bound, over 8 teacher-forced one-token steps."""
    import os
    import subprocess
    import sys

    from llama_p2p_amd import synth

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    shape = synth.SHAPES["test-8b-ffn"]
    ids = _seq(shape, 24, seed=13)
    outs = []
    for off in (False, True):
        out = str(tmp_path / f"pql_{w}_{int(off)}.npy")
        script = tmp_path / f"pql_{w}_{int(off)}.py"
        script.write_text(_PQL_CHILD.format(root=root, w=w, ids=[int(t) for t in ids], out=out))
        env = {k: v for k, v in os.environ.items() if k != "MX_NO_Q8_PERS_QL"}
        if off:
            env["MX_NO_Q8_PERS_QL"] = "1"
        subprocess.run([sys.executable, str(script)], check=True, env=env, timeout=240)
        outs.append(np.load(out))
    assert outs[0].tobytes() == outs[1].tobytes(), f"{w}: max |d| {np.abs(outs[0] - outs[1]).max()}"
    om = oracle_mod.OracleModel(shape, seed=0)
    (om.quantize_q4_0 if w == "q4_0" else om.quantize_q8)()
    ref = om.context(64).eval(ids, 0, all_logits=True)[16:]
    oracle_mod.q8_jitter(1e-6)
    try:
        om2 = oracle_mod.OracleModel(shape, seed=0)
        (om2.quantize_q4_0 if w == "q4_0" else om2.quantize_q8)()
        jit = om2.context(64).eval(ids, 0, all_logits=True)[16:]
    finally:
        oracle_mod.q8_jitter(0.0)
    err, self_dev = np.abs(outs[0] - ref).max(), np.abs(jit - ref).max()
    assert_logits_close(outs[0], ref, f"test-8b-ffn {w} one-token")
    assert err <= 2 * self_dev + 1e-4 * np.abs(ref).max(), (err, self_dev)
    print(f"test-8b-ffn {w}: persistent == one-tile groups bitwise; vs oracle max|d| {err:.3g} "
          f"(oracle under 1e-6 noise {self_dev:.3g})")
