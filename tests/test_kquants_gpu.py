"""K-quant / Q4_0 / F16 GGUF files on the GPU: the engine dequantises every
matrix at load (dequant_bf16_kernel) and runs the bf16 path.  Checks: (1) a Q4_K_M / Q5_K_M / Q4_0 /
F16 file gives bit-identical logits to a BF16 file holding numpy's dequantisation of the same blocks
(gguf.dequantize, pinned to ggml's loops by tests/test_kquants.py) -- so the device decoder equals
the host one bit for bit; (2) those logits follow the CPU oracle built from the same bf16 weights."""
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


@pytest.mark.parametrize("wtype", ["q4_k_m", "q5_k_m", "q4_0", "f16"])
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
