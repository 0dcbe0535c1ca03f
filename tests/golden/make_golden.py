"""Generate the golden vectors under tests/golden/ (committed; re-run to refresh).

    python tests/golden/make_golden.py

Why: the reference's arithmetic lives in llama-cpp-python/llama.cpp, which is
not vendored in /root/reference and is not installed here, and
the reference has no tests or fixtures of its own.  To pin the CPU oracle's
layout conventions we use an *independent* implementation of the same model,
transformers' ``LlamaForCausalLM`` (5.15, local code, built from a config --
no download), over the very same bf16 synthetic weights:

  * GGUF stores attn_q / attn_k rows permuted for interleaved-pair RoPE
    (llama.cpp convert_hf_to_gguf ``permute``); HF expects the unpermuted rows
    with rotate-half RoPE.  We feed HF the inverse permutation of the GGUF rows.
  * HF runs in float32 (``attn_implementation="eager"``); the oracle in its
    ORC_EXACT mode does fp32 math over the same weights, so the two must agree
    to ~1e-5 of the logit scale.  The oracle's default (ggml) mode adds bf16
    activation rounding and f16 KV/q/probs; it must agree within the bf16
    tolerance stated in the tests.

Each fixture holds: ``ids`` (teacher-forced token sequence), ``logits`` (HF
fp32 logits at every position, float32), and the shape name/seed.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from llama_p2p_amd import synth  # noqa: E402

SHAPES = ["test-tiny", "test-gqa8", "test-d128", "test-h4096"]
SEQ_LEN = 40
SEED = 0


def unpermute_rows(w: np.ndarray, n_head: int) -> np.ndarray:
    """Inverse of llama.cpp's permute(w, n_head, n_head): GGUF rows -> HF rows."""
    out_dim = w.shape[0]
    d = out_dim // n_head
    return w.reshape(n_head, d // 2, 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def permute_rows(w: np.ndarray, n_head: int) -> np.ndarray:
    out_dim = w.shape[0]
    d = out_dim // n_head
    return w.reshape(n_head, 2, d // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def hf_model(shape, seed, rope_parameters=None):
    import torch
    from transformers import LlamaConfig, LlamaForCausalLM

    extra = {"rope_parameters": dict(rope_parameters, rope_theta=shape.rope_base)} if rope_parameters else {}
    cfg = LlamaConfig(vocab_size=shape.n_vocab, hidden_size=shape.n_embd, intermediate_size=shape.n_ff,
                      num_hidden_layers=shape.n_layer, num_attention_heads=shape.n_head,
                      num_key_value_heads=shape.n_head_kv, rms_norm_eps=shape.eps, rope_theta=shape.rope_base,
                      max_position_embeddings=4096, tie_word_embeddings=False, attn_implementation="eager", **extra)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg).float().eval()
    t = {name: (kind, arr) for name, kind, arr in synth.synth_tensors(shape, seed)}

    def W(name):
        kind, arr = t[name]
        if kind == "bf16":
            return torch.from_numpy(synth.bf16_bits_to_f32(arr).copy())
        return torch.from_numpy(arr.copy())

    sd = {"model.embed_tokens.weight": W("token_embd.weight"), "model.norm.weight": W("output_norm.weight"),
          "lm_head.weight": W("output.weight")}
    for l in range(shape.n_layer):
        p, q = f"blk.{l}.", f"model.layers.{l}."
        wq = unpermute_rows(W(p + "attn_q.weight").numpy(), shape.n_head)
        wk = unpermute_rows(W(p + "attn_k.weight").numpy(), shape.n_head_kv)
        sd[q + "self_attn.q_proj.weight"] = torch.from_numpy(np.ascontiguousarray(wq))
        sd[q + "self_attn.k_proj.weight"] = torch.from_numpy(np.ascontiguousarray(wk))
        sd[q + "self_attn.v_proj.weight"] = W(p + "attn_v.weight")
        sd[q + "self_attn.o_proj.weight"] = W(p + "attn_output.weight")
        sd[q + "mlp.gate_proj.weight"] = W(p + "ffn_gate.weight")
        sd[q + "mlp.up_proj.weight"] = W(p + "ffn_up.weight")
        sd[q + "mlp.down_proj.weight"] = W(p + "ffn_down.weight")
        sd[q + "input_layernorm.weight"] = W(p + "attn_norm.weight")
        sd[q + "post_attention_layernorm.weight"] = W(p + "ffn_norm.weight")
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if "rotary" not in m]
    assert not missing and not unexpected, (missing, unexpected)
    return model


def make(shape_name: str):
    import torch

    shape = synth.SHAPES[shape_name]
    rng = np.random.default_rng(1234)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, SEQ_LEN - 1)]).astype(np.int32)
    model = hf_model(shape, SEED)
    with torch.no_grad():
        out = model(torch.from_numpy(ids.astype(np.int64))[None], use_cache=False)
    logits = out.logits[0].float().numpy().astype(np.float32)
    path = os.path.join(HERE, f"hf_{shape_name}.npz")
    np.savez_compressed(path, ids=ids, logits=logits, shape=shape_name, seed=SEED)
    print(f"wrote {path}: ids {ids.shape}, logits {logits.shape}, max|logit| {np.abs(logits).max():.3f}")


# RoPE scaling (SURVEY §8a a8 for Llama-3.1 GGUFs): transformers' "llama3" rope type
# (its inv_freq is the base frequencies divided by llama.cpp's rope_freqs.weight factors -- stored
# here as ff = base_inv_freq / hf_inv_freq, what convert_hf_to_gguf writes) and "linear" (llama.cpp
# freq_scale = 1 / factor).  original_max_position_embeddings is small so the scaled band reaches
# frequencies that matter within the 40-token sequence.
ROPE_CASES = {
    "llama3": {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
               "original_max_position_embeddings": 32},
    "linear": {"rope_type": "linear", "factor": 4.0},
}


def make_rope(shape_name: str, case: str):
    import torch

    shape = synth.SHAPES[shape_name]
    params = ROPE_CASES[case]
    rng = np.random.default_rng(4321)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, SEQ_LEN - 1)]).astype(np.int32)
    model = hf_model(shape, SEED, params)
    d = shape.head_dim
    base_inv = 1.0 / (shape.rope_base ** (np.arange(0, d, 2, dtype=np.float64) / d))
    hf_inv = model.model.rotary_emb.inv_freq.double().numpy()
    if case == "linear":
        ff, freq_scale = np.ones(d // 2, np.float32), np.float32(1.0 / params["factor"])
    else:
        ff, freq_scale = (base_inv / hf_inv).astype(np.float32), np.float32(1.0)
    with torch.no_grad():
        out = model(torch.from_numpy(ids.astype(np.int64))[None], use_cache=False)
    logits = out.logits[0].float().numpy().astype(np.float32)
    path = os.path.join(HERE, f"hf_{shape_name}_rope_{case}.npz")
    np.savez_compressed(path, ids=ids, logits=logits, shape=shape_name, seed=SEED, rope_ff=ff, freq_scale=freq_scale)
    print(f"wrote {path}: factors {ff.min():.3f}..{ff.max():.3f}, freq_scale {freq_scale}")


if __name__ == "__main__":
    for s in SHAPES:
        make(s)
    for case in ROPE_CASES:
        make_rope("test-tiny", case)
