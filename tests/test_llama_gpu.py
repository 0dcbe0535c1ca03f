"""The ``Llama`` drop-in (llama-p2p_amd/llama.py) end to end on the GPU: a GGUF file on disk (bf16
and Q8_0, with tokenizer metadata) -> ``Llama(model_path=...)`` (p2p:19) -> ``llm(prompt,
max_tokens=...)["choices"][0]["text"]`` (p2p:125).  Greedy output must follow the CPU oracle on
the same tokenised prompt; the reference's own call (default sampling, max_tokens=100) must return
a completion dict of the llama-cpp-python shape."""
import os

import numpy as np
import pytest

from conftest import check_greedy_chain

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wtype", ["bf16", "q8_0"])
def test_llama_dropin_greedy_vs_oracle(oracle_mod, tmp_path, wtype):
    from llama_p2p_amd import gguf, synth
    from llama_p2p_amd.llama import Llama

    shape = synth.SHAPES["test-d128"]
    path = str(tmp_path / f"d128_{wtype}.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=4, wtype=wtype)
    llm = Llama(model_path=path, n_ctx=256, verbose=False)
    prompt = "hello world, the llama peer network"
    ids = llm.tokenize(prompt.encode(), add_bos=True, special=True)
    assert ids[0] == 1 and len(ids) > 3

    out = llm(prompt, max_tokens=12, temperature=0.0)
    assert out["object"] == "text_completion" and out["usage"]["prompt_tokens"] == len(ids)
    n_gen = out["usage"]["completion_tokens"]
    assert 1 <= n_gen <= 12 and out["choices"][0]["finish_reason"] in ("length", "stop")

    toks, _ = llm._engine.generate(ids, 12, temperature=0.0, ignore_eos=True)
    om = oracle_mod.OracleModel(shape, seed=4)
    if wtype == "q8_0":
        om.quantize_q8()  # the same blocks the GGUF holds (tests/test_q8.py pins the two quantisers)
    assert check_greedy_chain(om.context(256), np.array(ids, np.int32), toks, f"Llama {wtype}") >= 10
    # the text of the public call is the detokenised greedy continuation (up to an end-of-generation)
    stop = next((i for i, t in enumerate(toks) if llm.tokenizer_.is_eog(t)), len(toks))
    want = llm.detokenize(toks[:stop], prev_tokens=ids).decode("utf-8", errors="ignore")
    assert out["choices"][0]["text"] == want

    # the reference's call: default sampling (temperature 0.8, top-k 40, top-p 0.95, min-p 0.05)
    res = llm(prompt, max_tokens=100)
    assert isinstance(res["choices"][0]["text"], str) and res["usage"]["completion_tokens"] <= 100
    llm.close()


def test_sampling_device_topk_equals_host_chain():
    """The decode loop's sampler takes its top-k candidates from the device (launch_topk); with fixed
    seeds the completions must be identical to the all-host chain (an engine created with
    MX_NO_DEV_TOPK=1: full logits rows, partial sort) -- same candidates, same order, same draws --
    at the reference's default sampling and at other top-k / top-p / min-p / temperature settings,
    for 1 and 3 concurrent requests."""
    from llama_p2p_amd import engine

    def run(host_only):
        if host_only:
            os.environ["MX_NO_DEV_TOPK"] = "1"
        try:
            eng = engine.Engine("synthetic:test-d128:seed=0", n_ctx=256, n_seq_max=4)
        finally:
            os.environ.pop("MX_NO_DEV_TOPK", None)
        rng = np.random.default_rng(5)
        prompts = [[1] + [int(t) for t in rng.integers(3, 2000, 12 + 5 * i)] for i in range(3)]
        out = []
        for kw in ({"temperature": 0.8, "top_k": 40, "top_p": 0.95, "min_p": 0.05},   # llama-cpp defaults
                   {"top_k": 5, "temperature": 1.3}, {"top_k": 64, "top_p": 0.8, "min_p": 0.0, "temperature": 0.5}):
            out.append(list(eng.generate(prompts[0], 24, seed=7, ignore_eos=True, **kw)[0]))
            # submitted atomically: one admission round, so the batch composition (and with it the
            # kernel path of every step) is the same in both engines
            reqs = eng.submit_many(prompts, 16, seeds=[11 + i for i in range(len(prompts))], ignore_eos=True, **kw)
            out += [list(eng.wait(r)[0]) for r in reqs]
        eng.close()
        return out

    dev, host = run(False), run(True)
    assert dev == host
    assert len({tuple(o) for o in dev}) > 3  # sampling actually varied the completions
