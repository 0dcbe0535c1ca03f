"""The ``Llama`` drop-in (llama-p2p_amd/llama.py) end to end on the GPU: a GGUF file on disk (bf16
and Q8_0, with tokenizer metadata) -> ``Llama(model_path=...)`` (p2p:19) -> ``llm(prompt,
max_tokens=...)["choices"][0]["text"]`` (p2p:125).  Greedy output must follow the CPU oracle on
the same tokenised prompt; the reference's own call (default sampling, max_tokens=100) must return
a completion dict of the llama-cpp-python shape."""
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
