"""The drop-in node serving concurrent requests from the wire on the GPU engine:
32 requests through ``handle_requests`` (p2p:84-98) over REP contexts -> ``cached_inference``
(p2p:120-133) -> the model, micro-batched by the engine's scheduler; every greedy completion must
follow the CPU oracle (teacher-forced chain), and the replies must match their requests."""
import json
import threading

import numpy as np
import pytest

from conftest import check_chain_batched

pytestmark = pytest.mark.gpu


class GreedyRecorder:
    """The node's model: ``model(prompt, max_tokens=100)`` -> completion dict, greedy, recording
    the prompt ids and generated ids for the oracle check."""

    def __init__(self, llm):
        self.llm, self.rec, self.lock = llm, {}, threading.Lock()

    def __call__(self, prompt, max_tokens=16, **kw):
        ids = self.llm.tokenize(prompt.encode(), add_bos=True, special=True)
        toks, _ = self.llm._engine.generate(ids, max_tokens, temperature=0.0, ignore_eos=True)
        with self.lock:
            self.rec[prompt] = (ids, toks)
        return {"choices": [{"text": self.llm.detokenize(toks, prev_tokens=ids).decode("utf-8", errors="ignore")}]}


def test_32_requests_through_handle_requests_vs_oracle(oracle_mod):
    from llama_p2p_amd import synth
    from llama_p2p_amd.llama import Llama
    from llama_p2p_amd.node import LlamaP2PNode, LocalTransport

    shape = synth.SHAPES["test-d128"]
    llm = Llama(model_path="synthetic:test-d128", n_ctx=256, n_seq_max=32, verbose=False)
    model = GreedyRecorder(llm)
    tr = LocalTransport()
    node = LlamaP2PNode("synthetic:test-d128", 5000, cache_size=100, secret_key="k", model=model, transport=tr,
                        n_contexts=32)
    th = threading.Thread(target=node.handle_requests, daemon=True)
    th.start()
    rng = np.random.default_rng(9)
    words = ["peer", "node", "cache", "token", "graph", "layer", "gossip", "stream"]
    prompts = [f"req {i}: " + " ".join(words[int(j)] for j in rng.integers(0, 8, int(rng.integers(3, 25))))
               for i in range(32)]
    replies = {}

    def client(i):
        msg = json.dumps({"type": "inference", "prompt": prompts[i], "secret_key": "k"}).encode()
        replies[i] = json.loads(tr.request(msg, timeout=120))

    cs = [threading.Thread(target=client, args=(i,)) for i in range(32)]
    for c in cs:
        c.start()
    for c in cs:
        c.join()
    node.active = False
    th.join(timeout=5)
    assert len(replies) == 32 and len(model.rec) == 32
    om = oracle_mod.OracleModel(shape, seed=0)
    exact = 0
    for i, p in enumerate(prompts):
        ids, toks = model.rec[p]
        assert len(toks) == 100
        text = llm.detokenize(toks, prev_tokens=ids).decode("utf-8", errors="ignore")
        assert replies[i] == {"result": text}, f"reply {i} does not belong to its request"
        e, _ = check_chain_batched(om.context(256), np.array(ids, np.int32), toks, f"request {i}")
        exact += e
    assert exact >= 0.9 * 32 * 100
    st = llm._engine.stats()
    assert st["generated_tokens"] >= 3200
    llm.close()
