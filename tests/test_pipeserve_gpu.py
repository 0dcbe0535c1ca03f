"""Pipeline serving on one GPU: S stage engines of one model in one process (pipeserve.local_pipeline_llama),
requests through the Llama-compatible front (submit / wait via create_completion and through the node's
handle_requests -> cached_inference), hand-offs in bf16.  Greedy outputs are teacher-forced through the
CPU oracle (every pick the oracle's argmax or a near tie); sampled outputs are reproducible per seed.
The S-GPU launch uses the same server with RCCL between processes (bench.py --gpus N / serve_pipeline);
its schedule is covered on CPU over gloo and a strict rendezvous transport (test_pipeserve_cpu.py).
"""
import json
import threading

import numpy as np
import pytest

from conftest import check_chain_batched

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,parts,handoff_bf16", [
    ("test-gqa8", [(0, 1), (1, 3)], True),
    ("test-8b-v128k", [(0, 1), (1, 2)], True),
    ("test-gqa8", [(0, 1), (1, 2), (2, 3)], False),
])
def test_pipeline_requests_vs_oracle(oracle_mod, name, parts, handoff_bf16):
    from llama_p2p_amd import pipeserve, synth

    sh = synth.SHAPES[name]
    llm = pipeserve.local_pipeline_llama(f"synthetic:{name}:seed=0", parts, lanes=len(parts), rows=4, n_ctx=256,
                                         handoff_bf16=handoff_bf16)
    rng = np.random.default_rng(9)
    prompts = [[1] + rng.integers(3, sh.n_vocab, int(rng.integers(4, 90))).tolist() for _ in range(10)]
    outs = [None] * len(prompts)

    def run(i):  # concurrent callers: micro-batched into the lanes
        outs[i] = llm._engine.generate(prompts[i], 12, temperature=0.0, ignore_eos=True)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(prompts))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    om = oracle_mod.OracleModel(sh, seed=0)
    exact = 0
    for p, (toks, fin) in zip(prompts, outs):
        assert len(toks) == 12 and fin == 0
        e, _ = check_chain_batched(om.context(256), np.array(p, np.int32), toks, f"{name} pipeline")
        exact += e
    assert exact >= 0.85 * 12 * len(prompts)
    # sampling on the device (default chain, fixed seed): reproducible, same length
    a = llm._engine.generate(prompts[0], 16, temperature=0.8, top_k=40, top_p=0.95, min_p=0.05, seed=123,
                             ignore_eos=True)
    b = llm._engine.generate(prompts[0], 16, temperature=0.8, top_k=40, top_p=0.95, min_p=0.05, seed=123,
                             ignore_eos=True)
    assert a == b and len(a[0]) == 16
    lanes_used = llm.scheduler.board.stats()
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    assert sum(v["success"] for v in lanes_used.values()) == len(prompts) + 2


def test_node_over_pipeline():
    """The reference node's handler (p2p:84-98) and cached_inference (p2p:120-133) on a sharded model:
    concurrent JSON requests over REP contexts, then the same prompts again as cache hits."""
    from llama_p2p_amd import pipeserve
    from llama_p2p_amd.node import LlamaP2PNode, LocalTransport

    llm = pipeserve.local_pipeline_llama("synthetic:test-gqa8:seed=0", [(0, 2), (2, 3)], lanes=2, rows=4,
                                         n_ctx=256)
    tr = LocalTransport()
    node = LlamaP2PNode("synthetic:test-gqa8:seed=0", 5000, cache_size=100, secret_key="k", model=llm,
                        transport=tr, n_contexts=8)
    threading.Thread(target=node.handle_requests, daemon=True).start()
    prompts = [f"question {i}: which peer holds the layers" for i in range(6)]
    replies = [None] * len(prompts)

    def ask(i):
        replies[i] = json.loads(tr.request(json.dumps({"type": "inference", "prompt": prompts[i],
                                                       "secret_key": "k"}).encode()))

    for _ in range(2):
        th = [threading.Thread(target=ask, args=(i,)) for i in range(len(prompts))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert all("result" in r for r in replies), replies
    assert len(node.cache) == len(prompts)
    node.active = False
    llm.close()


def test_pipeline_sampling_chain_equals_single_engine():
    """Seeded sampled requests (penalties, top_k <= 64) through the pipeline's device chain
    (mx_stage_rows_pick's first draw, the window / draw-count hand-over of newly admitted rows in
    run_round) give the tokens of the same requests through one engine's scheduler (Engine.submit),
    with greedy and sampled rows mixed in one lane.  f32 hand-off (stage splits are bitwise equal to
    one engine), the same admission round on both sides, and counter-based draws that do not depend
    on the schedule (K steps per round): the tokens must be identical."""
    from llama_p2p_amd import pipeserve, synth
    from llama_p2p_amd.engine import Engine

    name = "test-gqa8"
    sh = synth.SHAPES[name]
    path = f"synthetic:{name}:seed=0"
    rng = np.random.default_rng(17)
    prompts = [[1] + rng.integers(3, sh.n_vocab, int(rng.integers(6, 40))).tolist() for _ in range(6)]
    kws = [dict(temperature=0.8, top_k=40, top_p=0.95, min_p=0.05, seed=101),
           dict(temperature=0.0),
           dict(temperature=1.1, top_k=12, top_p=0.9, min_p=0.02, repeat_penalty=1.3, repeat_last_n=16, seed=7),
           dict(temperature=0.7, top_k=64, top_p=1.0, min_p=0.0, frequency_penalty=0.4, presence_penalty=0.3,
                seed=99),
           dict(temperature=0.0, repeat_penalty=1.2, repeat_last_n=32, seed=5),
           dict(temperature=0.9, top_k=5, seed=12345)]
    # both sides admit the six requests in ONE round (one batched prefill of the same rows, then one
    # decode batch), so every logit is computed by the same kernels at the same row counts
    eng = Engine(path, n_ctx=256, n_seq_max=8)
    rids = eng.submit_many(prompts, 20, per_request=[dict(kw, ignore_eos=True) for kw in kws])
    ref = [eng.wait(r)[0] for r in rids]
    eng.close()
    # one lane of 8 rows: every request shares it (greedy and sampled rows mixed)
    llm = pipeserve.local_pipeline_llama(path, [(0, 1), (1, 3)], lanes=1, rows=8, n_ctx=256, handoff_bf16=False)
    front = llm._engine
    with llm.scheduler.cv:  # queued atomically: the next round admits all of them
        rids = [front.submit(p, 20, ignore_eos=True, **kw) for p, kw in zip(prompts, kws)]
    outs = [front.wait(r)[0] for r in rids]
    placements = list(llm.scheduler.placements)
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    assert {lane for _, lane, _, _ in placements} == {0}
    for i, (a, b) in enumerate(zip(outs, ref)):
        assert a == b, f"request {i} ({kws[i]}): pipeline {a} vs engine {b}"
