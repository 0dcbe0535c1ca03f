"""The stage planner's applied re-split on HIP stage engines (the reference's score-driven peer choice,
/root/reference/llama_p2p_network.py:156-168, turned into stage placement).

A 4-stage in-process TinyLlama-1.1B pipeline (pipeserve.local_pipeline_llama, f32 hand-off) starts from
a skewed split (13 of 22 layers on stage 0).  Requests of wave A are admitted; then the re-split to the
byte-balanced ``partition_layers`` split is forced through the scheduler's drain (the same call the
planner makes: admit nothing, let the lanes finish, every stage rebuilds its engine on the new range,
resume) while wave B waits in the queue.  Both waves' greedy tokens must equal those of one engine
holding all 22 layers (f32 hand-off: a stage split is bitwise equal to one engine), and the pipeline
must end on the new split.  A second check runs the planner itself on the skewed start: it must
re-split on measured stage times (one stage at a time on the shared GPU) toward the balanced split.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAME = "tinyllama-1.1b"
PATH = f"synthetic:{NAME}:seed=0"
SKEW = [(0, 13), (13, 16), (16, 19), (19, 22)]


def _prompts(seed, n):
    from llama_p2p_amd import synth

    sh = synth.SHAPES[NAME]
    rng = np.random.default_rng(seed)
    return [[1] + rng.integers(3, sh.n_vocab, int(rng.integers(6, 60))).tolist() for _ in range(n)]


def _balanced():
    from llama_p2p_amd import synth
    from llama_p2p_amd.pipeline import partition_layers

    sh = synth.SHAPES[NAME]
    layer = 2 * (2 * sh.n_embd ** 2 + 2 * sh.n_embd * sh.n_embd_kv + 3 * sh.n_embd * sh.n_ff)
    return [tuple(p) for p in partition_layers(sh.n_layer, layer, 2 * sh.n_vocab * sh.n_embd, 4)]


def _engine_tokens(prompts, n_tok):
    from llama_p2p_amd.engine import Engine

    eng = Engine(PATH, n_ctx=256, n_seq_max=4)  # a fresh engine per wave: no prefix reuse across waves
    rids = eng.submit_many(prompts, n_tok, per_request=[dict(temperature=0.0, ignore_eos=True)] * len(prompts))
    out = [eng.wait(r)[0] for r in rids]
    eng.close()
    return out


def test_forced_resplit_mid_stream_tokens_equal_one_engine():
    from llama_p2p_amd import pipeserve

    target = _balanced()
    assert target != SKEW
    wave_a, wave_b = _prompts(31, 4), _prompts(32, 4)
    ref_a, ref_b = _engine_tokens(wave_a, 24), _engine_tokens(wave_b, 24)

    llm = pipeserve.local_pipeline_llama(PATH, SKEW, lanes=1, rows=4, n_ctx=256, handoff_bf16=False)
    front, sched = llm._engine, llm.scheduler
    with sched.cv:  # wave A in one admission round
        ra = [front.submit(p, 24, temperature=0.0, ignore_eos=True) for p in wave_a]
    front.poll(ra[0], 0)  # wave A is admitted and decoding before the drain begins
    sched.begin_drain(target)  # the planner's call: drain, rebuild every stage, resume
    with sched.cv:  # wave B waits in the queue through the drain and is admitted after the rebuild
        rb = [front.submit(p, 24, temperature=0.0, ignore_eos=True) for p in wave_b]
    out_a = [front.wait(r)[0] for r in ra]
    out_b = [front.wait(r)[0] for r in rb]
    parts = [tuple(p) for p in llm.parts]
    planner_parts = [tuple(p) for p in llm.planner.parts]
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    print({"from": SKEW, "to": parts, "target": target})
    assert parts == target and planner_parts == target
    for i, (a, b) in enumerate(zip(out_a, ref_a)):
        assert a == b, f"wave A request {i}: pipeline {a} vs engine {b}"
    for i, (a, b) in enumerate(zip(out_b, ref_b)):
        assert a == b, f"wave B request {i} (after the re-split): pipeline {a} vs engine {b}"


def test_planner_resplits_skewed_start_on_measured_times():
    from llama_p2p_amd import pipeserve

    target = _balanced()
    llm = pipeserve.local_pipeline_llama(PATH, SKEW, lanes=2, rows=4, n_ctx=256, handoff_bf16=False,
                                         repartition=True, planner_kw=dict(max_resplits=1), stage_time_every=2)
    front = llm._engine
    prompts = _prompts(40, 48)
    outs = [None] * len(prompts)

    def run(i):
        outs[i] = front.generate(prompts[i], 64, temperature=0.0, ignore_eos=True)

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(prompts))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    hist = list(llm.planner.history)
    last = llm.planner.last
    parts = [tuple(p) for p in llm.parts]
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    print({"history": [{k: h[k] for k in ("from", "to", "gain", "needed", "samples")} for h in hist], "last": last,
           "target": target})
    assert all(len(o[0]) == 64 for o in outs)
    assert hist, f"no re-split from the skewed start: {last}"
    sizes, want = [le - lb for lb, le in parts], [le - lb for lb, le in target]
    assert sizes[0] < 13  # stage 0 gave layers away
    assert max(abs(a - b) for a, b in zip(sizes, want)) <= 2, (parts, target)
