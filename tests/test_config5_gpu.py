"""BASELINE config 5 at its own workload: Llama-3-70B bf16 as an 8-stage pipeline with gossip-score-driven
request placement under a synthetic Poisson request stream of 256 requests, prompts U[32, 512], 128 greedy
tokens each (/root/reference/llama_p2p_network.py:135-168: forward each request to the best-scored peer;
here the peers are the pipeline's micro-batch lanes).

On one GPU the 8 stages are in-process stage engines (pipeserve.local_pipeline_llama; the 8-GPU launch
runs the same server with RCCL between processes), f32 hand-offs.  The Poisson stream (config 5's
generator, arrival clock compressed) goes through the Llama-compatible front; every admission is placed
by the lanes' PeerScoreboard (score_aware: p2p:159's score divided by mean latency x (1 + in flight)).
Checked:
  * every request completes with its 128 tokens;
  * every placement equals the policy replayed from the logged scoreboard state (success / failure /
    mean latency / in flight of each lane at that moment), and the lanes are spread;
  * tokens: a seeded sample of 16 requests, generated again by ONE engine holding all 80 layers
    (mx_submit_batch, 16 rows at a time), gives the pipeline's tokens exactly.  That holds because a
    request's result does not depend on what it is batched with (DESIGN.md §1 "batch invariance":
    GEMM prefill with one K range per output, canonical K order of the decode GEMVs at every row count)
    and because an f32 stage hand-off is the residual stream itself.
"""
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_REQ, LO, HI, GEN, N_CTX = 256, 32, 512, 128, 640


@pytest.mark.timeout(900)
def test_config5_70b_poisson_placement_and_tokens_vs_one_engine():
    import torch

    from llama_p2p_amd import pipeserve, synth
    from llama_p2p_amd.engine import Engine
    from llama_p2p_amd.pipeline import partition_layers
    from llama_p2p_amd.placement import PeerScoreboard, poisson_schedule

    sh = synth.SHAPES["llama3-70b"]
    h, kv, ff = sh.n_embd, sh.n_embd_kv, sh.n_ff
    parts = partition_layers(sh.n_layer, 2 * (2 * h * h + 2 * h * kv + 3 * h * ff), 2 * sh.n_vocab * h, 8)
    t_build = time.perf_counter()
    llm = pipeserve.local_pipeline_llama("synthetic:llama3-70b:seed=0", parts, lanes=8, rows=32, n_ctx=N_CTX,
                                         policy="score_aware", seed=0, handoff_bf16=False)
    front, sched = llm._engine, llm.scheduler
    stream = poisson_schedule(16.0, N_REQ, seed=3, prompt_lo=LO, prompt_hi=HI, vocab=sh.n_vocab)
    out, workers, t0 = [None] * len(stream), [], time.perf_counter()
    t_build = t0 - t_build
    for i, (ta, prompt) in enumerate(stream):
        d = ta - (time.perf_counter() - t0)
        if d > 0:
            time.sleep(d)
        w = threading.Thread(target=lambda i=i, p=prompt: out.__setitem__(
            i, front.generate(p.tolist(), GEN, temperature=0.0, ignore_eos=True)))
        w.start()
        workers.append(w)
    for w in workers:
        w.join()
    t_serve = time.perf_counter() - t0
    placements, states = list(sched.placements), list(sched.placement_state)
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    assert all(o is not None and len(o[0]) == GEN for o in out)
    assert len(placements) == len(stream) == len(states)
    for (rid, lane, cands, snap), (avg, inflight) in zip(placements, states):
        b = PeerScoreboard(list(range(8)), policy="score_aware")
        for t, (succ, fail) in snap.items():
            b.perf[t] = {"success": succ, "failure": fail, "avg_time": avg[t]}
        for t, n in inflight.items():
            b.inflight[t] = n
        assert b.select(candidates=cands) == lane, (rid, lane, cands, snap, avg, inflight)
    used = {lane for _, lane, _, _ in placements}
    assert len(used) >= 4

    # the same requests on one engine holding every layer
    del llm, front, sched
    torch.cuda.empty_cache()
    sample = sorted(np.random.default_rng(7).choice(N_REQ, 16, replace=False).tolist())
    eng = Engine("synthetic:llama3-70b:seed=0", n_ctx=N_CTX, n_seq_max=16)
    t1 = time.perf_counter()
    reqs = eng.submit_many([stream[i][1].tolist() for i in sample], GEN, ignore_eos=True)
    ref = [eng.wait(r)[0] for r in reqs]
    t_one = time.perf_counter() - t1
    eng.close()
    diff = [i for i, r in zip(sample, ref) if r != out[i][0]]
    gen_tokens = N_REQ * GEN
    print({"lanes_used": sorted(used), "placements": len(placements), "build_s": round(t_build, 1),
           "serve_s": round(t_serve, 1), "serve_tok_s": round(gen_tokens / t_serve, 1),
           "prompt_tokens": int(sum(len(p) for _, p in stream)), "one_engine_s": round(t_one, 1),
           "sample": sample, "token_mismatch": diff})
    assert not diff, f"requests {diff}: the pipeline's tokens differ from one engine's"
