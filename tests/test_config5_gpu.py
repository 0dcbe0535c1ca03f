"""BASELINE config 5 on its own model: Llama-3-70B bf16 as an 8-stage pipeline with gossip-score-driven
request placement under a synthetic Poisson request stream (/root/reference/llama_p2p_network.py:135-168:
forward each request to the best-scored peer; here the peers are the pipeline's micro-batch lanes).

On one GPU the 8 stages are in-process stage engines (pipeserve.local_pipeline_llama; the 8-GPU launch
runs the same server with RCCL between processes).  A Poisson stream (config 5's generator, compressed
clock) goes through the Llama-compatible front; every admission is placed by the lanes' PeerScoreboard
(score_aware: p2p:159's score divided by mean latency x (1 + in flight)).  Checked: every request
completes with its tokens, every placement equals the policy replayed from the logged scoreboard state
(success / failure / mean latency / in flight of each lane at that moment), and several lanes are used.
(Tokens are not compared across requests: a prompt's prefill rows share GEMM chunks with whatever else
was admitted in its round, and the chunk's row count picks the GEMM's K split.)
"""
import threading
import time

import pytest

pytestmark = pytest.mark.gpu


def test_config5_70b_poisson_score_placement():
    from llama_p2p_amd import pipeserve, synth
    from llama_p2p_amd.pipeline import partition_layers
    from llama_p2p_amd.placement import PeerScoreboard, poisson_schedule

    sh = synth.SHAPES["llama3-70b"]
    h, kv, ff = sh.n_embd, sh.n_embd_kv, sh.n_ff
    parts = partition_layers(sh.n_layer, 2 * (2 * h * h + 2 * h * kv + 3 * h * ff), 2 * sh.n_vocab * h, 8)
    llm = pipeserve.local_pipeline_llama("synthetic:llama3-70b:seed=0", parts, lanes=8, rows=4, n_ctx=512,
                                         policy="score_aware", seed=0)
    front, sched = llm._engine, llm.scheduler
    stream = poisson_schedule(2.0, 24, seed=3, prompt_lo=32, prompt_hi=200, vocab=sh.n_vocab)
    out, workers, t0 = [None] * len(stream), [], time.perf_counter()
    for i, (ta, prompt) in enumerate(stream):
        d = ta * 0.25 - (time.perf_counter() - t0)  # arrival clock compressed 4x
        if d > 0:
            time.sleep(d)
        w = threading.Thread(target=lambda i=i, p=prompt: out.__setitem__(
            i, front.generate(p.tolist(), 16, temperature=0.0, ignore_eos=True)))
        w.start()
        workers.append(w)
    for w in workers:
        w.join()
    placements, states = list(sched.placements), list(sched.placement_state)
    parts_after = list(llm.parts)
    llm.close()
    assert not llm._stage_errors, llm._stage_errors
    assert all(o is not None and len(o[0]) == 16 for o in out)
    assert len(placements) == len(stream) == len(states)
    for (rid, lane, cands, snap), (avg, inflight) in zip(placements, states):
        b = PeerScoreboard(list(range(8)), policy="score_aware")
        for t, (succ, fail) in snap.items():
            b.perf[t] = {"success": succ, "failure": fail, "avg_time": avg[t]}
        for t, n in inflight.items():
            b.inflight[t] = n
        assert b.select(candidates=cands) == lane, (rid, lane, cands, snap, avg, inflight)
    used = {lane for _, lane, _, _ in placements}
    print({"lanes_used": sorted(used), "placements": len(placements), "parts": parts_after})
    assert len(used) >= 4
