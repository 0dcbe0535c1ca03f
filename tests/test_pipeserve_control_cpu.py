"""Pipeline-serving control plane on CPU (pipeserve.py): stage re-partition from measured stage
scores, failure propagation, the round-length rule and the partition DP's cost.

* Re-partition (the reference's select_peer / update_peer_performance, p2p:156-168, applied to
  stages): over gloo at world 3 and 4 one rank's toy stage is slowed per layer; the planner's proposed
  split is applied (drain the lanes, every rank rebuilds its stage on the new layer range) while
  requests keep arriving, and every request's tokens still equal the one-stage run.
* Failure: a stage that raises in the middle of a round fails every outstanding request (admitted
  and still queued), later submissions are refused, and -- on another rank -- the peers' blocked
  receives are released (LocalComm abort in-process, the gloo process group over TCP).
"""
import os
import queue
import threading
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llama_p2p_amd import pipeserve as P
from llama_p2p_amd.pipeline import TorchComm, partition_layers
from test_pipeserve_cpu import L, N_CTX, V, H, ToyLane, ToyServeEngine, _free_port


class SlowEngine(ToyServeEngine):
    """The toy stage on a slower "GPU": every lane step sleeps ``delay`` seconds per layer held."""

    def __init__(self, lb, le, n_slots, delay=0.0, fail_at=None):
        super().__init__(lb, le, n_slots)
        self.delay, self.fail_at, self.steps = delay, fail_at, 0

    def make_lane(self, slots, kmax):
        return SlowLane(self, slots)


class SlowLane(ToyLane):
    def step_tensors(self, x_in=None, x_out=None):
        self.eng.steps += 1
        if self.eng.fail_at is not None and self.eng.steps == self.eng.fail_at:
            raise RuntimeError("injected stage failure")
        if self.eng.delay:
            time.sleep(self.eng.delay * (self.eng.le - self.eng.lb))
        super().step_tensors(x_in, x_out)


WAVE1 = [(list(range(3 + i, 9 + i)), 36) for i in range(6)]
WAVE2 = [(list(range(20 + i, 24 + 2 * i)), 10) for i in range(6)]


def _serve_waves(rank, world, parts, comm, out_q, slow_rank=-1, lanes=3, rows=3):
    delay = lambda r: 0.004 if r == slow_rank else 0.0  # noqa: E731

    def runner_for(ps):
        lb, le = ps[rank]
        return P.StageRunner(SlowEngine(lb, le, lanes * rows, delay(rank)), comm, rank, world, lanes, rows, kmax=4,
                             device=torch.device("cpu"), stage_time_every=2)

    runner = runner_for(parts)
    if rank != 0:
        P.serve_loop(runner, comm, None, N_CTX, rebuild=runner_for)
        return
    sched = P.Scheduler(lanes, rows, N_CTX, -1, kmax=4, seed=11)
    planner = P.StagePlanner(parts, head_layers=0.0, min_gain=0.10, min_samples=4, enabled=world > 1)
    front = P.PipelineFront(runner, comm, sched, N_CTX, V, H, rebuild=lambda f, ps: runner_for(ps), planner=planner)
    res = {}

    def one(key, ids, mt):
        res[key] = front.generate(ids, mt, temperature=0.0)

    th = [threading.Thread(target=one, args=(("a", i), ids, mt)) for i, (ids, mt) in enumerate(WAVE1)]
    for t in th:
        t.start()
    t0 = time.time()
    while world > 1 and not planner.history and time.time() - t0 < 60 and any(t.is_alive() for t in th):
        time.sleep(0.01)
    # the second wave arrives while the lanes drain (it waits in the queue) or after the re-split
    th2 = [threading.Thread(target=one, args=(("b", i), ids, mt)) for i, (ids, mt) in enumerate(WAVE2)]
    for t in th2:
        t.start()
    for t in th + th2:
        t.join()
    front.close()
    out_q.put({"tokens": {f"{k[0]}{k[1]}": v[0] for k, v in res.items()}, "history": planner.history,
               "parts": planner.parts})


def _worker(rank, world, port, parts, slow_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _serve_waves(rank, world, parts, TorchComm(rank, world), q, slow_rank)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,slow,expect", [(3, 1, [(0, 2), (2, 4), (4, 6)]),
                                               (4, 2, [(0, 1), (1, 2), (2, 4), (4, 6)])])
def test_repartition_applied_and_tokens_unchanged(world, slow, expect):
    q1 = queue.Queue()
    _serve_waves(0, 1, [(0, L)], None, q1)
    ref = q1.get()
    parts = partition_layers(L, 1.0, 0.0, world)
    assert parts == expect
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, parts, slow, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got["history"], "the slowed stage's scores never produced a re-split"
    first = got["history"][0]
    assert [tuple(x) for x in first["from"]] == parts
    # the first re-split shrinks the slowed stage (a second one, allowed by max_resplits = 2, may move a
    # layer back when the timings say so: the test checks the evidence-driven first move)
    sizes = [le - lb for lb, le in first["to"]]
    assert sizes[slow] < 2 and sum(sizes) == L and min(sizes) >= 1
    final = [le - lb for lb, le in got["parts"]]
    assert sum(final) == L and min(final) >= 1
    assert first["predicted_max_to"] <= 0.9 * first["predicted_max_from"]
    assert got["tokens"] == ref["tokens"]
    assert all(len(got["tokens"][f"a{i}"]) == WAVE1[i][1] for i in range(len(WAVE1)))


def test_planner_needs_gain_and_samples():
    parts = [(0, 4), (4, 8)]
    pl = P.StagePlanner(parts, min_gain=0.10, min_samples=2, z=0.0)
    assert pl.observe([1.0, 1.05]) is None  # one sample each: not yet
    assert pl.observe([1.0, 1.05]) is None  # balanced within 10 %: keep
    pl2 = P.StagePlanner(parts, min_gain=0.10, min_samples=2, z=0.0)
    assert pl2.observe([1.0, 2.0]) is None
    new = pl2.observe([1.0, 2.0])
    assert new is not None and new[1][1] - new[1][0] < 4
    assert pl2.history and pl2.history[0]["gain"] >= 0.10
    pl2.applied(new)
    assert pl2.parts == new and not pl2.board.stats()  # fresh scores after a re-split
    assert all(not x for x in pl2.samples)


def test_planner_waits_for_evidence():
    """Default thresholds: 8 samples per stage, a gain beyond 3x the stage times' relative standard
    error, a cooldown after a re-split and at most 2 re-splits."""
    parts = [(0, 4), (4, 8)]
    pl = P.StagePlanner(parts)
    for _ in range(7):  # stage 1 twice as slow, but only 7 samples
        assert pl.observe([1.0, 2.0]) is None
    assert pl.observe([1.0, 2.0]) is not None
    # the same mean imbalance inside large noise: no re-split
    noisy = P.StagePlanner(parts)
    rng = np.random.default_rng(0)
    for _ in range(12):
        assert noisy.observe([float(rng.uniform(0.2, 3.0)), float(rng.uniform(0.2, 3.0)) * 1.3]) is None
    assert noisy.last["needed"] > noisy.min_gain
    # proposed once while it drains (observations keep coming until every stage has rebuilt)
    once = P.StagePlanner(parts)
    got = [once.observe([1.0, 2.0]) for _ in range(12)]
    assert sum(g is not None for g in got) == 1 and len(once.history) == 1
    # re-splits are capped, and each needs a cooldown after the previous one
    cap = P.StagePlanner(parts, max_resplits=1)
    for _ in range(8):
        got = cap.observe([1.0, 2.0])
    assert got is not None
    cap.applied(got)
    for _ in range(20):
        assert cap.observe([1.0, 3.0]) is None


def test_partition_dp_80_layers_8_stages_is_fast():
    from llama_p2p_amd.placement import PeerScoreboard

    parts = partition_layers(80, 1.0, 2.3, 8)
    b = PeerScoreboard(list(range(8)))
    for s, t in enumerate([1.0, 1.0, 1.0, 1.6, 1.0, 1.0, 1.0, 1.0]):
        b.update(s, True, t * (parts[s][1] - parts[s][0] + (2.3 if s == 7 else 0)))
    t0 = time.perf_counter()
    new = P.proposed_partition(b, parts, head_layers=2.3)
    assert time.perf_counter() - t0 < 2.0
    sizes = [le - lb for lb, le in new]
    assert sum(sizes) == 80 and new[0][0] == 0 and new[-1][1] == 80
    assert sizes[3] < parts[3][1] - parts[3][0]
    w = P.stage_weights(b, parts, 2.3)
    # the DP is optimal: no single-boundary move lowers the predicted slowest stage
    best = P.predicted_max(w, new, 2.3)
    for i in range(7):
        for d in (-1, 1):
            alt = [list(p) for p in new]
            alt[i][1] += d
            alt[i + 1][0] += d
            if all(b_ < e_ for b_, e_ in alt):
                assert P.predicted_max(w, [tuple(p) for p in alt], 2.3) >= best - 1e-9


def test_round_length_shortened_while_requests_queue():
    s = P.Scheduler(1, 2, N_CTX, -1, kmax=8)
    for mt in (3, 20, 20):
        s.submit([1, 2, 3], mt, {"temperature": 0.0}, 0)
    plan = s.next_plan(idle_s=0)
    assert len(plan["admit"]) == 2 and len(s.pending) == 1
    # the admitted 3-token request has 2 decode tokens left after its prefill pick
    assert plan["K"] == 2
    s2 = P.Scheduler(1, 2, N_CTX, -1, kmax=8)
    for mt in (3, 20):
        s2.submit([1, 2, 3], mt, {"temperature": 0.0}, 0)
    assert s2.next_plan(idle_s=0)["K"] == 8  # nothing queued: full rounds


def _front_one_stage(fail_at, lanes=2, rows=2):
    runner = P.StageRunner(SlowEngine(0, L, lanes * rows, fail_at=fail_at), None, 0, 1, lanes, rows, kmax=4,
                           device=torch.device("cpu"))
    sched = P.Scheduler(lanes, rows, N_CTX, -1, kmax=4)
    return P.PipelineFront(runner, None, sched, N_CTX, V, H), sched


def _outcomes(front, reqs):
    res = [None] * len(reqs)

    def one(i):
        try:
            res[i] = front.generate(reqs[i][0], reqs[i][1], temperature=0.0)
        except RuntimeError as e:
            res[i] = e

    th = [threading.Thread(target=one, args=(i,)) for i in range(len(reqs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "a request never returned"
    return res


def test_failed_round_fails_admitted_and_queued_requests():
    front, sched = _front_one_stage(fail_at=5)
    reqs = [([1, 2, 3 + i], 20) for i in range(7)]  # 4 rows: 3 requests stay queued
    res = _outcomes(front, reqs)
    assert all(isinstance(r, RuntimeError) and "injected stage failure" in str(r) for r in res), res
    with pytest.raises(RuntimeError, match="failed"):
        front.submit([1, 2], 4)
    front.close()


def test_peer_stage_failure_releases_rank0_in_process():
    """Stage 1 of 3 (in-process, LocalComm) raises mid-round: stage 0 and 2, blocked in receives,
    are released by the abort, and every request on rank 0 returns the error."""
    world, lanes, rows = 3, 3, 2
    parts = partition_layers(L, 1.0, 0.0, world)
    hub = P.LocalHub()
    comms = [P.LocalComm(hub, r, world, timeout=60) for r in range(world)]
    errs = []

    def stage(r):
        run = P.StageRunner(SlowEngine(*parts[r], lanes * rows, fail_at=4 if r == 1 else None), comms[r], r, world,
                            lanes, rows, kmax=4, device=torch.device("cpu"))
        try:
            P.serve_loop(run, comms[r], None, N_CTX)
        except Exception as e:  # noqa: BLE001
            errs.append((r, e))

    th = [threading.Thread(target=stage, args=(r,), daemon=True) for r in (1, 2)]
    for t in th:
        t.start()
    run0 = P.StageRunner(SlowEngine(*parts[0], lanes * rows), comms[0], 0, world, lanes, rows, kmax=4,
                         device=torch.device("cpu"))
    sched = P.Scheduler(lanes, rows, N_CTX, -1, kmax=4)
    front = P.PipelineFront(run0, comms[0], sched, N_CTX, V, H)
    res = _outcomes(front, [([1, 2, 3 + i], 12) for i in range(8)])
    assert all(isinstance(r, RuntimeError) for r in res), res
    for t in th:
        t.join(timeout=30)
    assert {r for r, _ in errs} == {1, 2}
    assert any("injected stage failure" in repr(e) for r, e in errs if r == 1)
    front.close()


def _fail_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lanes, rows = 2, 2
    parts = partition_layers(L, 1.0, 0.0, world)
    comm = TorchComm(rank, world)
    run = P.StageRunner(SlowEngine(*parts[rank], lanes * rows, fail_at=3 if rank == 1 else None), comm, rank, world,
                        lanes, rows, kmax=4, device=torch.device("cpu"))
    if rank != 0:
        try:
            P.serve_loop(run, comm, None, N_CTX)
        except Exception:  # noqa: BLE001 -- the injected failure; the abort has been sent
            pass
        os._exit(0)
    sched = P.Scheduler(lanes, rows, N_CTX, -1, kmax=4)
    front = P.PipelineFront(run, comm, sched, N_CTX, V, H)
    res = _outcomes(front, [([1, 2, 3 + i], 12) for i in range(6)])
    q.put([isinstance(r, RuntimeError) for r in res])
    q.close()
    q.join_thread()  # flush the queue's feeder thread before the hard exit
    os._exit(0)


def test_peer_failure_over_gloo_releases_rank0():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert got and all(got)
