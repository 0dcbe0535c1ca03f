"""Pipeline serving (pipeserve.py) on CPU: the request API over S stages, world 2 and 4 over gloo.

Rank 0 runs the Scheduler + PipelineFront (engine.Engine's submit / poll / cancel / wait), every
rank a StageRunner over a toy executor with the serving interface of pipeserve.EngineExecutor:
an embedding, layers whose output depends on a per-(slot, position) running state that stands in
for the KV cache (a row at position p reads the state its sequence left at p-1, so mis-routed
slots, positions or lanes change the tokens; pad rows past a prompt are overwritten before they are
read, as in the engine), and a greedy head.  Requests submitted concurrently through the S-stage
pipeline must give the tokens of the same requests served by ONE stage holding every layer, under
both placement policies; cancel-before-admission and max_tokens / EOS handling are checked too.
An in-process strict-rendezvous transport (test_pipeline_cpu._Hub) shows the serving schedule
cannot deadlock under RCCL's blocking-send semantics.
"""
import os
import time
import queue
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llama_p2p_amd import pipeserve as P
from llama_p2p_amd.pipeline import TorchComm, partition_layers
from llama_p2p_amd.placement import PeerScoreboard

H, V, L, N_CTX = 16, 50, 6, 64


def _params():
    g = torch.Generator().manual_seed(0)
    E = torch.randn(V, H, generator=g)
    A = [torch.randn(H, H, generator=g) * 0.3 for _ in range(L)]
    W = torch.randn(H, V, generator=g)
    return E, A, W


class ToyServeEngine:
    """Serving executor on torch CPU tensors (f32 hand-off)."""

    prefill_chunk = 7  # small: prompts cross hand-off chunk boundaries

    def __init__(self, lb, le, n_slots):
        self.E, self.A, self.W = _params()
        self.lb, self.le = lb, le
        self.first, self.last = lb == 0, le == L
        self.state = torch.zeros(L, n_slots, N_CTX, H)

    def layers(self, x, slots, pos):
        for i, (sl, p) in enumerate(zip(slots, pos)):
            xi = x[i:i + 1]
            for l in range(self.lb, self.le):
                prev = self.state[l, sl, p - 1] if p > 0 else torch.zeros(H)
                s = prev * 0.5 + xi[0]
                self.state[l, sl, p] = s
                xi = xi + torch.tanh(s @ self.A[l]) * 0.5
            x[i:i + 1] = xi
        return x

    def alloc_x(self, rows):
        return torch.empty((rows, H), dtype=torch.float32)

    def prefill(self, slots, pos, ids, x_in, x_out, rowmap, samp):
        x = self.E[torch.tensor(ids).long()] if x_in is None else x_in.clone()
        x = self.layers(x, slots, pos)
        if x_out is not None:
            x_out.copy_(x)
            return []
        return [int(t) for t in (x[list(rowmap)] @ self.W).argmax(-1)] if rowmap else []

    def make_lane(self, slots, kmax):
        return ToyLane(self, slots)

    def samplers(self, rows):
        assert all(s.get("temperature", 0.0) <= 0 for s, _, _, _ in rows), "the toy head is greedy"
        return rows


class ToyLane:
    def __init__(self, eng, slots):
        self.eng, self.slots = eng, list(slots)
        self.ids = torch.zeros(len(slots), dtype=torch.int32)
        self.pos = [0] * len(slots)
        self.hist = []

    def bind_ids_tensor(self, t):
        t.copy_(self.ids)
        self.ids = t

    def reset(self, pos, ids=None, samplers=None):
        self.pos = list(pos)
        if ids is not None:
            self.ids.copy_(torch.tensor(ids, dtype=torch.int32))
        self.hist = []

    def step_tensors(self, x_in=None, x_out=None):
        x = self.eng.E[self.ids.long()] if x_in is None else x_in.clone()
        x = self.eng.layers(x, self.slots, self.pos)
        if x_out is not None:
            x_out.copy_(x)
        else:
            tok = (x @ self.eng.W).argmax(-1).to(torch.int32)
            self.ids.copy_(tok)
            self.hist.append(tok.clone())
        self.pos = [min(p + 1, N_CTX - 1) for p in self.pos]

    def tokens(self):
        return torch.stack(self.hist, 1).numpy() if self.hist else np.zeros((len(self.slots), 0), np.int32)

    def close(self):
        pass


def _requests(n=12, seed=5):
    rng = np.random.default_rng(seed)
    return [(rng.integers(0, V, int(rng.integers(2, 20))).tolist(), int(rng.integers(1, 14))) for _ in range(n)]


def _serve(rank, world, parts, lanes, rows, policy, comm, out_q, eos=-1, cancel_first=False):
    """One rank: rank 0 submits every request from its own thread (all at once) and reports the tokens."""
    lb, le = parts[rank]
    ex = ToyServeEngine(lb, le, lanes * rows)
    runner = P.StageRunner(ex, comm, rank, world, lanes, rows, kmax=4, device=torch.device("cpu"),
                           stage_time_every=3)
    if rank != 0:
        P.serve_loop(runner, comm, None, N_CTX)
        return
    sched = P.Scheduler(lanes, rows, N_CTX, eos, kmax=4, policy=policy, seed=11)
    stage_board = PeerScoreboard(list(range(world)))
    front = P.PipelineFront(runner, comm, sched, N_CTX, V, H, stage_board)
    reqs = _requests()
    res = [None] * len(reqs)
    if cancel_first:  # a request cancelled before any round admits it returns no tokens
        with sched.cv:
            rid = front.submit(reqs[0][0], 5)
            front.cancel(rid)
        res_c = front.wait(rid)
        assert res_c == ([], P.FINISH_STOP), res_c

    def one(i):
        ids, mt = reqs[i]
        res[i] = front.generate(ids, mt, temperature=0.0)

    th = [threading.Thread(target=one, args=(i,)) for i in range(len(reqs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    front.close()
    out_q.put({"tokens": [r[0] for r in res], "finish": [r[1] for r in res], "lanes": sched.board.stats(),
               "stages": stage_board.stats(), "rounds": sched.rounds})


def _worker(rank, world, port, parts, lanes, rows, policy, q, eos):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _serve(rank, world, parts, lanes, rows, policy, TorchComm(rank, world), q, eos)
    finally:
        dist.destroy_process_group()


def _reference(lanes, rows, eos=-1):
    q = queue.Queue()
    _serve(0, 1, [(0, L)], lanes, rows, "score_aware", None, q, eos)
    return q.get()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,policy", [(2, "score_aware"), (4, "reference"), (4, "score_aware")])
def test_pipeline_serving_equals_single_stage(world, policy):
    lanes, rows = world, 3
    ref = _reference(lanes, rows)
    parts = partition_layers(L, 1.0, 1.5, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, parts, lanes, rows, policy, q, -1))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reqs = _requests()
    for i, (ids, mt) in enumerate(reqs):
        assert len(got["tokens"][i]) == mt and got["finish"][i] == P.FINISH_LENGTH
    assert got["tokens"] == ref["tokens"]
    assert sum(v["success"] for v in got["lanes"].values()) == len(reqs)
    assert set(got["stages"]) == set(range(world))  # every stage reported its busy time


def test_eos_and_cancel_single_stage():
    """One stage (world 1): a request cancelled before admission returns nothing; with an EOS id
    chosen from the reference's outputs, requests stop at it (finish STOP, EOS kept in the ids, as the
    engine returns them)."""
    q = queue.Queue()
    _serve(0, 1, [(0, L)], 2, 3, "score_aware", None, q, -1, cancel_first=True)
    ref = q.get()
    toks = [t for seq in ref["tokens"] for t in seq]
    eos = max(set(toks), key=toks.count)
    q2 = queue.Queue()
    _serve(0, 1, [(0, L)], 2, 3, "score_aware", None, q2, eos)
    got = q2.get()
    for a, b, fin in zip(ref["tokens"], got["tokens"], got["finish"]):
        k = a.index(eos) + 1 if eos in a else len(a)
        assert b == a[:k]
        assert fin == (P.FINISH_STOP if eos in a else P.FINISH_LENGTH)


class _RdvComm:
    """test_pipeline_cpu's strict rendezvous transport + in-process object passing."""

    def __init__(self, hub, rank, world, boxes):
        from test_pipeline_cpu import RendezvousComm

        self.t = RendezvousComm(hub, rank)
        self.rank, self.world, self.boxes = rank, world, boxes

    def exchange(self, sends, recvs):
        self.t.exchange(sends, recvs)

    def send(self, t, dst):
        self.t.send(t, dst)

    def recv(self, t, src):
        self.t.recv(t, src)

    def drain(self):
        pass

    def bcast_obj(self, obj, src=0):
        if self.rank == src:
            for r in range(self.world):
                if r != src:
                    self.boxes[(src, r)].put(obj)
            return obj
        return self.boxes[(src, self.rank)].get(timeout=30)

    def send_obj(self, obj, dst):
        self.boxes[(self.rank, dst)].put(obj)

    def recv_obj(self, src):
        return self.boxes[(src, self.rank)].get(timeout=30)


@pytest.mark.parametrize("world", [2, 3])
def test_serving_schedule_under_rendezvous_transport(world):
    from collections import defaultdict

    from test_pipeline_cpu import _Hub

    lanes, rows = world, 2
    ref = _reference(lanes, rows)
    hub = _Hub(20)
    boxes = defaultdict(queue.Queue)
    parts = partition_layers(L, 1.0, 1.5, world)
    q, errs = queue.Queue(), []

    def run(r):
        try:
            _serve(r, world, parts, lanes, rows, "score_aware", _RdvComm(hub, r, world, boxes), q)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert q.get(timeout=5)["tokens"] == ref["tokens"]


def test_reference_policy_concentrates_score_aware_spreads():
    """Lane placement: p2p:159's score (reference policy) keeps sending requests to the lane that
    answered first while it has room; the score-aware policy spreads them by requests in flight."""
    ref_b = PeerScoreboard(list(range(4)), policy="reference", seed=1)
    aware = PeerScoreboard(list(range(4)), policy="score_aware")
    for b in (ref_b, aware):
        t = b.select()
        b.update(t, True, 0.5)
    picks_ref = [ref_b.select(candidates=[0, 1, 2, 3]) for _ in range(6)]
    picks_aw = [aware.select(candidates=[0, 1, 2, 3]) for _ in range(6)]
    assert len(set(picks_ref)) == 1  # every request to the lane with stats (p2p:159)
    assert len(set(picks_aw)) == 4   # untried lanes first, then by in-flight load
    # a full lane is not a candidate: the reference policy falls back to a random free lane
    assert ref_b.select(candidates=[2, 3]) in (2, 3)


def test_proposed_partition_follows_stage_scores():
    """Stage placement from measured scores: a stage measured twice as slow per layer gets fewer
    layers in the proposed split; equal scores keep a balanced split."""
    parts = [(0, 4), (4, 8), (8, 12), (12, 16)]
    b = PeerScoreboard(list(range(4)))
    for s, t in enumerate([1.0, 1.0, 2.0, 1.0]):
        b.update(s, True, t)
    new = P.proposed_partition(b, parts)
    sizes = [le - lb for lb, le in new]
    assert new[0][0] == 0 and new[-1][1] == 16 and sum(sizes) == 16
    assert sizes[2] < 4 and min(sizes) >= 1
    b2 = PeerScoreboard(list(range(4)))
    for s in range(4):
        b2.update(s, True, 1.0)
    assert P.proposed_partition(b2, parts) == parts


def _p2p159(snap, cands):
    """select_peer (p2p:156-159) over the candidate lanes that have stats: argmax success/(s+f+1)."""
    known = [t for t in snap if t in cands]
    if not known:
        return None  # random among the candidates
    return max(known, key=lambda t: snap[t][0] / (snap[t][0] + snap[t][1] + 1))


@pytest.mark.parametrize("policy", ["reference", "score_aware"])
def test_poisson_stream_placed_on_lanes(policy):
    """Config 5's driver shape on the toy pipeline (world 4 in-process, strict rendezvous): a Poisson
    stream (compressed clock) whose requests the peer scoreboard places onto the pipeline's lanes.
    Under the reference policy every placement is p2p:159's pick among the lanes with a free row."""
    from collections import defaultdict

    from llama_p2p_amd.placement import poisson_schedule
    from test_pipeline_cpu import _Hub

    world, lanes, rows = 4, 4, 2
    parts = partition_layers(L, 1.0, 1.5, world)
    hub, boxes = _Hub(30), defaultdict(queue.Queue)
    comms = [_RdvComm(hub, r, world, boxes) for r in range(world)]
    sched = P.Scheduler(lanes, rows, N_CTX, -1, kmax=4, policy=policy, seed=3)
    runners = [P.StageRunner(ToyServeEngine(*parts[r], lanes * rows), comms[r], r, world, lanes, rows, 4,
                             torch.device("cpu")) for r in range(world)]
    th = [threading.Thread(target=P.serve_loop, args=(runners[r], comms[r], None, N_CTX), daemon=True)
          for r in range(1, world)]
    for t in th:
        t.start()
    front = P.PipelineFront(runners[0], comms[0], sched, N_CTX, V, H)
    stream = poisson_schedule(2.0, 24, seed=3, prompt_lo=4, prompt_hi=30, vocab=V, bos=1)
    t0, out, workers = time.perf_counter(), [None] * len(stream), []
    for i, (ta, prompt) in enumerate(stream):
        d = ta * 0.02 - (time.perf_counter() - t0)  # clock compressed 50x
        if d > 0:
            time.sleep(d)
        w = threading.Thread(target=lambda i=i, p=prompt: out.__setitem__(i, front.generate(p.tolist(), 6)))
        w.start()
        workers.append(w)
    for w in workers:
        w.join()
    front.close()
    for t in th:
        t.join(timeout=30)
    assert all(o is not None and len(o[0]) == 6 for o in out)
    placements = list(sched.placements)
    assert len(placements) == len(stream)
    if policy == "reference":
        for rid, lane, cands, snap in placements:
            want = _p2p159(snap, cands)
            assert lane in cands and (want is None or lane == want)
    used = {lane for _, lane, _, _ in placements}
    assert used <= set(range(lanes))
