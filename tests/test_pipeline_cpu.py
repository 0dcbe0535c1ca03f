"""Pipeline schedule on CPU: world_size 2 (and 4) over gloo with a stand-in executor.

The executor is a tiny deterministic "model" on torch CPU tensors with the same
tensor interface as the GPU engine (engine.EngineAdapter / engine.Batch): an
embedding, layers whose output depends on a per-(slot, layer) running state
(standing in for the KV cache, so mis-routed micro-batches or slots change the
tokens), and a greedy head.  The S-stage pipeline must produce exactly the
tokens of the 1-stage run.  The stage partition is checked separately.

RCCL's ncclSend may block until the peer posts the matching ncclRecv (gloo
buffers sends, so the gloo runs cannot show a deadlock).  The same schedule is
therefore also run over an in-process transport with strict rendezvous
semantics: every op of a group completes only when each of its ops has been
matched by the peer's op of the same direction, in order.
"""
import collections
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llama_p2p_amd.pipeline import Stage, TorchComm, partition_layers

H, V, L = 16, 50, 6


def _params():
    g = torch.Generator().manual_seed(0)
    E = torch.randn(V, H, generator=g)
    A = [torch.randn(H, H, generator=g) * 0.3 for _ in range(L)]
    W = torch.randn(H, V, generator=g)
    return E, A, W


class ToyBatch:
    def __init__(self, eng, slots, pos, ids, max_steps):
        self.eng, self.slots, self.pos = eng, list(slots), list(pos)
        self.ids = torch.tensor(ids if ids is not None else [0] * len(slots), dtype=torch.int32)
        self.hist = []
        self.max_steps = max_steps

    def bind_ids_tensor(self, t):
        t.copy_(self.ids)
        self.ids = t

    def step_tensors(self, x_in=None, x_out=None):
        x = self.eng.E[self.ids.long()] if x_in is None else x_in.clone()
        x = self.eng.layers(x, self.slots)
        if x_out is not None:
            x_out.copy_(x)
        else:
            tok = (x @ self.eng.W).argmax(-1).to(torch.int32)
            self.ids.copy_(tok)
            self.hist.append(tok.clone())
        self.pos = [p + 1 for p in self.pos]

    def tokens(self):
        return torch.stack(self.hist, 1).numpy() if self.hist else np.zeros((len(self.slots), 0), np.int32)

    def close(self):
        pass


class ToyEngine:
    def __init__(self, lb, le, n_slots):
        self.E, self.A, self.W = _params()
        self.lb, self.le = lb, le
        self.state = torch.zeros(L, n_slots, H)

    def layers(self, x, slots):
        idx = torch.tensor(slots)
        for l in range(self.lb, self.le):
            s = self.state[l, idx] * 0.5 + x
            self.state[l, idx] = s
            x = x + torch.tanh(s @ self.A[l]) * 0.5
        return x

    def stage_rows_tensors(self, slots, pos, ids, x_in, x_out):
        x = self.E[torch.tensor(ids).long()] if x_in is None else x_in.clone()
        # rows of one sequence are consumed in order, exactly like prompt prefill
        for i in range(len(slots)):
            x[i:i + 1] = self.layers(x[i:i + 1], [slots[i]])
        if x_out is not None:
            x_out.copy_(x)

    def batch(self, slots, pos, ids, max_steps):
        return ToyBatch(self, slots, pos, ids, max_steps)


def _workload(S, M, seed=3):
    rng = np.random.default_rng(seed)
    mb_rows, mb_state = [], []
    for mb in range(S):
        rows = ([], [], [])
        st = ([], [], [])
        for i in range(M):
            n = int(rng.integers(2, 7))
            ids = rng.integers(0, V, n).tolist()
            sl = mb * M + i
            rows[0].extend([sl] * (n - 1)); rows[1].extend(range(n - 1)); rows[2].extend(ids[:-1])
            st[0].append(sl); st[1].append(n - 1); st[2].append(ids[-1])
        mb_rows.append(rows)
        mb_state.append(st)
    return mb_rows, mb_state


def _run_stage(rank, world, parts, S, M, steps, q, comm=None):
    lb, le = parts[rank]
    if comm is None:
        comm = TorchComm(rank, world) if world > 1 else None
    eng = ToyEngine(lb, le, S * M)
    st = Stage(eng, comm, rank, world, H, torch.device("cpu"), S)
    mb_rows, mb_state = _workload(S, M)
    st.prefill(mb_rows, chunk=5)
    st.setup_decode(mb_state, max_steps=steps)
    st.decode_steps(2, 0)
    st.finish()
    st.decode_steps(steps - 2, 2)
    st.finish()
    toks = st.tokens()
    if toks is not None:
        q.put(np.stack(toks))


def _worker(rank, world, port, parts, S, M, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run_stage(rank, world, parts, S, M, steps, q)
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_pipeline_tokens_equal_single_stage(world):
    S, M, steps = world, 3, 6
    q1 = mp.get_context("spawn").Queue()
    # reference: one stage holding every layer, same micro-batches
    import queue

    qq = queue.Queue()
    _run_stage(0, 1, [(0, L)], S, M, steps, qq)
    ref = qq.get()
    parts = partition_layers(L, 1.0, 1.5, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, parts, S, M, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got.shape == ref.shape == (S, M, steps)
    assert np.array_equal(got, ref)


def test_partition_balances_bytes():
    # Llama-3-8B: 32 layers x 436 MB, lm_head 1.05 GB
    layer = 2 * (2 * 4096 ** 2 + 2 * 4096 * 1024 + 3 * 4096 * 14336)
    head = 2 * 128256 * 4096
    for S in (1, 2, 4, 8):
        parts = partition_layers(32, layer, head, S)
        assert parts[0][0] == 0 and parts[-1][1] == 32
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        assert all(le > lb for lb, le in parts)
        costs = [(le - lb) * layer + (head if i == S - 1 else 0) for i, (lb, le) in enumerate(parts)]
        assert max(costs) <= (32 * layer + head) / S + layer  # within one layer of perfect balance
    p8 = partition_layers(32, layer, head, 8)
    assert p8[-1][1] - p8[-1][0] < p8[0][1] - p8[0][0]  # the head stage holds fewer layers
    with pytest.raises(ValueError):
        partition_layers(4, 1.0, 1.0, 5)


class _Hub:
    """Rendezvous matching of sends/receives per ordered (src, dst) pair."""

    def __init__(self, timeout):
        self.cv = threading.Condition()
        self.sends = collections.defaultdict(collections.deque)
        self.recvs = collections.defaultdict(collections.deque)
        self.timeout = timeout

    def group(self, rank, sends, recvs):
        ops = []
        with self.cv:
            for t, d in sends:
                ops.append([t, False])
                self.sends[(rank, d)].append(ops[-1])
            for t, s in recvs:
                ops.append([t, False])
                self.recvs[(s, rank)].append(ops[-1])
            for key in list(self.sends):
                qs, qr = self.sends[key], self.recvs[key]
                while qs and qr:
                    snd, rcv = qs.popleft(), qr.popleft()
                    rcv[0].copy_(snd[0])
                    snd[1] = rcv[1] = True
            self.cv.notify_all()
            if not self.cv.wait_for(lambda: all(o[1] for o in ops), timeout=self.timeout):
                raise TimeoutError(f"rank {rank}: rendezvous deadlock")


class RendezvousComm:
    def __init__(self, hub, rank, grouped=True):
        self.hub, self.rank, self.grouped = hub, rank, grouped

    def exchange(self, sends, recvs):
        if self.grouped:
            self.hub.group(self.rank, sends, recvs)
        else:  # every op alone, in the order the ungrouped schedule issued them
            for snd in sends:
                self.hub.group(self.rank, [snd], [])
            for rcv in recvs:
                self.hub.group(self.rank, [], [rcv])

    def send(self, t, dst):
        self.hub.group(self.rank, [(t, dst)], [])

    def recv(self, t, src):
        self.hub.group(self.rank, [], [(t, src)])

    def drain(self):
        pass


def _run_rendezvous(world, grouped, timeout):
    import queue

    S, M, steps = world, 3, 6
    parts = partition_layers(L, 1.0, 1.5, world)
    hub = _Hub(timeout)
    q, errs = queue.Queue(), []

    def run(r):
        try:
            _run_stage(r, world, parts, S, M, steps, q, comm=RendezvousComm(hub, r, grouped))
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            with hub.cv:  # wake the other ranks so they time out too
                hub.cv.notify_all()

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=4 * timeout + 30)
    return errs, (q.get() if not q.empty() else None)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_pipeline_schedule_under_rendezvous_transport(world):
    import queue

    qq = queue.Queue()
    _run_stage(0, 1, [(0, L)], world, 3, 6, qq)
    ref = qq.get()
    errs, got = _run_rendezvous(world, grouped=True, timeout=20)
    assert not errs, errs
    assert np.array_equal(got, ref)


def test_ungrouped_schedule_deadlocks_under_rendezvous():
    # the transport is strict enough to catch the hazard: the same ops, each posted alone
    errs, _ = _run_rendezvous(2, grouped=False, timeout=2)
    assert errs and all(isinstance(e, TimeoutError) for e in errs)


def test_70b_eight_stage_plan_fits():
    """Config 5: Llama-3-70B bf16 over 8 stages, n_seq_max = S*M = 8 x 32 slots of 512 positions per
    stage: byte-balanced contiguous layers (every layer on exactly one stage, lm_head on the last)
    and every stage within one MI355X's 288 GB; the whole model would also fit one GPU."""
    from llama_p2p_amd import pipeline, synth

    sh = synth.SHAPES["llama3-70b"]
    plan = pipeline.stage_plan(sh, 8, 32, 512)
    assert [p["layers"][0] for p in plan][0] == 0 and plan[-1]["layers"][1] == sh.n_layer
    assert all(plan[i]["layers"][1] == plan[i + 1]["layers"][0] for i in range(7))
    w = [p["weight_bytes"] for p in plan]
    assert max(w) < 1.15 * (sum(w) / 8) + 2 * sh.n_vocab * sh.n_embd  # balanced by bytes
    assert all(p["total_bytes"] < 288e9 for p in plan)
    single = pipeline.stage_plan(sh, 1, 32, 512)
    assert single[0]["total_bytes"] < 288e9  # config 5's model also fits one GPU (bench llama3_70b)
    with pytest.raises(ValueError):
        pipeline.stage_plan(sh, 1, 32, 512, hbm_bytes=100 * 10 ** 9)
