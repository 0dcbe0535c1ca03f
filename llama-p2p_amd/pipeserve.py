"""Pipeline serving: the reference's request path on a model sharded over S GPU stages.

The reference node answers a request with ``self.model(prompt, max_tokens=100)`` on a model it
holds whole (/root/reference/llama_p2p_network.py:125, :19) and scales by forwarding whole
requests to peers (:135-154).  On one 8xMI355X node the peers are GPUs holding contiguous layer
shards (pipeline.py), and this module puts the same request API on top of that sharded model:

  * ``PipelineLlama`` (rank 0) has ``Llama``'s contract (llama.py: create_completion, tokenize, the
    completion dict), so ``cached_inference`` / ``handle_requests`` (p2p:84-133) run unchanged on a
    sharded model; ranks 1..S-1 run ``serve_stage``.
  * Requests are admitted into S micro-batch *lanes* of M rows (KV slot = lane*M + row); the lane is
    chosen by the reference's peer scoreboard (placement.PeerScoreboard: p2p:156-168's score, or the
    score-aware policy), so the gossip scores drive request placement onto the pipeline.
  * Rounds: rank 0 broadcasts a plan (admissions, every active lane's positions and samplers, K);
    the admitted prompts are prefilled through all stages in GEMM chunks (hand-off per chunk) and
    the last stage picks each first token; then K decode steps of every active lane run around the
    ring with grouped send/recv (pipeline.Stage's deadlock-free schedule) while the tokens stay on
    the device (last stage -> stage 0); the last stage returns the K tokens per row to rank 0.
  * Token picks are on the device (greedy argmax, or the device sampling chain: penalties, top-k,
    top-p, min-p, temperature, counter-based draws), so sampling requests run K steps per round too.
  * Hidden states cross stage boundaries in bf16 (``handoff_bf16``: half the bytes of f32).
  * Per-stage busy time is reported to rank 0 every few rounds into a second scoreboard whose mean
    times give ``proposed_partition`` (stage placement from measured scores); when the proposed
    split predicts a markedly lower slowest-stage time, ``StagePlanner`` has the scheduler drain the
    lanes and every rank rebuilds its stage on the new layer range (``serve_loop``'s ``rebuild``).
  * A failure on any rank fails every outstanding request and aborts the peers' transport, so no
    caller or peer stays blocked.

Transport- and executor-agnostic like pipeline.Stage: tests drive it on CPU over gloo (and an
in-process rendezvous) with a toy executor, and on one GPU with in-process stage engines.
"""
from __future__ import annotations

import collections
import itertools
import logging
import threading
import time
from typing import Dict, List, Optional

import numpy as np

from .placement import PeerScoreboard

FINISH_LENGTH, FINISH_STOP = 0, 1


_log = logging.getLogger("llama_p2p_amd.pipeserve")

class PRequest:
    __slots__ = ("id", "prompt", "samp", "seed", "max_tokens", "out", "done", "finish", "cancel", "lane", "row",
                 "pos", "t0", "error")

    def __init__(self, rid, prompt, samp, seed, max_tokens):
        self.id, self.prompt, self.samp, self.seed, self.max_tokens = rid, list(prompt), samp, seed, max_tokens
        self.out: List[int] = []
        self.done, self.finish, self.cancel = False, None, False
        self.lane = self.row = -1
        self.pos = 0
        self.t0 = time.perf_counter()
        self.error = None


def _sampling_rows(reqs, firsts=None):
    """Per-row sampler specs for the last stage: (settings, seed, tokens sampled so far, penalty window)."""
    rows = []
    for i, r in enumerate(reqs):
        if r is None:
            rows.append(None)
            continue
        out = r.out if firsts is None else r.out + [firsts[i]]
        hist = (r.prompt + out)[-64:]
        rows.append((dict(r.samp), r.seed, len(out), hist))
    return rows


class Scheduler:
    """Rank 0: pending queue, lane table, placement, round plans, token bookkeeping."""

    def __init__(self, lanes: int, rows: int, n_ctx: int, eos: int, kmax: int = 8, policy: str = "score_aware",
                 seed: Optional[int] = None):
        self.S, self.M, self.n_ctx, self.eos, self.kmax = lanes, rows, n_ctx, eos, kmax
        self.table: List[List[Optional[PRequest]]] = [[None] * rows for _ in range(lanes)]
        self.pending: collections.deque = collections.deque()
        self.reqs: Dict[int, PRequest] = {}
        self.cv = threading.Condition()
        self.ids = itertools.count(1)
        self.board = PeerScoreboard(list(range(lanes)), policy=policy, seed=seed)
        self.stop = False
        self.failed: Optional[str] = None
        self.drain_to = None  # new stage ranges: admit nothing until the lanes are empty, then re-split
        self.rounds = 0
        # placement decisions: (request id, lane, candidate lanes, scoreboard snapshot before the pick)
        self.placements = collections.deque(maxlen=100000)
        self.placement_state = collections.deque(maxlen=100000)  # (avg_time per lane, in flight per lane)

    # ---- request side (any thread)
    def submit(self, prompt, max_tokens, samp, seed):
        with self.cv:
            if self.failed is not None:
                raise RuntimeError(f"pipeline server failed: {self.failed}")
            if self.stop:
                raise RuntimeError("pipeline server shutting down")
            r = PRequest(next(self.ids), prompt, samp, seed, max_tokens)
            self.reqs[r.id] = r
            self.pending.append(r)
            self.cv.notify_all()
            return r.id

    def wait(self, rid):
        with self.cv:
            r = self.reqs[rid]
            self.cv.wait_for(lambda: r.done)
            del self.reqs[rid]
        if r.error:
            raise RuntimeError(f"request failed: {r.error}")
        return list(r.out), r.finish

    def poll(self, rid, n_have):
        with self.cv:
            r = self.reqs[rid]
            self.cv.wait_for(lambda: r.done or len(r.out) > n_have)
            return list(r.out), r.done

    def cancel(self, rid):
        with self.cv:
            self.reqs[rid].cancel = True

    def shutdown(self):
        with self.cv:
            self.stop = True
            self.cv.notify_all()

    def fail_all(self, err: str):
        """A round (or a peer) failed: every queued and admitted request returns the error, and the
        scheduler refuses new ones."""
        with self.cv:
            self.failed = err
            self.stop = True
            for r in list(self.pending) + [x for ln in self.table for x in ln if x is not None]:
                r.error, r.done = err, True
            self.pending.clear()
            self.table = [[None] * self.M for _ in range(self.S)]
            self.cv.notify_all()

    def begin_drain(self, parts):
        with self.cv:
            self.drain_to = [tuple(p) for p in parts]
            self.cv.notify_all()

    def end_drain(self):
        with self.cv:
            self.drain_to = None
            self.cv.notify_all()

    # ---- server side (the round loop)
    def _free_lanes(self):
        return [l for l in range(self.S) if any(x is None for x in self.table[l])]

    def _active(self):
        return [l for l in range(self.S) if any(x is not None for x in self.table[l])]

    def next_plan(self, idle_s: float = 1.0):
        """Block until there is work (or idle_s passed: a heartbeat plan keeps the peers' collectives
        alive); admit pending requests into lanes; return the round plan."""
        with self.cv:
            self.cv.wait_for(lambda: self.stop or self.pending or self._active(), timeout=idle_s)
            if self.stop:
                for r in list(self.pending) + [x for ln in self.table for x in ln if x is not None]:
                    r.error, r.done = "pipeline server shutting down", True
                self.cv.notify_all()
                return {"stop": True}
            if self.drain_to is not None and not self._active():
                return {"repartition": list(self.drain_to)}
            admit = []
            while self.pending and self.drain_to is None:
                r = self.pending[0]
                if r.cancel:  # cancelled before admission: no tokens
                    self.pending.popleft()
                    r.done, r.finish = True, FINISH_STOP
                    continue
                free = self._free_lanes()
                if not free:
                    break
                self.pending.popleft()
                st = self.board.stats()
                snap = {t: (p["success"], p["failure"]) for t, p in st.items()}
                # the rest of what score_aware reads (running mean latency, requests in flight): a
                # placement can be replayed from the log (tests/test_config5_gpu.py)
                self.placement_state.append(({t: p["avg_time"] for t, p in st.items()}, dict(self.board.inflight)))
                lane = self.board.select(candidates=free)
                self.placements.append((r.id, lane, free, snap))
                row = self.table[lane].index(None)
                r.lane, r.row, r.pos = lane, row, len(r.prompt)
                self.table[lane][row] = r
                admit.append(r)
            self.cv.notify_all()
            active = self._active()
            if not admit and not active:
                return {"idle": True}
            room, need = self.kmax, 1
            for l in active:
                for r in self.table[l]:
                    if r is not None and r not in admit:
                        room = min(room, self.n_ctx - r.pos)
                        need = max(need, r.max_tokens - len(r.out))
                    elif r is not None:
                        room = min(room, self.n_ctx - r.pos)
                        need = max(need, r.max_tokens - 1)
            K = max(1, min(room, need))
            if self.pending:
                # requests wait for a row: end the round when the first row runs out of tokens, so
                # its row is free for the next round's admissions (EOS cannot be foreseen)
                soon = min(r.max_tokens - len(r.out) if r not in admit else r.max_tokens - 1
                           for l in active for r in self.table[l] if r is not None)
                K = max(1, min(K, soon))
            lanes = []
            for l in active:
                pos, ids, new = [], [], []
                for row, r in enumerate(self.table[l]):
                    if r is None:
                        pos.append(0), ids.append(0), new.append(False)
                    else:
                        pos.append(r.pos), ids.append(r.out[-1] if r.out else -1), new.append(r in admit)
                lanes.append({"lane": l, "pos": pos, "ids": ids, "new": new,
                              "samp": _sampling_rows(self.table[l])})
            self.rounds += 1
            return {"admit": [{"lane": r.lane, "row": r.row, "ids": r.prompt, "samp": dict(r.samp), "seed": r.seed}
                              for r in admit],
                    "lanes": lanes, "K": K}

    def apply_first(self, plan, firsts):
        """First tokens of the admitted requests (prefill picks), in plan["admit"] order."""
        with self.cv:
            for a, t in zip(plan["admit"], firsts):
                r = self.table[a["lane"]][a["row"]]
                r.out.append(int(t))
            self.cv.notify_all()
        return {(a["lane"], a["row"]): int(t) for a, t in zip(plan["admit"], firsts)}

    def apply_round(self, plan, tokens):
        """tokens[lane] = int array [M][K] (the K decode tokens of every row of that lane).  A row stops
        at EOS, max_tokens, n_ctx or a cancel; tokens after that within the round are discarded."""
        now = time.perf_counter()
        with self.cv:
            for ln in plan["lanes"]:
                l = ln["lane"]
                tk = tokens[l]
                for row, r in enumerate(self.table[l]):
                    if r is None:
                        continue
                    if self._finished(r):  # finished by its first token (prefill pick)
                        self._release(r, now)
                        continue
                    for k in range(plan["K"]):
                        r.pos += 1
                        r.out.append(int(tk[row][k]))
                        if self._finished(r):
                            break
                    if r.done:
                        self._release(r, now)
            self.cv.notify_all()

    def _finished(self, r):
        if r.done:
            return True
        t = r.out[-1] if r.out else None
        if (t == self.eos and not r.samp.get("ignore_eos", False)) or r.cancel:
            r.done, r.finish = True, FINISH_STOP
        elif len(r.out) >= r.max_tokens or r.pos >= self.n_ctx:
            r.done, r.finish = True, FINISH_LENGTH
        return r.done

    def _release(self, r, now):
        self.table[r.lane][r.row] = None
        self.board.update(r.lane, True, now - r.t0)


class StageRunner:
    """Executes round plans on one stage: pipelined prefill of admissions, lane resets, the K-step
    decode ring, and (last stage) the token return to rank 0."""

    def __init__(self, executor, comm, rank: int, world: int, lanes: int, rows: int, kmax: int, device,
                 stage_time_every: int = 8, timing_lock=None):
        import torch

        # stages sharing ONE GPU (local_pipeline_llama): lane steps are timed one stage at a time under
        # this lock, so a stage's event pair does not also count the other stages' kernels
        self.timing_lock = timing_lock

        self.ex, self.comm, self.rank, self.world = executor, comm, rank, world
        self.first, self.last = rank == 0, rank == world - 1
        self.S, self.M, self.kmax, self.device = lanes, rows, kmax, device
        self.torch = torch
        self.stage_time_every = stage_time_every
        self.busy_s, self.rounds = 0.0, 0
        self._events = []  # (start, end) CUDA events around this stage's lane steps
        self.host_exchange_s, self.host_step_s, self.micro_steps = 0.0, 0.0, 0  # host issue cost of the ring
        self.lanes, self.x_in, self.x_out, self.tok = [], [], [], []
        for l in range(lanes):
            b = executor.make_lane([l * rows + i for i in range(rows)], kmax)
            t = torch.zeros(rows, dtype=torch.int32, device=device)
            if self.first or self.last:
                b.bind_ids_tensor(t)
            self.lanes.append(b)
            self.tok.append(t)
            self.x_in.append(executor.alloc_x(rows))
            self.x_out.append(executor.alloc_x(rows))
        self.chunk = executor.prefill_chunk
        self.buf_in = executor.alloc_x(self.chunk)
        self.buf_out = executor.alloc_x(self.chunk)

    # ---- prefill of the admitted prompts: rows of every prompt back to back (each padded to a
    # multiple of 16 rows so chunks form 16-position blocks whatever else is admitted), in hand-off chunks
    def _prefill(self, admit, M, n_ctx):
        slots, pos, ids, ends = [], [], [], []
        for a in admit:
            sl = a["lane"] * M + a["row"]
            n = len(a["ids"])
            slots += [sl] * n
            pos += list(range(n))
            ids += a["ids"]
            ends.append(len(slots) - 1)
            pad = (16 - n % 16) % 16  # near n_ctx: copies of the last row (engine.cpp blocked_rows)
            slots += [sl] * pad
            pos += list(range(n, n + pad)) if n + pad <= n_ctx else [n - 1] * pad
            ids += [a["ids"][-1]] * pad
        samp = [(a["samp"], a["seed"], 0, a["ids"][-64:]) for a in admit]
        firsts: List[int] = []
        k0 = 0
        for i in range(0, len(slots), self.chunk):
            n = min(self.chunk, len(slots) - i)
            xin = xout = None
            if not self.first:
                self.comm.recv(self.buf_in[:n], self.rank - 1)
                xin = self.buf_in[:n]
            if not self.last:
                xout = self.buf_out[:n]
            k1 = k0
            while k1 < len(ends) and ends[k1] < i + n:
                k1 += 1
            rowmap = [e - i for e in ends[k0:k1]] if self.last else []
            toks = self.ex.prefill(slots[i:i + n], pos[i:i + n], ids[i:i + n] if self.first else None, xin, xout,
                                   rowmap, samp[k0:k1] if self.last else None)
            firsts += toks
            k0 = k1
            if not self.last:
                self.comm.send(xout, self.rank + 1)
                self.comm.drain()  # buf_out is reused by the next chunk
        return firsts

    def _step(self, b, x_in=None, x_out=None):
        """One lane step, bracketed by events on the work stream (after the hand-off waits were
        enqueued, so the pair times this stage's kernels only): the stage's busy time."""
        if self.world == 1:  # one stage: no placement to inform
            b.step_tensors(x_in, x_out)
        elif self.device.type == "cuda" and self.timing_lock is not None:
            with self.timing_lock:
                e0, e1 = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
                self.torch.cuda.current_stream().synchronize()  # the hand-off copies before the step
                e0.record()
                b.step_tensors(x_in, x_out)
                e1.record()
                e1.synchronize()
            self.busy_s += e0.elapsed_time(e1) / 1e3
        elif self.device.type == "cuda":
            e0, e1 = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
            e0.record()
            b.step_tensors(x_in, x_out)
            e1.record()
            self._events.append((e0, e1))
        else:
            t = time.perf_counter()
            b.step_tensors(x_in, x_out)
            self.busy_s += time.perf_counter() - t

    def take_busy(self):
        """Seconds this stage spent in its lane steps since the last call (synchronises)."""
        if self._events:
            self._events[-1][1].synchronize()
            self.busy_s += sum(a.elapsed_time(b) for a, b in self._events) / 1e3
            self._events.clear()
        t, self.busy_s = self.busy_s, 0.0
        return t

    def _ring(self, active, K):
        """K decode steps of the active lanes around the ring (pipeline.Stage.decode_steps' grouped
        schedule: the send of micro-step k is posted with the receive of micro-step k+1)."""
        if self.world == 1:
            for _ in range(K):
                for l in active:
                    self._step(self.lanes[l])
            return
        deferred, pending_tokens = [], False
        for _ in range(K):
            for l in active:
                b = self.lanes[l]
                if self.first:
                    recvs = [(self.tok[l], self.world - 1)] if pending_tokens else []
                else:
                    recvs = [(self.x_in[l], self.rank - 1)]
                t0 = time.perf_counter()
                self.comm.exchange(deferred, recvs)
                t1 = time.perf_counter()
                if self.first:
                    self._step(b, None, self.x_out[l])
                    deferred = [(self.x_out[l], 1)]
                elif self.last:
                    self._step(b, self.x_in[l], None)
                    deferred = [(self.tok[l], 0)]
                else:
                    self._step(b, self.x_in[l], self.x_out[l])
                    deferred = [(self.x_out[l], self.rank + 1)]
                self.host_exchange_s += t1 - t0
                self.host_step_s += time.perf_counter() - t1
                self.micro_steps += 1
            pending_tokens = True
        recvs = [(self.tok[l], self.world - 1) for l in active] if self.first else []
        self.comm.exchange(deferred, recvs)

    def run_round(self, plan, sched: Optional[Scheduler] = None, n_ctx: int = 512):
        """One round on this stage.  Rank 0 passes its Scheduler (bookkeeping)."""
        firsts = {}
        if plan["admit"]:
            toks = self._prefill(plan["admit"], self.M, n_ctx)
            if self.last and not self.first:
                self.comm.send_obj(toks, 0)
            if self.first and not self.last:
                toks = self.comm.recv_obj(self.world - 1)
            if self.first:
                firsts = sched.apply_first(plan, toks)
            elif self.last:
                firsts = {(a["lane"], a["row"]): t for a, t in zip(plan["admit"], toks)}
        active = [ln["lane"] for ln in plan["lanes"]]
        for ln in plan["lanes"]:
            l = ln["lane"]
            ids = None
            if self.first:  # next token per row: the prefill pick for rows admitted now, else the last one
                ids = [firsts[(l, r)] if (l, r) in firsts else max(0, t) for r, t in enumerate(ln["ids"])]
            samplers = None
            if self.last:
                rows = []
                for r, spec in enumerate(ln["samp"]):
                    if spec is None:
                        rows.append(({"temperature": 0.0}, 0, 0, []))
                    elif ln["new"][r]:  # its first token was just picked: one draw used, window grows
                        s, seed, nd, win = spec
                        rows.append((s, seed, nd + 1, (list(win) + [firsts[(l, r)]])[-64:]))
                    else:
                        rows.append(spec)
                samplers = self.ex.samplers(rows)
            self.lanes[l].reset(ln["pos"], ids, samplers)
        self._ring(active, plan["K"])
        tokens = None
        if self.last:
            tokens = {l: self.lanes[l].tokens()[:, :plan["K"]] for l in active}
            if not self.first:
                self.comm.send_obj(tokens, 0)
        if self.first and not self.last:
            tokens = self.comm.recv_obj(self.world - 1)
        if self.first:
            sched.apply_round(plan, tokens)
        self.rounds += 1
        return tokens

    def host_stats(self):
        """Host microseconds per decode micro-step: issuing the grouped hand-off (a blocking transport
        waits for its peer inside it) and the lane step (graph replay + events)."""
        n = max(1, self.micro_steps)
        return {"micro_steps": self.micro_steps, "exchange_us": round(self.host_exchange_s / n * 1e6, 1),
                "step_launch_us": round(self.host_step_s / n * 1e6, 1)}

    def close(self):
        for b in self.lanes:
            b.close()


def _abort_peers(comm, err: str):
    """Best effort: make the peers' blocked receives fail instead of waiting forever."""
    abort = getattr(comm, "abort", None)
    if abort is not None:
        try:
            abort(err)
        except Exception:  # noqa: BLE001 -- already failing
            pass


def serve_loop(runner: StageRunner, comm, sched: Optional[Scheduler], n_ctx: int, stage_board=None,
               rebuild=None, planner: Optional["StagePlanner"] = None):
    """The round loop of every rank: rank 0 plans (sched) and broadcasts, every rank runs the plan.
    Per-stage busy time is gathered every runner.stage_time_every rounds into the planner's board
    (or stage_board) on rank 0.  A ``repartition`` plan (the planner's drained re-split) makes every
    rank replace its stage: ``rebuild(new_parts) -> StageRunner``.  Returns the last runner."""
    if planner is not None:
        stage_board = planner.board
    while True:
        try:
            plan = sched.next_plan() if runner.first else None
            if runner.world > 1:
                plan = comm.bcast_obj(plan, 0)
            if plan.get("stop"):
                return runner
            if plan.get("idle"):
                continue
            if "repartition" in plan:
                parts = [tuple(p) for p in plan["repartition"]]
                if rebuild is None:
                    raise RuntimeError("repartition plan on a stage without a rebuild callback")
                runner = rebuild(parts)
                if runner.first:
                    if planner is not None:
                        planner.applied(parts)
                        stage_board = planner.board
                    sched.end_drain()
                continue
            runner.run_round(plan, sched, n_ctx)
            if runner.world > 1 and runner.rounds % runner.stage_time_every == 0:
                busy = runner.take_busy()
                if runner.first:
                    times = [busy] + [comm.recv_obj(r) for r in range(1, runner.world)]
                    if planner is not None:
                        new = planner.observe(times, runner.stage_time_every)
                        if new is not None:
                            sched.begin_drain(new)
                    elif stage_board is not None:
                        for st, t in enumerate(times):
                            stage_board.update(st, True, t / runner.stage_time_every)
                else:
                    comm.send_obj(busy, 0)
        except Exception as e:  # a failed round (or peer) fails every request and the peers' transport
            if sched is not None:
                sched.fail_all(repr(e))
            _abort_peers(comm, repr(e))
            raise


def proposed_partition(stage_board: PeerScoreboard, parts, head_layers: float = 0.0):
    """Stage placement from measured scores: each stage's mean round time / its layer count (the
    last stage's counting the head as ``head_layers`` layers) gives a per-layer cost on that GPU;
    the min-max DP over (stage, first layer) -- O(S * L^2) -- re-splits the layers so that the
    slowest stage's predicted time is minimal (ties: smaller sum of squares).  Returns the current
    ranges unless the new split is strictly better."""
    w = stage_weights(stage_board, parts, head_layers)
    if w is None:
        return list(parts)
    S, n_layer = len(parts), parts[-1][1]
    new = _minmax_split(w, n_layer, head_layers)
    if predicted_max(w, new, head_layers) < predicted_max(w, parts, head_layers) * (1 - 1e-9):
        return new
    return list(parts)


def stage_weights(stage_board: PeerScoreboard, parts, head_layers: float = 0.0):
    """Relative per-layer cost of each stage's GPU (mean 1) from the measured stage times, or None."""
    st = stage_board.stats()
    S = len(parts)
    speeds = []
    for s, (lb, le) in enumerate(parts):
        t = st.get(s, {}).get("avg_time", 0.0) or 0.0
        n = le - lb + (head_layers if s == S - 1 else 0.0)
        speeds.append(t / n if t > 0 else None)
    known = [v for v in speeds if v]
    if not known:
        return None
    mean = sum(known) / len(known)
    return [v / mean if v else 1.0 for v in speeds]


def predicted_max(w, parts, head_layers: float = 0.0) -> float:
    S = len(parts)
    return max(w[s] * (le - lb + (head_layers if s == S - 1 else 0.0)) for s, (lb, le) in enumerate(parts))


def _minmax_split(w, n_layer: int, head_layers: float):
    S = len(w)
    INF = float("inf")
    # best[s][lb] = (max, sumsq, next boundary) for layers [lb, n_layer) over stages s..S-1
    best = [[(INF, INF, -1)] * (n_layer + 1) for _ in range(S)]
    for lb in range(n_layer):
        c = w[S - 1] * (n_layer - lb + head_layers)
        best[S - 1][lb] = (c, c * c, n_layer)
    for s in range(S - 2, -1, -1):
        for lb in range(s, n_layer - (S - 1 - s)):
            cur = (INF, INF, -1)
            for le in range(lb + 1, n_layer - (S - 2 - s)):
                c = w[s] * (le - lb)
                m, q, _ = best[s + 1][le]
                cand = (max(c, m), c * c + q, le)
                if (round(cand[0], 9), cand[1]) < (round(cur[0], 9), cur[1]):
                    cur = cand
            best[s][lb] = cur
    out, lb = [], 0
    for s in range(S):
        le = best[s][lb][2]
        out.append((lb, le))
        lb = le
    return out


class StagePlanner:
    """Rank 0's stage placement (the reference's select_peer / update_peer_performance,
    p2p:156-168, applied to stages): per-stage busy times go into a PeerScoreboard (and a sample list
    per stage).  A proposed split is returned -- the scheduler then drains the lanes and every rank
    rebuilds its stage -- only on evidence:
      * every stage has ``min_samples`` samples since the last re-split (and ``cooldown``
        observations have passed since it),
      * the predicted slowest-stage time drops by at least ``min_gain`` AND by more than ``z`` times
        the largest relative standard error of a stage's mean time (a gain inside the noise of the
        measurement is no reason to rebuild every stage),
      * at most ``max_resplits`` re-splits over the planner's life.
    Every decision that returns a split is logged and kept in ``history``; ``last`` holds the most
    recent evaluation."""

    SAMPLE_WINDOW = 512

    def __init__(self, parts, head_layers: float = 0.0, min_gain: float = 0.10, min_samples: int = 8,
                 enabled: bool = True, z: float = 3.0, max_resplits: int = 2, cooldown: int = 8):
        self.parts = [tuple(p) for p in parts]
        self.head_layers, self.min_gain, self.min_samples, self.enabled = head_layers, min_gain, min_samples, enabled
        self.z, self.max_resplits, self.cooldown = z, max_resplits, cooldown
        self.board = PeerScoreboard(list(range(len(parts))), policy="score_aware")
        # the most recent SAMPLE_WINDOW stage times per stage (bounded for a long-lived server)
        self.samples = [collections.deque(maxlen=self.SAMPLE_WINDOW) for _ in parts]
        self.n_obs, self.obs_at_resplit, self.resplits = 0, 0, 0
        self.history = []  # every re-split returned: parts before / after, predicted times, evidence
        self.last: Optional[dict] = None
        self.pending = None  # a returned re-split not yet applied (the lanes are draining)

    @staticmethod
    def _rse(xs) -> float:
        """Relative standard error of the mean of xs."""
        n = len(xs)
        if n < 2:
            return float("inf")
        m = sum(xs) / n
        if m <= 0:
            return float("inf")
        var = sum((x - m) ** 2 for x in xs) / (n - 1)
        return (var ** 0.5) / m / n ** 0.5

    def observe(self, times, rounds_per_sample: int = 1):
        planning = self.enabled and self.resplits < self.max_resplits
        for s, t in enumerate(times):
            v = t / rounds_per_sample
            self.board.update(s, True, v)
            if planning:  # no samples kept once no re-split can follow
                self.samples[s].append(v)
        self.n_obs += 1
        if not planning or self.pending is not None:
            return None  # (pending: a re-split is draining; it is proposed once)
        if self.resplits and self.n_obs - self.obs_at_resplit < self.cooldown:
            return None
        if any(len(x) < self.min_samples for x in self.samples):
            return None
        w = stage_weights(self.board, self.parts, self.head_layers)
        if w is None:
            return None
        new = proposed_partition(self.board, self.parts, self.head_layers)
        cur_t, new_t = predicted_max(w, self.parts, self.head_layers), predicted_max(w, new, self.head_layers)
        gain = 1.0 - new_t / cur_t if cur_t > 0 else 0.0
        noise = max(self._rse(x) for x in self.samples)
        need = max(self.min_gain, self.z * noise)
        self.last = {"from": list(self.parts), "proposed": list(new), "predicted_max_from": cur_t,
                     "predicted_max_to": new_t, "gain": gain, "noise_rse": noise, "needed": need,
                     "samples": min(len(x) for x in self.samples)}
        if new != self.parts and gain >= need:
            self.history.append(dict(self.last, to=list(new), weights=w, t=time.time()))
            self.resplits += 1
            self.pending = list(new)
            _log.warning("stage planner: re-split %s -> %s (predicted slowest stage %.3g -> %.3g, gain %.1f%% "
                         "> needed %.1f%%, %d samples per stage)", self.parts, new, cur_t, new_t, 100 * gain,
                         100 * need, self.last["samples"])
            return new
        return None

    def applied(self, parts):
        self.pending = None
        self.parts = [tuple(p) for p in parts]
        self.board = PeerScoreboard(list(range(len(parts))), policy="score_aware")
        self.samples = [collections.deque(maxlen=self.SAMPLE_WINDOW) for _ in parts]
        self.obs_at_resplit = self.n_obs


# ------------------------------------------------------------------------------ engine executor
class EngineExecutor:
    """The MI355X engine as a pipeline-serving stage (engine.Engine with a layer range)."""

    def __init__(self, eng, device, prefill_chunk: int = 1024):
        import torch

        from .engine import row_samplers, sampling, torch_stream_handle

        self.eng, self.device, self.torch = eng, device, torch
        self._row_samplers, self._sampling, self._stream = row_samplers, sampling, torch_stream_handle
        self.first, self.last = bool(eng.info.has_embed), bool(eng.info.has_head)
        self.n_embd = eng.n_embd
        self.dtype = torch.bfloat16 if eng.handoff_bf16 else torch.float32
        self.prefill_chunk = prefill_chunk

    def alloc_x(self, rows):
        return self.torch.empty((rows, self.n_embd), dtype=self.dtype, device=self.device)

    def prefill(self, slots, pos, ids, x_in, x_out, rowmap, samp):
        samplers = self.samplers(samp) if samp else None
        return self.eng.stage_rows_pick(slots, pos, ids, x_in.data_ptr() if x_in is not None else 0,
                                        x_out.data_ptr() if x_out is not None else 0, rowmap, samplers,
                                        self._stream())

    def make_lane(self, slots, kmax):
        return _EngineLane(self.eng.batch(slots, [0] * len(slots), [0] * len(slots) if self.first else None,
                                          max_steps=kmax), self._stream)

    def samplers(self, rows):
        return self._row_samplers([(self._sampling(**s), seed, nd, win) for s, seed, nd, win in rows])


class _EngineLane:
    def __init__(self, batch, stream):
        self.b, self._stream = batch, stream

    def reset(self, pos, ids=None, samplers=None):
        self.b.reset(pos, ids, samplers, self._stream())

    def step_tensors(self, x_in=None, x_out=None):
        self.b.step_tensors(x_in, x_out)

    def bind_ids_tensor(self, t):
        self.b.bind_ids_tensor(t)

    def tokens(self):
        return self.b.tokens()

    def close(self):
        self.b.close()


# ------------------------------------------------------------------------------ request front
SAMPLING_KEYS = ("temperature", "top_k", "top_p", "min_p", "repeat_penalty", "repeat_last_n", "ignore_eos",
                 "frequency_penalty", "presence_penalty")


class PipelineFront:
    """Rank 0's request API with engine.Engine's method names (submit / poll / cancel / wait), so
    llama.Llama.create_completion drives the pipeline unchanged.  The round loop runs on a thread."""

    def __init__(self, runner: StageRunner, comm, sched: Scheduler, n_ctx: int, n_vocab: int, n_embd: int,
                 stage_board: Optional[PeerScoreboard] = None, rebuild=None, planner: Optional[StagePlanner] = None):
        self.runner, self.comm, self.sched, self.n_ctx = runner, comm, sched, n_ctx
        self.n_vocab, self.n_embd = n_vocab, n_embd
        self.stage_board = stage_board
        self.planner = planner
        self._rebuild = rebuild
        self.engine = None  # this stage's engine, closed with the front
        self.stage_threads = []  # in-process stages (local_pipeline_llama): joined on close
        self.error = None
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def _loop(self):
        try:
            dev = self.runner.device
            if dev.type == "cuda":  # the round loop's own (non-default) stream: engine calls and hand-offs
                import torch

                torch.cuda.set_device(dev)
                torch.cuda.set_stream(torch.cuda.Stream(device=dev))
            rebuild = None
            if self._rebuild is not None:
                def rebuild(parts):
                    self.runner = self._rebuild(self, parts)
                    return self.runner
            self.runner = serve_loop(self.runner, self.comm, self.sched, self.n_ctx, self.stage_board,
                                     rebuild=rebuild, planner=self.planner)
        except Exception as e:  # noqa: BLE001 -- surfaced to callers through their requests
            self.error = e
            self.sched.fail_all(repr(e))

    def submit(self, ids, max_tokens, seed=None, **kw):
        import random

        samp = {k: kw[k] for k in SAMPLING_KEYS if k in kw}
        samp.setdefault("temperature", 0.0)
        tk, rl = samp.get("top_k", 40), samp.get("repeat_last_n", 64)
        sampling = samp["temperature"] > 0 or samp.get("repeat_penalty", 1.0) != 1.0 or \
            samp.get("frequency_penalty", 0.0) != 0.0 or samp.get("presence_penalty", 0.0) != 0.0
        if sampling and not (1 <= tk <= 64 and 0 <= rl <= 64):
            raise ValueError("pipeline serving samples on the device: top_k must be 1..64 and repeat_last_n 0..64")
        s = seed if seed is not None and seed >= 0 else random.getrandbits(63)
        mt = max_tokens if max_tokens and max_tokens > 0 else self.n_ctx - len(ids)
        # Scheduler.submit refuses under its lock once the round loop has failed (fail_all)
        return self.sched.submit(list(map(int, ids)), min(mt, self.n_ctx - len(ids)), samp, s)

    def poll(self, rid, n_have=0):
        return self.sched.poll(rid, n_have)

    def cancel(self, rid):
        self.sched.cancel(rid)

    def wait(self, rid, cap=None):
        return self.sched.wait(rid)

    def generate(self, ids, max_tokens, **kw):
        return self.wait(self.submit(ids, max_tokens, **kw))

    def close(self):
        self.sched.shutdown()
        self._thread.join(timeout=60)
        self.runner.close()
        if self.engine is not None:
            self.engine.close()
            self.engine = None
        # in-process stages leave serve_loop on the stop plan and free their engines: wait for them,
        # or the interpreter may finalise while a stage thread is still inside the HIP runtime
        for th in self.stage_threads:
            th.join(timeout=120)
        self.stage_threads = []


def _layer_costs(model_path):
    """(bytes per layer, head bytes) of a synthetic model path, or None for a GGUF."""
    from . import synth

    syn = synth.parse_synthetic_path(model_path)
    if syn is None:
        return None
    sh = syn[0]
    return 2 * (2 * sh.n_embd ** 2 + 2 * sh.n_embd * sh.n_embd_kv + 3 * sh.n_embd * sh.n_ff), 2 * sh.n_vocab * sh.n_embd


def _stage_setup(model_path, rank, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, parts=None):
    """Engine holding this rank's byte-balanced layer range, its executor and runner pieces."""
    from . import engine as E
    from .pipeline import partition_layers

    if parts is None:
        costs = _layer_costs(model_path)
        if costs is None:
            raise ValueError("pipeline serving of a GGUF needs explicit stage ranges (parts=...)")
        from . import synth

        sh = synth.parse_synthetic_path(model_path)[0]
        parts = partition_layers(sh.n_layer, costs[0], costs[1], world)
    lb, le = parts[rank]
    eng = E.Engine(model_path, n_ctx=n_ctx, n_seq_max=lanes * rows, layer_begin=lb, layer_end=le,
                   device=device.index if device.type == "cuda" else -1, handoff_bf16=handoff_bf16)
    return eng, parts


def serve_stage(model_path: str, comm, rank: int, world: int, lanes: int, rows: int = 32, n_ctx: int = 512,
                kmax: int = 8, device=None, handoff_bf16: bool = True, parts=None, timing_lock=None,
                stage_time_every: int = 8):
    """Ranks 1..S-1: hold a stage and execute rank 0's round plans until it stops (a repartition
    plan replaces the stage engine by one holding the new layer range)."""
    import torch

    device = device or torch.device("cuda", torch.cuda.current_device())
    eng, parts = _stage_setup(model_path, rank, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, parts)
    held = {"eng": eng, "runner": StageRunner(EngineExecutor(eng, device), comm, rank, world, lanes, rows, kmax,
                                              device, stage_time_every, timing_lock=timing_lock)}

    def rebuild(new_parts):
        held["runner"].close()
        held["eng"].close()
        held["runner"] = held["eng"] = None
        e2, _ = _stage_setup(model_path, rank, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, new_parts)
        held["eng"] = e2
        held["runner"] = StageRunner(EngineExecutor(e2, device), comm, rank, world, lanes, rows, kmax, device,
                                     stage_time_every, timing_lock=timing_lock)
        return held["runner"]

    try:
        serve_loop(held["runner"], comm, None, n_ctx, rebuild=rebuild)
    finally:
        if held["runner"] is not None:
            held["runner"].close()
        if held["eng"] is not None:
            held["eng"].close()


def pipeline_llama(model_path: str, comm, world: int, lanes: Optional[int] = None, rows: int = 32,
                   n_ctx: int = 512, kmax: int = 8, device=None, handoff_bf16: bool = True, parts=None,
                   policy: str = "score_aware", seed: Optional[int] = None, verbose: bool = False,
                   repartition: bool = False, min_gain: float = 0.10, timing_lock=None, planner_kw=None,
                   stage_time_every: int = 8):
    """Rank 0: a Llama-compatible object whose completions run on the S-stage pipeline (ranks 1..S-1
    run serve_stage with the same arguments).  ``repartition`` (opt-in): apply the stage planner's
    re-splits (drain, rebuild every stage -- a full weight reload -- resume) when the measured stage
    times predict >= ``min_gain`` lower slowest-stage time beyond their noise (StagePlanner;
    ``planner_kw`` overrides its evidence thresholds)."""
    import torch

    from .llama import Llama

    device = device or torch.device("cuda", torch.cuda.current_device())
    lanes = lanes or world
    eng, parts = _stage_setup(model_path, 0, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, parts)
    runner = StageRunner(EngineExecutor(eng, device), comm, 0, world, lanes, rows, kmax, device,
                         stage_time_every, timing_lock=timing_lock)
    sched = Scheduler(lanes, rows, n_ctx, eng.info.eos_id, kmax, policy=policy, seed=seed)
    costs = _layer_costs(model_path)
    head_layers = costs[1] / costs[0] if costs else 1.0
    planner = StagePlanner(parts, head_layers=head_layers, min_gain=min_gain, enabled=repartition, **(planner_kw or {}))

    def rebuild(front, new_parts):
        front.runner.close()
        front.engine.close()
        front.engine = None
        e2, _ = _stage_setup(model_path, 0, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, new_parts)
        front.engine = e2
        llm.parts = list(new_parts)
        return StageRunner(EngineExecutor(e2, device), comm, 0, world, lanes, rows, kmax, device,
                           stage_time_every, timing_lock=timing_lock)

    # vocabulary size from the model (stage 0 has no head: n_vocab comes from the model info)
    front = PipelineFront(runner, comm, sched, n_ctx, eng.info.n_vocab, eng.info.n_embd, planner.board,
                          rebuild=rebuild, planner=planner)
    llm = Llama.from_engine(model_path, front, n_ctx=n_ctx, verbose=verbose)
    front.engine = eng
    llm.parts, llm.stage_board, llm.scheduler, llm.planner = parts, planner.board, sched, planner
    return llm


# ------------------------------------------------------------------------------ in-process stages
class LocalHub:
    """Mailboxes between in-process stages (one queue per ordered (src, dst) pair)."""

    def __init__(self):
        import queue

        self._q = collections.defaultdict(queue.Queue)
        self.lock = threading.Lock()
        self.aborted: Optional[str] = None

    def q(self, src, dst):
        with self.lock:
            return self._q[(src, dst)]


class LocalComm:
    """Hand-offs between stages living in ONE process (S stage engines on one GPU, each stage a
    thread with its own stream): a send snapshots the tensor (clone on the sender's stream, then
    that stream is synchronised) into the receiver's mailbox, a receive copies it in on the
    receiver's stream; sends never block, so the grouped ring schedule cannot deadlock.  Control
    objects travel through the same mailboxes."""

    def __init__(self, hub: LocalHub, rank: int, world: int, timeout: float = 120.0):
        self.hub, self.rank, self.world, self.timeout = hub, rank, world, timeout

    def _get(self, src):
        """Next message from src; raises once any stage has aborted (or after the timeout)."""
        import queue

        q = self.hub.q(src, self.rank)
        t0 = time.time()
        while True:
            if self.hub.aborted is not None:
                raise RuntimeError(f"pipeline peer aborted: {self.hub.aborted}")
            try:
                return q.get(timeout=0.1)
            except queue.Empty:
                if time.time() - t0 > self.timeout:
                    raise TimeoutError(f"stage {self.rank}: nothing from stage {src} in {self.timeout:.0f}s")

    def abort(self, err: str):
        self.hub.aborted = self.hub.aborted or f"stage {self.rank}: {err}"

    def send(self, t, dst):
        import torch

        c = t.clone()
        if c.is_cuda:
            torch.cuda.current_stream().synchronize()
        self.hub.q(self.rank, dst).put(("t", c))

    def recv(self, t, src):
        kind, c = self._get(src)
        assert kind == "t", "hand-off order mismatch: expected a tensor"
        t.copy_(c)
        if c.is_cuda:  # the snapshot came from the sender stream's pool: it must not return there (and be
            import torch  # reused by the sender) before this stream's copy has run

            torch.cuda.current_stream().synchronize()

    def exchange(self, sends, recvs):
        for t, d in sends:
            self.send(t, d)
        for t, s in recvs:
            self.recv(t, s)

    def drain(self):
        pass

    def send_obj(self, obj, dst):
        self.hub.q(self.rank, dst).put(("o", obj))

    def recv_obj(self, src):
        kind, obj = self._get(src)
        assert kind == "o", "hand-off order mismatch: expected an object"
        return obj

    def bcast_obj(self, obj, src=0):
        if self.rank == src:
            for r in range(self.world):
                if r != src:
                    self.send_obj(obj, r)
            return obj
        return self.recv_obj(src)


def local_pipeline_llama(model_path: str, parts, lanes: int = 2, rows: int = 8, n_ctx: int = 512, kmax: int = 8,
                         device=None, handoff_bf16: bool = True, policy: str = "score_aware",
                         seed: Optional[int] = None, repartition: bool = False, min_gain: float = 0.10,
                         planner_kw=None, stage_time_every: int = 8):
    """S = len(parts) stage engines of one model in THIS process (one GPU), each served by its own
    thread and stream, behind one Llama-compatible front: the pipeline server end to end without a
    multi-GPU launch (tests; a 1-GPU rehearsal of the S-GPU layout).  With ``repartition`` the stages
    time their lane steps one at a time (a shared lock), so the planner sees each stage's own cost."""
    import torch

    torch.cuda.init()  # lazy CUDA init here, not raced by the stage threads below
    device = device or torch.device("cuda", torch.cuda.current_device())
    world = len(parts)
    hub = LocalHub()
    comms = [LocalComm(hub, r, world) for r in range(world)]
    ready, errors, threads = threading.Barrier(world), [], []
    timing_lock = threading.Lock() if repartition else None

    def stage(r):
        try:
            torch.cuda.set_device(device)
            torch.cuda.set_stream(torch.cuda.Stream(device=device))
            ready.wait()
            serve_stage(model_path, comms[r], r, world, lanes, rows, n_ctx, kmax, device, handoff_bf16, parts,
                        timing_lock=timing_lock, stage_time_every=stage_time_every)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    for r in range(1, world):
        th = threading.Thread(target=stage, args=(r,), daemon=True)
        th.start()
        threads.append(th)
    torch.cuda.set_stream(torch.cuda.Stream(device=device))
    ready.wait()
    llm = pipeline_llama(model_path, comms[0], world, lanes, rows, n_ctx, kmax, device, handoff_bf16, parts,
                         policy=policy, seed=seed, repartition=repartition, min_gain=min_gain,
                         timing_lock=timing_lock, planner_kw=planner_kw, stage_time_every=stage_time_every)
    llm._engine.stage_threads = threads
    llm._stage_threads, llm._stage_errors = threads, errors
    return llm
