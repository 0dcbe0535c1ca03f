"""Pipeline-parallel decode: the reference's peer mesh mapped onto one 8-GPU node.

The reference scales by forwarding whole requests to peers that each hold the
full model (/root/reference/llama_p2p_network.py:135-154).  On an MI355X node
the peers are GPUs and the model is sharded instead (BASELINE.json north_star,
SURVEY.md §8e): rank r holds a contiguous, byte-balanced range of layers
(stage r), hidden states go stage -> stage with send/recv (RCCL over xGMI on
GPUs, gloo in CPU tests), and the greedy token ids go from the last stage back
to stage 0.  S micro-batches are in flight so every stage is busy: aggregate
throughput ~ S x one stage's rate (weak scaling: per-GPU work is fixed).

This module is transport- and executor-agnostic: ``Stage`` drives any engine
object with the ``Engine``/``Batch`` tensor interface (engine.py), and tests
drive it on CPU with gloo and a numpy stand-in executor.
"""
from __future__ import annotations

import json
import os
import time
from typing import List, Sequence, Tuple


def partition_layers(n_layer: int, layer_cost: float, head_cost: float, n_stages: int,
                     embed_cost: float = 0.0) -> List[Tuple[int, int]]:
    """Contiguous layer ranges minimising the most expensive stage.

    Stage 0 also carries the embedding, the last stage the output norm + lm_head
    (1.05 GB for Llama-3-8B = 2.4 layers' worth of bytes), so stages are balanced
    by streamed bytes, not by layer count.  Every stage gets at least one layer.
    """
    if n_stages < 1 or n_stages > n_layer:
        raise ValueError(f"need 1 <= stages <= {n_layer}, got {n_stages}")

    def cost(lb, le, s):
        c = (le - lb) * layer_cost
        if s == 0:
            c += embed_cost
        if s == n_stages - 1:
            c += head_cost
        return c

    # DP over (stage, boundary): minimise the max stage cost, then the sum of squared
    # costs (spread the slack instead of dumping it on one stage)
    import functools

    @functools.lru_cache(maxsize=None)
    def best(s, lb):
        """Best split of layers [lb, n_layer) over stages s..n_stages-1 -> (max, sumsq, bounds)."""
        if s == n_stages - 1:
            c = cost(lb, n_layer, s)
            return (c, c * c, ((lb, n_layer),))
        out = None
        for le in range(lb + 1, n_layer - (n_stages - 1 - s) + 1):
            c = cost(lb, le, s)
            m, q, rest = best(s + 1, le)
            cand = (max(c, m), c * c + q, ((lb, le),) + rest)
            if out is None or (round(cand[0], 6), cand[1]) < (round(out[0], 6), out[1]):
                out = cand
        return out

    return [tuple(b) for b in best(0, 0)[2]]


def stage_plan(shape, n_stages: int, seqs_per_micro_batch: int, n_ctx: int, hbm_bytes: int = 288 * 10 ** 9):
    """Byte-balanced stages of ``shape`` and each stage's device memory: bf16 weights (+ the token
    embedding table on stage 0, output norm + lm_head on the last), the f16 KV cache for the
    S * M slots the pipeline keeps (n_seq_max = S micro-batches x M sequences, each of n_ctx
    positions rounded up to 64), and the engine's prefill-chunk activations.  Raises if a stage does
    not fit ``hbm_bytes`` (288 GB per MI355X)."""
    h, kv, ff, V = shape.n_embd, shape.n_embd_kv, shape.n_ff, shape.n_vocab
    layer_bytes = 2 * (2 * h * h + 2 * h * kv + 3 * h * ff) + 2 * h * 4
    head_bytes = 2 * V * h + h * 4
    parts = partition_layers(shape.n_layer, layer_bytes, head_bytes, n_stages, embed_cost=0)
    slots = n_stages * seqs_per_micro_batch
    ctx_stride = (n_ctx + 63) // 64 * 64
    kv_per_layer = 2 * slots * ctx_stride * kv * 2
    act = 4096 * (3 * h * 4 + 2 * h * 2 + ff * 2)  # PREFILL_ROWS rows: x, q, ssq-ish f32 + bf16 operands
    plan = []
    for s, (lb, le) in enumerate(parts):
        nl = le - lb
        w = nl * layer_bytes + (V * h * 2 if s == 0 else 0) + (head_bytes if s == n_stages - 1 else 0)
        total = w + nl * kv_per_layer + act
        if total > hbm_bytes:
            raise ValueError(f"stage {s} ({nl} layers) needs {total / 1e9:.1f} GB > {hbm_bytes / 1e9:.0f} GB")
        plan.append({"stage": s, "layers": (lb, le), "weight_bytes": w, "kv_bytes": nl * kv_per_layer,
                     "total_bytes": total})
    return plan


class TorchComm:
    """Point-to-point hand-offs over torch.distributed (nccl = RCCL on ROCm, or gloo).

    ``exchange`` posts a set of sends and receives as ONE group
    (``batch_isend_irecv`` = ncclGroupStart/End): RCCL's ncclSend may not complete
    until the peer has posted the matching ncclRecv, so ops that must progress
    together have to share a group (see ``Stage.decode_steps``).
    """

    def __init__(self, rank: int, world: int, obj_group=None, host_staged: bool = False):
        import torch.distributed as dist

        self.dist, self.rank, self.world = dist, rank, world
        self._pending = []
        # host_staged (gloo over device tensors: the multi-process rehearsal on ONE GPU, where RCCL
        # cannot run two ranks): each hand-off is copied to host memory, sent over gloo, copied back
        self.host_staged = host_staged
        # control-plane objects (round plans, token lists) go over a gloo group: host data, no device
        # round trip; on a gloo default group that group is reused
        if obj_group is None and world > 1 and dist.get_backend() != "gloo":
            obj_group = dist.new_group(backend="gloo")
        self.obj_group = obj_group

    def bcast_obj(self, obj, src: int = 0):
        box = [obj]
        self.dist.broadcast_object_list(box, src=src, group=self.obj_group)
        return box[0]

    def send_obj(self, obj, dst: int):
        self.dist.send_object_list([obj], dst=dst, group=self.obj_group)

    def recv_obj(self, src: int):
        box = [None]
        self.dist.recv_object_list(box, src=src, group=self.obj_group)
        return box[0]

    def _host(self, t):
        return t.cpu() if self.host_staged and t.is_cuda else t  # .cpu() waits for the stream's writes

    def send(self, t, dst: int):
        c = self._host(t)
        w = self.dist.isend(c, dst)
        self._pending.append((w, c))
        return w

    def recv(self, t, src: int):
        c = self._host(t) if t.is_cuda and self.host_staged else t
        self.dist.recv(c, src)
        if c is not t:
            t.copy_(c)

    def exchange(self, sends, recvs):
        """sends = [(tensor, dst)], recvs = [(tensor, src)]; returns when all completed
        (on nccl: the current stream waits for them)."""
        P = self.dist.P2POp
        sends = [(self._host(t), d) for t, d in sends]
        rbufs = [(self._host(t) if self.host_staged else t, t, s) for t, s in recvs]
        ops = [P(self.dist.isend, t, d) for t, d in sends] + [P(self.dist.irecv, c, s) for c, _, s in rbufs]
        if not ops:
            return
        for w in self.dist.batch_isend_irecv(ops):
            w.wait()
        for c, t, _ in rbufs:
            if c is not t:
                t.copy_(c)

    def drain(self):
        for w, _ in self._pending:
            w.wait()
        self._pending.clear()

    def abort(self, err: str = ""):
        """Tear the communicators down so that peers blocked in a receive fail instead of waiting
        forever (gloo: "connection closed by peer"; RCCL: the communicator abort)."""
        for g in ([self.obj_group] if self.obj_group is not None else []) + [None]:
            try:
                self.dist.distributed_c10d._abort_process_group(g)
            except Exception:  # noqa: BLE001 -- best effort on an already failing rank
                pass


class Stage:
    """One pipeline stage: S micro-batches of M sequences, greedy decode."""

    def __init__(self, eng, comm, rank: int, world: int, n_embd: int, device, micro_batches: int, dtype=None):
        import torch

        self.eng, self.comm, self.rank, self.world = eng, comm, rank, world
        self.first, self.last = rank == 0, rank == world - 1
        self.S = micro_batches
        self.n_embd = n_embd
        self.device = device
        self.torch = torch
        self.dtype = dtype or torch.float32  # hand-off dtype (the engine's handoff_bf16)
        self.batches = []
        self.x_in, self.x_out, self.tok = [], [], []
        self.pending_tokens = False  # stage 0 has not yet received the last step's tokens
        self.deferred = []  # sends of the previous micro-step, posted with the next receive
        # host seconds spent issuing hand-offs / lane steps, and micro-steps issued (the hand-off's
        # host cost per micro-step against the stage's device time, bench line "host_per_micro_step")
        self.host_exchange_s, self.host_step_s, self.micro_steps = 0.0, 0.0, 0

    # -- prefill (untimed): prompt rows through every stage, 64 rows per hand-off
    def prefill(self, mb_rows: Sequence[Tuple[List[int], List[int], List[int]]], chunk: int = 64):
        """mb_rows[mb] = (slots, positions, ids) of every prompt row of micro-batch mb."""
        torch = self.torch
        buf_in = torch.empty((chunk, self.n_embd), dtype=self.dtype, device=self.device)
        buf_out = torch.empty((chunk, self.n_embd), dtype=self.dtype, device=self.device)
        for slots, pos, ids in mb_rows:
            for i in range(0, len(slots), chunk):
                n = min(chunk, len(slots) - i)
                xin = None
                if not self.first:
                    self.comm.recv(buf_in[:n], self.rank - 1)
                    xin = buf_in[:n]
                xout = None if self.last else buf_out[:n]
                self.eng.stage_rows_tensors(slots[i:i + n], pos[i:i + n], ids[i:i + n] if self.first else None,
                                            xin, xout)
                if not self.last:
                    self.comm.send(xout, self.rank + 1)
                    self.comm.drain()  # buf_out is reused by the next chunk

    def setup_decode(self, mb_state: Sequence[Tuple[List[int], List[int], List[int]]], max_steps: int):
        """mb_state[mb] = (slots, positions of the next token, next token ids)."""
        torch = self.torch
        M = len(mb_state[0][0])
        for slots, pos, ids in mb_state:
            b = self.eng.batch(slots, pos, ids if self.first else None, max_steps=max_steps if self.last else 0)
            t = torch.tensor(ids if self.first else [0] * M, dtype=torch.int32, device=self.device)
            if self.first or self.last:
                b.bind_ids_tensor(t)
            self.batches.append(b)
            self.tok.append(t)
            self.x_in.append(torch.empty((M, self.n_embd), dtype=self.dtype, device=self.device))
            self.x_out.append(torch.empty((M, self.n_embd), dtype=self.dtype, device=self.device))

    def decode_steps(self, n_steps: int, step0: int = 0):
        """n_steps greedy tokens for every micro-batch, micro-batches interleaved.

        Per micro-step k a stage receives its input (x from stage r-1; on stage 0 the
        tokens of micro-step k-S from the last stage), computes, and sends its output.
        The send of micro-step k is deferred and posted in ONE group with the receive
        of micro-step k+1.  Under rendezvous semantics (an RCCL send completes only
        once its receive is posted) ungrouped ops deadlock as soon as S > 1: stage 0
        would block sending x of micro-batch 1 while the last stage blocks sending the
        tokens of micro-batch 0, each waiting for the other's next op.  Grouped, the
        wait graph has no cycle (tests/test_pipeline_cpu.py runs the schedule over a
        strict rendezvous transport)."""
        for st in range(step0, step0 + n_steps):
            for mb, b in enumerate(self.batches):
                if self.world == 1:
                    b.step_tensors()
                    continue
                if self.first:
                    recvs = [(self.tok[mb], self.world - 1)] if self.pending_tokens else []
                else:
                    recvs = [(self.x_in[mb], self.rank - 1)]
                t0 = time.perf_counter()
                self.comm.exchange(self.deferred, recvs)
                t1 = time.perf_counter()
                if self.first:
                    b.step_tensors(None, self.x_out[mb])
                    self.deferred = [(self.x_out[mb], 1)]
                elif self.last:
                    b.step_tensors(self.x_in[mb], None)
                    self.deferred = [(self.tok[mb], 0)]
                else:
                    b.step_tensors(self.x_in[mb], self.x_out[mb])
                    self.deferred = [(self.x_out[mb], self.rank + 1)]
                self.host_exchange_s += t1 - t0
                self.host_step_s += time.perf_counter() - t1
                self.micro_steps += 1
            self.pending_tokens = True

    def finish(self):
        """Drain the ring: post the deferred send, and stage 0 receives the tokens of the
        final step.  Must run before any device-wide synchronize, or the last stage's
        send of those tokens would never complete."""
        if self.world > 1:
            recvs = []
            if self.first and self.pending_tokens:
                recvs = [(self.tok[mb], self.world - 1) for mb in range(len(self.batches))]
            self.comm.exchange(self.deferred, recvs)
            self.deferred = []
        self.pending_tokens = False

    def tokens(self):
        return [b.tokens() for b in self.batches] if self.last else None


def bench_main(args, metric: str, make_prompts):
    """bench.py --gpus N, one pipeline stage per rank (started by torch.distributed.run or by
    launch.spawn_ranks).  ``args.dry_run``: the same schedule, timing and report on CPU over gloo
    with ``DryEngine`` standing in for the HIP engine (tests/test_bench_launch.py)."""
    import zlib

    import numpy as np
    import torch
    import torch.distributed as dist

    from . import synth

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dry = bool(getattr(args, "dry_run", False))
    host = bool(getattr(args, "host_handoff", False)) and not dry
    f32 = getattr(args, "handoff", "bf16") == "f32"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world == 1:
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if dry:
        device = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    elif host:  # rehearsal: real engines, ranks may share GPUs, hand-offs through host memory over gloo
        local = local % max(1, torch.cuda.device_count())
        device = torch.device("cuda", local)
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        device = torch.device("cuda", local)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    world_rd, backend = dist.get_world_size(), str(dist.get_backend())
    if world_rd != world:
        raise RuntimeError(f"torch.distributed world size {world_rd} != WORLD_SIZE {world}")
    shape = synth.SHAPES[args.model]
    layer_bytes = 2 * (2 * shape.n_embd ** 2 + 2 * shape.n_embd * shape.n_embd_kv + 3 * shape.n_embd * shape.n_ff)
    head_bytes = 2 * shape.n_vocab * shape.n_embd
    parts = partition_layers(shape.n_layer, layer_bytes, head_bytes, world, embed_cost=0)
    lb, le = parts[rank]
    S = int(getattr(args, "micro_batches", 0) or world)
    M = args.seqs
    comm = TorchComm(rank, world, host_staged=host) if world > 1 else None
    if dry:
        eng = DryEngine(lb, le, S * M, shape.n_layer)
        vocab = eng.V
        stage = Stage(eng, comm, rank, world, eng.H, device, S)
        sync = lambda: None  # noqa: E731
    else:
        from .engine import Engine

        eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=args.n_ctx, n_seq_max=S * M, layer_begin=lb,
                     layer_end=le, device=local, handoff_bf16=not f32)
        vocab = shape.n_vocab
        work_stream = torch.cuda.Stream(device=local)  # engine kernels and RCCL hand-offs are ordered on it
        torch.cuda.set_stream(work_stream)
        stage = Stage(EngineAdapter(eng), comm, rank, world, shape.n_embd, device, S,
                      dtype=torch.float32 if f32 else torch.bfloat16)  # hidden states cross stages in bf16
        sync = torch.cuda.synchronize
    # every rank's engine exists before any rank computes: a context or queue being created on the
    # same GPU while another rank's kernels run is when results were seen to vary
    sync()
    dist.barrier()
    prompts = make_prompts(vocab, S * M)
    mb_rows, mb_state = [], []
    for mb in range(S):
        slots, pos, ids, st = [], [], [], ([], [], [])
        for i in range(M):
            p = prompts[mb * M + i]
            sl = mb * M + i
            slots += [sl] * (len(p) - 1)
            pos += list(range(len(p) - 1))
            ids += [int(t) for t in p[:-1]]
            st[0].append(sl)
            st[1].append(len(p) - 1)
            st[2].append(int(p[-1]))
        mb_rows.append((slots, pos, ids))
        mb_state.append(st)
    stage.prefill(mb_rows, chunk=max(1, min(64, int(getattr(args, "prefill_chunk", 64) or 64))))
    stage.setup_decode(mb_state, max_steps=args.warmup + args.steps)
    sync()
    dist.barrier()
    stage.decode_steps(args.warmup, 0)
    stage.finish()
    sync()
    dist.barrier()
    stage.host_exchange_s = stage.host_step_s = 0.0
    stage.micro_steps = 0
    t0 = time.perf_counter()
    stage.decode_steps(args.steps, args.warmup)
    stage.finish()
    sync()
    dist.barrier()
    rdev = torch.device("cpu") if host else device  # gloo reduces host tensors
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=rdev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    # host cost of a micro-step (max over ranks): with RCCL both the grouped send/recv and the graph
    # replay only enqueue, so the stage's GPU stays fed while this stays below its device time
    hs = torch.tensor([stage.host_exchange_s, stage.host_step_s], dtype=torch.float64, device=rdev)
    dist.all_reduce(hs, op=dist.ReduceOp.MAX)
    n_micro = max(1, stage.micro_steps)
    # the generated tokens live on the last stage: their CRC goes to rank 0 for the line
    toks = stage.tokens()
    crc = zlib.crc32(np.ascontiguousarray(np.stack(toks).astype(np.int32)).tobytes()) if toks is not None else None
    if toks is not None and os.environ.get("MX_TOKENS_DUMP"):  # diagnosis: [S][M][steps] token ids
        np.save(os.environ["MX_TOKENS_DUMP"], np.stack(toks).astype(np.int32))
    if world > 1 and stage.last:
        comm.send_obj(crc, 0)
    elif world > 1 and rank == 0:
        crc = comm.recv_obj(world - 1)
    roof = None
    if not dry:
        us, wbytes = eng.profile_kernel(2, M, iters=2)
        kbytes = wbytes + M * shape.n_embd * 2 + M * shape.n_ff * 2
        roof = {"bound": "hbm", "achieved": round(kbytes / us / 1e3, 1), "peak": 8000.0, "unit": "GB/s",
                "frac": round(kbytes / us / 1e3 / 8000.0, 4), "traffic": traffic_bytes(args.model, M),
                "kernel": ("mm_wide_kernel" if M > 16 else "mm_kernel") +
                          "<EPI_SWIGLU> (ffn_gate+ffn_up+SiLU*up), rank 0",
                "us_per_launch": round(us, 2), "bytes_per_launch": int(kbytes)}
    wb = torch.tensor([float(eng.info.weight_bytes)], dtype=torch.float64, device=rdev)
    dist.all_reduce(wb)
    total_tokens = args.steps * S * M
    if rank == 0:
        ctx_sum = sum(len(p) + args.warmup + args.steps / 2 for p in prompts)
        step_bytes = float(wb.item()) * S + (ctx_sum + S * M) * shape.kv_bytes_per_pos() + S * M * shape.n_vocab * 4
        line = {
            "metric": metric, "value": round(total_tokens / dt, 2), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": ("dry run: toy CPU executor over gloo (schedule and launch check, not a measurement)" if dry else
                     "synthetic (seeded random bf16 weights of the exact shape; random prompt ids)"),
            "config": {"workload": f"{args.model} greedy decode, {world}-stage pipeline, {S} micro-batches x {M} "
                                   f"sequences in flight, prompts U[16,256] (seed 2), n_ctx {args.n_ctx}",
                       "model": args.model, "stages": world, "micro_batches": S, "seqs_per_micro_batch": M,
                       "layer_ranges": parts, "parallelism": f"pp{world}", "handoff": "f32" if f32 else "bf16"},
            "dist": {"backend": backend, "world_size": world_rd,
                     "launcher": os.environ.get("MX_LAUNCHER", "torch.distributed.run or external")},
            "tokens_crc32": crc,
            "step_hbm_gbs": round(step_bytes / dt * args.steps / 1e9, 1),
            "step_hbm_frac": round(step_bytes / (dt / args.steps) / 1e9 / 8000.0 / world, 4),
            "roofline": roof,
        }
        if world > 1:
            line["host_per_micro_step"] = {
                "exchange_us": round(float(hs[0].item()) / n_micro * 1e6, 1),
                "step_launch_us": round(float(hs[1].item()) / n_micro * 1e6, 1),
                "wall_us": round(dt / (args.steps * S) * 1e6, 1),
                "note": "host seconds per micro-step, max over ranks (exchange = grouped send/recv issue; "
                        "gloo waits inside it, RCCL only enqueues) vs wall time per micro-step"}
        if dry:
            line["dry_run"] = True
        if host:
            line["rehearsal"] = ("hand-offs staged through host memory over gloo, ranks sharing "
                                 f"{torch.cuda.device_count()} visible GPU(s): a schedule and parity check, "
                                 "not the RCCL measurement")
        print(json.dumps(line), flush=True)
    for b in stage.batches:
        b.close()
    if not dry:
        eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class DryEngine:
    """CPU stand-in for the HIP engine behind ``Stage`` (``bench.py --dry-run``): an embedding,
    ``n_layer`` layers whose output depends on a per-(slot, layer) running state (so a mis-routed
    micro-batch or slot changes the tokens, as a wrong KV cache would), and a greedy head; the stage
    holds layers [lb, le).  Same tensor interface as ``EngineAdapter`` / ``engine.Batch``."""

    H, V = 32, 512

    class _Info:
        def __init__(self, nbytes):
            self.weight_bytes = nbytes

    def __init__(self, lb: int, le: int, n_slots: int, n_layer: int):
        import torch

        self.torch = torch
        g = torch.Generator().manual_seed(0)
        self.E = torch.randn(self.V, self.H, generator=g)
        self.A = [torch.randn(self.H, self.H, generator=g) * 0.3 for _ in range(n_layer)]
        self.W = torch.randn(self.H, self.V, generator=g)
        self.lb, self.le = lb, le
        self.state = torch.zeros(n_layer, n_slots, self.H)
        self.info = DryEngine._Info(4 * self.H * self.H * (le - lb))

    def layers(self, x, slots):
        torch = self.torch
        idx = torch.tensor(slots)
        for l in range(self.lb, self.le):
            s = self.state[l, idx] * 0.5 + x
            self.state[l, idx] = s
            x = x + torch.tanh(s @ self.A[l]) * 0.5
        return x

    def stage_rows_tensors(self, slots, pos, ids, x_in, x_out):
        torch = self.torch
        x = self.E[torch.tensor(ids).long()] if x_in is None else x_in.clone()
        # one sequence's rows are consumed in order, as prompt prefill does
        for i in range(len(slots)):
            x[i:i + 1] = self.layers(x[i:i + 1], [slots[i]])
        if x_out is not None:
            x_out.copy_(x)

    def batch(self, slots, pos, ids, max_steps):
        return _DryBatch(self, slots, ids)


class _DryBatch:
    def __init__(self, eng, slots, ids):
        torch = eng.torch
        self.eng, self.slots = eng, list(slots)
        self.ids = torch.tensor(ids if ids is not None else [0] * len(slots), dtype=torch.int32)
        self.hist = []

    def bind_ids_tensor(self, t):
        t.copy_(self.ids)
        self.ids = t

    def step_tensors(self, x_in=None, x_out=None):
        torch = self.eng.torch
        x = self.eng.E[self.ids.long()] if x_in is None else x_in.clone()
        x = self.eng.layers(x, self.slots)
        if x_out is not None:
            x_out.copy_(x)
        else:
            tok = (x @ self.eng.W).argmax(-1).to(torch.int32)
            self.ids.copy_(tok)
            self.hist.append(tok.clone())

    def tokens(self):
        import numpy as np

        torch = self.eng.torch
        return torch.stack(self.hist, 1).numpy() if self.hist else np.zeros((len(self.slots), 0), np.int32)

    def close(self):
        pass


def traffic_bytes(model: str, M: int):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes (bench.py)."""
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    try:
        rec = json.load(open(path)).get(f"{model}/gate_up/M{M}")
    except (OSError, ValueError):
        return None
    return round(rec["traffic_bytes"]) if rec else None


class EngineAdapter:
    """Tensor-level view of engine.Engine used by Stage (device tensors in, device tensors out)."""

    def __init__(self, eng):
        self.eng = eng

    def stage_rows_tensors(self, slots, pos, ids, x_in, x_out):
        from .engine import torch_stream_handle

        stream = torch_stream_handle()
        self.eng.stage_rows(slots, pos, ids, x_in.data_ptr() if x_in is not None else 0,
                            x_out.data_ptr() if x_out is not None else 0, False, stream)

    def batch(self, slots, pos, ids, max_steps):
        return self.eng.batch(slots, pos, ids, max_steps=max_steps)
