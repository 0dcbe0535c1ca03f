#!/usr/bin/env python3
"""Diagnosis: the bench's pipeline schedule (pipeline.Stage) with real stage engines as THREADS of one
process (pipeserve.LocalComm hand-offs, device copies), against the one-stage run -- separates the
engine's stage-split numerics from the multi-process / host-staged transport of --host-handoff.

    python tools/rehearsal_threads.py [--stages 2] [--S 2] [--M 32] [--steps 5] [--chunk 64]
"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--S", type=int, default=2)
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--lo", type=int, default=16)
    ap.add_argument("--hi", type=int, default=256)
    ap.add_argument("--serial", action="store_true", help="one stage's GPU work at a time (device-wide lock)")
    ap.add_argument("--sync-only", action="store_true", help="device sync around every engine call, no lock")
    ap.add_argument("--lock-only", action="store_true", help="engine calls under one lock, no device sync")
    ap.add_argument("--one-stream", action="store_true", help="both stage threads enqueue on ONE stream")
    ap.add_argument("--serial-what", default="both", choices=["both", "prefill", "decode"],
                    help="which engine calls --serial covers")
    ap.add_argument("--repeat", action="store_true", help="also run the split twice (determinism)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from llama_p2p_amd import pipeserve, synth
    from llama_p2p_amd.engine import Engine
    from llama_p2p_amd.pipeline import EngineAdapter, Stage, partition_layers

    sh = synth.SHAPES[args.model]
    path = f"synthetic:{args.model}:seed=0"
    S, M = args.S, args.M
    prompts = bench.make_prompts(sh.n_vocab, S * M, lo=args.lo, hi=args.hi)
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
    if args.serial or args.sync_only or args.lock_only:  # every engine call runs alone on the GPU
        import contextlib

        from llama_p2p_amd import engine as E

        glock = threading.Lock() if not args.sync_only else contextlib.nullcontext()
        sync = not args.lock_only

        def locked(f):
            def g(*a, **k):
                with glock:
                    if sync:
                        torch.cuda.synchronize()
                    r = f(*a, **k)
                    if sync:
                        torch.cuda.synchronize()
                    return r
            return g

        if args.serial_what in ("both", "decode"):
            E.Batch.step = locked(E.Batch.step)
        if args.serial_what in ("both", "prefill"):
            E.Engine.stage_rows = locked(E.Engine.stage_rows)
    # per-run record of every prefill hand-off: CRC of stage 0's x_out and of stage 1's x_in per chunk
    import zlib

    rec = {}
    orig = EngineAdapter.stage_rows_tensors

    def traced(self, slots, pos, ids, x_in, x_out):
        orig(self, slots, pos, ids, x_in, x_out)
        torch.cuda.current_stream().synchronize()
        key = "in" if x_in is not None else "out"
        t = x_in if x_in is not None else x_out
        if t is not None:
            rec.setdefault(key, []).append(zlib.crc32(t.cpu().numpy().tobytes()))

    EngineAdapter.stage_rows_tensors = traced
    layer = 2 * (2 * sh.n_embd ** 2 + 2 * sh.n_embd * sh.n_embd_kv + 3 * sh.n_embd * sh.n_ff)
    dev = torch.device("cuda", 0)

    def run(world):
        parts = partition_layers(sh.n_layer, layer, 2 * sh.n_vocab * sh.n_embd, world)
        hub = pipeserve.LocalHub()
        out, errs = [None] * world, []
        # the engine captures each batch's graph at creation (thread-local capture mode), and a legacy-
        # stream copy on another thread breaks a capture on a blocking stream: batches are created
        # one thread at a time, between barriers
        bar, lock = threading.Barrier(world), threading.Lock()
        shared = torch.cuda.Stream(device=dev) if args.one_stream else None

        def rank(r):
            try:
                torch.cuda.set_device(dev)
                torch.cuda.set_stream(shared if shared is not None else torch.cuda.Stream(device=dev))
                lb, le = parts[r]
                eng = Engine(path, n_ctx=512, n_seq_max=S * M, layer_begin=lb, layer_end=le, device=0,
                             handoff_bf16=False)
                comm = pipeserve.LocalComm(hub, r, world) if world > 1 else None
                st = Stage(EngineAdapter(eng), comm, r, world, sh.n_embd, dev, S, dtype=torch.float32)
                st.prefill(mb_rows, chunk=args.chunk)
                torch.cuda.synchronize()
                bar.wait()
                with lock:
                    st.setup_decode(mb_state, max_steps=args.steps)
                    torch.cuda.synchronize()
                bar.wait()
                st.decode_steps(args.steps, 0)
                st.finish()
                torch.cuda.synchronize()
                out[r] = st.tokens()
                for b in st.batches:
                    b.close()
                eng.close()
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        r = dict(rec)
        rec.clear()
        return parts, np.stack(out[-1]), r

    _, ref, _ = run(1)
    parts, got, rec1 = run(args.stages)
    d = np.argwhere(ref != got)
    res = {"stages": args.stages, "parts": parts, "equal": bool(np.array_equal(ref, got)), "n_diff": len(d),
           "first": d[:10].tolist(), "chunk": args.chunk, "serial": args.serial,
           "sync_only": args.sync_only, "lock_only": args.lock_only,
           "serial_what": args.serial_what, "one_stream": args.one_stream, "graphs": not os.environ.get("MX_NO_GRAPHS")}
    res["handoff_in_equals_out"] = rec1.get("in") == rec1.get("out")
    if args.repeat:
        _, got2, rec2 = run(args.stages)
        res["split_repeat_equal"] = bool(np.array_equal(got, got2))
        for k in ("out", "in"):
            a, b = rec1.get(k, []), rec2.get(k, [])
            res[f"first_{k}_chunk_differing"] = next((i for i, (u, v) in enumerate(zip(a, b)) if u != v), None)
            res[f"n_{k}_chunks"] = len(a)
        _, ref2, _ = run(1)
        res["one_stage_repeat_equal"] = bool(np.array_equal(ref, ref2))
    print(res)


if __name__ == "__main__":
    main()
