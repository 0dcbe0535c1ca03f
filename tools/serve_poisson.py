#!/usr/bin/env python3
"""Config 5 driver: a Poisson request stream (rate λ, seed 3, prompt lengths
U[lo, hi], `gen` new tokens) placed by the reference's peer scoreboard (placement.PeerScoreboard,
p2p:156-168) onto serving targets:

  --stages S (default): the pipeline server (pipeserve.py) -- S stages, S micro-batch lanes; the
      scoreboard places every request on a lane with a free row, per-stage busy times feed a second
      scoreboard whose scores propose the next layer split.  Under torch.distributed.run (WORLD_SIZE
      > 1) every rank holds one stage on its own GPU with RCCL hand-offs; otherwise the S stages
      live in this process on one GPU (the 1-GPU rehearsal of the 8-GPU layout).
  --replicas: whole-model engine replicas, one per visible GPU (the reference's own scaling).

    python tools/serve_poisson.py --model llama3-70b --stages 8 --rate 2 --n 256 --time-scale 0.25
    python -m torch.distributed.run --nproc-per-node 8 tools/serve_poisson.py --model llama3-70b
One JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def drive(generate, schedule, gen, time_scale):
    """Replay the arrivals in (scaled) real time; each request on its own thread."""
    import numpy as np

    t0, lat, toks, workers = time.perf_counter(), [0.0] * len(schedule), [0] * len(schedule), []

    def one(i, prompt):
        ts = time.perf_counter()
        out, _ = generate(prompt, gen)
        lat[i], toks[i] = time.perf_counter() - ts, len(out)

    for i, (ta, prompt) in enumerate(schedule):
        d = ta * time_scale - (time.perf_counter() - t0)
        if d > 0:
            time.sleep(d)
        w = threading.Thread(target=one, args=(i, prompt.tolist()), daemon=True)
        w.start()
        workers.append(w)
    for w in workers:
        w.join()
    wall = time.perf_counter() - t0
    a = np.array(lat)
    return {"requests": len(schedule), "tokens": int(sum(toks)), "wall_s": round(wall, 3),
            "tok_s": round(sum(toks) / wall, 1), "p50_s": round(float(np.percentile(a, 50)), 3),
            "p99_s": round(float(np.percentile(a, 99)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rate", type=float, default=2.0, help="requests per second")
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--prompt-lo", type=int, default=32)
    ap.add_argument("--prompt-hi", type=int, default=512)
    ap.add_argument("--n-ctx", type=int, default=640)
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--rows", type=int, default=32, help="rows per pipeline lane")
    ap.add_argument("--lanes", type=int, default=0, help="micro-batch lanes (default: one per stage; on one GPU "
                    "the in-process stages run one after another, so every extra lane streams the weights again)")
    ap.add_argument("--replicas", action="store_true")
    ap.add_argument("--policy", default="score_aware", choices=["score_aware", "reference"])
    ap.add_argument("--time-scale", type=float, default=1.0, help="<1 compresses the arrival clock")
    ap.add_argument("--min-gain", type=float, default=0.10,
                    help="apply a stage re-split when it predicts this much lower slowest-stage time")
    ap.add_argument("--no-repartition", action="store_true")
    ap.add_argument("--stage-time-every", type=int, default=8, help="rounds per stage-time sample of the planner")
    ap.add_argument("--parts", default="", help="initial stage ranges 'lb:le,lb:le,...' (in-process stages; "
                    "default partition_layers by bytes) -- e.g. a skewed split for the planner to repair")
    args = ap.parse_args()
    from llama_p2p_amd import synth
    from llama_p2p_amd.placement import PeerScoreboard, poisson_schedule, serve

    shape = synth.SHAPES[args.model]
    path = f"synthetic:{args.model}:seed=0"
    sched = poisson_schedule(args.rate, args.n, seed=3, prompt_lo=args.prompt_lo, prompt_hi=args.prompt_hi,
                             vocab=shape.n_vocab)
    if args.replicas:
        from llama_p2p_amd.engine import Engine, device_count

        engines = {f"gpu{d}": Engine(path, n_ctx=args.n_ctx, n_seq_max=64, device=d)
                   for d in range(max(1, device_count()))}
        board = PeerScoreboard(list(engines), policy=args.policy, seed=0)
        res = serve(board, lambda t, p, g: len(engines[t].generate(p, g, temperature=0.0, ignore_eos=True)[0]),
                    sched, args.gen, time_scale=args.time_scale)
        res.pop("records")
        res.update({"model": args.model, "mode": "replicas", "replicas": len(engines), "policy": args.policy})
        print(json.dumps(res), flush=True)
        for e in engines.values():
            e.close()
        return

    import torch

    from llama_p2p_amd import pipeserve

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:  # one stage per rank/GPU, RCCL hand-offs
        import torch.distributed as dist

        from llama_p2p_amd.pipeline import TorchComm

        rank, local = int(os.environ["RANK"]), int(os.environ.get("LOCAL_RANK", os.environ["RANK"]))
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        comm = TorchComm(rank, world)
        torch.cuda.set_stream(torch.cuda.Stream())
        dev = torch.device("cuda", local)
        if rank != 0:
            pipeserve.serve_stage(path, comm, rank, world, world, args.rows, args.n_ctx, device=dev)
            dist.destroy_process_group()
            return
        llm = pipeserve.pipeline_llama(path, comm, world, world, args.rows, args.n_ctx, device=dev,
                                       policy=args.policy, seed=0, repartition=not args.no_repartition,
                                       min_gain=args.min_gain, stage_time_every=args.stage_time_every)
        mode = f"{world} stages, one GPU each (RCCL)"
    else:
        from llama_p2p_amd.pipeline import partition_layers

        h, kv, ff = shape.n_embd, shape.n_embd_kv, shape.n_ff
        parts = partition_layers(shape.n_layer, 2 * (2 * h * h + 2 * h * kv + 3 * h * ff), 2 * shape.n_vocab * h,
                                 args.stages)
        if args.parts:
            parts = [tuple(int(v) for v in r.split(":")) for r in args.parts.split(",")]
            if parts[0][0] != 0 or parts[-1][1] != shape.n_layer or any(a[1] != b[0] for a, b in zip(parts, parts[1:])):
                raise SystemExit(f"--parts must tile 0..{shape.n_layer}")
            args.stages = len(parts)
        initial_parts = list(parts)
        llm = pipeserve.local_pipeline_llama(path, parts, lanes=args.lanes or args.stages, rows=args.rows, n_ctx=args.n_ctx,
                                             policy=args.policy, seed=0, repartition=not args.no_repartition,
                                             min_gain=args.min_gain, stage_time_every=args.stage_time_every)
        mode = f"{args.stages} stages in one process on one GPU, {args.lanes or args.stages} lanes"
    from llama_p2p_amd.pipeline import partition_layers as _pl

    _h, _kv, _ff = shape.n_embd, shape.n_embd_kv, shape.n_ff
    balanced = [tuple(p) for p in _pl(shape.n_layer, 2 * (2 * _h * _h + 2 * _h * _kv + 3 * _h * _ff),
                                      2 * shape.n_vocab * _h, len(llm.parts))]
    front = llm._engine
    res = drive(lambda p, g: front.generate(p, g, temperature=0.0, ignore_eos=True), sched, args.gen,
                args.time_scale)
    lanes = {}
    for _, lane, _, _ in llm.scheduler.placements:
        lanes[lane] = lanes.get(lane, 0) + 1
    res.update({"model": args.model, "mode": mode, "policy": args.policy, "rate": args.rate,
                "time_scale": args.time_scale, "prompt_len": [args.prompt_lo, args.prompt_hi], "gen": args.gen,
                "initial_layer_ranges": initial_parts if world == 1 else None, "layer_ranges": llm.parts,
                "requests_per_lane": lanes, "lane_scores": llm.scheduler.board.stats(),
                "stage_scores": llm.planner.board.stats(),
                "proposed_partition": pipeserve.proposed_partition(llm.planner.board, llm.parts,
                                                                   llm.planner.head_layers),
                "repartitions": llm.planner.history, "planner_last": llm.planner.last,
                "byte_balanced": balanced,
                "max_layer_delta_vs_balanced": max(abs((b - a) - (d - c)) for (a, b), (c, d) in zip(llm.parts, balanced)),
                "rounds": llm.scheduler.rounds,
                "stage0_host_per_micro_step": front.runner.host_stats()})
    llm.close()
    print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
