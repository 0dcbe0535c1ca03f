#!/usr/bin/env python3
"""Config 5 driver: a Poisson request stream placed by the gossip scoreboard
(llama-p2p_amd/placement.py, the reference's p2p:156-168 bookkeeping) onto engine replicas, one
per visible GPU (several per GPU with --per-gpu).  Each replica micro-batches whatever it is given.

    python tools/serve_poisson.py --model llama3-8b --rate 2 --n 64 --gen 128 [--policy reference]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rate", type=float, default=2.0, help="requests per second")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--prompt-lo", type=int, default=32)
    ap.add_argument("--prompt-hi", type=int, default=512)
    ap.add_argument("--n-ctx", type=int, default=1024)
    ap.add_argument("--per-gpu", type=int, default=1)
    ap.add_argument("--policy", default="score_aware", choices=["score_aware", "reference"])
    ap.add_argument("--time-scale", type=float, default=1.0, help="<1 compresses the arrival clock")
    args = ap.parse_args()
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine, device_count
    from llama_p2p_amd.placement import PeerScoreboard, poisson_schedule, serve

    shape = synth.SHAPES[args.model]
    ngpu = max(1, device_count())
    engines = {f"gpu{d}.{k}": Engine(f"synthetic:{args.model}:seed=0", n_ctx=args.n_ctx, n_seq_max=64, device=d)
               for d in range(ngpu) for k in range(args.per_gpu)}
    sched = poisson_schedule(args.rate, args.n, seed=3, prompt_lo=args.prompt_lo, prompt_hi=args.prompt_hi,
                             vocab=shape.n_vocab)

    def run(tgt, prompt, gen):
        toks, _ = engines[tgt].generate(prompt, gen, temperature=0.0, ignore_eos=True)
        return len(toks)

    board = PeerScoreboard(list(engines), policy=args.policy, seed=0)
    res = serve(board, run, sched, args.gen, time_scale=args.time_scale)
    res.pop("records")
    res.update({"model": args.model, "replicas": len(engines), "rate": args.rate, "policy": args.policy})
    print(json.dumps(res), flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
