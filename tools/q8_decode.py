#!/usr/bin/env python3
"""Greedy decode on the Q8_0 quantisation of a synthetic model (for rocprofv3 kernel traces).

    python tools/q8_decode.py [--model llama3-8b] [--rows 1] [--steps 64] [--bf16]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--bf16", action="store_true")
    args = ap.parse_args()
    import numpy as np

    from llama_p2p_amd.engine import Engine

    eng = Engine(f"synthetic:{args.model}:seed=0" + ("" if args.bf16 else ":q8_0"), n_ctx=512,
                 n_seq_max=max(args.rows, 1))
    rng = np.random.default_rng(0)
    M, P = args.rows, 100
    for i in range(M):
        eng.forward_rows([i] * P, list(range(P)), [1] + [int(t) for t in rng.integers(3, 30000, P - 1)],
                         want_logits=False)
    b = eng.batch(slots=list(range(M)), pos=[P] * M, ids=[5] * M, max_steps=args.steps + 4)
    for _ in range(4):
        b.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.step()
    eng.sync()
    dt = (time.perf_counter() - t0) / args.steps
    print(f"rows {M}: {dt * 1e3:.3f} ms/step, {M / dt:.1f} tok/s", flush=True)
    b.close()
    eng.close()


if __name__ == "__main__":
    main()
