#!/usr/bin/env python3
"""Batched prefill timing (32 prompts x 128 tokens by default) for kernel profiling:
    rocprofv3 --kernel-trace -d gpurun_out/pp -- python3 tools/prefill_probe.py
--sweep L1,L2,..: one prompt of each length instead (best of 3), for every split-K target in
--targets (MX_GEMM_SPLIT_TARGET, read when the engine is built).
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--prompts", type=int, default=32)
    ap.add_argument("--len", type=int, default=128)
    ap.add_argument("--sweep", default="")
    ap.add_argument("--targets", default="256")
    ap.add_argument("--quant", default="", help="q8_0 | q4_0 | q4_k_m (synthetic quantised model)")
    args = ap.parse_args()
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    shape = synth.SHAPES[args.model]
    if args.sweep:
        rng = np.random.default_rng(3)
        for tgt in args.targets.split(","):
            os.environ["MX_GEMM_SPLIT_TARGET"] = tgt
            eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=2048, n_seq_max=2)
            for L in [int(v) for v in args.sweep.split(",")]:
                ids = rng.integers(3, shape.n_vocab, L).astype(np.int32)
                best = 1e9
                for _ in range(3):
                    eng.sync()
                    t0 = time.perf_counter()
                    eng.forward_rows([0] * L, list(range(L)), ids, want_logits=False)
                    eng.sync()
                    best = min(best, time.perf_counter() - t0)
                print(f"target {tgt:>4} rows {L:5d}: {best * 1e3:8.2f} ms  {L / best:9.0f} tok/s", flush=True)
            eng.close()
        return
    eng = Engine(f"synthetic:{args.model}:seed=0" + (f":{args.quant}" if args.quant else ""), n_ctx=512,
                 n_seq_max=args.prompts)
    rng = np.random.default_rng(3)
    slots = np.repeat(np.arange(args.prompts), args.len)
    pos = np.tile(np.arange(args.len), args.prompts)
    ids = rng.integers(3, shape.n_vocab, len(pos)).astype(np.int32)
    for _ in range(2):
        eng.sync()
        t0 = time.perf_counter()
        eng.forward_rows(slots, pos, ids, want_logits=False)
        eng.sync()
        dt = time.perf_counter() - t0
    print(f"{len(ids)} tokens in {dt * 1e3:.1f} ms: {len(ids) / dt:.0f} tok/s")
    eng.close()


if __name__ == "__main__":
    main()
