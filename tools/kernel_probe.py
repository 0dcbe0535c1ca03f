#!/usr/bin/env python3
"""Per-kernel timing on the GPU (HIP events, rotating through every layer's weights).

    python tools/kernel_probe.py [--model llama3-8b] [--rows 1,32] [--pos 255] [--wtype q4_k_m] [--kinds 0,2,3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

KINDS = {0: "qkv", 1: "attn_output", 2: "gate_up", 3: "down", 4: "lm_head", 5: "qkv+norm_on_load", 6: "gate_up+norm_on_load",
         7: "attention"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rows", default="1,32")
    ap.add_argument("--pos", type=int, default=255)
    ap.add_argument("--q8", action="store_true", help="the Q8_0 quantisation of the model")
    ap.add_argument("--wtype", default="", help="q8_0 / q4_0 / q4_k_m / q5_k_m (default bf16)")
    ap.add_argument("--kinds", default="", help="comma list of kernel kinds (default all)")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    os.environ["MX_PROF_POS"] = str(args.pos)
    from llama_p2p_amd.engine import Engine

    wtype = "q8_0" if args.q8 else args.wtype
    eng = Engine(f"synthetic:{args.model}:seed=0" + (f":{wtype}" if wtype else ""), n_ctx=512, n_seq_max=64)
    kinds = [int(x) for x in args.kinds.split(",")] if args.kinds else list(KINDS)
    for M in [int(x) for x in args.rows.split(",")]:
        for k in kinds:
            name = KINDS[k]
            if k in (5, 6) and (M > 4 or wtype):
                continue
            us, b = eng.profile_kernel(k, M, iters=args.iters)
            print(f"M={M:<3d} {name:14s} {us:9.2f} us  {b / us / 1e3:8.1f} GB/s", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
