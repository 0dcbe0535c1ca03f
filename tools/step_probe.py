#!/usr/bin/env python3
"""Per-kernel times of one decode layer at M rows (mx_profile_kernel), Llama-3-8B synthetic.

    python tools/step_probe.py [--M 32] [--pos 200] [--iters 20]

kinds: 0 q|k|v, 1 attn_output, 2 gate/up, 3 ffn_down, 4 lm_head, 7 attention, 8/9/10 RMS_NORM folding
4/8/0 split-K slabs.  Environment switches of the engine (MX_NO_WIDE, ...) apply.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--pos", type=int, default=200)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--kinds", default="0,7,1,8,2,3,9,10,4")
    ap.add_argument("--quant", default="", help="q8_0 | q4_0 | q4_k_m (synthetic quantised model)")
    args = ap.parse_args()
    os.environ["MX_PROF_POS"] = str(args.pos)
    from llama_p2p_amd.engine import Engine

    path = f"synthetic:{args.model}:seed=0" + (f":{args.quant}" if args.quant else "")
    eng = Engine(path, n_ctx=512, n_seq_max=64, device=0)
    names = {0: "qkv", 1: "attn_output", 2: "gate_up", 3: "ffn_down", 4: "lm_head", 7: "attention",
             8: "fold4_norm", 9: "fold8_norm", 10: "norm"}
    out = {"M": args.M, "pos": args.pos, "quant": args.quant, "env": {k: v for k, v in os.environ.items() if k.startswith("MX_")}}
    for k in [int(v) for v in args.kinds.split(",")]:
        us, nb = eng.profile_kernel(k, args.M, args.iters)
        out[names[k]] = {"us": round(us, 2), "GBps": round(nb / us / 1e3, 1)}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
