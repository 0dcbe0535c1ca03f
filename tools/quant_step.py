#!/usr/bin/env python3
"""bench.py's quantised decode section alone (32-sequence step and batch 1) for A/B runs:
    python tools/quant_step.py q4_k_m q8_0 q4_0
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("wtypes", nargs="+")
    ap.add_argument("--steps", type=int, default=32)
    a = ap.parse_args()
    import bench
    args = argparse.Namespace(model="llama3-8b", seqs=bench.MB_SEQS, n_ctx=512, prefill_prompts=0, prefill_len=128)
    for w in a.wtypes:
        out = bench.quant_bench(args, w, a.steps)
        print(json.dumps({"wtype": w, "env": {k: v for k, v in os.environ.items() if k.startswith("MX_")},
                          "decode": out[f"decode_M{args.seqs}"], "batch1": out["batch1"]}), flush=True)


if __name__ == "__main__":
    main()
