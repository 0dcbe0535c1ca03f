#!/usr/bin/env python3
"""Attention kernel timing (HIP events, every layer of the model, mx_profile_kernel kind 7) at a
few (rows, position) points -- one process per geometry variant (MX_ATTN_VARIANT / MX_ATTN_V1 are
read once per process).  Prints one JSON line per point.

    python tools/attn_probe.py [--model llama3-8b] [--rows 1,32] [--pos 150,300]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--rows", default="1,32")
    ap.add_argument("--pos", default="150,300")
    ap.add_argument("--n-ctx", type=int, default=512)
    a = ap.parse_args()
    from llama_p2p_amd.engine import Engine

    eng = Engine(f"synthetic:{a.model}:seed=0", n_ctx=a.n_ctx, n_seq_max=64)
    tag = os.environ.get("MX_ATTN_VARIANT", "v1" if os.environ.get("MX_ATTN_V1") else "1")
    for M in [int(x) for x in a.rows.split(",")]:
        for p in [int(x) for x in a.pos.split(",")]:
            os.environ["MX_PROF_POS"] = str(p)
            eng.profile_kernel(7, M, iters=2)  # warm
            us, by = eng.profile_kernel(7, M, iters=5)
            print(json.dumps({"variant": tag, "M": M, "pos": p, "us": round(us, 2),
                              "gbs": round(by / us / 1e3, 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
