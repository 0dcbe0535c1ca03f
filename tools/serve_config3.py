#!/usr/bin/env python3
"""BASELINE.json config 3 through the drop-in node, standalone: bench.py's ``serving`` section
(handle_requests on REP contexts -> cached_inference -> Llama(prompt, max_tokens=100), greedy, then
the same prompts again for the cache hits) with its own model / request count.  One JSON line.

    python tools/serve_config3.py [--model llama3-8b] [--n 32]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--n-ctx", type=int, default=512)
    args = ap.parse_args()
    import bench

    print(json.dumps(bench.serving_bench(args, args.n)), flush=True)


if __name__ == "__main__":
    main()
