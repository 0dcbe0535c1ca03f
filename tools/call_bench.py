#!/usr/bin/env python3
"""The reference's own call, end to end: Llama(model_path)(prompt, max_tokens=100) with
llama-cpp-python's default sampling (temperature 0.8, top-k 40, top-p 0.95, min-p 0.05), and
greedy for comparison.  tokens/s = completion tokens / wall time of the call."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="synthetic:llama3-8b")
    ap.add_argument("--max-tokens", type=int, default=100)
    args = ap.parse_args()
    from llama_p2p_amd.llama import Llama

    llm = Llama(model_path=args.model, verbose=False)
    prompt = "The quick brown fox jumps over the lazy dog. " * 4
    llm(prompt, max_tokens=4)  # warm: graphs, first allocation
    for name, kw in (("default sampling", {}), ("greedy", {"temperature": 0.0})):
        t0 = time.perf_counter()
        out = llm(prompt, max_tokens=args.max_tokens, seed=1, **kw)
        dt = time.perf_counter() - t0
        n = out["usage"]["completion_tokens"]
        print(f"{name}: {n} tokens in {dt * 1e3:.1f} ms = {n / dt:.1f} tok/s "
              f"(prompt {out['usage']['prompt_tokens']} tokens)", flush=True)
    llm.close()


if __name__ == "__main__":
    main()
