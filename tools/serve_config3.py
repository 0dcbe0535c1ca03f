#!/usr/bin/env python3
"""BASELINE.json config 3 through the drop-in node: Llama-3-8B bf16 serving 32
concurrent synthetic requests with the result cache on.

32 client threads call ``LlamaP2PNode.cached_inference(prompt)`` (p2p:120-133; the model call is
the reference's ``self.model(prompt, max_tokens=100)`` with llama-cpp-python's default sampling),
then the same 32 prompts are submitted again (all cache hits).  Reported: generated tokens/s of
the first wave (hits excluded), the second wave's hit rate and latency, and, for comparison, the
reference's serialised behaviour (one request at a time, as its lock around the model call does)
timed on a bounded sample of the same prompts.  One JSON line on stdout.

    python tools/serve_config3.py [--model synthetic:llama3-8b] [--n 32] [--serial 4]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


class _NoNet:
    """No gossip/RPC sockets: requests enter through cached_inference directly."""

    def __getattr__(self, name):
        return lambda *a, **k: None


class _Counting:
    """Wraps the Llama object to count completion tokens (cached_inference returns text only)."""

    def __init__(self, llm):
        self.llm, self.tokens, self.calls, self.lock = llm, 0, 0, threading.Lock()

    def __call__(self, prompt, **kw):
        out = self.llm(prompt, **kw)
        with self.lock:
            self.tokens += out["usage"]["completion_tokens"]
            self.calls += 1
        return out


def make_text_prompts(n, tokenize, seed=2, lo=16, hi=256):
    """n prompts of about U[lo, hi] tokens (config 3's lengths): random words, trimmed by the
    model's own tokenizer so that every prompt fits n_ctx 512 with 100 generated tokens."""
    import numpy as np

    rng = np.random.default_rng(seed)
    words = ["node", "peer", "model", "layer", "cache", "token", "request", "the", "of", "and", "gossip",
             "stage", "prompt", "answer", "question", "fast", "memory", "bandwidth", "graph", "stream"]
    out = []
    for i in range(n):
        L = int(rng.integers(lo, hi + 1))
        ws = [words[int(j)] for j in rng.integers(0, len(words), L)]
        while len(ws) > 1 and len(tokenize(f"Request {i}: " + " ".join(ws))) > L:
            ws = ws[:max(1, int(len(ws) * 0.9))]
        out.append(f"Request {i}: " + " ".join(ws))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="synthetic:llama3-8b")
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--serial", type=int, default=4, help="requests timed one at a time (reference lock)")
    args = ap.parse_args()
    from llama_p2p_amd.llama import Llama
    from llama_p2p_amd.node import LlamaP2PNode

    llm = Llama(model_path=args.model, verbose=False, n_seq_max=max(args.n, 1))
    llm("warm up", max_tokens=4)
    counting = _Counting(llm)
    node = LlamaP2PNode(args.model, 5000, cache_size=100, secret_key="k", model=counting, transport=_NoNet())
    tok = lambda t: llm.tokenize(t.encode(), add_bos=True, special=True)  # noqa: E731
    prompts = make_text_prompts(args.n, tok)

    def wave(ps):
        lat = [0.0] * len(ps)

        def run(i):
            t = time.perf_counter()
            node.cached_inference(ps[i])
            lat[i] = time.perf_counter() - t

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(ps))]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0, lat

    dt1, lat1 = wave(prompts)
    gen1, calls1 = counting.tokens, counting.calls
    dt2, lat2 = wave(prompts)
    hits = args.n - (counting.calls - calls1)

    # the reference's behaviour: its lock serialises every model call (p2p:121-133)
    serial = None
    if args.serial > 0:
        sp = make_text_prompts(args.serial, tok, seed=7)
        t0, tok0 = time.perf_counter(), counting.tokens
        for p in sp:
            counting(p, max_tokens=100)
        sdt = time.perf_counter() - t0
        serial = {"requests": args.serial, "tok_s": round((counting.tokens - tok0) / sdt, 1),
                  "s_per_request": round(sdt / args.serial, 3)}
    llm.close()
    print(json.dumps({
        "workload": f"config 3: {args.model}, {args.n} concurrent cached_inference calls "
                    f"(max_tokens=100, default sampling), then the same {args.n} again",
        "wave1": {"requests": args.n, "generated_tokens": gen1, "wall_s": round(dt1, 3),
                  "tok_s": round(gen1 / dt1, 1), "p50_latency_s": round(sorted(lat1)[len(lat1) // 2], 3)},
        "wave2": {"requests": args.n, "hit_rate": round(hits / args.n, 3), "wall_s": round(dt2, 4),
                  "max_latency_ms": round(max(lat2) * 1e3, 3)},
        "overall_hit_rate": round(hits / (2 * args.n), 3),
        "serialised_reference_behaviour": serial,
    }), flush=True)


if __name__ == "__main__":
    main()
