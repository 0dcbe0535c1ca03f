#!/usr/bin/env python3
"""BASELINE.json config 3 through the drop-in node: Llama-3-8B bf16 serving 32
concurrent synthetic requests with the result cache on.

32 clients send inference requests over the node's request socket at once (an in-process REP
transport with concurrent contexts, node.LocalTransport): ``handle_requests`` (p2p:84-98) ->
``cached_inference`` (p2p:120-133) -> the reference's ``self.model(prompt, max_tokens=100)``
(llama-cpp-python's default sampling, or greedy with --greedy), then the same 32 prompts are
sent again (all cache hits).  Reported: generated tokens/s of
the first wave (hits excluded), the second wave's hit rate and latency, and, for comparison, the
reference's serialised behaviour (one request at a time, as its lock around the model call does)
timed on a bounded sample of the same prompts.  One JSON line on stdout.

    python tools/serve_config3.py [--model synthetic:llama3-8b] [--n 32] [--serial 4] [--greedy]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


class _Counting:
    """Wraps the Llama object to count completion tokens (cached_inference returns text only)."""

    def __init__(self, llm, extra=None):
        self.llm, self.tokens, self.calls, self.lock = llm, 0, 0, threading.Lock()
        self.extra = extra or {}

    def __call__(self, prompt, **kw):
        out = self.llm(prompt, **kw, **self.extra)
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
    ap.add_argument("--greedy", action="store_true", help="temperature 0 (the parity setting) instead of the defaults")
    args = ap.parse_args()
    from llama_p2p_amd.llama import Llama
    from llama_p2p_amd.node import LlamaP2PNode, LocalTransport

    llm = Llama(model_path=args.model, verbose=False, n_seq_max=max(args.n, 1))
    llm("warm up", max_tokens=4)
    counting = _Counting(llm, {"temperature": 0.0} if args.greedy else None)
    tr = LocalTransport()
    node = LlamaP2PNode(args.model, 5000, cache_size=100, secret_key="k", model=counting, transport=tr,
                        n_contexts=args.n)
    threading.Thread(target=node.handle_requests, daemon=True).start()
    tok = lambda t: llm.tokenize(t.encode(), add_bos=True, special=True)  # noqa: E731
    prompts = make_text_prompts(args.n, tok)

    def wave(ps):
        lat = [0.0] * len(ps)

        def run(i):
            t = time.perf_counter()
            reply = json.loads(tr.request(json.dumps({"type": "inference", "prompt": ps[i], "secret_key": "k"}).encode()))
            assert "result" in reply, reply
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
    node.active = False
    llm.close()
    print(json.dumps({
        "workload": f"config 3: {args.model}, {args.n} concurrent requests through handle_requests "
                    f"(REP contexts) -> cached_inference (max_tokens=100, "
                    f"{'greedy' if args.greedy else 'default sampling'}), then the same {args.n} again",
        "wave1": {"requests": args.n, "generated_tokens": gen1, "wall_s": round(dt1, 3),
                  "tok_s": round(gen1 / dt1, 1), "p50_latency_s": round(sorted(lat1)[len(lat1) // 2], 3)},
        "wave2": {"requests": args.n, "hit_rate": round(hits / args.n, 3), "wall_s": round(dt2, 4),
                  "max_latency_ms": round(max(lat2) * 1e3, 3)},
        "overall_hit_rate": round(hits / (2 * args.n), 3),
        "serialised_reference_behaviour": serial,
    }), flush=True)


if __name__ == "__main__":
    main()
