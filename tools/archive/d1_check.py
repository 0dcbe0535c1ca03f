#!/usr/bin/env python3
"""Persistent one-token decode (decode1.hip) against the per-op kernels and the oracle, then timing.

    python tools/d1_check.py [--models test-gqa8,llama3-8b] [--steps 32]

For each model: a prompt prefilled through the engine, then one-token steps (forward_logits at the
next positions, teacher-forced) through an engine using decode1 and one with MX_NO_DECODE1=1; logits
compared with each other and (small models) with the CPU oracle; then batch-1 device-loop decode
timed both ways.  One JSON line per model.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def run(name, steps, check_oracle):
    import numpy as np

    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    sh = synth.SHAPES[name]
    rng = np.random.default_rng(7)
    prompt = np.concatenate([[1], rng.integers(3, sh.n_vocab, 40)]).astype(np.int32)
    out = {"model": name}
    res = {}
    for mode in ("decode1", "per_op"):
        if mode == "per_op":
            os.environ["MX_NO_DECODE1"] = "1"
        else:
            os.environ.pop("MX_NO_DECODE1", None)
            os.environ["MX_DECODE1"] = "1"
        eng = Engine(f"synthetic:{name}:seed=0", n_ctx=512, n_seq_max=2)
        n = len(prompt)
        eng.forward_rows([0] * (n - 8), list(range(n - 8)), [int(t) for t in prompt[:n - 8]], want_logits=False)
        lg = np.stack([eng.forward_logits(prompt[i:i + 1], i)[0] for i in range(n - 8, n)])  # one-token steps
        first = int(np.argmax(lg[-1]))
        b = eng.batch(slots=[0], pos=[n], ids=[first], max_steps=steps + 4)
        for _ in range(4):
            b.step()
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            b.step()
        eng.sync()
        dt = (time.perf_counter() - t0) / steps
        toks = b.tokens()[0].tolist()
        b.close()
        eng.close()
        res[mode] = (lg, toks, dt)
    d = float(np.abs(res["decode1"][0] - res["per_op"][0]).max())
    scale = float(np.abs(res["per_op"][0]).max())
    out["max_abs_diff_vs_per_op"] = round(d, 6)
    out["logit_scale"] = round(scale, 4)
    out["tokens_equal"] = res["decode1"][1] == res["per_op"][1]
    out["first_tokens"] = {k: v[1][:8] for k, v in res.items()}
    out["ms_per_token"] = {k: round(v[2] * 1e3, 4) for k, v in res.items()}
    out["speedup"] = round(res["per_op"][2] / res["decode1"][2], 4)
    by = sh.weight_bytes_per_token()
    out["hbm_frac"] = {k: round(by / v[2] / 8e12, 4) for k, v in res.items()}
    if check_oracle:
        import oracle as O

        om = O.OracleModel(sh, seed=0)
        ref = om.context(512).eval(prompt, 0, all_logits=True)[-8:]
        tol = 1e-2 * np.abs(ref) + 2e-2 * np.abs(ref).max(axis=-1, keepdims=True)
        out["oracle_ratio"] = {k: round(float((np.abs(v[0] - ref) / tol).max()), 4) for k, v in res.items()}
        om.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="test-gqa8,test-h4096,test-tiny-ffn,llama3-8b,tinyllama-1.1b")
    ap.add_argument("--steps", type=int, default=32)
    args = ap.parse_args()
    for m in args.models.split(","):
        run(m, args.steps, m.startswith("test-"))


if __name__ == "__main__":
    main()
