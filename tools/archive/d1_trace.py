#!/usr/bin/env python3
"""Phase timeline of the persistent one-token decode (decode1.hip) from its s_memrealtime stamps.

    python tools/d1_trace.py [--model llama3-8b] [--pos 200]

Per layer and op, over all work-groups (CUs): when compute starts (after the hand-off wait, gather and
norm) and when the work-group arrives; the loader's idle (ring full) and landing-wait ticks, and the
consumers' ring waits.  Times in us (100 MHz counter)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--pos", type=int, default=200)
    args = ap.parse_args()
    os.environ["MX_D1_TRACE"] = "1"
    os.environ["MX_DECODE1"] = "1"
    import numpy as np

    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    sh = synth.SHAPES[args.model]
    eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=512, n_seq_max=2)
    rng = np.random.default_rng(1)
    ids = rng.integers(3, sh.n_vocab, args.pos + 1).astype(np.int32)
    eng.forward_rows([0] * args.pos, list(range(args.pos)), ids[:args.pos].tolist(), want_logits=False)
    # steady state: the batch-1 decode graph replayed (as the bench times it); the trace keeps the
    # stamps of the last launch
    b = eng.batch(slots=[0], pos=[args.pos], ids=[int(ids[args.pos])], max_steps=16)
    for _ in range(16):
        b.step()
    eng.sync()
    b.close()
    tr = eng.decode1_trace().astype(np.int64)
    eng.close()
    L = sh.n_layer
    G = tr.shape[0]
    t0 = tr[:, L * 10 + 0].min()
    st = (tr[:, :L * 10].reshape(G, L, 5, 2) - t0) / 100.0  # us
    names = ["qkv", "att", "wo", "gu", "down"]
    rows = []
    for l in (0, 1, L // 2, L - 1):
        r = {"layer": l}
        for p, n in enumerate(names):
            s, e = st[:, l, p, 0], st[:, l, p, 1]
            m = e > 0 if p == 1 else np.ones(G, bool)
            if p == 1:
                m = (tr[:, l * 10 + 3] > 0)
            if not m.any():
                continue
            r[n] = {"start_min": round(float(s[m].min()), 2), "start_max": round(float(s[m].max()), 2),
                    "arrive_min": round(float(e[m].min()), 2), "arrive_max": round(float(e[m].max()), 2)}
        rows.append(r)
    end = (tr[:, L * 10 + 1] - t0) / 100.0
    lay = [(st[:, l, 4, 1].max() - (st[:, l - 1, 4, 1].max() if l else 0)) for l in range(L)]
    out = {"model": args.model, "work_groups": G, "kernel_us": round(float(end.max()), 2),
           "per_layer_us_mean": round(float(np.mean(lay[1:])), 2),
           "loader_idle_us_mean": round(float(tr[:, L * 10 + 2].mean() / 100), 2),
           "loader_landing_wait_us_mean": round(float(tr[:, L * 10 + 3].mean() / 100), 2),
           "consumer_ring_wait_us_mean": round(float(tr[:, L * 10 + 5].mean() / 100), 2),
           "layers": rows}
    # per-op means over layers 1..L-1: op span = max arrive - max arrive of the previous op
    seq = []
    for l in range(1, L):
        prev = st[:, l - 1, 4, 1].max()
        for p, n in enumerate(names):
            if p == 1:
                m = tr[:, l * 10 + 3] > 0
                a = st[m, l, p, 1].max()
            else:
                a = st[:, l, p, 1].max()
            seq.append((n, a - prev))
            prev = a
    for n in names:
        out[f"{n}_span_us"] = round(float(np.mean([d for k, d in seq if k == n])), 2)
    # gather/wait time: start of compute (max over WGs) minus previous op's last arrival
    for p, n in enumerate(names):
        if p == 1:
            continue
        w = []
        for l in range(1, L):
            prev = st[:, l, p - 1, 1].max() if p != 2 else st[tr[:, l * 10 + 3] > 0, l, 1, 1].max()
            if p == 0:
                prev = st[:, l - 1, 4, 1].max()
            w.append(np.median(st[:, l, p, 0]) - prev)
        out[f"{n}_handoff_to_compute_us_median"] = round(float(np.mean(w)), 2)
    # the last layer's attention body, per consumer wave of the attention work-groups: entry, q in
    # registers (q|k|v granules summed, RoPE, K/V stored, barrier), first chunk landed, chunk loop
    # done, partials merged in LDS; then the op's arrival -- us after the q|k|v op's last arrival
    nkv = sh.n_head_kv
    base = L * 10 + 8
    qkv_last = st[:, L - 1, 0, 1].max()
    att = {}
    for k, n in enumerate(["entry", "q_ready", "first_kv", "chunks_done", "merged"]):
        v = tr[:nkv, base + k:base + 24:8]
        v = v[v > 0]
        if v.size:
            att[n] = round(float(((v - t0) / 100.0 - qkv_last).mean()), 2)
    att["arrive"] = round(float((st[:nkv, L - 1, 1, 1] - qkv_last).mean()), 2)
    att["wo_compute_start_median"] = round(float(np.median(st[:, L - 1, 2, 0]) - qkv_last), 2)
    out["last_layer_attention_us_after_qkv"] = att
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
