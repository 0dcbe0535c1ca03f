#!/usr/bin/env python3
"""Diagnosis: GGUF-loaded vs synthesised K-quant model, and run-to-run determinism."""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from llama_p2p_amd import engine, gguf, synth

    ftype = sys.argv[1] if len(sys.argv) > 1 else "q4_k_m"
    shape = synth.SHAPES["test-tiny"]
    d = tempfile.mkdtemp()
    path = os.path.join(d, "t.gguf")
    gguf.write_synthetic_gguf(path, shape, seed=3, wtype=ftype)
    rng = np.random.default_rng(7)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, 23)]).astype(np.int32)
    a = engine.Engine(path, n_ctx=64, n_seq_max=2)
    b = engine.Engine(f"synthetic:test-tiny:seed=3:{ftype}", n_ctx=64, n_seq_max=2)
    print("weight bytes", a.info.weight_bytes, b.info.weight_bytes)
    for n in (1, 2, 8, 16, 17, 24):
        la = a.forward_logits(ids[:n])
        la2 = a.forward_logits(ids[:n])
        lb = b.forward_logits(ids[:n])
        rows = [int(r) for r in np.nonzero(np.abs(la - lb).max(-1) > 0)[0]]
        print(f"n={n}: |a-b| {np.abs(la - lb).max():.3g}  |a-a| {np.abs(la - la2).max():.3g}  max|a| "
              f"{np.abs(la).max():.3g}  rows differing {rows}")
    # 24 independent sequences at position 0 (attention over one position: the GEMVs only)
    a2 = engine.Engine(path, n_ctx=64, n_seq_max=24)
    b2 = engine.Engine(f"synthetic:test-tiny:seed=3:{ftype}", n_ctx=64, n_seq_max=24)
    for m in (1, 16, 17, 24):
        la = a2.forward_rows(list(range(m)), [0] * m, [int(t) for t in ids[:m]])
        lb = b2.forward_rows(list(range(m)), [0] * m, [int(t) for t in ids[:m]])
        l1 = np.concatenate([a2.forward_rows([i], [0], [int(ids[i])]) for i in range(m)])
        print(f"pos0 m={m}: |a-b| {np.abs(la - lb).max():.3g}  |m rows - 1 row| {np.abs(la - l1).max():.3g}")
    print("done")


if __name__ == "__main__":
    main()
