#!/usr/bin/env python3
"""K-quant persistent GEMV vs the one-tile-per-work-group kernel: max |d logit| per decode step."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run(name, ftype, ids):
    from llama_p2p_amd import engine

    eng = engine.Engine(f"synthetic:{name}:seed=0:{ftype}", n_ctx=64, n_seq_max=2)
    eng.forward_logits(ids[:8], 0, slot=0)
    out = [eng.forward_logits(ids[p:p + 1], p, slot=0) for p in range(8, 12)]
    eng.close()
    return out


def main():
    from llama_p2p_amd import synth

    for name, ftype in [("test-8b-ffn", "q4_k_m"), ("test-tiny-ffn", "q4_k_m"), ("test-8b-v128k", "q4_k_m")]:
        shape = synth.SHAPES[name]
        rng = np.random.default_rng(9)
        ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, 11)]).astype(np.int32)
        os.environ.pop("MX_NO_KQ_PERS", None)
        a = run(name, ftype, ids)
        a2 = run(name, ftype, ids)
        os.environ["MX_NO_KQ_PERS"] = "1"
        b = run(name, ftype, ids)
        b2 = run(name, ftype, ids)
        for i in range(4):
            print(name, ftype, i, "pers-vs-mkq", float(np.abs(a[i] - b[i]).max()), "pers-rerun", float(np.abs(a[i] - a2[i]).max()),
                  "mkq-rerun", float(np.abs(b[i] - b2[i]).max()), "max|l|", float(np.abs(b[i]).max()), flush=True)


if __name__ == "__main__":
    main()
