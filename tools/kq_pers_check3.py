#!/usr/bin/env python3
"""K-quant persistent vs one-tile kernels against the CPU oracle (test-8b-v128k Q4_K_M decode steps)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
from tools.kq_pers_check import run  # noqa: E402


def main():
    import oracle as O
    from llama_p2p_amd import synth

    name, ftype = "test-8b-v128k", "q4_k_m"
    shape = synth.SHAPES[name]
    rng = np.random.default_rng(9)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, 11)]).astype(np.int32)
    os.environ.pop("MX_NO_KQ_PERS", None)
    a = run(name, ftype, ids)
    os.environ["MX_NO_KQ_PERS"] = "1"
    b = run(name, ftype, ids)
    om = O.OracleModel(shape, seed=0)
    om.kq_synthetic(ftype, 0)
    ctx = om.context(64)
    ctx.eval(ids[:8], 0)
    for s, p in enumerate(range(8, 12)):
        r = ctx.eval(ids[p:p + 1], p)[0]
        print(f"step {s}: |pers-oracle| {np.abs(a[s][0] - r).max():.5f}  |mkq-oracle| {np.abs(b[s][0] - r).max():.5f}  "
              f"argmax pers {int(a[s][0].argmax())} mkq {int(b[s][0].argmax())} oracle {int(r.argmax())}", flush=True)


if __name__ == "__main__":
    main()
