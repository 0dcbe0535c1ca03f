#!/usr/bin/env python3
"""Which lm_head rows differ between the K-quant persistent kernel and mkq_kernel (test-8b-v128k)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tools.kq_pers_check import run  # noqa: E402


def main():
    from llama_p2p_amd import synth

    name, ftype = "test-8b-v128k", "q4_k_m"
    shape = synth.SHAPES[name]
    rng = np.random.default_rng(9)
    ids = np.concatenate([[1], rng.integers(3, shape.n_vocab, 11)]).astype(np.int32)
    os.environ.pop("MX_NO_KQ_PERS", None)
    a = run(name, ftype, ids)
    os.environ["MX_NO_KQ_PERS"] = "1"
    b = run(name, ftype, ids)
    G = 1002
    for s in range(4):
        d = np.abs(a[s][0] - b[s][0])
        rows = np.nonzero(d > 1e-4)[0]
        tiles = np.unique(rows // 16)
        print(f"step {s}: {len(rows)} rows differ > 1e-4, tiles {len(tiles)}: {tiles[:20].tolist()}", flush=True)
        if len(tiles):
            print("   tile%G (work-group):", sorted(set((tiles % G).tolist()))[:20], " tile//G (i):",
                  sorted(set((tiles // G).tolist())), " rows%16:", sorted(set((rows % 16).tolist())), flush=True)
            r = rows[0]
            print("   e.g. row", int(r), "pers", float(a[s][0][r]), "mkq", float(b[s][0][r]), flush=True)


if __name__ == "__main__":
    main()
