#!/usr/bin/env python3
"""Where does a persistent-decode-kernel step spend its time?  Per phase kind: median work time
(phase start -> work end) and barrier time (work end -> next phase start), max over work-groups.

    python tools/pdk_trace.py [--model llama3-8b] [--M 1] [--pos 200]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

KIND = ["qkv", "attention", "attn_output", "gate_up", "down"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--M", type=int, default=1)
    ap.add_argument("--pos", type=int, default=200)
    args = ap.parse_args()
    os.environ["MX_PDK"] = "1"
    from llama_p2p_amd.engine import Engine

    eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=512, n_seq_max=8)
    for _ in range(3):
        t = eng.pdk_trace(args.M, args.pos).astype(np.int64)
    G, NP, _ = t.shape
    t0 = t[:, 0, 0].min()
    start = t[:, :, 0] - t0  # [G, NP]
    img = t[:, :, 1] - t0
    end = t[:, :, 2] - t0
    total = (end[:, -1].max()) * 10 / 1e3  # us
    print(f"grid {G}, phases {NP}, step {total:.1f} us (100 MHz stamps)")
    # phase p spans [min start_p, max end_p]; barrier = next min start - max end
    work = (end.max(0) - start.min(0)) * 10 / 1e3
    work_med = np.median(end - start, axis=0) * 10 / 1e3
    img_med = np.median(img - start, axis=0) * 10 / 1e3
    bar = np.zeros(NP)
    bar[:-1] = (start.min(0)[1:] - end.max(0)[:-1]) * 10 / 1e3
    skew = (end.max(0) - end.min(0)) * 10 / 1e3
    L = (NP - 1) // 5
    for k in range(5):
        idx = [5 * l + k for l in range(L)]
        print(f"{KIND[k]:12s} span {work[idx].mean():7.2f} us  median-wg work {work_med[idx].mean():7.2f}  "
              f"image {img_med[idx].mean():6.2f}  end skew {skew[idx].mean():6.2f}  barrier after {bar[idx].mean():6.2f}")
    print(f"{'lm_head':12s} span {work[-1]:7.2f} us  median-wg work {work_med[-1]:7.2f}")
    eng.close()


if __name__ == "__main__":
    main()
