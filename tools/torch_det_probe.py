#!/usr/bin/env python3
"""Diagnosis: is a torch-only GPU workload bitwise repeatable while another process shares the GPU?
A chain of bf16 GEMMs + RMS-norms (hipBLASLt / torch kernels only), repeated; prints whether every
repetition equals the first."""
import sys

import torch


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    torch.manual_seed(0)
    ws = [torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(24)]
    x0 = torch.randn(64, 4096, device="cuda", dtype=torch.bfloat16)
    outs = []
    for _ in range(reps):
        x = x0
        for w in ws:
            x = x @ w
            x = (x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5)).to(torch.bfloat16)
        torch.cuda.synchronize()
        outs.append(x.float().cpu())
    print({"torch_reps_equal": [bool(torch.equal(outs[0], o)) for o in outs[1:]],
           "max_abs_diff": [float((outs[0] - o).abs().max()) for o in outs[1:]]}, flush=True)


if __name__ == "__main__":
    main()
