#!/usr/bin/env python3
"""Reference point for the prefill GEMMs: torch.matmul (hipBLASLt) on the Llama-3-8B prefill shapes at 4096
rows, bf16, timed with HIP events (plain GEMMs, no fused epilogue).  Prints one JSON line per shape."""
import json

import torch

shapes = {"qkv": (4096, 6144, 4096), "attn_output": (4096, 4096, 4096), "gate_up": (4096, 28672, 4096),
          "ffn_down": (4096, 4096, 14336)}
torch.manual_seed(0)
for name, (m, n, k) in shapes.items():
    a = torch.randn(m, k, dtype=torch.bfloat16, device="cuda")
    b = torch.randn(n, k, dtype=torch.bfloat16, device="cuda")
    for _ in range(3):
        c = a @ b.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        c = a @ b.t()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / it * 1e3
    tf = 2 * m * n * k / us / 1e6
    print(json.dumps({"gemm": name, "m": m, "n": n, "k": k, "us": round(us, 1), "tflops": round(tf, 1),
                      "frac_of_2500": round(tf / 2500, 3)}), flush=True)
