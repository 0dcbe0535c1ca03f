#!/usr/bin/env python3
"""Batch-1 and 32-row Llama-3-8B decode timed with the engine on /opt/rocm's HIP runtime (no PyTorch in
the process: `--no-torch`) or on PyTorch's bundled one (PyTorch initialised first, the product order).

    python tools/runtime_speed_probe.py [--no-torch]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
no_torch = "--no-torch" in sys.argv
from llama_p2p_amd import engine as E  # noqa: E402

if no_torch:
    E._torch_hip_first = lambda: None
import numpy as np  # noqa: E402

eng = E.Engine("synthetic:llama3-8b:seed=0", n_ctx=512, n_seq_max=32, device=0)
res = {"runtime": "/opt/rocm (no torch)" if no_torch else "torch bundled (torch first)",
       "torch_loaded": "torch" in sys.modules}
for M in (1, 32):
    b = eng.batch(slots=list(range(M)), pos=[100] * M, ids=[5] * M, max_steps=80)
    for _ in range(8):
        b.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(64):
        b.step()
    eng.sync()
    res[f"ms_per_step_M{M}"] = round((time.perf_counter() - t0) / 64 * 1e3, 4)
    b.close()
eng.close()
print(json.dumps(res), flush=True)
