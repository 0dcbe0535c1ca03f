#!/usr/bin/env python3
"""Two HIP runtimes share a process here: the engine links ROCm 7.2's libamdhip64.so.7 / libhsa-runtime64.so.1
(/opt/rocm), PyTorch loads its bundled ROCm 7.0 libamdhip64.so / libhsa-runtime64.so.  This probe initialises
them in the order given (engine|torch first) and reports whether the second one still sees the GPU.

    python tools/hip_runtime_order_probe.py engine-first | torch-first
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def engine_init():
    from llama_p2p_amd.engine import Engine

    e = Engine("synthetic:test-tiny:seed=0", n_ctx=64, n_seq_max=2)
    lg = e.eval([1, 5, 7]) if hasattr(e, "eval") else None
    e.close()
    return True


def torch_init():
    import torch

    torch.cuda.init()
    x = torch.ones(4, device="cuda")
    return float(x.sum()) == 4.0


order = sys.argv[1] if len(sys.argv) > 1 else "engine-first"
res = {"order": order}
for name, fn in ((("engine", engine_init), ("torch", torch_init)) if order == "engine-first"
                 else (("torch", torch_init), ("engine", engine_init))):
    try:
        res[name] = fn()
    except Exception as e:  # noqa: BLE001
        res[name] = repr(e)[:300]
print(json.dumps(res), flush=True)
