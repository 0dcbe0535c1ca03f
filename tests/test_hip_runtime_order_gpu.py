"""The engine's HIP runtime and PyTorch's in one process (round-5 regression).

libmxllama.so links /opt/rocm's libamdhip64.so.7; PyTorch loads its own bundled HIP runtime.  When the
engine's runtime opened the GPU first, PyTorch then saw no GPU ("No HIP GPUs are available") -- the
pipeline, the bench and the stage tests use both.  engine.lib() now initialises PyTorch's runtime
before loading the engine; this runs the order probe in a fresh process (where nothing has touched the
GPU yet) with the engine used first and PyTorch after it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_engine_first_then_torch_sees_the_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hip_runtime_order_probe.py"), "engine-first"],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["engine"] is True and res["torch"] is True, res
