"""Config 4's bench path with real stage engines in separate processes, on ONE GPU.

`python3 bench.py --gpus N` starts N ranks (launch.spawn_ranks), each building the HIP engine for its
layer range of Llama-3-8B and running the pipelined greedy decode (pipeline.Stage, S = N micro-batches
of 32 sequences).  RCCL cannot put two ranks on one GPU, so `--host-handoff` sends the hand-offs over
gloo through host memory -- everything else (launcher, partition, per-rank engines, the grouped
send/recv schedule, prefill hand-offs, token return, timing and the one JSON line) is the path the
8-GPU run takes.  With the f32 hand-off a stage split is bitwise equal to one engine, so
the CRC32 of every generated token must equal the one-stage run over the same micro-batches.

Prompt rows cross stages in 64-row chunks (the bench's default).  Round 4 had to narrow this to 16-row
chunks: with two processes on one GPU the 17-64-row one-sequence chunks were not run-to-run reproducible.
The cause was the packed-FP32 RoPE in qkv_finish_kernel (profiles/round5_rope_packed_hazard.txt), now
scalar; tests/test_gpu_sharing_gpu.py keeps the in-process two-stream form of the same check.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", "llama3-8b", "--steps", "4", "--warmup", "1",
           "--handoff", "f32", "--prefill-chunk", "64", "--no-cpu-baseline"] + list(extra)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_host_staged_pipeline_tokens_equal_one_stage(n):
    ref = _bench("--gpus", "1", "--force-pipeline", "--micro-batches", str(n))
    got = _bench("--gpus", str(n), "--host-handoff")
    print(json.dumps({"n": n, "ref_crc": ref["tokens_crc32"], "crc": got["tokens_crc32"],
                      "layer_ranges": got["config"]["layer_ranges"], "host": got.get("host_per_micro_step")}))
    assert got["n_gpus"] == n and got["dist"]["world_size"] == n and got["dist"]["backend"] == "gloo"
    assert got["config"]["micro_batches"] == n and got["config"]["handoff"] == "f32"
    assert len(got["config"]["layer_ranges"]) == n
    assert got["tokens_crc32"] == ref["tokens_crc32"]
    assert "rehearsal" in got
