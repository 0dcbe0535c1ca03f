"""`python3 bench.py --gpus N` starts its own N ranks (llama-p2p_amd/launch.py) -- CPU, gloo.

The driver may run the bench as the plain command.  With --dry-run the ranks run the real
pipeline schedule, timing (barrier + max over ranks) and report of pipeline.bench_main, with
pipeline.DryEngine in place of the HIP engine, over gloo.  Checked: exactly one JSON line on
stdout, n_gpus = N = the torch.distributed world size each rank read back, and the generated
tokens equal the one-stage run of the same micro-batches (CRC32 over every token).
"""
import json
import os
import subprocess
import sys

import pytest

from llama_p2p_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    return p


def _line(p):
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, f"stdout must be one JSON line, got {len(lines)}: {p.stdout[:2000]}"
    return json.loads(lines[0])


COMMON = ["--dry-run", "--steps", "5", "--warmup", "2", "--seqs", "3"]


@pytest.mark.parametrize("n", [2, 4])
def test_plain_command_starts_n_ranks(n):
    got = _line(_run(["--gpus", str(n)] + COMMON))
    assert got["n_gpus"] == n
    assert got["dist"]["world_size"] == n and got["dist"]["backend"] == "gloo"
    assert got["dist"]["launcher"].startswith("bench.py")
    assert got["config"]["stages"] == n and got["config"]["micro_batches"] == n
    assert len(got["config"]["layer_ranges"]) == n
    ref = _line(_run(["--gpus", "1", "--force-pipeline", "--micro-batches", str(n)] + COMMON))
    assert ref["n_gpus"] == 1 and ref["dist"]["world_size"] == 1
    assert got["tokens_crc32"] == ref["tokens_crc32"] is not None


def test_external_launcher_is_not_doubled():
    """Under torch.distributed.run (WORLD_SIZE set) bench.py must not start ranks of its own."""
    assert launch.needs_launch(2, {}) and not launch.needs_launch(1, {})
    assert not launch.needs_launch(8, {"WORLD_SIZE": "8"})
    port = launch.free_port()
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2"] + COMMON
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    e.update(env)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=e, cwd=ROOT)
    got = _line(p)
    assert got["n_gpus"] == 2 and got["dist"]["world_size"] == 2
    assert not got["dist"]["launcher"].startswith("bench.py")


def test_failing_rank_fails_the_launch():
    p = _run(["--gpus", "2", "--dry-run", "--model", "no-such-model", "--steps", "1", "--warmup", "0"], timeout=120)
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.strip()]


_HANG = r"""
import os, sys, time
sys.path.insert(0, {root!r})
from llama_p2p_amd import launch
if os.environ.get("RANK") is not None:          # a rank: report its pid, then hang
    launch.rank_init()                          # as bench.py's ranks: die with the launcher
    open(os.path.join({tmp!r}, "rank" + os.environ["RANK"]), "w").write(str(os.getpid()))
    time.sleep(600)
    sys.exit(0)
sys.exit(launch.spawn_ranks(2, [__file__], grace={grace}))
"""


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:  # a zombie is not a live rank
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except FileNotFoundError:
        return False


def _ranks(tmp, n=2, t_max=60):
    import time

    t0 = time.time()
    while time.time() - t0 < t_max:
        got = [os.path.join(tmp, f"rank{r}") for r in range(n)]
        if all(os.path.exists(g) and open(g).read() for g in got):
            return [int(open(g).read()) for g in got]
        time.sleep(0.1)
    raise AssertionError("ranks did not start")


def test_sigterm_to_launcher_stops_every_rank(tmp_path):
    """A launcher killed by the driver (SIGTERM) must not leave ranks holding GPUs and the port."""
    import signal
    import time

    script = tmp_path / "hang.py"
    script.write_text(_HANG.format(root=ROOT, tmp=str(tmp_path), grace=300))
    p = subprocess.Popen([sys.executable, str(script)], cwd=ROOT)
    pids = _ranks(str(tmp_path))
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    t0 = time.time()
    while any(_alive(q) for q in pids) and time.time() - t0 < 20:
        time.sleep(0.1)
    assert not any(_alive(q) for q in pids)


def test_sigkill_to_launcher_still_stops_ranks(tmp_path):
    """Even when the launcher dies without running its handlers, PR_SET_PDEATHSIG (set by each rank's
    launch.rank_init) ends its ranks."""
    import signal
    import time

    script = tmp_path / "hang.py"
    script.write_text(_HANG.format(root=ROOT, tmp=str(tmp_path), grace=300))
    p = subprocess.Popen([sys.executable, str(script)], cwd=ROOT)
    pids = _ranks(str(tmp_path))
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=30)
    t0 = time.time()
    while any(_alive(q) for q in pids) and time.time() - t0 < 20:
        time.sleep(0.1)
    assert not any(_alive(q) for q in pids)
