"""Start one process per GPU for ``bench.py --gpus N`` when no launcher did.

The driver may start the bench as ``torch.distributed.run --nproc-per-node N bench.py --gpus N``
(RANK / WORLD_SIZE set: nothing to do here) or as the plain ``python3 bench.py --gpus N``.  In the
second case the parent becomes a launcher: it starts N children of the same command with the
torch.distributed env:// variables set (MASTER_ADDR 127.0.0.1, a free port, RANK = LOCAL_RANK = i),
forwards rank 0's stdout (the one JSON line) and sends every other rank's stdout to stderr, then
exits with the first failing child's status.

The parent never imports torch or touches the GPU: the children are started as new processes
(no fork of a GPU-initialised process, no exec), which is the only safe shape on this pool.  This
replaces the reference's peer forwarding (``/root/reference/llama_p2p_network.py:135-154``): the
peers are the node's GPUs, one pipeline stage each.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_launch(n: int, env=None) -> bool:
    """True when ``--gpus n`` asks for ranks that no launcher has started."""
    env = os.environ if env is None else env
    return n > 1 and "WORLD_SIZE" not in env


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PYTHONUNBUFFERED": "1",
                "MX_LAUNCHER_PID": str(os.getpid())})
    return env


class _Terminated(Exception):
    pass


def _raise_terminated(signum, frame):
    raise _Terminated(signum)


def rank_init() -> None:
    """Called by a rank's own entry code (bench.py, first thing, before torch): die with the launcher
    (PR_SET_PDEATHSIG = SIGTERM), so a killed launcher cannot leave ranks holding the GPUs and the
    rendezvous port.  Set here rather than in a ``preexec_fn``: that hook runs Python in a forked copy
    of the launcher before exec, and the launcher may itself be a GPU-initialised process (a profiler's
    preload initialises the GPU before the program starts).  If the launcher is already gone (it died
    between the spawn and this call), the rank exits at once."""
    parent = os.environ.get("MX_LAUNCHER_PID")
    if not parent:
        return
    try:
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM, 0, 0, 0)  # PR_SET_PDEATHSIG
    except OSError:
        return
    if os.getppid() != int(parent):
        os._exit(128 + signal.SIGTERM)


def spawn_ranks(n: int, argv: Sequence[str], timeout: Optional[float] = None, stdout=None,
                grace: float = 300.0) -> int:
    """Run ``[python] + argv`` as ranks 0..n-1; returns the exit status (0, or the first failure's).

    A rank that fails ends the others (by their exact PIDs: SIGTERM, then SIGKILL after 10 s), so a
    stuck RCCL rendezvous cannot outlive a crashed peer; once any rank has exited, the rest get
    ``grace`` seconds.  SIGTERM / SIGINT to the launcher stop every rank before it exits, and each
    rank also gets SIGTERM if the launcher dies without running its handlers (``rank_init``)."""
    port = free_port()
    out = sys.stdout if stdout is None else stdout
    out.flush()
    procs: List[subprocess.Popen] = []
    old = {sig: signal.signal(sig, _raise_terminated) for sig in (signal.SIGTERM, signal.SIGINT)}
    status = 0
    try:
        for r in range(n):
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, n, port),
                                          stdout=out if r == 0 else sys.stderr, stderr=sys.stderr))
        t0 = time.time()
        first_exit = None
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if first_exit is None:
                    first_exit = time.time()
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"[launch] rank {procs.index(p)} exited with {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    _stop(live)
            if live and timeout is not None and time.time() - t0 > timeout:
                print(f"[launch] ranks still running after {timeout:.0f}s; stopping them", file=sys.stderr, flush=True)
                _stop(live)
                status = status or 124
            if live and first_exit is not None and time.time() - first_exit > grace:
                print(f"[launch] ranks still running {grace:.0f}s after the first exit; stopping them",
                      file=sys.stderr, flush=True)
                _stop(live)
                status = status or 124
            time.sleep(0.05)
    except _Terminated as e:
        print(f"[launch] signal {e.args[0]}: stopping every rank", file=sys.stderr, flush=True)
        status = 128 + int(e.args[0])
    finally:
        # a second SIGTERM / SIGINT while the ranks are being stopped must not escape this block (the
        # old handlers would stay replaced and ranks that ignore SIGTERM would not be SIGKILLed)
        for sig in old:
            signal.signal(sig, signal.SIG_IGN)
        _stop(procs)
        for sig, h in old.items():
            signal.signal(sig, h)
    return status


def _stop(procs):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t = time.time()
    while any(p.poll() is None for p in procs) and time.time() - t < 10:
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait()
