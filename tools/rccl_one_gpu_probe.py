#!/usr/bin/env python3
"""Can RCCL put two ranks on one GPU here?  Two processes, both on cuda:0, nccl backend, one send/recv of a
32x4096 bf16 hand-off (the pipeline's micro-step payload), timed; prints one JSON line per rank or the error.

    python tools/rccl_one_gpu_probe.py            (spawns its 2 ranks; MASTER_ADDR 127.0.0.1)
"""
import json
import os
import sys
import time


def rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    out = {"rank": rank}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((32, 4096), float(rank + 1), dtype=torch.bfloat16, device="cuda")
        for it in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 200
            for _ in range(n):
                if rank == 0:
                    dist.send(x, 1)
                else:
                    dist.recv(x, 0)
            torch.cuda.synchronize()
            out[f"us_per_hop_{it}"] = round((time.perf_counter() - t0) / n * 1e6, 2)
        out["ok"] = bool(rank == 0 or float(x[0, 0]) == 1.0)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)[:500]
    q.put(out)


def main():
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    for _ in ps:
        try:
            res.append(q.get(timeout=120))
        except Exception as e:  # noqa: BLE001
            res.append({"error": f"no result: {e!r}"})
    for p in ps:
        p.join(10)
        if p.is_alive():
            p.kill()
    for r in res:
        print(json.dumps(r), flush=True)
    sys.exit(0)


if __name__ == "__main__":
    main()
