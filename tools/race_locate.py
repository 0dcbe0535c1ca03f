#!/usr/bin/env python3
"""Diagnosis: which kernel of the 17..64-row one-sequence forward gives different results from run to
run while another process uses the GPU (profiles/round4_gpu_sharing.txt)?

    python tools/race_locate.py --out gpurun_out/loc.json [--load] [--stops -1,1,2,3,4,5,6,7,8]
                                [--reps 3] [--layers 1] [--chunk 64] [--sync]

The parent (never touches the GPU) starts an optional LOAD process that repeats the same chunked
prefill on its own engine, waits until it runs, then starts the PROBE process.  The probe, for every
stop value n (-1: the whole forward), repeats the chunked prefill `reps` times with the engine's
forward ending after n launches (mx_debug op 0) and records, after every chunk, a CRC of each internal
buffer's live rows, and after the whole prefill a CRC of the K and V caches.  Per stop value it
reports the first (chunk, buffer) where a repetition differs from the first: the first stop value
whose last-written buffer differs names the kernel.  Launch order of one layer (wide path, rows of
one sequence): 1 resid_norm(attn) -> xn, 2 qkv split-K -> slabs, 3 qkv_finish -> q, K/V,
4 attention -> attn_out, 5 attn_output split-K -> slabs, 6 resid_norm(ffn) -> x, xn, 7 gate/up -> act,
8 ffn_down -> slabs.
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rows_of(args):
    import numpy as np

    rng = np.random.default_rng(2)
    lens = rng.integers(args.lo, args.hi + 1, args.M)
    prompts = [np.concatenate([[1], rng.integers(3, 128000, L - 1)]).astype(np.int32) for L in lens]
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * len(p)
        pos += list(range(len(p)))
        ids += [int(t) for t in p]
    return slots, pos, ids


def make_engine(args):
    from llama_p2p_amd.engine import Engine

    kw = dict(layer_begin=0, layer_end=args.layers) if args.layers else {}
    return Engine(f"synthetic:{args.model}:seed=0", n_ctx=512, n_seq_max=args.M, device=0, **kw)


def prefill(eng, rows, chunk, per_chunk=None):
    from llama_p2p_amd.engine import MX_DEBUG_STOPPED, MxError

    slots, pos, ids = rows
    for i in range(0, len(slots), chunk):
        k = min(chunk, len(slots) - i)
        try:
            eng.stage_rows(slots[i:i + k], pos[i:i + k], ids[i:i + k], 0, 0, False, 0)
        except MxError as e:  # a forward cut short by mx_debug op 0 reports MX_DEBUG_STOPPED
            if e.code != MX_DEBUG_STOPPED:
                raise
        if per_chunk:
            per_chunk(k)


def role_load(args):
    eng = make_engine(args)
    rows = rows_of(args)
    open(args.ready, "w").write("ok")
    while not os.path.exists(args.stopfile):
        prefill(eng, rows, args.load_chunk)
    eng.close()


def role_probe(args):
    import numpy as np

    eng = make_engine(args)
    rows = rows_of(args)
    h, ff = 4096, 14336
    if args.model != "llama3-8b":
        from llama_p2p_amd import synth

        sh = synth.SHAPES[args.model]
        h, ff = sh.n_embd, sh.n_ff
    nq = h + 2 * 1024 if args.model == "llama3-8b" else None
    if args.sync:
        eng.debug_sync(True)
    res = {"args": vars(args), "stops": {}}
    t0 = time.time()
    for stop in args.stops:
        eng.debug_stop(stop)
        reps = []
        for r in range(args.reps):
            rec = []

            dumps = {}

            def per_chunk(k):
                if stop == args.dump_stop and len(rec) < 2:  # full buffers of the first chunks
                    for name, nb in (("q", k * h * 4), ("pos", k * 4), ("slot", k * 4), ("slabs", 4 * 64 * (nq or h) * 4)):
                        dumps[f"{name}{len(rec)}"] = eng.debug_read(name, nb).copy()
                    dumps[f"rope{len(rec)}"] = np.array([zlib.crc32(eng.debug_read("rope_cs", 512 * 128 * 4).tobytes())])
                d = {}
                for name, nb in (("x", k * h * 4), ("q", k * h * 4), ("xn", k * h * 2), ("attn_out", k * h * 2),
                                 ("act", k * ff * 2), ("slabs", 4 * 64 * (nq or h) * 4)):
                    d[name] = zlib.crc32(eng.debug_read(name, nb).tobytes())
                rec.append(d)

            prefill(eng, rows, args.chunk, per_chunk)
            kv = {n: zlib.crc32(eng.debug_read(n, 64 << 20).tobytes()) for n in ("kcache", "vcache")}
            reps.append((rec, kv))
            if dumps:
                np.savez(args.out.replace(".json", f"_dump_rep{r}.npz"), **dumps)
        first = []
        for r in range(1, args.reps):
            rec, kv = reps[r]
            f = None
            for ci, (a, b) in enumerate(zip(reps[0][0], rec)):
                bad = [n for n in a if a[n] != b[n]]
                if bad:
                    f = {"chunk": ci, "buffers": bad}
                    break
            kvd = [n for n in kv if kv[n] != reps[0][1][n]]
            first.append({"first": f, "kv_differs": kvd})
        res["stops"][str(stop)] = first
        res.setdefault("rep0", {})[str(stop)] = reps[0]  # to compare runs (e.g. MX_POISON=1 vs not)
        print(f"stop {stop}: {first}  ({time.time() - t0:.0f} s)", flush=True)
        json.dump(res, open(args.out, "w"), indent=1)
    eng.debug_stop(-1)
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", default="parent", choices=["parent", "load", "probe"])
    ap.add_argument("--out", default="gpurun_out/race_locate.json")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--lo", type=int, default=16)
    ap.add_argument("--hi", type=int, default=256)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--load-chunk", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stops", default="-1,1,2,3,4,5,6,7,8")
    ap.add_argument("--load", action="store_true")
    ap.add_argument("--dump-stop", type=int, default=-99, help="save q / pos / slot / slabs of the first chunks")
    ap.add_argument("--sync", action="store_true", help="stream sync after every launch of the probe's forward")
    ap.add_argument("--ready", default="")
    ap.add_argument("--stopfile", default="")
    args = ap.parse_args()
    if isinstance(args.stops, str):
        args.stops = [int(v) for v in args.stops.split(",")]
    if args.role == "load":
        return role_load(args)
    if args.role == "probe":
        return role_probe(args)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)) or ".", exist_ok=True)
    base = [sys.executable, os.path.abspath(__file__), "--model", args.model, "--layers", str(args.layers),
            "--M", str(args.M), "--lo", str(args.lo), "--hi", str(args.hi), "--chunk", str(args.chunk),
            "--load-chunk", str(args.load_chunk), "--dump-stop=" + str(args.dump_stop)]
    load = None
    tag = f"/tmp/race_locate_{os.getpid()}"
    ready, stopfile = tag + ".ready", tag + ".stop"
    for f in (ready, stopfile):
        if os.path.exists(f):
            os.remove(f)
    try:
        if args.load:
            load = subprocess.Popen(base + ["--role", "load", "--ready", ready, "--stopfile", stopfile])
            t = time.time()
            while not os.path.exists(ready):
                if load.poll() is not None or time.time() - t > 300:
                    raise RuntimeError("load process did not start")
                time.sleep(0.5)
        cmd = base + ["--role", "probe", "--out", args.out, "--reps", str(args.reps),
                      "--stops=" + ",".join(map(str, args.stops))] + (["--sync"] if args.sync else [])
        rc = subprocess.call(cmd)
    finally:
        open(stopfile, "w").write("stop")
        if load is not None:
            try:
                load.wait(60)
            except subprocess.TimeoutExpired:
                load.send_signal(signal.SIGKILL)
                load.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
