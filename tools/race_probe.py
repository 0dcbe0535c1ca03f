#!/usr/bin/env python3
"""Diagnosis: are the engine's results independent of what else runs on the GPU?

    python tools/race_probe.py [--model llama3-8b] [--reps 4] [--load]

Prefill (64-row chunks, as pipeline.Stage does) then one 32-row step with logits, repeated `reps`
times on the same inputs (the same KV slots are rewritten), with --load a second stream running
large GEMMs all the while.  Prints, per phase, whether every repetition is bitwise identical.
"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--load", action="store_true")
    ap.add_argument("--mem-load", action="store_true", help="the second stream streams 2 GiB copies (HBM-bound)")
    ap.add_argument("--alloc-load", action="store_true",
                    help="the second thread allocates and frees 1 GiB device buffers in a loop (page-table updates)")
    ap.add_argument("--engine-load", type=int, default=0,
                    help="the load is a SECOND engine (layers [0, N)) prefilling in chunks of --load-chunk rows")
    ap.add_argument("--load-chunk", type=int, default=64)
    ap.add_argument("--load-from", type=int, default=0,
                    help="the load engine is a LATER stage: layers [N, n_layer) + head fed random x_in rows")
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--lo", type=int, default=16)
    ap.add_argument("--hi", type=int, default=256)
    ap.add_argument("--layers", type=int, default=0, help="stage of the first N layers only (0: all + head)")
    ap.add_argument("--decode", type=int, default=0, help="then N greedy steps of one 32-row decode batch")
    ap.add_argument("--from-layer", type=int, default=0,
                    help="a later stage: layers [L, n_layer) + head fed seeded random x_in rows (f32 hand-off)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    sh = synth.SHAPES[args.model]
    torch.cuda.set_stream(torch.cuda.Stream())
    M = args.M
    prompts = bench.make_prompts(sh.n_vocab, M, lo=args.lo, hi=args.hi)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    kw = dict(layer_begin=0, layer_end=args.layers) if args.layers else {}
    if args.from_layer:
        kw = dict(layer_begin=args.from_layer, layer_end=sh.n_layer, handoff_bf16=False)
        g = torch.Generator(device="cuda").manual_seed(5)
        xin_all = torch.randn((len(slots) + M, sh.n_embd), generator=g, device="cuda", dtype=torch.float32)
    eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=512, n_seq_max=M, device=0, **kw)
    stop = threading.Event()

    def load():
        torch.cuda.set_stream(torch.cuda.Stream())
        if args.alloc_load:
            while not stop.is_set():
                t = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
                t[:4096].zero_()
                torch.cuda.current_stream().synchronize()
                del t
                torch.cuda.empty_cache()
            return
        if args.engine_load or args.load_from:
            if args.load_from:
                e2 = Engine(f"synthetic:{args.model}:seed=0", n_ctx=512, n_seq_max=M, device=0,
                            layer_begin=args.load_from, layer_end=sh.n_layer, handoff_bf16=False)
                g2 = torch.Generator(device="cuda").manual_seed(9)
                xi2 = torch.randn((64, sh.n_embd), generator=g2, device="cuda", dtype=torch.float32)
            else:
                e2 = Engine(f"synthetic:{args.model}:seed=1", n_ctx=512, n_seq_max=M, device=0, layer_begin=0,
                            layer_end=args.engine_load)
            xo2 = torch.empty((64, sh.n_embd), dtype=torch.float32, device="cuda")
            st2 = torch.cuda.current_stream().cuda_stream
            ready.set()
            while not stop.is_set():
                for i in range(0, len(slots), args.load_chunk):
                    k = min(args.load_chunk, len(slots) - i)
                    if args.load_from:
                        e2.stage_rows(slots[i:i + k], pos[i:i + k], None, xi2.data_ptr(), 0, False, st2)
                    else:
                        e2.stage_rows(slots[i:i + k], pos[i:i + k], ids[i:i + k], 0, xo2.data_ptr(), False, st2)
                    if stop.is_set():
                        break
            e2.close()
            return
        if args.mem_load:
            a = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
            b = torch.empty_like(a)
            while not stop.is_set():
                for _ in range(4):
                    b.copy_(a)
                    a.copy_(b)
                torch.cuda.current_stream().synchronize()
            return
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        while not stop.is_set():
            for _ in range(8):
                a = (a @ a).clamp_(-1, 1)
            torch.cuda.current_stream().synchronize()

    ready = threading.Event()
    th = threading.Thread(target=load, daemon=True) if (args.load or args.mem_load or args.engine_load or
                                                        args.load_from or args.alloc_load) else None
    if th:
        th.start()
        if args.engine_load or args.load_from:
            ready.wait(300)
    dp, di = [len(p) - 1 for p in prompts], [int(p[-1]) for p in prompts]
    rows = list(range(M))
    xo = torch.empty((64, sh.n_embd), dtype=torch.float32, device="cuda")
    outs = []
    for r in range(args.reps):
        st = torch.cuda.current_stream().cuda_stream
        for i in range(0, len(slots), args.chunk):
            k = min(args.chunk, len(slots) - i)
            if args.from_layer:
                eng.stage_rows(slots[i:i + k], pos[i:i + k], None, xin_all[i:i + k].data_ptr(), 0, False, st)
            else:
                eng.stage_rows(slots[i:i + k], pos[i:i + k], ids[i:i + k], 0,
                               xo.data_ptr() if args.layers else 0, False, st)
        if args.from_layer:
            outs.append(eng.stage_rows(rows, dp, None, xin_all[len(slots):].data_ptr(), 0, True, st))
        elif args.layers:
            eng.stage_rows(rows, dp, di, 0, xo.data_ptr(), False, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append(xo[:M].cpu().numpy().copy())
        elif args.decode:
            b = eng.batch(rows, dp, di, max_steps=args.decode)
            for _ in range(args.decode):
                b.step(stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append(b.tokens().astype(np.float32))
            b.close()
        else:
            outs.append(eng.stage_rows(rows, dp, di, 0, 0, True, torch.cuda.current_stream().cuda_stream))
    stop.set()
    if th:
        th.join()
    same = [bool(np.array_equal(outs[0], o)) for o in outs[1:]]
    diff = [float(np.abs(outs[0] - o).max()) for o in outs[1:]]
    print({"model": args.model, "load": args.load, "mem_load": args.mem_load, "alloc_load": args.alloc_load, "engine_load": args.engine_load,
           "load_chunk": args.load_chunk, "load_from": args.load_from, "layers": args.layers or "all", "reps_equal": same,
           "max_abs_diff": diff, "chunk": args.chunk, "decode": args.decode, "from_layer": args.from_layer, "prompts": [args.lo, args.hi]})
    eng.close()


if __name__ == "__main__":
    main()
