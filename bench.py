#!/usr/bin/env python3
"""Decode throughput benchmark (BASELINE.json metric) for the MI355X engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model llama3-8b]

Workload (BASELINE.json configs[2]/[3]): Llama-3-8B bf16 with
synthetic weights (seed 0; no checkpoint exists offline), 32 concurrent
sequences per micro-batch, prompts U[16,256] tokens from seed 2 (prefilled,
untimed), then K greedy decode steps timed.  A "step" = one decode token for
every sequence of every micro-batch.

N = 1: one GPU runs the whole model, one micro-batch of 32 sequences.
N > 1: launched by torch.distributed.run, one rank per GPU; rank r holds a
contiguous, byte-balanced layer shard (pipeline stage r); N micro-batches of 32
sequences are in flight; hidden states go stage->stage with RCCL send/recv
over xGMI and the sampled token ids go back from the last stage to stage 0
(llama-p2p_amd/pipeline.py).  Per-GPU work is fixed as N grows (weak scaling).

Output: one JSON line (rank 0) with value = total decode tokens/s over all
GPUs, the dominant kernel's roofline (HIP-event timed, same stream) and the CPU
oracle timed on this host's cores (N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decode tokens/sec (node) + % HBM roofline, Llama-3-8B at 1/2/4/8-stage"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
MFMA_PEAK_BF16 = 2.5e15  # dense bf16 MFMA, MI355X spec (MI355X_MICROARCH.md; no sparsity)
MB_SEQS = 32


def make_prompts(vocab: int, n: int, seed: int = 2, lo: int = 16, hi: int = 256):
    import numpy as np

    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n)
    return [np.concatenate([[1], rng.integers(3, vocab, L - 1)]).astype(np.int32) for L in lens]


def measured_traffic(label: str):
    """HBM bytes per launch of the dominant kernel, from the PMC passes committed under
    profiles/ (tools/prof_summary.py traffic); None when that configuration was not profiled."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(path)).get(label)
    except (OSError, ValueError):
        return None


def cpu_baseline(shape_name: str, n_prompt: int = 4, n_decode: int = 6):
    """The CPU oracle (C/OpenMP restatement of llama.cpp's CPU forward, bf16
    weights, f32 accumulation) doing what the reference does: batch-1 greedy
    decode, timed on this host's cores.  Bounded sample: n_decode tokens."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from llama_p2p_amd import synth

    shape = synth.SHAPES[shape_name]
    t0 = time.time()
    m = O.OracleModel(shape, seed=0)
    ctx = m.context(64)
    t_gen = time.time() - t0
    prompt = make_prompts(shape.n_vocab, 1, seed=5, lo=n_prompt, hi=n_prompt)[0]
    lg = ctx.eval(prompt, 0)
    tok = int(lg[0].argmax())
    t1 = time.time()
    for i in range(n_decode):
        lg = ctx.eval([tok], n_prompt + i)
        tok = int(lg[0].argmax())
    dt = time.time() - t1
    cores = O.lib().orc_num_threads()
    ctx.close()
    m.close()
    return {"value": round(n_decode / dt, 3), "unit": "tokens/s", "cores": cores, "kind": "port",
            "sample": f"{shape_name} bf16, batch 1 (the reference's serial path), {n_prompt}-token prompt then "
                      f"{n_decode} greedy decode tokens timed; weight synthesis {t_gen:.1f}s untimed"}


def run_single(args):
    import numpy as np

    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    shape = synth.SHAPES[args.model]
    M = args.seqs
    eng = Engine(f"synthetic:{args.model}:seed=0", n_ctx=args.n_ctx, n_seq_max=max(M, 1))
    prompts = make_prompts(shape.n_vocab, M)
    # prefill (untimed): all but the last prompt token of every sequence, 64 rows per
    # forward; the first decode step then consumes the last prompt token
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    for i in range(0, len(slots), 64):
        eng.stage_rows(slots[i:i + 64], pos[i:i + 64], ids[i:i + 64])
    b = eng.batch(slots=list(range(M)), pos=[len(p) - 1 for p in prompts], ids=[int(p[-1]) for p in prompts],
                  max_steps=args.warmup + args.steps)
    for _ in range(args.warmup):
        b.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.step()
    eng.sync()
    dt = time.perf_counter() - t0
    toks = b.tokens()
    assert toks.shape[1] == args.warmup + args.steps
    # algorithmic bytes per decode step: weights + KV read/write + logits
    ctx_sum = sum(len(p) + args.warmup + args.steps / 2 for p in prompts)
    step_bytes = eng.info.weight_bytes + ctx_sum * shape.kv_bytes_per_pos() + M * shape.kv_bytes_per_pos() + \
        M * shape.n_vocab * 4
    res = {"tok_s": M * args.steps / dt, "ms_per_step": dt * 1e3 / args.steps,
           "step_gbs": step_bytes / (dt / args.steps) / 1e9, "step_bytes": step_bytes}
    # dominant kernel: ffn gate/up (fused, 2 x n_ff x n_embd bf16 per layer) -- HIP events on the engine stream
    us, wbytes = eng.profile_kernel(2, M, iters=3)
    kbytes = wbytes + M * shape.n_embd * 2 + M * shape.n_ff * 2  # weights + activations in/out
    traffic = measured_traffic(f"{args.model}/gate_up/M{M}")
    res["roofline"] = {"bound": "hbm", "achieved": round(kbytes / us / 1e3, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(kbytes / us / 1e3 / HBM_PEAK_GBS, 4),
                       "traffic": round(traffic["traffic_bytes"]) if traffic else None,
                       "traffic_source": (f"profiles/traffic.json: {traffic['kernel']} ({traffic['method']})"
                                          if traffic else None),
                       "kernel": ("mm_wide_kernel" if M > 16 else "mm_kernel") + "<EPI_SWIGLU> (ffn_gate+ffn_up+SiLU*up)", "us_per_launch": round(us, 2),
                       "bytes_per_launch": int(kbytes)}
    # batch-1 decode (the north_star's 70% target), same engine
    if args.batch1_steps > 0:
        b1 = eng.batch(slots=[0], pos=[len(prompts[0]) - 1 + args.warmup + args.steps], ids=[int(toks[0, -1])],
                       max_steps=args.batch1_steps + 4)
        for _ in range(4):
            b1.step()
        eng.sync()
        t0 = time.perf_counter()
        for _ in range(args.batch1_steps):
            b1.step()
        eng.sync()
        d1 = (time.perf_counter() - t0) / args.batch1_steps
        b1_bytes = eng.info.weight_bytes + (len(prompts[0]) + 4 + args.batch1_steps / 2) * shape.kv_bytes_per_pos()
        res["batch1"] = {"tok_s": round(1.0 / d1, 2), "ms_per_token": round(d1 * 1e3, 3),
                         "hbm_frac": round(b1_bytes / d1 / 1e9 / HBM_PEAK_GBS, 4),
                         "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / b1_bytes, 1)}
        # its dominant kernel: gate/up with the ffn RMS_NORM on load (row-tile-persistent GEMV)
        us1, wb1 = eng.profile_kernel(6, 1, iters=3)
        kb1 = wb1 + shape.n_embd * 4 + shape.n_ff * 2
        res["batch1"]["gate_up"] = {"kernel": "mm_pers_kernel<EPI_SWIGLU, norm on load>", "us_per_launch": round(us1, 2),
                                    "bytes_per_launch": int(kb1), "achieved_gbs": round(kb1 / us1 / 1e3, 1),
                                    "frac": round(kb1 / us1 / 1e3 / HBM_PEAK_GBS, 4)}
        b1.close()
    b.close()
    if args.prefill_prompts > 0:
        res["prefill"] = prefill_bench(eng, shape, args.prefill_prompts, args.prefill_len)
    eng.close()
    return res


def q8_bench(args):
    """The same model quantised to Q8_0 (a llama.cpp Q8_0 GGUF): batch-1 and
    M-sequence greedy decode, and the Q8 gate/up kernel against the HBM roofline.  Algorithmic
    bytes = the Q8_0 weights (1.0625 B/weight in packed tiles) + K/V + logits."""
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    shape = synth.SHAPES[args.model]
    M = args.seqs
    eng = Engine(f"synthetic:{args.model}:seed=0:q8_0", n_ctx=args.n_ctx, n_seq_max=max(M, 1))
    assert eng.info.weight_type == 8
    prompts = make_prompts(shape.n_vocab, M)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    out = {"model": f"{args.model} Q8_0 (quantisation of the same synthetic bf16 weights)",
           "weight_bytes": int(eng.info.weight_bytes)}
    steps = args.q8_steps
    b = eng.batch(slots=list(range(M)), pos=[len(p) - 1 for p in prompts], ids=[int(p[-1]) for p in prompts],
                  max_steps=4 + steps)
    for _ in range(4):
        b.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step()
    eng.sync()
    dt = (time.perf_counter() - t0) / steps
    toks = b.tokens()
    b.close()
    ctx_sum = sum(len(p) + 4 + steps / 2 for p in prompts)
    step_bytes = eng.info.weight_bytes + ctx_sum * shape.kv_bytes_per_pos() + M * shape.n_vocab * 4
    out[f"decode_M{M}"] = {"tok_s": round(M / dt, 1), "ms_per_step": round(dt * 1e3, 3),
                           "hbm_frac": round(step_bytes / dt / 1e9 / HBM_PEAK_GBS, 4)}
    b1 = eng.batch(slots=[0], pos=[len(prompts[0]) + 3 + steps], ids=[int(toks[0, -1])], max_steps=steps + 4)
    for _ in range(4):
        b1.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        b1.step()
    eng.sync()
    d1 = (time.perf_counter() - t0) / steps
    b1.close()
    b1_bytes = eng.info.weight_bytes + (len(prompts[0]) + 8 + steps * 1.5) * shape.kv_bytes_per_pos()
    out["batch1"] = {"tok_s": round(1.0 / d1, 2), "ms_per_token": round(d1 * 1e3, 3),
                     "hbm_frac": round(b1_bytes / d1 / 1e9 / HBM_PEAK_GBS, 4),
                     "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / b1_bytes, 1)}
    for m in (1, M):
        us, wbytes = eng.profile_kernel(2, m, iters=3)
        kb = wbytes + m * shape.n_embd + m * shape.n_embd // 8 + m * shape.n_ff * 4
        out[f"gate_up_M{m}"] = {"kernel": "mq8_kernel<EPI_SWIGLU>", "us_per_launch": round(us, 2),
                                "bytes_per_launch": int(kb), "achieved_gbs": round(kb / us / 1e3, 1),
                                "frac": round(kb / us / 1e3 / HBM_PEAK_GBS, 4)}
    eng.close()
    return out


def tiny_bench(args):
    """BASELINE.json config 2: TinyLlama-1.1B on one MI355X -- batch-1 greedy decode of 128 tokens
    on a fixed prompt (BOS + 31 ids uniform in [3, 32000) from seed 1) and batched
    prefill of 32 prompts x 128 tokens, against the HBM and MFMA rooflines."""
    import numpy as np

    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    name = "tinyllama-1.1b"
    shape = synth.SHAPES[name]
    eng = Engine(f"synthetic:{name}:seed=0", n_ctx=512, n_seq_max=32)
    rng = np.random.default_rng(1)
    prompt = [1] + [int(t) for t in rng.integers(3, shape.n_vocab, 31)]
    n_gen = args.tiny_tokens
    eng.forward_rows([0] * 31, list(range(31)), prompt[:31], want_logits=False)
    b = eng.batch(slots=[0], pos=[31], ids=[prompt[31]], max_steps=n_gen + 4)
    for _ in range(4):
        b.step()
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(n_gen):
        b.step()
    eng.sync()
    d1 = (time.perf_counter() - t0) / n_gen
    b.close()
    by = eng.info.weight_bytes + (36 + n_gen / 2) * shape.kv_bytes_per_pos() + shape.n_vocab * 4
    out = {"model": f"{name} bf16 (synthetic weights, seed 0)",
           "batch1": {"tok_s": round(1.0 / d1, 1), "ms_per_token": round(d1 * 1e3, 4), "tokens": n_gen,
                      "hbm_frac": round(by / d1 / 1e9 / HBM_PEAK_GBS, 4),
                      "roofline_tok_s": round(HBM_PEAK_GBS * 1e9 / by, 1)}}
    if args.prefill_prompts > 0:
        out["prefill"] = prefill_bench(eng, shape, args.prefill_prompts, args.prefill_len)
    eng.close()
    return out


def copy_peak(gib: int = 4, iters: int = 10):
    """Measured HBM copy ceiling: the engine's streaming copy kernel (16 B per lane,
    mx_probe_copy) over two gib-GiB buffers, (read + write) bytes / HIP-event time on its stream.
    Reported next to the 8 TB/s spec that the roofline fractions use."""
    from llama_p2p_amd import engine

    gbs = engine.probe_copy(0, gib, iters)
    rd = engine.probe_copy(0, gib, iters, read_only=True)
    return {"gbs": round(gbs, 1), "frac_of_spec": round(gbs / HBM_PEAK_GBS, 4),
            "read_gbs": round(rd, 1), "read_frac_of_spec": round(rd / HBM_PEAK_GBS, 4),
            "method": f"mx_probe_copy / mx_probe_read: 16-B/lane streaming kernels, {gib} GiB x {iters}, "
                      "(read + write) or read bytes / HIP-event time"}


def prefill_bench(eng, shape, n_prompts: int, plen: int):
    """Batched prefill: n_prompts prompts of plen tokens (seed 3) pushed through the
    engine's GEMM path (chunks of up to PREFILL_ROWS = 4096 rows) with no lm_head (logits of prompt tokens are not needed), timed on the
    host around the whole pass.  MFMA utilisation = achieved dense bf16 FLOP/s / 2.5 PFLOP/s."""
    import numpy as np

    rng = np.random.default_rng(3)
    slots, pos, ids = [], [], []
    for i in range(n_prompts):
        slots += [i] * plen
        pos += list(range(plen))
        ids += [1] + [int(t) for t in rng.integers(3, shape.n_vocab, plen - 1)]
    eng.forward_rows(slots[:64], pos[:64], ids[:64], want_logits=False)  # warm
    eng.sync()
    t0 = time.perf_counter()
    eng.forward_rows(slots, pos, ids, want_logits=False)
    eng.sync()
    dt = time.perf_counter() - t0
    n_tok = len(ids)
    h, ff, L = shape.n_embd, shape.n_ff, shape.n_layer
    kv = h // shape.n_head * shape.n_head_kv
    linear = L * (h * (h + 2 * kv) + h * h + 3 * h * ff)
    attn = 4 * L * h * n_prompts * plen * (plen + 1) // 2  # QK^T + PV, causal
    flops = 2 * n_tok * linear + attn
    return {"tok_s": round(n_tok / dt, 1), "ms": round(dt * 1e3, 2), "tokens": n_tok,
            "tflops": round(flops / dt / 1e12, 1), "mfma_frac": round(flops / dt / MFMA_PEAK_BF16, 4),
            "sample": f"{n_prompts} prompts x {plen} tokens, 4096-row GEMM chunks, no lm_head"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seqs", type=int, default=MB_SEQS, help="sequences per micro-batch")
    ap.add_argument("--n-ctx", type=int, default=512)
    ap.add_argument("--batch1-steps", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prefill-prompts", type=int, default=32)
    ap.add_argument("--prefill-len", type=int, default=128)
    ap.add_argument("--q8-steps", type=int, default=32, help="Q8_0 decode steps (0: skip the Q8_0 section)")
    ap.add_argument("--tiny-tokens", type=int, default=128,
                    help="TinyLlama-1.1B batch-1 tokens (config 2; 0: skip the section)")
    ap.add_argument("--force-pipeline", action="store_true", help="run the torch.distributed pipeline path even at N=1")
    ap.add_argument("--copy-peak-only", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.copy_peak_only:
        print(json.dumps(copy_peak()), flush=True)
        return

    # stdout carries exactly the one JSON line: native libraries that write to fd 1 (the RCCL
    # version banner at communicator init, HIP runtime notes) are sent to stderr, and Python's
    # sys.stdout keeps the original descriptor
    real_stdout = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(real_stdout, "w", buffering=1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1 or args.force_pipeline:
        from llama_p2p_amd import pipeline

        return pipeline.bench_main(args, METRIC, make_prompts)

    res = run_single(args)
    try:
        copy = copy_peak()
    except Exception as ex:  # report, never hide
        copy = {"error": repr(ex)}
    line = {
        "metric": METRIC, "value": round(res["tok_s"], 2), "unit": "tokens/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(res["ms_per_step"], 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded random bf16 weights of the exact shape; random prompt ids)",
        "config": {"workload": f"{args.model} greedy decode, {args.seqs} concurrent sequences, prompts U[16,256] "
                               f"(seed 2), n_ctx {args.n_ctx}", "model": args.model, "stages": 1,
                   "micro_batches": 1, "seqs_per_micro_batch": args.seqs, "parallelism": "pp1"},
        "step_hbm_gbs": round(res["step_gbs"], 1), "step_hbm_frac": round(res["step_gbs"] / HBM_PEAK_GBS, 4),
        "roofline": res["roofline"],
    }
    if "batch1" in res:
        line["batch1"] = res["batch1"]
    if "prefill" in res:
        line["prefill"] = res["prefill"]
    if args.q8_steps > 0:
        try:
            line["q8_0"] = q8_bench(args)
        except Exception as ex:  # report, never hide
            line["q8_0"] = {"error": repr(ex)}
    if args.tiny_tokens > 0:
        try:
            line["tinyllama"] = tiny_bench(args)
        except Exception as ex:  # report, never hide
            line["tinyllama"] = {"error": repr(ex)}
    line["hbm_copy_peak"] = copy
    if "gbs" in copy:
        line["roofline"]["frac_of_copy_peak"] = round(line["roofline"]["achieved"] / copy["gbs"], 4)
        line["roofline"]["frac_of_read_peak"] = round(line["roofline"]["achieved"] / copy["read_gbs"], 4)
    if not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(args.model)
        except Exception as ex:  # report, never hide
            line["cpu_baseline"] = {"error": repr(ex)}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
