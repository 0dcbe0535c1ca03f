#!/usr/bin/env python3
"""Decode throughput benchmark (BASELINE.json metric) for the MI355X engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model llama3-8b]

Workload (BASELINE.json configs[2]/[3]): Llama-3-8B bf16 with
synthetic weights (seed 0; no checkpoint exists offline), 32 concurrent
sequences per micro-batch, prompts U[16,256] tokens from seed 2 (prefilled,
untimed), then K greedy decode steps timed.  A "step" = one decode token for
every sequence of every micro-batch.

N = 1: one GPU runs the whole model, one micro-batch of 32 sequences.
N > 1: one rank per GPU (started by torch.distributed.run, or -- for the plain
`python3 bench.py --gpus N` -- by this script itself, llama-p2p_amd/launch.py); rank r holds a
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
MFMA_PEAK_I8 = 5.0e15  # dense int8 MFMA: the K=64 / 32x32x32 forms at 2x the bf16 rate (MI355X_MICROARCH.md)
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


def tiny_prompt(vocab: int = 32000):
    """SURVEY §8d config 1/2 fixed prompt: BOS + 31 ids uniform in [3, vocab) from seed 1."""
    import numpy as np

    rng = np.random.default_rng(1)
    return np.array([1] + [int(t) for t in rng.integers(3, vocab, 31)], np.int32)


def cpu_baseline(shape_name: str, n_prompt: int = 16, n_decode: int = 24, tiny_tokens: int = 128):
    """The CPU oracle (C/OpenMP restatement of llama.cpp's CPU forward: bf16 weights, f32
    accumulation) doing what the reference does -- one request at a time, batch-1 greedy decode
    (its lock serialises every request, p2p:121) -- timed on this host's cores.  Bounded samples:
    the bench model (n_decode tokens after an n_prompt-token prompt), and BASELINE config 1
    (TinyLlama-1.1B, 128 greedy tokens on the fixed prompt, whole generate() call timed)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from llama_p2p_amd import synth

    shape = synth.SHAPES[shape_name]
    t0 = time.time()
    m = O.OracleModel(shape, seed=0)
    ctx = m.context(128)
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
    out = {"value": round(n_decode / dt, 3), "unit": "tokens/s", "cores": cores, "kind": "port",
           "sample": f"{shape_name} bf16, batch 1 (the reference serialises requests, p2p:121), {n_prompt}-token "
                     f"prompt then {n_decode} greedy decode tokens timed; weight synthesis {t_gen:.1f}s untimed"}
    if tiny_tokens > 0:
        ts = synth.SHAPES["tinyllama-1.1b"]
        tm = O.OracleModel(ts, seed=0)
        tc = tm.context(512)
        t2 = time.time()
        toks = tc.generate_greedy(tiny_prompt(ts.n_vocab), tiny_tokens)
        d2 = time.time() - t2
        tc.close()
        tm.close()
        out["config1"] = {"value": round(tiny_tokens / d2, 2), "unit": "tokens/s", "cores": cores, "kind": "port",
                          "seconds": round(d2, 3), "first_tokens": [int(t) for t in toks[:8]],
                          "sample": f"BASELINE config 1: tinyllama-1.1b bf16, {tiny_tokens} greedy tokens on the "
                                    "fixed prompt (BOS + 31 ids, seed 1), prompt eval + decode timed"}
    return out


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
    eng.forward_rows(slots, pos, ids, want_logits=False)  # GEMM prefill chunks
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


def quant_bench(args, wtype: str, steps: int):
    """The same model shape as a llama.cpp quantised GGUF: "q8_0" (the Q8_0
    quantisation of the synthetic bf16 weights) or "q4_k_m" (llama.cpp's Q4_K_M recipe: Q4_K with
    Q6_K attn_v / ffn_down on the use_more_bits layers and a Q6_K output, synthetic K-quant blocks).
    Batch-1 and M-sequence greedy decode and the gate/up kernel against the HBM roofline.
    Algorithmic bytes = the packed weights (Q8_0 1.0625 B/weight; K-quants their GGUF block bytes,
    +2.8% for byte-aligned Q4_K scales) + K/V + logits."""
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    shape = synth.SHAPES[args.model]
    M = args.seqs
    eng = Engine(f"synthetic:{args.model}:seed=0:{wtype}", n_ctx=args.n_ctx, n_seq_max=max(M, 1))
    assert eng.info.weight_type == {"q8_0": 8, "q4_k_m": 12, "q4_0": 2}[wtype]
    prompts = make_prompts(shape.n_vocab, M)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    desc = {"q8_0": "Q8_0 (quantisation of the same synthetic bf16 weights)",
            "q4_k_m": "Q4_K_M (llama.cpp recipe types, synthetic K-quant blocks; native int8-MFMA K-quant path)",
            "q4_0": "Q4_0 layers (quantize_row_q4_0_ref of the same synthetic bf16 weights), Q8_0 embd/output"}
    out = {"model": f"{args.model} {desc[wtype]}", "weight_bytes": int(eng.info.weight_bytes)}
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
    h = shape.n_embd
    for m in (1, M):
        us, wbytes = eng.profile_kernel(2, m, iters=3)
        if wtype in ("q8_0", "q4_0"):
            kb = wbytes + m * h + m * h // 8 + m * shape.n_ff * 4   # int8 rows + scales in, f32 act out
        else:
            kb = wbytes + m * h + m * h // 64 + m * h // 8 + m * shape.n_ff * 4  # Q8_K rows, d, sub-block sums
        kname = {"q8_0": "mq8_kernel" if m <= 16 else "mq8_wide_kernel",
                 "q4_0": "mq8_kernel<Q4>" if m <= 16 else "mq8_wide_kernel<Q4>",
                 "q4_k_m": "mkq_pers_kernel" if m <= 16 else "mkq_wide_kernel"}[wtype]
        if m == 1:  # one token: the form the decode runs, RMS_NORM + quantisation done on load in the GEMV
            kname += "<quantise-on-load>"
        out[f"gate_up_M{m}"] = {"kernel": kname + "<EPI_SWIGLU>",
                                "us_per_launch": round(us, 2), "bytes_per_launch": int(kb),
                                "achieved_gbs": round(kb / us / 1e3, 1), "frac": round(kb / us / 1e3 / HBM_PEAK_GBS, 4)}
    if args.prefill_prompts > 0:
        # > 64-row chunks: K-quant as dequantised bf16 GEMMs; Q8_0 as grouped Q8_0 GEMVs (ggml's
        # arithmetic), or dequantised bf16 GEMMs with MX_Q8_GEMM_PREFILL=1
        # Q8_0 / Q4_0 chunks run the int8-MFMA GEMM (q8gemm_kernel): utilisation against the int8 peak
        out["prefill"] = prefill_bench(eng, shape, args.prefill_prompts, args.prefill_len,
                                       int8=wtype in ("q8_0", "q4_0"))
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


def geometry_bench(args, name: str = "llama2-7b", steps: int = 16):
    """A non-Llama-3 geometry (Llama-2-7B: MHA, ff 11008, V 32000) at batch 1 and 32 rows: the
    shape-specialised fast paths (row-tile-persistent GEMVs for K 2048/4096/8192 with Llama-3 tile
    counts) do not apply to its gate/up (1376 tiles) and ffn_down (K 11008), so this measures the
    generic GEMV fallbacks against the same HBM roofline."""
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    shape = synth.SHAPES[name]
    M = args.seqs
    eng = Engine(f"synthetic:{name}:seed=0", n_ctx=512, n_seq_max=M)
    prompts = make_prompts(shape.n_vocab, M, lo=16, hi=128)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    out = {"model": f"{name} bf16 (synthetic weights, seed 0)", "weight_bytes": int(eng.info.weight_bytes)}
    for m in (1, M):
        b = eng.batch(slots=list(range(m)), pos=[len(p) - 1 for p in prompts[:m]],
                      ids=[int(p[-1]) for p in prompts[:m]], max_steps=steps + 2)
        for _ in range(2):
            b.step()
        eng.sync()
        t1 = time.perf_counter()
        for _ in range(steps):
            b.step()
        eng.sync()
        dt = (time.perf_counter() - t1) / steps
        b.close()
        ctx_sum = sum(len(p) + 2 + steps / 2 for p in prompts[:m])
        by = eng.info.weight_bytes + ctx_sum * shape.kv_bytes_per_pos() + m * shape.n_vocab * 4
        out[f"decode_M{m}"] = {"tok_s": round(m / dt, 2), "ms_per_step": round(dt * 1e3, 3),
                               "hbm_frac": round(by / dt / 1e9 / HBM_PEAK_GBS, 4)}
        us, wbytes = eng.profile_kernel(2, m, iters=2)
        kb = wbytes + m * shape.n_embd * 2 + m * shape.n_ff * 2
        out[f"gate_up_M{m}"] = {"us_per_launch": round(us, 2), "frac": round(kb / us / 1e3 / HBM_PEAK_GBS, 4)}
    eng.close()
    return out


def big_bench(args):
    """BASELINE config 5's model on ONE MI355X (141 GB of bf16 weights fit in 288 GB): Llama-3-70B
    synthetic, batch-1 and M-sequence greedy decode tok/s against the HBM roofline, and its gate/up
    GEMV (the dominant kernel) at both widths.  The 8-stage pipeline itself needs the 8-GPU node."""
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine

    name = "llama3-70b"
    shape = synth.SHAPES[name]
    M = args.seqs
    t0 = time.time()
    eng = Engine(f"synthetic:{name}:seed=0", n_ctx=512, n_seq_max=M)
    t_load = time.time() - t0
    prompts = make_prompts(shape.n_vocab, M, lo=16, hi=64)
    slots, pos, ids = [], [], []
    for i, p in enumerate(prompts):
        slots += [i] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
    eng.forward_rows(slots, pos, ids, want_logits=False)
    out = {"model": f"{name} bf16 (synthetic weights, seed 0)", "weight_bytes": int(eng.info.weight_bytes),
           "load_s": round(t_load, 1)}
    steps = args.big_steps
    for m in (1, M):
        b = eng.batch(slots=list(range(m)), pos=[len(p) - 1 for p in prompts[:m]], ids=[int(p[-1]) for p in prompts[:m]],
                      max_steps=steps + 2)
        for _ in range(2):
            b.step()
        eng.sync()
        t1 = time.perf_counter()
        for _ in range(steps):
            b.step()
        eng.sync()
        dt = (time.perf_counter() - t1) / steps
        b.close()
        ctx_sum = sum(len(p) + 2 + steps / 2 for p in prompts[:m])
        by = eng.info.weight_bytes + ctx_sum * shape.kv_bytes_per_pos() + m * shape.n_vocab * 4
        out[f"decode_M{m}"] = {"tok_s": round(m / dt, 2), "ms_per_step": round(dt * 1e3, 3),
                               "hbm_frac": round(by / dt / 1e9 / HBM_PEAK_GBS, 4),
                               "roofline_tok_s": round(m * HBM_PEAK_GBS * 1e9 / by, 1)}
        us, wbytes = eng.profile_kernel(2 if m > 1 else 6, m, iters=2)
        kb = wbytes + m * shape.n_embd * 2 + m * shape.n_ff * 2
        out[f"gate_up_M{m}"] = {"us_per_launch": round(us, 2), "bytes_per_launch": int(kb),
                                "achieved_gbs": round(kb / us / 1e3, 1), "frac": round(kb / us / 1e3 / HBM_PEAK_GBS, 4)}
        if m == M:
            break
    eng.close()
    return out


def hbm_probe(gib: int = 4, iters: int = 8):
    """Measured HBM streaming rates: the best of the engine's streaming probe
    variants (16 B per lane; 4/8/16 loads in flight x 1024-4096 work-groups x non-temporal or not)
    over gib-GiB buffers, bytes / HIP-event time.  Reported next to the 8 TB/s spec that the
    roofline fractions use; a reference stream, not a hard ceiling."""
    from llama_p2p_amd import engine

    cp, cdesc = engine.probe_copy(0, gib, iters)
    rd, rdesc = engine.probe_copy(0, gib, iters, read_only=True)
    return {"copy_gbs": round(cp, 1), "copy_frac_of_spec": round(cp / HBM_PEAK_GBS, 4), "copy_variant": cdesc,
            "read_gbs": round(rd, 1), "read_frac_of_spec": round(rd / HBM_PEAK_GBS, 4), "read_variant": rdesc,
            "method": f"mx_probe_copy / mx_probe_read: best of {gib} GiB x {iters} passes per variant, "
                      "(read + write) or read bytes / HIP-event time"}


def prefill_bench(eng, shape, n_prompts: int, plen: int, int8: bool = False):
    """Batched prefill: n_prompts prompts of plen tokens (seed 3) pushed through the
    engine's GEMM path (chunks of up to PREFILL_ROWS = 4096 rows) with no lm_head (logits of prompt tokens are not needed), timed on the
    host around the whole pass.  MFMA utilisation = achieved dense FLOP/s (OP/s) / the dense peak of
    the arithmetic the GEMMs run in: bf16 2.5 PFLOP/s, or for the Q8_0 / Q4_0 int8 GEMM (int8=True)
    the int8 dense peak of 5 POPS."""
    import numpy as np

    rng = np.random.default_rng(3)
    slots, pos, ids = [], [], []
    for i in range(n_prompts):
        slots += [i] * plen
        pos += list(range(plen))
        ids += [1] + [int(t) for t in rng.integers(3, shape.n_vocab, plen - 1)]
    eng.forward_rows(slots[:2 * plen], pos[:2 * plen], ids[:2 * plen], want_logits=False)  # warm (GEMM path)
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
    peak = MFMA_PEAK_I8 if int8 else MFMA_PEAK_BF16
    return {"tok_s": round(n_tok / dt, 1), "ms": round(dt * 1e3, 2), "tokens": n_tok,
            "tflops": round(flops / dt / 1e12, 1), "mfma_frac": round(flops / dt / peak, 4),
            "mfma_peak": {"dtype": "int8" if int8 else "bf16", "tflops": peak / 1e12},
            "sample": f"{n_prompts} prompts x {plen} tokens, 4096-row GEMM chunks, no lm_head"}


def make_text_prompts(n, tokenize, seed=2, lo=16, hi=256):
    """n text prompts of about U[lo, hi] tokens (config 3's lengths): random words, trimmed by the
    model's own tokenizer so that every prompt fits n_ctx 512 with the reference's 100 new tokens."""
    import numpy as np

    rng = np.random.default_rng(seed)
    words = ["node", "peer", "model", "layer", "cache", "token", "request", "the", "of", "and", "gossip",
             "stage", "prompt", "answer", "question", "fast", "memory", "bandwidth", "graph", "stream"]
    out = []
    for i in range(n):
        L = int(rng.integers(lo, hi + 1))
        ws = [words[int(j)] for j in rng.integers(0, len(words), L)]
        while len(ws) > 1 and len(tokenize(f"Request {i}: " + " ".join(ws))) > L:
            ws = ws[:max(1, int(len(ws) * 0.9))]
        out.append(f"Request {i}: " + " ".join(ws))
    return out


class _CountingModel:
    """The node's ``self.model``: forwards to Llama and counts completion tokens (cached_inference
    itself returns text only).  greedy: temperature 0 (the parity setting); otherwise the reference's
    literal call, llama-cpp-python's defaults (temperature 0.8, top_k 40, top_p 0.95, min_p 0.05)."""

    def __init__(self, llm, greedy: bool = True):
        import threading

        self.llm, self.tokens, self.calls, self.lock = llm, 0, 0, threading.Lock()
        self.kw = {"temperature": 0.0} if greedy else {}

    def __call__(self, prompt, **kw):
        out = self.llm(prompt, **self.kw, **kw)
        with self.lock:
            self.tokens += out["usage"]["completion_tokens"]
            self.calls += 1
        return out


def serving_bench(args, n: int = 32, greedy: bool = True):
    """BASELINE config 3 as worded -- Llama-3-8B bf16 serving 32 concurrent synthetic requests with the
    result cache on -- through the drop-in node: n client threads send JSON inference requests at once
    over an in-process REP transport with concurrent contexts (node.LocalTransport) ->
    handle_requests (p2p:84-98) -> cached_inference (p2p:120-133) -> Llama(prompt, max_tokens=100)
    (p2p:125; greedy) -> mx_submit/mx_wait.  A warm-up wave of other prompts runs first (the serving
    engine is long-lived: its decode graphs exist); then wave 1 (n new prompts: tokenize, batched
    prefill, micro-batched decode, detokenize, cache insert) is timed, then the same n prompts again
    (all hits).  tok/s = generated tokens of wave 1 / its wall time, prefill included."""
    import json as _json
    import threading

    from llama_p2p_amd.llama import Llama
    from llama_p2p_amd.node import LlamaP2PNode, LocalTransport

    path = f"synthetic:{args.model}"
    llm = Llama(model_path=path, verbose=False, n_seq_max=max(n, 1), n_ctx=args.n_ctx)
    model = _CountingModel(llm, greedy)
    tr = LocalTransport()
    node = LlamaP2PNode(path, 5000, cache_size=100, secret_key="k", model=model, transport=tr, n_contexts=n)
    threading.Thread(target=node.handle_requests, daemon=True).start()
    tok = lambda t: llm.tokenize(t.encode(), add_bos=True, special=True)  # noqa: E731

    def wave(ps):
        lat = [0.0] * len(ps)
        err = []

        def run(i):
            t = time.perf_counter()
            reply = _json.loads(tr.request(_json.dumps({"type": "inference", "prompt": ps[i],
                                                        "secret_key": "k"}).encode()))
            if "result" not in reply:
                err.append(reply)
            lat[i] = time.perf_counter() - t

        th = [threading.Thread(target=run, args=(i,)) for i in range(len(ps))]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            raise RuntimeError(f"serving: error replies {err[:2]}")
        return time.perf_counter() - t0, lat

    wave(make_text_prompts(n, tok, seed=11))  # warm-up (distinct prompts: no cache hits later)
    prompts = make_text_prompts(n, tok, seed=2)
    n_prompt_tok = sum(len(tok(p)) for p in prompts)
    tok0, calls0 = model.tokens, model.calls
    dt1, lat1 = wave(prompts)
    gen1 = model.tokens - tok0
    calls1 = model.calls
    dt2, lat2 = wave(prompts)
    hits = n - (model.calls - calls1)
    node.active = False
    llm.close()
    lat1.sort()
    how = "greedy" if greedy else "llama-cpp-python default sampling (temperature 0.8, top_k 40, top_p 0.95, min_p 0.05)"
    return {"workload": f"config 3: {path} bf16, {n} concurrent requests through handle_requests (REP contexts) "
                        f"-> cached_inference -> Llama(prompt, max_tokens=100), {how}; then the same {n} again",
            "wave1": {"requests": n, "calls": calls1 - calls0, "prompt_tokens": n_prompt_tok,
                      "generated_tokens": gen1, "wall_s": round(dt1, 4), "tok_s": round(gen1 / dt1, 1),
                      "p50_latency_s": round(lat1[len(lat1) // 2], 4), "max_latency_s": round(lat1[-1], 4)},
            "wave2": {"requests": n, "hit_rate": round(hits / n, 3), "wall_s": round(dt2, 4),
                      "max_latency_ms": round(max(lat2) * 1e3, 3)},
            "overall_hit_rate": round(hits / (2 * n), 3)}


class Sections:
    """Runs the bench sections in order with wall-clock timings on stderr.  The headline section
    raises on failure; optional ones report their error in the line, and are skipped once the
    run has used its time budget (so the default run always ends inside the driver's limit)."""

    def __init__(self, budget_s: float):
        self.t0 = time.time()
        self.budget = budget_s
        self.seconds = {}

    def run(self, name, fn, optional=True):
        if optional and time.time() - self.t0 > self.budget:
            print(f"[bench] {name}: skipped (time budget {self.budget:.0f}s used)", file=sys.stderr, flush=True)
            return {"skipped": f"time budget of {self.budget:.0f}s used"}
        t = time.time()
        print(f"[bench] {name} ...", file=sys.stderr, flush=True)
        try:
            res = fn()
        except Exception as ex:  # report, never hide
            if not optional:
                raise
            res = {"error": repr(ex)}
        self.seconds[name] = round(time.time() - t, 1)
        print(f"[bench] {name}: {self.seconds[name]}s", file=sys.stderr, flush=True)
        return res


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
    ap.add_argument("--kq-steps", type=int, default=32, help="Q4_K_M decode steps (0: skip the Q4_K_M section)")
    ap.add_argument("--q40-steps", type=int, default=32, help="Q4_0 decode steps (0: skip the Q4_0 section)")
    ap.add_argument("--tiny-tokens", type=int, default=128,
                    help="TinyLlama-1.1B batch-1 tokens (config 2; 0: skip the section)")
    ap.add_argument("--big-steps", type=int, default=8, help="Llama-3-70B decode steps (0: skip the section)")
    ap.add_argument("--geometry-steps", type=int, default=16,
                    help="Llama-2-7B-geometry decode steps (generic GEMV paths; 0: skip the section)")
    ap.add_argument("--serve-requests", type=int, default=32,
                    help="config 3 through the node's handler: concurrent requests (0: skip the section)")
    ap.add_argument("--budget", type=float, default=360.0,
                    help="seconds after which optional sections are skipped")
    ap.add_argument("--force-pipeline", action="store_true", help="run the torch.distributed pipeline path even at N=1")
    ap.add_argument("--micro-batches", type=int, default=0, help="pipeline micro-batches in flight (0: one per stage)")
    ap.add_argument("--dry-run", action="store_true",
                    help="pipeline path on CPU over gloo with a toy executor (launcher / schedule check, no GPU)")
    ap.add_argument("--handoff", default="bf16", choices=["bf16", "f32"],
                    help="stage hand-off dtype (f32: stage splits bitwise equal to one engine)")
    ap.add_argument("--prefill-chunk", type=int, default=64, help="pipeline prefill rows per hand-off (<= 64)")
    ap.add_argument("--host-handoff", action="store_true",
                    help="pipeline rehearsal: gloo with host-staged hand-offs, ranks may share a GPU (not RCCL)")
    ap.add_argument("--probe-only", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    from llama_p2p_amd import launch

    if launch.needs_launch(args.gpus):
        # plain `python3 bench.py --gpus N`: start the N ranks here (before anything touches the GPU)
        os.environ["MX_LAUNCHER"] = "bench.py (launch.spawn_ranks)"
        sys.exit(launch.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    launch.rank_init()  # a rank started by spawn_ranks dies with its launcher
    if args.probe_only:
        print(json.dumps(hbm_probe()), flush=True)
        return

    # stdout carries exactly the one JSON line: native libraries that write to fd 1 (the RCCL
    # version banner at communicator init, HIP runtime notes) are sent to stderr, and Python's
    # sys.stdout keeps the original descriptor
    real_stdout = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(real_stdout, "w", buffering=1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1 or args.force_pipeline or args.dry_run:
        from llama_p2p_amd import pipeline

        return pipeline.bench_main(args, METRIC, make_prompts)

    sec = Sections(args.budget)
    res = sec.run("decode", lambda: run_single(args), optional=False)
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
    for k in ("batch1", "prefill"):
        if k in res:
            line[k] = res[k]
    if args.serve_requests > 0:
        sv = sec.run("serving", lambda: serving_bench(args, args.serve_requests))
        if "wave1" in sv:
            sv["ratio_to_value"] = round(sv["wave1"]["tok_s"] / line["value"], 4)
        line["serving"] = sv
        # the reference's literal call (p2p:125): Llama(prompt, max_tokens=100) with its default sampling
        sd = sec.run("serving_default_sampling", lambda: serving_bench(args, args.serve_requests, greedy=False))
        if "wave1" in sd:
            sd["ratio_to_value"] = round(sd["wave1"]["tok_s"] / line["value"], 4)
            if "wave1" in sv:
                sd["ratio_to_greedy_serving"] = round(sd["wave1"]["tok_s"] / sv["wave1"]["tok_s"], 4)
        line["serving_default_sampling"] = sd
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = sec.run("cpu_baseline", lambda: cpu_baseline(args.model))
    if args.tiny_tokens > 0:
        line["tinyllama"] = sec.run("tinyllama", lambda: tiny_bench(args))
    line["hbm_probe"] = sec.run("hbm_probe", hbm_probe)
    if args.q8_steps > 0:
        line["q8_0"] = sec.run("q8_0", lambda: quant_bench(args, "q8_0", args.q8_steps))
    if args.kq_steps > 0:
        line["q4_k_m"] = sec.run("q4_k_m", lambda: quant_bench(args, "q4_k_m", args.kq_steps))
    if args.q40_steps > 0:
        line["q4_0"] = sec.run("q4_0", lambda: quant_bench(args, "q4_0", args.q40_steps))
    if args.big_steps > 0:
        line["llama3_70b"] = sec.run("llama3_70b", lambda: big_bench(args))
    if args.geometry_steps > 0:
        line["llama2_7b_geometry"] = sec.run("llama2_7b_geometry", lambda: geometry_bench(args, steps=args.geometry_steps))
    line["section_seconds"] = sec.seconds
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
