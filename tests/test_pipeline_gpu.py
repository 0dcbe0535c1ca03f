"""Pipeline stages on one GPU: engines holding layer ranges, hand-offs done in-process.

The 8-GPU run uses RCCL between processes (one GPU each), which a 1-GPU box
cannot host; the send/recv schedule itself is covered on CPU (gloo) by
test_pipeline_cpu.py.  Here the *engine side* is checked: stage engines with
layer ranges, device hidden-state hand-off (x_in / x_out), the last stage's
on-device greedy head writing into a bound id buffer, per-stage position
advance, and the prefill path (mx_stage_rows) -- the S-stage result must equal
the one-engine run token for token.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(prompts, base_slot=0):
    slots, pos, ids, st = [], [], [], ([], [], [])
    for i, p in enumerate(prompts):
        sl = base_slot + i
        slots += [sl] * (len(p) - 1)
        pos += list(range(len(p) - 1))
        ids += [int(t) for t in p[:-1]]
        st[0].append(sl); st[1].append(len(p) - 1); st[2].append(int(p[-1]))
    return (slots, pos, ids), st


@pytest.mark.parametrize("wtype", ["bf16", "q8_0"])
@pytest.mark.parametrize("splits", [[(0, 1), (1, 3)], [(0, 1), (1, 2), (2, 3)]])
def test_stage_engines_match_full_model(splits, wtype):
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine
    from llama_p2p_amd.pipeline import EngineAdapter

    name = "test-gqa8"
    sh = synth.SHAPES[name]
    rng = np.random.default_rng(5)
    M, steps = 4, 10
    prompts = [np.concatenate([[1], rng.integers(3, sh.n_vocab, int(rng.integers(5, 30)))]) for _ in range(M)]
    (slots, pos, ids), st = _rows(prompts)
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream())

    path = f"synthetic:{name}:seed=0:{wtype}"  # Q8_0: stage x_in feeds the quantise-on-load GEMVs
    full = Engine(path, n_ctx=128, n_seq_max=M)
    fa = EngineAdapter(full)
    for i in range(0, len(slots), 64):
        fa.stage_rows_tensors(slots[i:i + 64], pos[i:i + 64], ids[i:i + 64], None, None)
    fb = full.batch(st[0], st[1], st[2], max_steps=steps)
    for _ in range(steps):
        fb.step()
    ref = fb.tokens()

    engs = [Engine(path, n_ctx=128, n_seq_max=M, layer_begin=lb, layer_end=le)
            for lb, le in splits]
    ads = [EngineAdapter(e) for e in engs]
    S = len(engs)
    buf = [torch.empty((64, sh.n_embd), dtype=torch.float32, device=dev) for _ in range(S)]
    for i in range(0, len(slots), 64):
        n = min(64, len(slots) - i)
        for s in range(S):
            xin = buf[s - 1][:n] if s > 0 else None
            xout = buf[s][:n] if s < S - 1 else None
            ads[s].stage_rows_tensors(slots[i:i + n], pos[i:i + n], ids[i:i + n] if s == 0 else None, xin, xout)
    batches = [a.batch(st[0], st[1], st[2] if s == 0 else None, steps if s == S - 1 else 0) for s, a in enumerate(ads)]
    tok = torch.tensor(st[2], dtype=torch.int32, device=dev)
    batches[0].bind_ids_tensor(tok)
    batches[-1].bind_ids_tensor(torch.zeros(M, dtype=torch.int32, device=dev))
    xs = [torch.empty((M, sh.n_embd), dtype=torch.float32, device=dev) for _ in range(S)]
    for _ in range(steps):
        for s in range(S):
            xin = xs[s - 1] if s > 0 else None
            xout = xs[s] if s < S - 1 else None
            batches[s].step_tensors(xin, xout)
        tok.copy_(batches[-1]._ids_tensor)  # the "send" of the sampled ids back to stage 0
    torch.cuda.synchronize()
    got = batches[-1].tokens()
    assert np.array_equal(got, ref), (got, ref)
    for b in batches + [fb]:
        b.close()
    for e in engs + [full]:
        e.close()


def test_stage_engines_32_rows_128k_head(oracle_mod):
    """The width the pipeline bench runs: M = 32 sequences per micro-batch (the 17-64-row wide path
    fed by a stage's x_in through ssq_kernel), a 2-stage split of the Llama-3-8B-geometry test model
    whose last stage holds the 128256-token lm_head.  Stage tokens == one-engine tokens, and the
    chains follow the oracle."""
    from conftest import check_chain_batched
    from llama_p2p_amd import synth
    from llama_p2p_amd.engine import Engine
    from llama_p2p_amd.pipeline import EngineAdapter

    name = "test-8b-v128k"
    sh = synth.SHAPES[name]
    rng = np.random.default_rng(7)
    M, steps = 32, 6
    prompts = [np.concatenate([[1], rng.integers(3, sh.n_vocab, int(rng.integers(4, 40)))]) for _ in range(M)]
    (slots, pos, ids), st = _rows(prompts)
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream())
    path = f"synthetic:{name}:seed=0"
    full = Engine(path, n_ctx=128, n_seq_max=M)
    fa = EngineAdapter(full)
    for i in range(0, len(slots), 64):
        fa.stage_rows_tensors(slots[i:i + 64], pos[i:i + 64], ids[i:i + 64], None, None)
    fb = full.batch(st[0], st[1], st[2], max_steps=steps)
    for _ in range(steps):
        fb.step()
    ref = fb.tokens()
    fb.close()
    full.close()

    engs = [Engine(path, n_ctx=128, n_seq_max=M, layer_begin=lb, layer_end=le) for lb, le in [(0, 1), (1, 2)]]
    ads = [EngineAdapter(e) for e in engs]
    buf = torch.empty((64, sh.n_embd), dtype=torch.float32, device=dev)
    for i in range(0, len(slots), 64):
        n = min(64, len(slots) - i)
        ads[0].stage_rows_tensors(slots[i:i + n], pos[i:i + n], ids[i:i + n], None, buf[:n])
        ads[1].stage_rows_tensors(slots[i:i + n], pos[i:i + n], None, buf[:n], None)
    b0 = ads[0].batch(st[0], st[1], st[2], 0)
    b1 = ads[1].batch(st[0], st[1], None, steps)
    tok = torch.tensor(st[2], dtype=torch.int32, device=dev)
    b0.bind_ids_tensor(tok)
    b1.bind_ids_tensor(torch.zeros(M, dtype=torch.int32, device=dev))
    x = torch.empty((M, sh.n_embd), dtype=torch.float32, device=dev)
    for _ in range(steps):
        b0.step_tensors(None, x)
        b1.step_tensors(x, None)
        tok.copy_(b1._ids_tensor)
    torch.cuda.synchronize()
    got = b1.tokens()
    assert np.array_equal(got, ref), (got, ref)
    om = oracle_mod.OracleModel(sh, seed=0)
    for i in (0, 13, 31):
        check_chain_batched(om.context(128), prompts[i], got[i].tolist(), f"stage chain seq {i}")
    for b in (b0, b1):
        b.close()
    for e in engs:
        e.close()
