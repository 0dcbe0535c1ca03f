"""A request's result does not depend on what it is batched with (bf16 models; DESIGN.md §1 "batch
invariance").

The reference computes every prompt alone under its node lock (/root/reference/llama_p2p_network.py:
121-125) and caches the text per prompt (``cached_inference``, :120-133), so one prompt must give one
answer whatever else the engine is serving.  Bitwise, on the full 32-layer Llama-3-8B:

  * decode: the logits of a row are the same bits at every row count -- 1 (persistent GEMVs, RMS_NORM
    on load), 3, 4 (on load), 5..16 (norm launch + 16-wave GEMVs), 17..64 (mm_wide, split-K slabs,
    FIN attention): the canonical K slices + grouped fold (kernels.hip kfold / mm_wide slice_fold) and
    the canonical RMS_NORM sums (device_common.h ssq16 / ssq_lane / ssq_wave);
  * prefill: a prompt's hidden states after the last layer are the same bits alone and inside a chunk
    with 31 other prompts (mx_stage_rows_pick: the GEMM path at every row count, one K range per
    output, prompts padded to 16-row blocks for the prefill attention);
  * end to end through the request API (mx_submit vs mx_submit_batch): the same greedy tokens alone and
    among 31 other requests whose max_tokens make the decode batch shrink through 32 -> 16 -> 4 -> 1 rows.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_CTX = 512


@pytest.fixture(scope="module")
def eng8b():
    from llama_p2p_amd.engine import Engine

    e = Engine("synthetic:llama3-8b:seed=0", n_ctx=N_CTX, n_seq_max=64)
    yield e
    e.close()


def _prompts(vocab, n, seed, lo, hi):
    import bench

    return [list(map(int, p)) for p in bench.make_prompts(vocab, n, seed=seed, lo=lo, hi=hi)]


@pytest.mark.parametrize("model", ["llama3-8b", "tinyllama-1.1b", "test-tiny"])
def test_decode_logits_bitwise_at_every_row_count(model, request):
    """Llama-3-8B; TinyLlama (ffn_down K = 5632: canonical slices of 11 K-tiles end inside mm_wide's
    4-tile activation chunks); test-tiny (K = 256 < 512: empty slices)."""
    from llama_p2p_amd.engine import Engine

    if model == "llama3-8b":
        e, own = request.getfixturevalue("eng8b"), False
    else:
        e, own = Engine(f"synthetic:{model}:seed=0", n_ctx=128, n_seq_max=64), True
    try:
        _decode_rows_bitwise(e)
    finally:
        if own:
            e.close()


def _decode_rows_bitwise(e):
    ps = _prompts(e.n_vocab, 40, 21, 5, 60)
    for i, p in enumerate(ps):  # KV of each prompt but its last token
        e.forward_rows([i] * (len(p) - 1), list(range(len(p) - 1)), p[:-1], want_logits=False)
    slots = list(range(len(ps)))
    pos = [len(p) - 1 for p in ps]
    ids = [p[-1] for p in ps]
    ref = {}
    for i in (0, 3, 17, 39):
        ref[i] = e.forward_rows([slots[i]], [pos[i]], [ids[i]])[0]
        assert np.isfinite(ref[i]).all() and ref[i].std() > 0
    checked = 0
    for M in (2, 3, 4, 5, 8, 16, 17, 24, 32, 33, 40):
        lg = e.forward_rows(slots[:M], pos[:M], ids[:M])
        for i, r in ref.items():
            if i < M:
                d = np.flatnonzero(lg[i].view(np.uint32) != r.view(np.uint32))
                assert d.size == 0, f"row {i} at M={M}: {d.size} logits differ, max |d| {np.abs(lg[i] - r).max()}"
                checked += 1
    # a row alone after the 40-row step rewrote every KV position: still the same bits
    again = e.forward_rows([slots[17]], [pos[17]], [ids[17]])[0]
    assert np.array_equal(again.view(np.uint32), ref[17].view(np.uint32))
    print({"rows_checked": checked})


def _rows(prompts, slot0, n_ctx=N_CTX):
    """The scheduler's prefill layout (engine.cpp prefill_batch, pipeserve._prefill): each prompt from a
    16-row block boundary, padded to whole blocks; returns rows and each prompt's row range."""
    slots, pos, ids, spans = [], [], [], []
    for k, p in enumerate(prompts):
        n = len(p)
        r0 = len(slots)
        slots += [slot0 + k] * n
        pos += list(range(n))
        ids += p
        spans.append((r0, r0 + n))
        pad = (16 - n % 16) % 16
        slots += [slot0 + k] * pad
        pos += list(range(n, n + pad)) if n + pad <= n_ctx else [n - 1] * pad
        ids += [p[-1]] * pad
    return slots, pos, ids, spans


def test_prefill_hidden_states_bitwise_alone_and_in_a_chunk(eng8b):
    import torch

    e = eng8b
    others = _prompts(e.n_vocab, 31, 5, 16, 256)
    targets = [p[:L] for p, L in zip(_prompts(e.n_vocab, 5, 9, 300, 300), (7, 16, 40, 100, 300))]
    targets.append(_prompts(e.n_vocab, 1, 13, N_CTX - 3, N_CTX - 3)[0])  # padded with copies near n_ctx
    dev = torch.device("cuda", 0)
    for ti, t in enumerate(targets):
        s, p, i, sp = _rows([t], 0)
        xa = torch.empty((len(s), e.n_embd), dtype=torch.float32, device=dev)
        e.stage_rows_pick(s, p, i, x_out=xa.data_ptr())
        torch.cuda.synchronize()
        alone = xa[sp[0][0]:sp[0][1]].cpu().numpy()
        batch = others[:ti * 5] + [t] + others[ti * 5:]
        s, p, i, sp = _rows(batch, 1)
        xb = torch.empty((len(s), e.n_embd), dtype=torch.float32, device=dev)
        e.stage_rows_pick(s, p, i, x_out=xb.data_ptr())
        torch.cuda.synchronize()
        r0, r1 = sp[ti * 5]
        mixed = xb[r0:r1].cpu().numpy()
        d = np.flatnonzero(alone.view(np.uint32) != mixed.view(np.uint32))
        assert d.size == 0, f"prompt of {len(t)} tokens: {d.size} hidden values differ ({len(s)}-row batch)"
        assert np.isfinite(alone).all() and alone.std() > 0


def test_request_tokens_alone_and_among_31_others(eng8b):
    e = eng8b
    others = _prompts(e.n_vocab, 31, 7, 16, 256)
    targets = _prompts(e.n_vocab, 3, 3, 9, 200)
    rng = np.random.default_rng(4)
    T = 40
    for k, t in enumerate(targets):
        alone, fin = e.generate(t, T, ignore_eos=True)
        assert len(alone) == T
        # the others end at different steps: the decode batch shrinks through the 16- and 4-row regimes
        mts = [int(m) for m in rng.integers(2, 48, len(others))]
        pos = k * 10
        prompts = others[:pos] + [t] + others[pos:]
        reqs = e.submit_many(prompts, mts[:pos] + [T] + mts[pos:], ignore_eos=True)
        outs = [e.wait(r)[0] for r in reqs]
        mixed = outs[pos]
        first = next((i for i, (a, b) in enumerate(zip(alone, mixed)) if a != b), None)
        assert mixed == alone, f"target {k} ({len(t)} tokens): first difference at generated token {first}"
