"""Stage engines sharing ONE GPU on TWO streams give the one-engine tokens bitwise (round-5 regression).

Round 4 found that 17-64-row prompt chunks of one sequence were not run-to-run reproducible when a
second queue (another process, or another stream of the same process) used the GPU.  Round 5 located it
(profiles/round5_rope_packed_hazard.txt): the packed-FP32 RoPE of qkv_finish_kernel computed one element
of a quad wrong in lanes 32-63 while other waves shared the CU; the RoPE is now four scalar fmas
(device_common.h rope4).  This test is the in-process form of the failing rehearsal: the full 32-layer
Llama-3-8B split into two stage engines, each driven by its own thread on its own torch stream
(pipeline.Stage with pipeserve.LocalComm device hand-offs, f32), prompts prefilled in 64-row chunks, then
5 pipelined greedy decode steps of 2 micro-batches x 32 sequences -- the generated tokens must equal the
one-engine run bit for bit, twice.  The schedule is what bench.py runs across GPUs
(/root/reference/llama_p2p_network.py:125 is the call it serves).
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(world, model="synthetic:llama3-8b:seed=0", S=2, M=32, steps=5, chunk=64):
    import torch

    import bench
    from llama_p2p_amd import pipeserve, synth
    from llama_p2p_amd.engine import Engine
    from llama_p2p_amd.pipeline import EngineAdapter, Stage, partition_layers

    sh = synth.SHAPES["llama3-8b"]
    prompts = bench.make_prompts(sh.n_vocab, S * M, lo=16, hi=256)
    mb_rows, mb_state = [], []
    for mb in range(S):
        slots, pos, ids, st = [], [], [], ([], [], [])
        for i in range(M):
            p, sl = prompts[mb * M + i], mb * M + i
            slots += [sl] * (len(p) - 1)
            pos += list(range(len(p) - 1))
            ids += [int(t) for t in p[:-1]]
            st[0].append(sl)
            st[1].append(len(p) - 1)
            st[2].append(int(p[-1]))
        mb_rows.append((slots, pos, ids))
        mb_state.append(st)
    layer = 2 * (2 * sh.n_embd ** 2 + 2 * sh.n_embd * sh.n_embd_kv + 3 * sh.n_embd * sh.n_ff)
    parts = partition_layers(sh.n_layer, layer, 2 * sh.n_vocab * sh.n_embd, world)
    dev = torch.device("cuda", 0)
    torch.cuda.init()  # torch's lazy CUDA init in the main thread, not raced by the two stage threads
    hub = pipeserve.LocalHub()
    out, errs = [None] * world, []
    bar, lock = threading.Barrier(world), threading.Lock()

    def rank(r):
        try:
            torch.cuda.set_device(dev)
            torch.cuda.set_stream(torch.cuda.Stream(device=dev))  # one stream per stage
            lb, le = parts[r]
            eng = Engine(model, n_ctx=512, n_seq_max=S * M, layer_begin=lb, layer_end=le,
                         device=0, handoff_bf16=False)
            comm = pipeserve.LocalComm(hub, r, world) if world > 1 else None
            st = Stage(EngineAdapter(eng), comm, r, world, sh.n_embd, dev, S, dtype=torch.float32)
            st.prefill(mb_rows, chunk=chunk)
            torch.cuda.synchronize()
            bar.wait()
            with lock:  # batches capture graphs at creation: one thread at a time
                st.setup_decode(mb_state, max_steps=steps)
                torch.cuda.synchronize()
            bar.wait()
            st.decode_steps(steps, 0)
            st.finish()
            torch.cuda.synchronize()
            out[r] = st.tokens()
            for b in st.batches:
                b.close()
            eng.close()
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))
            bar.abort()

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    return np.stack(out[-1])


def test_two_stage_engines_on_two_streams_bitwise_with_64_row_chunks():
    ref = _run(1)
    a = _run(2)
    b = _run(2)
    print({"tokens": ref.shape, "split_equal": bool(np.array_equal(ref, a)), "repeat_equal": bool(np.array_equal(a, b))})
    assert np.array_equal(ref, a), np.argwhere(ref != a)[:10]
    assert np.array_equal(a, b), np.argwhere(a != b)[:10]


# Round 6: the other kernel families under sharing -- the <= 16-row decode GEMVs
# (M = 8: norm launch + 16-wave GEMVs; M = 2: RMS_NORM on load, persistent GEMVs) and the quantised
# models' 17..64-row prompt chunks and 32-row decode (Q8_0: mq8_* kernels; Q4_K_M: mkq_* kernels).  The
# product build has no packed-FP32 instruction left (tools/isa_scan.py); these legs
# check the families the round-5 fix did not touch.
@pytest.mark.parametrize("model,M", [("synthetic:llama3-8b:seed=0", 8), ("synthetic:llama3-8b:seed=0", 2),
                                     ("synthetic:llama3-8b:seed=0:q8_0", 32),
                                     ("synthetic:llama3-8b:seed=0:q4_0", 32),
                                     ("synthetic:llama3-8b:seed=0:q4_k_m", 32)])
def test_two_streams_bitwise_other_kernel_families(model, M):
    ref = _run(1, model=model, M=M)
    a = _run(2, model=model, M=M)
    print({"model": model, "M": M, "tokens": ref.shape, "split_equal": bool(np.array_equal(ref, a))})
    assert np.array_equal(ref, a), np.argwhere(ref != a)[:10]
