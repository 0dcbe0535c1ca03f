"""ctypes binding of the engine's C ABI (include/mx_engine.h).

The shared library is built in-tree (``llama-p2p_amd/libmxllama.so``, see
build.py).  There is deliberately no fallback: if the library is missing or no
GPU is visible, every entry point raises -- the product never computes on the
CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MX_LIB") or os.path.join(HERE, "libmxllama.so")  # MX_LIB: A/B builds only

MX_OK = 0
MX_ERR_ARG, MX_ERR_HIP, MX_ERR_MODEL, MX_ERR_CTX, MX_ERR_NOTFOUND, MX_ERR_STATE = -1, -2, -3, -4, -5, -6
MX_DEBUG_STOPPED = 1  # a forward cut short by debug_stop (include/mx_engine.h): raised, never silent
FINISH_LENGTH, FINISH_STOP, FINISH_ERROR = 0, 1, 2

# every symbol include/mx_engine.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "mx_opts_default", "mx_sampling_default", "mx_last_error", "mx_engine_create", "mx_engine_destroy", "mx_gguf_check",
    "mx_engine_info", "mx_forward_logits", "mx_forward_rows", "mx_forward_topk", "mx_submit", "mx_wait", "mx_submit_batch", "mx_poll", "mx_cancel", "mx_batch_create",
    "mx_batch_step", "mx_batch_ids_device", "mx_batch_bind_ids", "mx_batch_tokens", "mx_batch_destroy", "mx_stage_rows",
    "mx_profile_kernel", "mx_sync", "mx_device_count", "mx_engine_stats", "mx_batch_reset", "mx_stage_rows_pick",
    "mx_probe_copy", "mx_probe_read", "mx_debug",
]


class MxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mx error {code}: {msg}")
        self.code = code


class MxOpts(ctypes.Structure):
    _fields_ = [("n_ctx", ctypes.c_int32), ("n_seq_max", ctypes.c_int32), ("layer_begin", ctypes.c_int32),
                ("layer_end", ctypes.c_int32), ("device", ctypes.c_int32), ("use_graphs", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("handoff_bf16", ctypes.c_int32)]


class MxModelInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("n_embd", "n_layer", "n_head", "n_head_kv", "head_dim", "n_ff",
                                              "n_vocab", "n_ctx_train")] + \
               [("eps", ctypes.c_float), ("rope_base", ctypes.c_float)] + \
               [(n, ctypes.c_int32) for n in ("bos_id", "eos_id", "n_ctx", "n_seq_max", "layer_begin",
                                              "layer_end", "has_embed", "has_head")] + \
               [("weight_bytes", ctypes.c_uint64), ("weight_type", ctypes.c_int32)]


class MxSampling(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("top_k", ctypes.c_int32), ("top_p", ctypes.c_float),
                ("min_p", ctypes.c_float), ("repeat_penalty", ctypes.c_float), ("repeat_last_n", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("ignore_eos", ctypes.c_int32),
                ("frequency_penalty", ctypes.c_float), ("presence_penalty", ctypes.c_float)]


class MxRowSampler(ctypes.Structure):
    _fields_ = [("s", MxSampling), ("seed", ctypes.c_uint64), ("n_drawn", ctypes.c_int32), ("n_win", ctypes.c_int32),
                ("win", ctypes.c_int32 * 64)]


def sampling(temperature: float = 0.0, top_k: int = 40, top_p: float = 0.95, min_p: float = 0.05,
             repeat_penalty: float = 1.0, repeat_last_n: int = 64, seed: Optional[int] = None,
             ignore_eos: bool = False, frequency_penalty: float = 0.0, presence_penalty: float = 0.0) -> MxSampling:
    """An mx_sampling with llama-cpp-python's defaults for the unspecified fields."""
    s = MxSampling()
    lib().mx_sampling_default(ctypes.byref(s))
    s.temperature, s.top_k, s.top_p, s.min_p = temperature, top_k, top_p, min_p
    s.repeat_penalty, s.repeat_last_n, s.ignore_eos = repeat_penalty, repeat_last_n, int(ignore_eos)
    s.frequency_penalty, s.presence_penalty = frequency_penalty, presence_penalty
    if seed is not None and seed >= 0:
        s.seed = seed
    return s


def row_samplers(rows) -> "ctypes.Array":
    """rows: [(MxSampling, seed, n_drawn, window tokens)] -> mx_row_sampler[len(rows)]."""
    arr = (MxRowSampler * len(rows))()
    for i, (smp, seed, n_drawn, win) in enumerate(rows):
        win = list(win)[-64:]
        arr[i].s = smp
        arr[i].seed = seed
        arr[i].n_drawn = n_drawn
        arr[i].n_win = len(win)
        for j, t in enumerate(win):
            arr[i].win[j] = int(t)
    return arr


_lib = None
_lib_lock = threading.Lock()


def _torch_hip_first():
    """Initialise PyTorch's HIP runtime before loading the engine, so the process has ONE runtime.
    libmxllama.so NEEDs libamdhip64.so.7; PyTorch's libc10_hip.so NEEDs libamdhip64.so and loads its
    bundled copy, whose SONAME is also libamdhip64.so.7 -- loaded after PyTorch, the engine binds to that
    copy (and PyTorch stream handles passed to mx_batch_step are objects of the same runtime).  Loaded
    first, the engine pulled in /opt/rocm's copy and PyTorch's second copy then saw no GPU ("No HIP GPUs
    are available"; tools/hip_runtime_order_probe.py).  Nothing to do without a GPU."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def lib() -> ctypes.CDLL:
    """Load libmxllama.so (raises if it was not built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not found: build it with `python llama-p2p_amd/build.py` "
                              "(the engine has no CPU fallback)")
        _torch_hip_first()
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
        P = ctypes.POINTER
        L.mx_opts_default.argtypes = [P(MxOpts)]
        L.mx_sampling_default.argtypes = [P(MxSampling)]
        L.mx_last_error.restype = ctypes.c_char_p
        L.mx_engine_create.argtypes = [ctypes.c_char_p, P(MxOpts), P(vp)]
        L.mx_engine_destroy.argtypes = [vp]
        L.mx_gguf_check.argtypes = [ctypes.c_char_p]
        L.mx_engine_info.argtypes = [vp, P(MxModelInfo)]
        L.mx_forward_logits.argtypes = [vp, i32, vp, i32, i32, vp]
        L.mx_forward_rows.argtypes = [vp, i32, vp, vp, vp, vp]
        L.mx_forward_topk.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp]
        L.mx_submit.argtypes = [vp, vp, i32, P(MxSampling), i32, P(u64)]
        L.mx_wait.argtypes = [vp, u64, vp, i32, P(i32), P(i32)]
        L.mx_submit_batch.argtypes = [vp, i32, vp, vp, vp, vp, P(u64)]
        L.mx_poll.argtypes = [vp, u64, i32, vp, i32, P(i32), P(i32)]
        L.mx_cancel.argtypes = [vp, u64]
        L.mx_batch_create.argtypes = [vp, i32, vp, vp, vp, i32, P(vp)]
        L.mx_batch_step.argtypes = [vp, vp, vp, vp, vp]
        L.mx_batch_ids_device.argtypes = [vp]
        L.mx_batch_ids_device.restype = vp
        L.mx_batch_tokens.argtypes = [vp, vp, vp, i32, P(i32)]
        L.mx_batch_bind_ids.argtypes = [vp, vp, vp]
        L.mx_batch_destroy.argtypes = [vp, vp]
        L.mx_stage_rows.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp]
        L.mx_profile_kernel.argtypes = [vp, i32, i32, i32, P(ctypes.c_double), P(ctypes.c_double)]
        L.mx_sync.argtypes = [vp]
        L.mx_probe_copy.argtypes = [i32, ctypes.c_size_t, i32, P(ctypes.c_double), ctypes.c_char_p, i32]
        L.mx_probe_read.argtypes = [i32, ctypes.c_size_t, i32, P(ctypes.c_double), ctypes.c_char_p, i32]
        L.mx_device_count.argtypes = [P(i32)]
        L.mx_engine_stats.argtypes = [vp, P(MxStats)]
        L.mx_batch_reset.argtypes = [vp, vp, vp, vp, vp, vp]
        L.mx_stage_rows_pick.argtypes = [vp, i32, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp]
        L.mx_debug.argtypes = [vp, i32, ctypes.c_longlong, vp, ctypes.c_size_t]
        for name in EXPORTS:
            if name not in ("mx_opts_default", "mx_sampling_default", "mx_last_error", "mx_engine_destroy",
                            "mx_batch_destroy", "mx_batch_ids_device"):
                getattr(L, name).restype = i32
        _lib = L
        return L


class MxStats(ctypes.Structure):
    _fields_ = [("prompt_tokens", ctypes.c_uint64), ("reused_prompt_tokens", ctypes.c_uint64),
                ("generated_tokens", ctypes.c_uint64)]


def device_count() -> int:
    n = ctypes.c_int32()
    _check(lib().mx_device_count(ctypes.byref(n)))
    return n.value


def gguf_check(path: str):
    """Validate a GGUF container (no GPU needed); raises MxError(MX_ERR_MODEL) with the reason."""
    _check(lib().mx_gguf_check(path.encode()))


def probe_copy(device: int = 0, gib: int = 4, iters: int = 10, read_only: bool = False):
    """Best streaming rate in GB/s over the probe variants: (read + write) bytes / s of a copy or,
    with read_only, bytes read / s.  Returns (gbs, description of the winning variant)."""
    gbs = ctypes.c_double()
    desc = ctypes.create_string_buffer(160)
    fn = lib().mx_probe_read if read_only else lib().mx_probe_copy
    _check(fn(device, gib << 30, iters, ctypes.byref(gbs), desc, len(desc)))
    return gbs.value, desc.value.decode()


def _check(rc: int):
    if rc != MX_OK:
        raise MxError(rc, lib().mx_last_error().decode(errors="replace"))


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


class Engine:
    """One engine instance = one GPU, one model (or one pipeline stage of it)."""

    def __init__(self, model_path: str, n_ctx: int = 512, n_seq_max: int = 64, layer_begin: int = 0,
                 layer_end: int = -1, device: int = -1, use_graphs: bool = True, seed: int = 0,
                 handoff_bf16: bool = False):
        L = lib()
        opts = MxOpts()
        L.mx_opts_default(ctypes.byref(opts))
        opts.n_ctx, opts.n_seq_max = n_ctx, n_seq_max
        opts.layer_begin, opts.layer_end, opts.device = layer_begin, layer_end, device
        opts.use_graphs, opts.seed = int(use_graphs), seed
        opts.handoff_bf16 = int(handoff_bf16)
        self.handoff_bf16 = bool(handoff_bf16)
        h = ctypes.c_void_p()
        _check(L.mx_engine_create(model_path.encode(), ctypes.byref(opts), ctypes.byref(h)))
        self._h = h
        info = MxModelInfo()
        _check(L.mx_engine_info(self._h, ctypes.byref(info)))
        self.info = info
        self.n_vocab = info.n_vocab
        self.n_embd = info.n_embd
        self.n_ctx = info.n_ctx

    # -- parity hooks --------------------------------------------------------
    def forward_logits(self, ids: Sequence[int], pos0: int = 0, slot: int = 0) -> np.ndarray:
        ids = _i32(ids)
        out = np.empty((len(ids), self.n_vocab), dtype=np.float32)
        _check(lib().mx_forward_logits(self._h, slot, ids.ctypes.data, len(ids), pos0, out.ctypes.data))
        return out

    def forward_rows(self, slots, pos, ids, want_logits: bool = True) -> Optional[np.ndarray]:
        """Rows forward (chunked by 64); want_logits=False skips lm_head (prefill)."""
        slots, pos, ids = _i32(slots), _i32(pos), _i32(ids)
        out = np.empty((len(ids), self.n_vocab), dtype=np.float32) if want_logits else None
        _check(lib().mx_forward_rows(self._h, len(ids), slots.ctypes.data, pos.ctypes.data, ids.ctypes.data,
                                     out.ctypes.data if out is not None else None))
        return out

    def forward_topk(self, slots, pos, ids, k: int):
        """Rows forward (<= 64) + the device top-k kernel: (values [n][k], ids [n][k])."""
        slots, pos, ids = _i32(slots), _i32(pos), _i32(ids)
        vals = np.empty((len(ids), k), dtype=np.float32)
        idx = np.empty((len(ids), k), dtype=np.int32)
        _check(lib().mx_forward_topk(self._h, len(ids), slots.ctypes.data, pos.ctypes.data, ids.ctypes.data, k,
                                     vals.ctypes.data, idx.ctypes.data))
        return vals, idx

    def stage_rows(self, slots, pos, ids, x_in: int = 0, x_out: int = 0, want_logits: bool = False,
                   stream: int = 0) -> Optional[np.ndarray]:
        slots, pos = _i32(slots), _i32(pos)
        ids_p = _i32(ids).ctypes.data if ids is not None else None
        ids_keep = _i32(ids) if ids is not None else None
        if ids_keep is not None:
            ids_p = ids_keep.ctypes.data
        out = np.empty((len(slots), self.n_vocab), dtype=np.float32) if want_logits else None
        _check(lib().mx_stage_rows(self._h, len(slots), slots.ctypes.data, pos.ctypes.data, ids_p,
                                   x_in or None, x_out or None, out.ctypes.data if out is not None else None,
                                   stream or None))
        return out

    def stage_rows_pick(self, slots, pos, ids, x_in: int = 0, x_out: int = 0, rowmap=(), samplers=None,
                        stream: int = 0):
        """Pipelined prefill of any number of rows; on the last stage the rows in `rowmap` pick a token
        each (samplers: row_samplers() array or None for greedy).  Returns the tokens (list)."""
        slots, pos = _i32(slots), _i32(pos)
        ids_a = _i32(ids) if ids is not None else None
        rm = _i32(rowmap)
        tok = np.zeros(max(1, len(rm)), dtype=np.int32)
        _check(lib().mx_stage_rows_pick(self._h, len(slots), slots.ctypes.data, pos.ctypes.data,
                                        ids_a.ctypes.data if ids_a is not None else None, x_in or None, x_out or None,
                                        len(rm), rm.ctypes.data if len(rm) else None, samplers,
                                        tok.ctypes.data if len(rm) else None, stream or None))
        return tok[:len(rm)].tolist()

    # -- request API ---------------------------------------------------------
    def submit(self, ids: Sequence[int], max_tokens: int, temperature: float = 0.0, top_k: int = 40,
               top_p: float = 0.95, min_p: float = 0.05, repeat_penalty: float = 1.0, repeat_last_n: int = 64,
               seed: Optional[int] = None, ignore_eos: bool = False, frequency_penalty: float = 0.0,
               presence_penalty: float = 0.0) -> int:
        ids = _i32(ids)
        s = MxSampling()
        lib().mx_sampling_default(ctypes.byref(s))
        s.temperature, s.top_k, s.top_p, s.min_p = temperature, top_k, top_p, min_p
        s.repeat_penalty, s.repeat_last_n, s.ignore_eos = repeat_penalty, repeat_last_n, int(ignore_eos)
        s.frequency_penalty, s.presence_penalty = frequency_penalty, presence_penalty
        if seed is not None and seed >= 0:
            s.seed = seed
        req = ctypes.c_uint64()
        _check(lib().mx_submit(self._h, ids.ctypes.data, len(ids), ctypes.byref(s), max_tokens, ctypes.byref(req)))
        return req.value

    def submit_many(self, prompts, max_tokens: int, seeds=None, per_request=None, **kw):
        """Several requests queued atomically (one scheduler round admits them all); same sampling
        keywords as submit() (or ``per_request``: one keyword dict per prompt), one seed per prompt,
        max_tokens one value or one per prompt.  Returns the request ids."""
        n = len(prompts)
        arrs = [_i32(p) for p in prompts]
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
        lens = _i32([len(a) for a in arrs])
        mts = _i32(list(max_tokens) if hasattr(max_tokens, "__len__") else [max_tokens] * n)
        samp = (MxSampling * n)()
        base = kw
        for i in range(n):
            kw = dict(base, **per_request[i]) if per_request is not None else base
            if per_request is not None and "seed" in kw:
                seeds = list(seeds) if seeds is not None else [None] * n
                seeds[i] = kw["seed"]
            lib().mx_sampling_default(ctypes.byref(samp[i]))
            s = samp[i]
            s.temperature, s.top_k = kw.get("temperature", 0.0), kw.get("top_k", 40)
            s.top_p, s.min_p = kw.get("top_p", 0.95), kw.get("min_p", 0.05)
            s.repeat_penalty, s.repeat_last_n = kw.get("repeat_penalty", 1.0), kw.get("repeat_last_n", 64)
            s.ignore_eos = int(kw.get("ignore_eos", False))
            s.frequency_penalty, s.presence_penalty = kw.get("frequency_penalty", 0.0), kw.get("presence_penalty", 0.0)
            if seeds is not None and seeds[i] is not None and seeds[i] >= 0:
                s.seed = seeds[i]
        reqs = (ctypes.c_uint64 * n)()
        _check(lib().mx_submit_batch(self._h, n, ptrs, lens.ctypes.data, samp, mts.ctypes.data, reqs))
        return list(reqs)

    def wait(self, req: int, cap: Optional[int] = None):
        """Block until the request finishes; (generated ids, finish reason).  The buffer holds the
        whole context by default; a request that generated more is kept and re-read larger."""
        cap = cap or self.n_ctx
        n, fin = ctypes.c_int32(), ctypes.c_int32()
        while True:
            out = np.empty(cap, dtype=np.int32)
            rc = lib().mx_wait(self._h, req, out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(fin))
            if rc == MX_ERR_ARG and n.value > cap:
                cap = n.value
                continue
            _check(rc)
            return out[: min(n.value, cap)].tolist(), fin.value

    def poll(self, req: int, n_have: int = 0):
        """Block until the request holds more than n_have ids or finishes: (ids so far, done)."""
        cap = self.n_ctx
        out = np.empty(cap, dtype=np.int32)
        n, done = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().mx_poll(self._h, req, n_have, out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(done)))
        return out[: min(n.value, cap)].tolist(), bool(done.value)

    def cancel(self, req: int):
        """End the request after its current step (finish reason STOP); release it with wait()."""
        _check(lib().mx_cancel(self._h, req))

    def generate(self, ids, max_tokens: int, **kw):
        return self.wait(self.submit(ids, max_tokens, **kw))

    # -- device-resident batches (bench, pipeline) ---------------------------
    def batch(self, slots, pos, ids=None, max_steps: int = 0) -> "Batch":
        return Batch(self, slots, pos, ids, max_steps)

    def profile_kernel(self, kind: int, M: int, iters: int = 3):
        us, nb = ctypes.c_double(), ctypes.c_double()
        _check(lib().mx_profile_kernel(self._h, kind, M, iters, ctypes.byref(us), ctypes.byref(nb)))
        return us.value, nb.value

    def stats(self) -> dict:
        st = MxStats()
        _check(lib().mx_engine_stats(self._h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in MxStats._fields_}

    def sync(self):
        _check(lib().mx_sync(self._h))

    # -- diagnosis (include/mx_engine.h mx_debug) -------------------------------
    DEBUG_BUFFERS = {"x": 0, "q": 1, "xn": 2, "attn_out": 3, "act": 4, "slabs": 5, "kcache": 6, "vcache": 7,
                     "ssq": 8, "pos": 9, "slot": 10, "rope_cs": 11}

    def debug_stop(self, n: int):
        """End every 17..64-row forward after n launches (-1: never)."""
        _check(lib().mx_debug(self._h, 0, n, None, 0))

    def debug_sync(self, on: bool):
        """Synchronise the stream after every launch of a 17..64-row forward."""
        _check(lib().mx_debug(self._h, 1, int(on), None, 0))

    def debug_read(self, name: str, nbytes: int) -> np.ndarray:
        """The first nbytes of an internal buffer (after a device synchronize), as uint8."""
        out = np.zeros(nbytes, dtype=np.uint8)  # past the buffer's end: zeros
        _check(lib().mx_debug(self._h, 2, self.DEBUG_BUFFERS[name], out.ctypes.data, nbytes))
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().mx_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def torch_stream_handle() -> int:
    """hipStream_t of torch's current stream.  The engine's C ABI reads a NULL stream as
    "the engine's own stream", so the legacy default stream (handle 0) is refused: work
    enqueued there would not be ordered with the engine's kernels."""
    import torch

    h = torch.cuda.current_stream().cuda_stream
    if not h:
        raise RuntimeError("run engine tensor calls inside `with torch.cuda.stream(s):` (a non-default stream)")
    return h


class Batch:
    def __init__(self, eng: Engine, slots, pos, ids, max_steps: int):
        self.eng = eng
        slots, pos = _i32(slots), _i32(pos)
        self.M = len(slots)
        ids_a = _i32(ids) if ids is not None else None
        h = ctypes.c_void_p()
        _check(lib().mx_batch_create(eng._h, self.M, slots.ctypes.data, pos.ctypes.data,
                                     ids_a.ctypes.data if ids_a is not None else None, max_steps, ctypes.byref(h)))
        self._h = h
        self.max_steps = max_steps

    @property
    def ids_device_ptr(self) -> int:
        return lib().mx_batch_ids_device(self._h)

    def step(self, x_in: int = 0, x_out: int = 0, stream: int = 0):
        _check(lib().mx_batch_step(self.eng._h, self._h, x_in or None, x_out or None, stream or None))

    def reset(self, pos, ids=None, samplers=None, stream: int = 0):
        """Re-arm for the next run (graphs kept): positions, optional next ids, per-row samplers
        (row_samplers() array; None = greedy argmax); the token history restarts."""
        pos = _i32(pos)
        ids_a = _i32(ids) if ids is not None else None
        _check(lib().mx_batch_reset(self.eng._h, self._h, pos.ctypes.data,
                                    ids_a.ctypes.data if ids_a is not None else None, samplers, stream or None))

    def bind_ids(self, ids_device_ptr: int):
        _check(lib().mx_batch_bind_ids(self.eng._h, self._h, ids_device_ptr))

    # tensor-level interface used by the pipeline driver (torch device tensors)
    def step_tensors(self, x_in=None, x_out=None):
        stream = torch_stream_handle()
        self.step(x_in.data_ptr() if x_in is not None else 0, x_out.data_ptr() if x_out is not None else 0,
                  stream)

    def bind_ids_tensor(self, t):
        self._ids_tensor = t  # keep alive
        self.bind_ids(t.data_ptr())

    def tokens(self) -> np.ndarray:
        out = np.zeros((self.M, max(1, self.max_steps)), dtype=np.int32)
        n = ctypes.c_int32()
        _check(lib().mx_batch_tokens(self.eng._h, self._h, out.ctypes.data, out.shape[1], ctypes.byref(n)))
        return out[:, : min(n.value, self.max_steps)]

    def close(self):
        if getattr(self, "_h", None) and self.eng._h:
            lib().mx_batch_destroy(self.eng._h, self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
