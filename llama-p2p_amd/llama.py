"""``Llama`` -- drop-in for ``llama_cpp.Llama`` as the reference node uses it.

    self.model = Llama(model_path=model_path)                          p2p:19
    result = self.model(prompt, max_tokens=100)["choices"][0]["text"]  p2p:125

(p2p = /root/reference/llama_p2p_network.py.)  Constructor keywords,
``__call__``/``create_completion`` keywords and defaults, the returned
completion dict, ``tokenize``/``detokenize`` and the ``ValueError`` raised for
a prompt that does not fit ``n_ctx`` follow llama-cpp-python (~0.3.1, the
version current at the reference's date).  The
compute runs in the MI355X engine (engine.py -> libmxllama.so); calls release
the GIL, and concurrent calls from several threads are micro-batched by the
engine's scheduler instead of being serialised.
"""
from __future__ import annotations

import os
import threading
import time
import uuid
from typing import Any, Dict, Iterator, List, Optional, Sequence, Union

from . import engine as _engine
from . import synth as _synth
from .tokenizer import Tokenizer

LLAMA_DEFAULT_SEED = 0xFFFFFFFF


class Llama:
    def __init__(self, model_path: str, *, n_gpu_layers: int = -1, seed: int = LLAMA_DEFAULT_SEED, n_ctx: int = 512,
                 n_batch: int = 512, n_threads: Optional[int] = None, n_threads_batch: Optional[int] = None,
                 verbose: bool = True, n_seq_max: int = 64, device: int = -1, synthetic_seed: int = 0,
                 **kwargs: Any):
        # n_gpu_layers / n_threads / n_batch are accepted for signature compatibility: the whole model
        # always runs on the GPU, and prompts are processed in 64-row chunks.
        self.model_path = model_path
        self.verbose = verbose
        self._seed = seed
        if n_ctx == 0:
            n_ctx = 4096
        syn = _synth.parse_synthetic_path(model_path)
        if syn is None and not os.path.exists(model_path):
            raise ValueError(f"Model path does not exist: {model_path}")
        self._engine = _engine.Engine(model_path, n_ctx=n_ctx, n_seq_max=n_seq_max, device=device,
                                      seed=synthetic_seed)
        self._n_ctx = n_ctx
        self._init_tokenizer(model_path, self._engine.info.n_vocab)

    @classmethod
    def from_engine(cls, model_path: str, engine, n_ctx: int = 512, seed: int = LLAMA_DEFAULT_SEED,
                    verbose: bool = True) -> "Llama":
        """A Llama over another engine object with Engine's request methods (submit / poll / cancel /
        wait, n_vocab, n_embd) -- the pipeline server's rank-0 front (pipeserve.py)."""
        self = cls.__new__(cls)
        self.model_path, self.verbose, self._seed = model_path, verbose, seed
        self._engine, self._n_ctx = engine, n_ctx
        self._init_tokenizer(model_path, engine.n_vocab)
        return self

    def _init_tokenizer(self, model_path: str, n_vocab: int):
        if _synth.parse_synthetic_path(model_path) is None:
            from .gguf import GGUFReader

            md = GGUFReader(model_path).metadata
            self.metadata = {k: v for k, v in md.items() if not isinstance(v, list)}
            self.tokenizer_ = Tokenizer.from_gguf_metadata(md)
        else:
            from .gguf import synthetic_spm_vocab

            toks, scores, types = synthetic_spm_vocab(n_vocab)
            self.tokenizer_ = Tokenizer(toks, scores, types, "llama", bos_id=1, eos_id=2)
            self.metadata = {"general.architecture": "llama", "general.name": model_path}
        self._lock = threading.Lock()

    # ---------------------------------------------------------------- info
    def n_ctx(self) -> int:
        return self._n_ctx

    def n_vocab(self) -> int:
        return self._engine.n_vocab

    def n_embd(self) -> int:
        return self._engine.n_embd

    def token_bos(self) -> int:
        return self.tokenizer_.bos_id

    def token_eos(self) -> int:
        return self.tokenizer_.eos_id

    # ----------------------------------------------------------- tokenizer
    def tokenize(self, text: bytes, add_bos: bool = True, special: bool = False) -> List[int]:
        return self.tokenizer_.tokenize(text, add_bos=add_bos, special=special)

    def detokenize(self, tokens: Sequence[int], prev_tokens: Optional[Sequence[int]] = None,
                   special: bool = False) -> bytes:
        return self.tokenizer_.detokenize(tokens, prev_tokens=prev_tokens, special=special)

    # ---------------------------------------------------------- completion
    def create_completion(self, prompt: Union[str, List[int]], suffix: Optional[str] = None, max_tokens: Optional[int] = 16,
                          temperature: float = 0.8, top_p: float = 0.95, min_p: float = 0.05, typical_p: float = 1.0,
                          logprobs: Optional[int] = None, echo: bool = False,
                          stop: Optional[Union[str, List[str]]] = [], frequency_penalty: float = 0.0,
                          presence_penalty: float = 0.0, repeat_penalty: float = 1.0, top_k: int = 40,
                          stream: bool = False, seed: Optional[int] = None,
                          **kwargs: Any) -> Union[Dict[str, Any], Iterator[Dict[str, Any]]]:
        if logprobs is not None:
            raise NotImplementedError("logprobs are not supported")
        if typical_p != 1.0:
            raise NotImplementedError("typical_p != 1.0 is not supported (llama-cpp-python's default 1.0 is)")
        created = int(time.time())
        cid = f"cmpl-{uuid.uuid4()}"
        if isinstance(prompt, str):
            prompt_tokens = self.tokenize(prompt.encode("utf-8"), add_bos=True, special=True)
        else:
            prompt_tokens = list(prompt)
        if len(prompt_tokens) >= self._n_ctx:
            raise ValueError(f"Requested tokens ({len(prompt_tokens)}) exceed context window of {self._n_ctx}")
        if max_tokens is None or max_tokens <= 0:
            max_tokens = self._n_ctx - len(prompt_tokens)
        max_tokens = min(max_tokens, self._n_ctx - len(prompt_tokens))
        sd = seed if seed is not None else self._seed
        req = self._engine.submit(prompt_tokens, max_tokens, temperature=temperature, top_k=top_k, top_p=top_p,
                                  min_p=min_p, repeat_penalty=repeat_penalty, frequency_penalty=frequency_penalty,
                                  presence_penalty=presence_penalty, seed=None if sd == LLAMA_DEFAULT_SEED else sd)
        stops = [s for s in ([stop] if isinstance(stop, str) else list(stop or [])) if s]
        if stream:
            return self._stream(req, prompt_tokens, stops, cid, created, echo)
        if stops:  # stop strings end generation as soon as one appears (llama-cpp-python's check per token)
            n = 0
            while True:
                toks, done = self._engine.poll(req, n)
                n = len(toks)
                text = self.detokenize(toks, prev_tokens=prompt_tokens).decode("utf-8", errors="ignore")
                if done or any(s in text for s in stops):
                    break
            if not done:
                self._engine.cancel(req)
        toks, finish = self._engine.wait(req)
        finish_reason = "stop" if finish == _engine.FINISH_STOP else "length"
        if toks and self.tokenizer_.is_eog(toks[-1]) and finish == _engine.FINISH_STOP:
            toks = toks[:-1]
        text = self.detokenize(toks, prev_tokens=prompt_tokens).decode("utf-8", errors="ignore")
        cut = min((text.find(s) for s in stops if s in text), default=-1)
        if cut >= 0:
            text = text[:cut]
            finish_reason = "stop"
            # the cancel lands after the scheduler's current round (up to 8 greedy steps), so tokens past
            # the stop may have been generated: count only those up to the one completing the stop
            # string, as llama-cpp-python does (its check runs after every token)
            for k in range(1, len(toks) + 1):
                t = self.detokenize(toks[:k], prev_tokens=prompt_tokens).decode("utf-8", errors="ignore")
                if any(s in t for s in stops):
                    toks = toks[:k]
                    break
        if echo:
            text = self.detokenize(prompt_tokens).decode("utf-8", errors="ignore") + text
        if suffix is not None:
            text = text + suffix
        return {
            "id": cid, "object": "text_completion", "created": created, "model": self.model_path,
            "choices": [{"text": text, "index": 0, "logprobs": None, "finish_reason": finish_reason}],
            "usage": {"prompt_tokens": len(prompt_tokens), "completion_tokens": len(toks),
                      "total_tokens": len(prompt_tokens) + len(toks)},
        }

    def _chunk(self, cid: str, created: int, text: str, finish_reason: Optional[str]) -> Dict[str, Any]:
        return {"id": cid, "object": "text_completion", "created": created, "model": self.model_path,
                "choices": [{"text": text, "index": 0, "logprobs": None, "finish_reason": finish_reason}]}

    def _stream(self, req: int, prompt_tokens: List[int], stops: List[str], cid: str, created: int,
                echo: bool) -> Iterator[Dict[str, Any]]:
        """stream=True (llama-cpp-python's chunk stream): text as the engine's scheduler produces tokens
        (up to 8 per round for greedy requests), each chunk the text decoded since the last one; text
        that could still become a stop string is held back, a stop string ends the stream there, and
        the last chunk carries the finish reason.  The chunks' texts joined equal the text of the
        same call without stream (tests/test_llama_stream.py)."""
        if echo:
            yield self._chunk(cid, created, self.detokenize(prompt_tokens).decode("utf-8", errors="ignore"), None)
        sent, n, cut, ended = 0, 0, -1, False
        try:
            while True:
                toks, done = self._engine.poll(req, n)
                n = len(toks)
                body = toks[:-1] if toks and self.tokenizer_.is_eog(toks[-1]) else toks
                text = self.detokenize(body, prev_tokens=prompt_tokens).decode("utf-8", errors="ignore")
                cut = min((text.find(s) for s in stops if s in text), default=-1)
                if cut >= 0:
                    if cut > sent:
                        yield self._chunk(cid, created, text[sent:cut], None)
                    sent = cut
                    ended = done
                    break
                # hold back the longest tail that is a proper prefix of a stop string
                hold = max((k for s in stops for k in range(1, len(s)) if text.endswith(s[:k])), default=0)
                if done:
                    hold = 0
                if len(text) - hold > sent:
                    yield self._chunk(cid, created, text[sent:len(text) - hold], None)
                    sent = len(text) - hold
                if done:
                    ended = True
                    break
        finally:  # a stop string, or a consumer that closed the stream: end the request, then release it
            if not ended:
                self._engine.cancel(req)
            toks, finish = self._engine.wait(req)
        yield self._chunk(cid, created, "", "stop" if cut >= 0 or finish == _engine.FINISH_STOP else "length")

    def __call__(self, prompt: Union[str, List[int]], *args, **kwargs) -> Dict[str, Any]:
        return self.create_completion(prompt, *args, **kwargs)

    def close(self):
        if getattr(self, "_engine", None) is not None:
            self._engine.close()
            self._engine = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
