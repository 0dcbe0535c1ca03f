"""Host logic of the Llama drop-in (llama.py) on CPU: stop strings, cancellation and usage counts.

The engine is replaced by a scripted stand-in with the request API of engine.Engine (submit / poll /
cancel / wait) that generates a fixed token stream in scheduler rounds of 8 tokens, as the real
scheduler does for greedy requests (engine.cpp SCHED_KMAX).  What is checked is llama-cpp-python's
create_completion contract that the reference's call (p2p:125) sees: generation ends at the first stop
string, the text is cut there, finish_reason is "stop", and usage counts the tokens up to the one that
completed the stop string.
"""
import pytest

from llama_p2p_amd import engine as E
from llama_p2p_amd.gguf import synthetic_spm_vocab
from llama_p2p_amd.llama import Llama
from llama_p2p_amd.tokenizer import Tokenizer


class ScriptedEngine:
    ROUND = 8

    def __init__(self, stream, n_ctx=512):
        self.stream, self.n_ctx = list(stream), n_ctx
        self.n_vocab = 512
        self.reqs = {}
        self.cancelled = []
        self.next = 1

    def submit(self, ids, max_tokens, **kw):
        r = self.next
        self.next += 1
        self.reqs[r] = {"max": max_tokens, "out": [], "cancel": False, "done": False}
        self.last_kw = kw
        return r

    def _round(self, r):
        q = self.reqs[r]
        if q["done"]:
            return
        if q["cancel"]:  # the cancel lands at the start of the next round
            q["done"], q["fin"] = True, E.FINISH_STOP
            return
        for _ in range(self.ROUND):
            if len(q["out"]) >= min(q["max"], len(self.stream)):
                q["done"], q["fin"] = True, E.FINISH_LENGTH
                return
            q["out"].append(self.stream[len(q["out"])])

    def poll(self, r, n_have=0):
        q = self.reqs[r]
        while len(q["out"]) <= n_have and not q["done"]:
            self._round(r)
        return list(q["out"]), q["done"]

    def cancel(self, r):
        self.cancelled.append(r)
        self.reqs[r]["cancel"] = True

    def wait(self, r, cap=None):
        q = self.reqs[r]
        self._round(r)  # the round already in flight when the cancel arrived
        while not q["done"]:
            self._round(r)
        del self.reqs[r]
        return list(q["out"]), q["fin"]


def make_llama(stream):
    llm = Llama.__new__(Llama)
    toks, scores, types = synthetic_spm_vocab(512)
    llm.tokenizer_ = Tokenizer(toks, scores, types, "llama", bos_id=1, eos_id=2)
    llm._engine = ScriptedEngine(stream)
    llm._n_ctx, llm._seed, llm.model_path, llm.verbose = 512, 0xFFFFFFFF, "scripted", False
    return llm


def pieces(llm, text):
    return llm.tokenize(text.encode(), add_bos=False)


def test_stop_string_ends_generation_and_counts_tokens():
    llm0 = make_llama([])
    words = pieces(llm0, " alpha beta gamma delta epsilon zeta eta theta iota kappa lambda")
    llm = make_llama(words)
    out = llm("p", max_tokens=64, stop=["delta"], temperature=0.0)
    ch = out["choices"][0]
    assert ch["finish_reason"] == "stop"
    full = llm.detokenize(words, prev_tokens=llm.tokenize(b"p")).decode()
    assert ch["text"] == full[:full.index("delta")] and ch["text"].endswith("alpha beta gamma ")
    # tokens up to and including the one that completes "delta" -- not the whole scheduler round
    k = next(k for k in range(1, len(words) + 1) if "delta" in llm.detokenize(words[:k]).decode())
    assert out["usage"]["completion_tokens"] == k < len(words)
    assert llm._engine.cancelled, "the request was not cancelled at the stop string"
    assert "delta" in full


def test_stop_string_absent_runs_to_length():
    llm0 = make_llama([])
    words = pieces(llm0, " one two three")
    llm = make_llama(words)
    out = llm("p", max_tokens=len(words), stop="zzz", temperature=0.0)
    assert out["choices"][0]["finish_reason"] == "length"
    assert out["usage"]["completion_tokens"] == len(words)
    assert not llm._engine.cancelled


def test_sampling_keywords_reach_the_engine():
    llm = make_llama([5, 6, 7])
    out = llm("p", max_tokens=3, temperature=0.7, top_k=12, repeat_penalty=1.1, frequency_penalty=0.25,
              presence_penalty=0.5, seed=9)
    assert llm._engine.last_kw == {"temperature": 0.7, "top_k": 12, "top_p": 0.95, "min_p": 0.05,
                                   "repeat_penalty": 1.1, "frequency_penalty": 0.25, "presence_penalty": 0.5,
                                   "seed": 9}
    assert out["usage"]["completion_tokens"] == 3 and not llm._engine.reqs


def test_prompt_too_long_raises_value_error():
    llm = make_llama([5])
    llm._n_ctx = 8
    with pytest.raises(ValueError):
        llm(list(range(3, 20)), max_tokens=4)
