"""Llama(..., stream=True): llama-cpp-python's chunk stream over the engine's request API
(llama.py Llama._stream).  CPU only: a scripted engine hands out the tokens of a request a few
at a time, as the scheduler does (up to 8 greedy steps per round).  The joined chunk texts equal
the text of the same call without stream, stop strings end the stream (and cancel the request)
with the same text, held-back stop prefixes are released when they do not complete, and a
consumer that closes the stream early cancels its request."""
import itertools

import pytest

from llama_p2p_amd import engine as E
from llama_p2p_amd.llama import Llama

pytestmark = pytest.mark.timeout(60)


class ScriptedEngine:
    """submit/poll/cancel/wait of Engine; each poll releases `step` more of the scripted tokens."""

    n_vocab, n_embd = 512, 256

    def __init__(self, tokens, step=3, eos=None):
        self.script, self.step, self.eos = list(tokens), step, eos
        self.reqs, self.ids = {}, itertools.count(1)
        self.cancelled = []

    def submit(self, ids, max_tokens, **kw):
        r = next(self.ids)
        toks = self.script[:max_tokens]
        finish = E.FINISH_LENGTH
        if self.eos is not None and len(self.script) < max_tokens:
            toks, finish = toks + [self.eos], E.FINISH_STOP
        self.reqs[r] = {"toks": toks, "have": 0, "finish": finish}
        return r

    def poll(self, r, n_have=0):
        q = self.reqs[r]
        q["have"] = min(len(q["toks"]), max(q["have"], n_have) + self.step)
        return q["toks"][:q["have"]], q["have"] == len(q["toks"])

    def cancel(self, r):
        q = self.reqs[r]
        self.cancelled.append(r)
        q["toks"], q["finish"] = q["toks"][:q["have"] + 2], E.FINISH_STOP  # lands a little later

    def wait(self, r):
        q = self.reqs.pop(r)
        return q["toks"], q["finish"]


def make(tokens, step=3, eos=None):
    eng = ScriptedEngine(tokens, step, eos)
    return Llama.from_engine("synthetic:test-tiny:seed=0", eng, n_ctx=512), eng


SCRIPT = list(range(40, 100))


@pytest.mark.parametrize("step", [1, 3, 8])
def test_stream_joins_to_the_plain_text(step):
    llm, _ = make(SCRIPT, step)
    plain = llm("hello", max_tokens=30)
    chunks = list(llm("hello", max_tokens=30, stream=True))
    assert all(c["object"] == "text_completion" for c in chunks)
    assert "".join(c["choices"][0]["text"] for c in chunks) == plain["choices"][0]["text"]
    assert [c["choices"][0]["finish_reason"] for c in chunks[:-1]] == [None] * (len(chunks) - 1)
    assert chunks[-1]["choices"][0]["finish_reason"] == plain["choices"][0]["finish_reason"] == "length"
    assert len(chunks) > 2


def test_stream_eos_finishes_with_stop():
    llm, eng = make(SCRIPT[:10], 4, eos=2)
    plain = llm("hello", max_tokens=30)
    chunks = list(llm("hello", max_tokens=30, stream=True))
    assert "".join(c["choices"][0]["text"] for c in chunks) == plain["choices"][0]["text"]
    assert chunks[-1]["choices"][0]["finish_reason"] == "stop" == plain["choices"][0]["finish_reason"]


def test_stream_stop_string_cuts_and_cancels():
    llm, eng = make(SCRIPT, 2)
    full = llm("hello", max_tokens=40)["choices"][0]["text"]
    stop = full[len(full) // 2: len(full) // 2 + 3]
    assert stop and stop in full
    plain = llm("hello", max_tokens=40, stop=[stop])
    chunks = list(llm("hello", max_tokens=40, stop=[stop], stream=True))
    text = "".join(c["choices"][0]["text"] for c in chunks)
    assert text == plain["choices"][0]["text"] == full[: full.find(stop)]
    assert chunks[-1]["choices"][0]["finish_reason"] == "stop"
    assert eng.cancelled and not eng.reqs


def test_stream_releases_a_stop_prefix_that_does_not_complete():
    llm, _ = make(SCRIPT, 1)
    full = llm("hello", max_tokens=30)["choices"][0]["text"]
    stop = full[5] + "\x00never"  # its first character occurs, the rest never does
    chunks = list(llm("hello", max_tokens=30, stop=[stop], stream=True))
    assert "".join(c["choices"][0]["text"] for c in chunks) == full


def test_closing_the_stream_cancels_the_request():
    llm, eng = make(SCRIPT, 2)
    it = llm("hello", max_tokens=50, stream=True)
    next(it)
    it.close()
    assert eng.cancelled and not eng.reqs


def test_echo_streams_the_prompt_first():
    llm, _ = make(SCRIPT, 5)
    plain = llm("hello", max_tokens=10, echo=True)
    chunks = list(llm("hello", max_tokens=10, echo=True, stream=True))
    assert "".join(c["choices"][0]["text"] for c in chunks) == plain["choices"][0]["text"]
