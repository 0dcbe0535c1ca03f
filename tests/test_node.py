"""The node's drop-in boundary (★B) reproduces the reference's behaviour.

Fixtures: tests/golden/node_fixtures.json, captured from
/root/reference/llama_p2p_network.py itself by tests/golden/make_node_fixtures.py.
CPU-only: the model is an injected stand-in (the GPU engine is tested elsewhere).
"""
import hashlib
import json
import os
import threading
import time

import pytest

from llama_p2p_amd.node import LlamaP2PNode, Timeout

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "node_fixtures.json")))


class FakeModel:
    def __init__(self, delay=0.0):
        self.calls = []
        self.delay = delay
        self.lock = threading.Lock()

    def __call__(self, prompt, *args, **kwargs):
        with self.lock:
            self.calls.append({"prompt": prompt, "args": list(args), "kwargs": kwargs})
        if self.delay:
            time.sleep(self.delay)
        return {"choices": [{"text": f"<{prompt}>"}]}


class FakeTransport:
    def __init__(self, replies=None):
        self.inbox, self.outbox, self.published, self.connected = [], [], [], []
        self.replies = replies or {}
        self.gossip = []

    def connect(self, peer): self.connected.append(peer)
    def publish(self, msg): self.published.append(msg)
    def poll_gossip(self): return self.gossip.pop(0) if self.gossip else None

    def recv(self, timeout=100):
        if not self.inbox:
            raise Timeout()
        return self.inbox.pop(0)

    def send(self, data): self.outbox.append(data)

    def request(self, peer, data):
        r = self.replies[peer]
        if isinstance(r, Exception):
            raise r
        return r

    def close(self): pass


@pytest.fixture
def model_file(tmp_path):
    p = tmp_path / "m.gguf"
    p.write_bytes(bytes(range(256)) * 40 + b"tail")
    return str(p)


def make(model_file, peers=None, cache_size=3, replies=None, model=None):
    return LlamaP2PNode(model_file, 5000, peers, cache_size=cache_size, secret_key="k",
                        model=model or FakeModel(), transport=FakeTransport(replies))


def test_model_hash(model_file):
    n = make(model_file)
    assert n.model_hash == FX["model_hash"]["node_hash"] == hashlib.md5(open(model_file, "rb").read()).hexdigest()


def test_cache_sequence_matches_reference(model_file):
    m = FakeModel()
    n = make(model_file, cache_size=FX["cache_sequence"]["cache_size"], model=m)
    for step in FX["cache_sequence"]["steps"]:
        before = len(m.calls)
        assert n.cached_inference(step["prompt"]) == step["result"]
        assert (len(m.calls) > before) == step["model_called"]
        assert list(n.cache.keys()) == step["cache_keys"]
        assert list(n.cache_queue) == step["queue"]
    assert m.calls[0] == FX["cache_sequence"]["model_call_args"]  # model(prompt, max_tokens=100)


def test_handler_replies(model_file):
    n = make(model_file)
    for case in FX["handler"]:
        n.transport.outbox.clear()
        try:
            n.handle_one(case["request"].encode())
        except Exception:
            pass  # the reference logs and sends nothing
        got = n.transport.outbox[0].decode() if n.transport.outbox else None
        assert got == case["reply"], case


def test_handler_loop_survives_bad_json(model_file):
    n = make(model_file)
    n.transport.inbox += [b"{bad", json.dumps({"type": "inference", "prompt": "q", "secret_key": "k"}).encode()]
    t = threading.Thread(target=n.handle_requests, daemon=True)
    t.start()
    for _ in range(100):
        if n.transport.outbox:
            break
        time.sleep(0.01)
    n.active = False
    t.join(timeout=2)
    assert [json.loads(o) for o in n.transport.outbox] == [{"result": "<q>"}]


def test_peer_performance(model_file):
    n = make(model_file, peers=["a:1", "b:2"])
    n.update_peer_performance("a:1", True, 1.0)
    n.update_peer_performance("a:1", True, 3.0)
    n.update_peer_performance("b:2", False)
    n.update_peer_performance("c:3", True, 0.0)
    assert {k: dict(v) for k, v in n.peer_performance.items()} == FX["peer_performance"]["stats"]
    assert n.select_peer() == FX["peer_performance"]["selected"]


def test_forward_paths(model_file):
    n = make(model_file, peers=["x:9"], replies={"x:9": RuntimeError("refused")})
    assert n.distributed_inference("fwd") == FX["forward_fail"]["result"]
    assert sorted(n.peers) == FX["forward_fail"]["peers_after"]
    assert {k: dict(v) for k, v in n.peer_performance.items()} == FX["forward_fail"]["perf"]

    n = make(model_file, peers=["y:8"], replies={"y:8": json.dumps({"result": "remote!"}).encode()})
    assert n.distributed_inference("fwd2") == FX["forward_ok"]["result"]
    assert sorted(n.peers) == FX["forward_ok"]["peers_after"]
    assert list(n.cache) == FX["forward_ok"]["local_cache"]
    assert n.peer_performance["y:8"]["success"] == FX["forward_ok"]["success"]

    n = make(model_file, peers=["z:7"], replies={"z:7": json.dumps({"error": "Unauthorized"}).encode()})
    assert n.distributed_inference("fwd3") == FX["forward_unauthorized"]["result"]
    assert sorted(n.peers) == FX["forward_unauthorized"]["peers_after"]
    assert n.peer_performance["z:7"]["failure"] == FX["forward_unauthorized"]["failure"]


def test_gossip_adds_peer(model_file):
    n = make(model_file)
    n.on_gossip({"type": "gossip", "node_id": "abc", "port": 7, "peers": [], "model_hash": "other"})
    assert "abc:7" in n.peers and n.transport.connected == ["abc:7"]


def test_concurrent_prompts_overlap_but_identical_prompts_compute_once(model_file):
    """The engine lock is gone: different prompts run concurrently (they batch on
    the GPU); identical prompts still reach the model once, like the reference."""
    m = FakeModel(delay=0.2)
    n = make(model_file, cache_size=10, model=m)
    res = {}

    def run(p, k):
        res[k] = n.cached_inference(p)

    ts = [threading.Thread(target=run, args=(p, i)) for i, p in enumerate(["a", "b", "c", "a", "a"])]
    t0 = time.time()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.time() - t0
    assert dt < 0.5, "different prompts were serialised"
    assert sorted(c["prompt"] for c in m.calls) == ["a", "b", "c"]
    assert [res[i] for i in range(5)] == ["<a>", "<b>", "<c>", "<a>", "<a>"]


def _serve(n):
    t = threading.Thread(target=n.handle_requests, daemon=True)
    t.start()
    return t


@pytest.mark.parametrize("n_contexts", [1, 32])
def test_concurrent_handler_contexts(model_file, n_contexts):
    """handle_requests over REP contexts: 32 clients on the wire at once are served concurrently
    (n_contexts > 1), each gets its own reply; with one context the handler is the reference's
    lock-step loop (requests serialised)."""
    from llama_p2p_amd.node import LocalTransport

    m = FakeModel(delay=0.1)
    tr = LocalTransport()
    n = LlamaP2PNode(model_file, 5000, cache_size=100, secret_key="k", model=m, transport=tr, n_contexts=n_contexts)
    th = _serve(n)
    out = {}

    def client(i):
        req = {"type": "inference", "prompt": f"p{i}", "secret_key": "k" if i % 8 else "bad"}
        out[i] = json.loads(tr.request(json.dumps(req).encode()))

    cs = [threading.Thread(target=client, args=(i,)) for i in range(32)]
    t0 = time.time()
    for c in cs:
        c.start()
    for c in cs:
        c.join()
    dt = time.time() - t0
    n.active = False
    th.join(timeout=2)
    for i in range(32):
        assert out[i] == ({"result": f"<p{i}>"} if i % 8 else {"error": "Unauthorized"})
    if n_contexts > 1:
        assert dt < 1.0, f"32 requests took {dt:.2f}s: not served concurrently"
    else:
        assert dt > 2.5, "one context must serialise (28 model calls x 0.1 s)"
    assert len(m.calls) == 28


def test_handler_context_bad_json_gets_no_reply(model_file):
    from llama_p2p_amd.node import LocalTransport

    tr = LocalTransport()
    n = LlamaP2PNode(model_file, 5000, secret_key="k", model=FakeModel(), transport=tr, n_contexts=4)
    th = _serve(n)
    with pytest.raises(TimeoutError):
        tr.request(b"{bad", timeout=0.5)  # the reference logs the error and sends nothing
    assert json.loads(tr.request(json.dumps({"type": "inference", "prompt": "q", "secret_key": "k"}).encode())) == \
        {"result": "<q>"}
    n.active = False
    th.join(timeout=2)
