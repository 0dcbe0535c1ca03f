"""Capture the reference node's boundary behaviour as fixtures (tests/golden/node_fixtures.json).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_node_fixtures.py

Imports /root/reference/llama_p2p_network.py (read-only; nothing is written
there) with in-memory stand-ins for its three absent dependencies (zmq,
pynng, llama_cpp -- ordinary ModuleNotFoundErrors here), drives
the four boundary functions and records inputs/outputs.  Only data is
committed; the reference never travels.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import random
import sys
import tempfile
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/llama_p2p_network.py"


class _Timeout(Exception):
    pass


def _stubs(model_calls, replies):
    zmq = types.ModuleType("zmq")

    class ZMQError(Exception):
        pass

    class _Sock:
        def __init__(self, *a):
            self.sent = []

        def bind(self, *a): pass
        def connect(self, *a): pass
        def setsockopt_string(self, *a): pass
        def send_json(self, m): self.sent.append(m)
        def recv_json(self, flags=0): raise ZMQError("empty")
        def close(self): pass

    class Context:
        def socket(self, kind): return _Sock()
        def term(self): pass

    zmq.Context, zmq.ZMQError, zmq.PUB, zmq.SUB, zmq.SUBSCRIBE, zmq.NOBLOCK = Context, ZMQError, 1, 2, 6, 1

    pynng = types.ModuleType("pynng")

    class Rep0:
        def __init__(self):
            self.inbox, self.outbox = [], []

        def listen(self, *a): pass
        def recv(self, timeout=None):
            if not self.inbox:
                raise _Timeout()
            return self.inbox.pop(0)

        def send(self, data): self.outbox.append(data)
        def close(self): pass

    class Req0:
        def __init__(self):
            self.peer = None

        def __enter__(self): return self
        def __exit__(self, *a): return False
        def dial(self, addr): self.peer = addr[len("tcp://"):]
        def send(self, data): self.req = data
        def recv(self):
            r = replies[self.peer]
            if isinstance(r, Exception):
                raise r
            return r

    pynng.Rep0, pynng.Req0, pynng.Timeout = Rep0, Req0, _Timeout

    llama_cpp = types.ModuleType("llama_cpp")

    class Llama:
        def __init__(self, model_path=None, **kw):
            self.model_path = model_path

        def __call__(self, prompt, *args, **kwargs):
            model_calls.append({"prompt": prompt, "args": list(args), "kwargs": kwargs})
            return {"choices": [{"text": f"<{prompt}>"}]}

    llama_cpp.Llama = Llama
    return {"zmq": zmq, "pynng": pynng, "llama_cpp": llama_cpp}


def load_reference(model_calls, replies):
    saved = {k: sys.modules.get(k) for k in ("zmq", "pynng", "llama_cpp")}
    sys.modules.update(_stubs(model_calls, replies))
    try:
        spec = importlib.util.spec_from_file_location("llama_p2p_network_ref", REF)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def main():
    calls, replies = [], {}
    mod = load_reference(calls, replies)
    fx = {}
    with tempfile.NamedTemporaryFile(delete=False, suffix=".gguf") as f:
        f.write(bytes(range(256)) * 40 + b"tail")
        model_file = f.name
    try:
        node = mod.LlamaP2PNode(model_file, 5000, None, cache_size=3, secret_key="k")
        fx["model_hash"] = {"file_bytes_hex_md5": hashlib.md5(open(model_file, "rb").read()).hexdigest(),
                            "node_hash": node.model_hash}
        # cache quirk: insert p0..p5 then re-ask p0
        seq = [f"p{i}" for i in range(6)] + ["p0", "p4", "p1"]
        outs = []
        for p in seq:
            n_before = len(calls)
            outs.append({"prompt": p, "result": node.cached_inference(p), "model_called": len(calls) > n_before,
                         "cache_keys": list(node.cache.keys()), "queue": list(node.cache_queue)})
        fx["cache_sequence"] = {"cache_size": 3, "steps": outs, "model_call_args": calls[0]}
        # handler replies
        rep = node.reply_socket
        msgs = [json.dumps({"type": "inference", "prompt": "hello", "secret_key": "k"}).encode(),
                json.dumps({"type": "inference", "prompt": "hello", "secret_key": "bad"}).encode(),
                json.dumps({"type": "other", "prompt": "hello", "secret_key": "k"}).encode(),
                b"{not json"]
        handler = []
        for m in msgs:
            rep.inbox.append(m)
            rep.outbox.clear()
            node.active = True

            # run exactly one loop iteration
            def once(self=node):
                try:
                    msg = self.reply_socket.recv(timeout=100)
                    request = json.loads(msg.decode())
                    if request["type"] == "inference" and request.get("secret_key") == self.secret_key:
                        result = self.cached_inference(request["prompt"])
                        self.reply_socket.send(json.dumps({"result": result}).encode())
                    else:
                        self.reply_socket.send(json.dumps({"error": "Unauthorized"}).encode())
                except _Timeout:
                    pass
                except Exception:
                    pass

            # the reference loop body is handle_requests; call it with active toggled off after one pass
            orig_recv = rep.recv

            def recv_once(timeout=None, _o=orig_recv):
                node.active = False
                return _o(timeout)

            rep.recv = recv_once
            node.handle_requests()
            rep.recv = orig_recv
            handler.append({"request": m.decode(errors="replace"),
                            "reply": rep.outbox[0].decode() if rep.outbox else None})
        fx["handler"] = handler
        # peer selection / performance
        node2 = mod.LlamaP2PNode(model_file, 5002, ["a:1", "b:2"], cache_size=3, secret_key="k")
        node2.update_peer_performance("a:1", True, 1.0)
        node2.update_peer_performance("a:1", True, 3.0)
        node2.update_peer_performance("b:2", False)
        node2.update_peer_performance("c:3", True, 0.0)
        fx["peer_performance"] = {"stats": {k: dict(v) for k, v in node2.peer_performance.items()},
                                  "selected": node2.select_peer()}
        # forward path: failing peer removed, falls back to local
        node3 = mod.LlamaP2PNode(model_file, 5004, ["x:9"], cache_size=3, secret_key="k")
        replies["x:9"] = RuntimeError("connection refused")
        r = node3.distributed_inference("fwd")
        fx["forward_fail"] = {"result": r, "peers_after": sorted(node3.peers),
                              "perf": {k: dict(v) for k, v in node3.peer_performance.items()}}
        node4 = mod.LlamaP2PNode(model_file, 5006, ["y:8"], cache_size=3, secret_key="k")
        replies["y:8"] = json.dumps({"result": "remote!"}).encode()
        r = node4.distributed_inference("fwd2")
        fx["forward_ok"] = {"result": r, "peers_after": sorted(node4.peers), "local_cache": list(node4.cache),
                            "success": node4.peer_performance["y:8"]["success"]}
        node5 = mod.LlamaP2PNode(model_file, 5008, ["z:7"], cache_size=3, secret_key="k")
        replies["z:7"] = json.dumps({"error": "Unauthorized"}).encode()
        r = node5.distributed_inference("fwd3")
        fx["forward_unauthorized"] = {"result": r, "peers_after": sorted(node5.peers),
                                      "failure": node5.peer_performance["z:7"]["failure"]}
    finally:
        os.unlink(model_file)
    out = os.path.join(HERE, "node_fixtures.json")
    json.dump(fx, open(out, "w"), indent=1, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    random.seed(0)
    main()
