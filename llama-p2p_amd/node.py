"""LlamaP2PNode -- the reference node with its local model swapped for the MI355X engine.

Mirror of /root/reference/llama_p2p_network.py:17-190.  The four functions the
drop-in boundary is drawn around keep the reference's signatures and visible
behaviour:

  handle_requests(self)               p2p:84-98   JSON REQ -> {"result"} / {"error": "Unauthorized"}
  cached_inference(self, prompt)      p2p:120-133 result cache, incl. its eviction quirk (§4.1)
  distributed_inference(self, prompt) p2p:135-154 forward-or-local decision
  compute_model_hash(self, path)      p2p:177-182 MD5 of the model file

Deliberate difference: the reference holds ``self.lock`` across the whole
model call (p2p:121-133), serialising every generation on the node.  Here the
lock guards only the cache; concurrent *different* prompts reach the engine
together and are micro-batched on the GPU, while concurrent *identical*
prompts still compute once (the second waits for the first, as with the lock).
The cache contents and eviction order are unchanged.

The request handler keeps its signature but no longer answers one message at a
time: the reference's single lock-step ``Rep0`` loop (p2p:84-98) becomes
``n_contexts`` concurrent REP contexts (nng's ``Rep0`` contexts; SURVEY.md §8f
item 1), each a worker that receives, runs ``cached_inference`` and replies on
its own context, so concurrent requests from the wire reach the engine together
and are micro-batched.  A transport without contexts keeps the lock-step loop.

The gossip (zmq PUB/SUB) and RPC (nng REQ/REP) transports are the reference's
control plane and are out of scope; they are imported
lazily, and tests inject in-process transports instead.
"""
from __future__ import annotations

import hashlib
import json
import logging
import random
import secrets
import threading
import time
from collections import defaultdict, deque

log = logging.getLogger("llama_p2p_amd.node")


class Timeout(Exception):
    """Raised by a reply transport's recv when nothing arrived (pynng.Timeout)."""


class Closed(Exception):
    """Raised by a reply context's recv once its socket is closed (pynng.Closed): the worker exits."""


class LlamaP2PNode:
    def __init__(self, model_path, port, known_peers=None, cache_size=100, secret_key=None, *, model=None,
                 transport=None, llama_kwargs=None, n_contexts=64):
        """``model`` injects an already-built Llama; ``transport`` injects the networking
        (an object with gossip/subscriber/reply sockets and ``dial(peer)``); without
        it, zmq + pynng are used as in the reference (p2p:24-31)."""
        if model is None:
            from .llama import Llama

            model = Llama(model_path=model_path, **(llama_kwargs or {}))
        self.model = model
        self.model_hash = self.compute_model_hash(model_path)
        self.port = port
        self.peers = set(known_peers) if known_peers else set()
        self.node_id = hashlib.sha256(f"{port}_{random.randint(1, 1000000)}".encode()).hexdigest()[:10]
        self.transport = transport if transport is not None else _NetTransport(port)
        self.cache = {}
        self.cache_queue = deque(maxlen=cache_size)
        self.lock = threading.Lock()
        self._inflight = {}
        self.active = True
        self.secret_key = secret_key or secrets.token_hex(16)
        self.peer_performance = defaultdict(lambda: {"success": 0, "failure": 0, "avg_time": 0})
        self.n_contexts = n_contexts

    # ------------------------------------------------------------ lifecycle
    def start(self, cli: bool = True):
        for peer in self.peers:
            self.connect_to_peer(peer)
        threading.Thread(target=self.gossip_loop, daemon=True).start()
        threading.Thread(target=self.listen_loop, daemon=True).start()
        threading.Thread(target=self.handle_requests, daemon=True).start()
        log.info(f"Node {self.node_id} started on port {self.port}")
        if cli:
            self.cli_loop()

    def connect_to_peer(self, peer):
        try:
            self.transport.connect(peer)
            log.info(f"Connected to peer: {peer}")
        except Exception as e:
            log.error(f"Failed to connect to peer {peer}: {e}")

    def gossip_loop(self):
        while self.active:
            message = {"type": "gossip", "node_id": self.node_id, "port": self.port, "peers": list(self.peers),
                       "model_hash": self.model_hash}
            self.transport.publish(message)
            time.sleep(5)

    def listen_loop(self):
        while self.active:
            try:
                message = self.transport.poll_gossip()
                if message is None:
                    time.sleep(0.1)
                    continue
                self.on_gossip(message)
            except Exception:
                time.sleep(0.1)

    def on_gossip(self, message):
        """One received gossip message (p2p:73-80)."""
        if message["type"] == "gossip":
            new_peer = f"{message['node_id']}:{message['port']}"
            if new_peer not in self.peers and new_peer != f"{self.node_id}:{self.port}":
                log.info(f"Discovered new peer: {new_peer}")
                self.peers.add(new_peer)
                self.connect_to_peer(new_peer)
            if message["model_hash"] != self.model_hash:
                log.warning(f"Peer {new_peer} has a different model hash")

    # ------------------------------------------------------- drop-in boundary
    def handle_requests(self):
        """p2p:84-98.  With a transport that opens REP contexts: n_contexts workers, each receiving
        on its own context and replying on it, so requests are served concurrently; otherwise the
        reference's lock-step loop on the one reply socket."""
        new_context = getattr(self.transport, "new_context", None)
        if new_context is None or self.n_contexts <= 1:
            while self.active:
                try:
                    msg = self.transport.recv(timeout=100)
                    self.handle_one(msg)
                except Timeout:
                    continue
                except Exception as e:
                    log.error(f"Error handling request: {e}")
            return
        workers = [threading.Thread(target=self._context_loop, args=(new_context(),), daemon=True)
                   for _ in range(self.n_contexts)]
        for w in workers:
            w.start()
        for w in workers:
            w.join()

    def _context_loop(self, ctx):
        while self.active:
            try:
                msg = ctx.recv(timeout=100)
            except Timeout:
                continue
            except Closed:
                break
            except Exception as e:
                log.error(f"Error handling request: {e}")
                continue
            try:
                self.handle_one(msg, reply=ctx)
            except Exception as e:  # as the reference: logged, no reply on this context
                log.error(f"Error handling request: {e}")
        close = getattr(ctx, "close", None)
        if close:
            close()

    def handle_one(self, msg: bytes, reply=None):
        """Body of the handler loop for one message (p2p:88-94); raises like the reference.
        ``reply``: the REP context the message came from (default: the transport's socket)."""
        out = reply if reply is not None else self.transport
        request = json.loads(msg.decode())
        if request["type"] == "inference" and request.get("secret_key") == self.secret_key:
            result = self.cached_inference(request["prompt"])
            response = {"result": result}
            out.send(json.dumps(response).encode())
        else:
            out.send(json.dumps({"error": "Unauthorized"}).encode())

    def cached_inference(self, prompt):
        with self.lock:
            if prompt in self.cache:
                return self.cache[prompt]
            ev = self._inflight.get(prompt)
            owner = ev is None
            if owner:
                ev = self._inflight[prompt] = threading.Event()
        if not owner:  # an identical prompt is being generated: wait for it (the reference's lock did this)
            ev.wait()
            with self.lock:
                if prompt in self.cache:
                    return self.cache[prompt]
            return self.cached_inference(prompt)
        try:
            result = self.model(prompt, max_tokens=100)["choices"][0]["text"]
            with self.lock:
                self.cache[prompt] = result
                self.cache_queue.append(prompt)
                if len(self.cache) > self.cache_queue.maxlen:
                    oldest = self.cache_queue.popleft()
                    del self.cache[oldest]
            return result
        finally:
            with self.lock:
                self._inflight.pop(prompt, None)
            ev.set()

    def distributed_inference(self, prompt):
        if not self.peers:
            return self.cached_inference(prompt)
        peer = self.select_peer()
        try:
            start_time = time.time()
            response = self.transport.request(peer, json.dumps(
                {"type": "inference", "prompt": prompt, "secret_key": self.secret_key}).encode())
            elapsed_time = time.time() - start_time
            result = json.loads(response.decode())["result"]
            self.update_peer_performance(peer, True, elapsed_time)
            return result
        except Exception as e:
            log.error(f"Error communicating with peer {peer}: {e}")
            self.update_peer_performance(peer, False)
            self.peers.remove(peer)
            return self.distributed_inference(prompt)

    def select_peer(self):
        if not self.peer_performance:
            return random.choice(list(self.peers))
        return max(self.peer_performance, key=lambda x: self.peer_performance[x]["success"] / (
            self.peer_performance[x]["success"] + self.peer_performance[x]["failure"] + 1))

    def update_peer_performance(self, peer, success, elapsed_time=None):
        with self.lock:
            if success:
                self.peer_performance[peer]["success"] += 1
                if elapsed_time:
                    p = self.peer_performance[peer]
                    p["avg_time"] = (p["avg_time"] * (p["success"] - 1) + elapsed_time) / p["success"]
            else:
                self.peer_performance[peer]["failure"] += 1

    def compute_model_hash(self, model_path):
        hasher = hashlib.md5()
        if model_path.startswith("synthetic:"):  # no file: hash the synthetic model's spec string
            hasher.update(model_path.encode())
            return hasher.hexdigest()
        with open(model_path, "rb") as f:
            for chunk in iter(lambda: f.read(1 << 22), b""):
                hasher.update(chunk)
        return hasher.hexdigest()

    # --------------------------------------------------------------- misc
    def cli_loop(self):
        while self.active:
            command = input("Enter command (infer/peers/cache/performance/exit): ")
            if command == "infer":
                prompt = input("Enter prompt: ")
                print(f"Result: {self.distributed_inference(prompt)}")
            elif command == "peers":
                print(f"Known peers: {self.peers}")
            elif command == "cache":
                print(f"Cache size: {len(self.cache)}")
                print(f"Cache items: {list(self.cache.keys())}")
            elif command == "performance":
                self.print_performance_stats()
            elif command == "exit":
                self.shutdown()
                break
            else:
                print("Unknown command")

    def print_performance_stats(self):
        for peer, stats in self.peer_performance.items():
            print(f"Peer {peer}:")
            print(f"  Success: {stats['success']}")
            print(f"  Failure: {stats['failure']}")
            print(f"  Avg Time: {stats['avg_time']:.2f}s")

    def shutdown(self):
        log.info(f"Shutting down node {self.node_id}")
        self.active = False
        self.transport.close()


class _NetTransport:
    """The reference's zmq PUB/SUB + nng REQ/REP wiring (p2p:24-31, :52, :66, :72, :87, :92, :142-145)."""

    def __init__(self, port):
        import pynng  # noqa: F401  (absent on this machine: control plane is out of scope)
        import zmq

        self._zmq, self._pynng = zmq, pynng
        self.context = zmq.Context()
        self.gossip_socket = self.context.socket(zmq.PUB)
        self.gossip_socket.bind(f"tcp://*:{port}")
        self.subscriber = self.context.socket(zmq.SUB)
        self.subscriber.setsockopt_string(zmq.SUBSCRIBE, "")
        self.reply_socket = pynng.Rep0()
        self.reply_socket.recv_timeout = 100  # ms: lets the context workers notice shutdown
        self.reply_socket.listen(f"tcp://0.0.0.0:{port + 1}")

    def connect(self, peer):
        self.subscriber.connect(f"tcp://{peer}")

    def publish(self, msg):
        self.gossip_socket.send_json(msg)

    def poll_gossip(self):
        try:
            return self.subscriber.recv_json(flags=self._zmq.NOBLOCK)
        except self._zmq.ZMQError:
            return None

    def recv(self, timeout=100):
        try:
            return self.reply_socket.recv(timeout=timeout)
        except self._pynng.Timeout:
            raise Timeout()

    def send(self, data):
        self.reply_socket.send(data)

    def new_context(self):
        """A REP context of the reply socket (nng: each context has its own receive/reply state,
        so several requests are in progress at once on one socket)."""
        return _NetContext(self.reply_socket.new_context(), self._pynng)

    def request(self, peer, data):
        with self._pynng.Req0() as s:
            s.dial(f"tcp://{peer}")
            s.send(data)
            return s.recv()

    def close(self):
        self.gossip_socket.close()
        self.subscriber.close()
        self.reply_socket.close()
        self.context.term()


class _NetContext:
    """One REP context.  UNVERIFIED here (pynng is not importable in this container): the receive
    timeout is set on the context itself where pynng exposes it, and otherwise inherited from the
    socket's recv_timeout; ``close()`` of the socket is the shutdown path either way -- a blocked
    recv then raises pynng.Closed, which ends the worker instead of being logged and retried."""

    def __init__(self, ctx, pynng, timeout_ms=100):
        self._ctx, self._pynng = ctx, pynng
        try:
            ctx.recv_timeout = timeout_ms
        except Exception:  # older pynng: contexts take the socket's option
            pass

    def recv(self, timeout=100):
        try:
            return self._ctx.recv()
        except self._pynng.Timeout:
            raise Timeout()
        except self._pynng.Closed:
            raise Closed()

    def send(self, data):
        self._ctx.send(data)

    def close(self):
        self._ctx.close()


class LocalTransport:
    """In-process stand-in for the node's nng REP socket with concurrent contexts: clients call
    ``request(data)`` (blocking, like a Req0 round trip); the node's context workers receive the
    messages in arrival order and each reply goes back to the client that sent that message.
    Used to drive ``handle_requests`` without a network (tests, tools/serve_config3.py)."""

    def __init__(self):
        import queue

        self._q = queue.Queue()
        self._queue_mod = queue

    # client side
    def request(self, data: bytes, timeout: float = 600.0) -> bytes:
        box = {"ev": threading.Event(), "reply": None}
        self._q.put((data, box))
        if not box["ev"].wait(timeout):
            raise TimeoutError("no reply")
        return box["reply"]

    # node side (the reference's control-plane calls are no-ops here)
    def connect(self, peer): pass
    def publish(self, msg): pass
    def poll_gossip(self): return None
    def close(self): pass

    def recv(self, timeout=100):  # lock-step mode: the one context
        return self._ctx.recv(timeout)

    def send(self, data):
        self._ctx.send(data)

    @property
    def _ctx(self):
        if not hasattr(self, "_default"):
            self._default = self.new_context()
        return self._default

    def new_context(self):
        return _LocalContext(self)


class _LocalContext:
    def __init__(self, t: LocalTransport):
        self._t = t
        self._box = None

    def recv(self, timeout=100):
        try:
            data, self._box = self._t._q.get(timeout=timeout / 1000.0)
        except self._t._queue_mod.Empty:
            raise Timeout()
        return data

    def send(self, data):
        box, self._box = self._box, None
        if box is None:
            raise RuntimeError("send without a received request (REP state machine)")
        box["reply"] = data
        box["ev"].set()
