"""Gossip-score request placement and the Poisson serving driver (BASELINE.json configs[4],
SURVEY.md §8d config 5, §8f item 2).

The reference's load balancer is the node's peer scoreboard:
  peer_performance = defaultdict(lambda: {"success": 0, "failure": 0, "avg_time": 0})   p2p:37
  select_peer: random peer while no stats exist, else argmax success/(success+failure+1)  p2p:156-159
  update_peer_performance: success/failure counts, running mean of avg_time              p2p:161-168
On one 8xMI355X node the "peers" are serving targets -- one engine replica per GPU, or the
micro-batch lanes of a pipeline -- and the same scoreboard drives where each request goes.

Two policies share that bookkeeping:
  * ``reference`` -- p2p:156-159 exactly, quirks included: the score ignores avg_time and only
    peers that already have stats compete, so the first target to succeed keeps every request.
  * ``score_aware`` -- the default for serving: untried targets are explored first, then the
    reference score is divided by the target's running mean latency and by (1 + requests it
    has in flight), so a fast, idle replica wins and a failing one is avoided.
"""
from __future__ import annotations

import random
import threading
import time
from collections import defaultdict
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np


class PeerScoreboard:
    """peer_performance + select_peer + update_peer_performance (p2p:37, p2p:156-168)."""

    def __init__(self, targets: Sequence, policy: str = "score_aware", seed: Optional[int] = None):
        if policy not in ("reference", "score_aware"):
            raise ValueError(f"unknown placement policy {policy!r}")
        self.targets = list(targets)
        self.policy = policy
        self.perf: Dict = defaultdict(lambda: {"success": 0, "failure": 0, "avg_time": 0})
        self.inflight: Dict = defaultdict(int)
        self.lock = threading.Lock()
        self.rng = random.Random(seed)

    @staticmethod
    def score(p) -> float:
        """p2p:159: success / (success + failure + 1)."""
        return p["success"] / (p["success"] + p["failure"] + 1)

    def select(self, candidates: Optional[Sequence] = None):
        """The next target.  candidates: the targets able to take a request now (e.g. pipeline lanes
        with a free row); default all.  The reference policy picks among the candidates that have
        stats exactly as p2p:156-159 does among its peers, and a random candidate when none has."""
        with self.lock:
            cands = list(self.targets) if candidates is None else list(candidates)
            if not cands:
                raise ValueError("no placement target available")
            if self.policy == "reference":
                known = [x for x in self.perf if x in cands]
                if not known:
                    t = self.rng.choice(cands)
                else:
                    t = max(known, key=lambda x: self.score(self.perf[x]))
            else:
                untried = [t for t in cands if t not in self.perf and self.inflight[t] == 0]
                if untried:
                    t = untried[0]
                else:
                    def value(x):
                        p = self.perf[x] if x in self.perf else {"success": 0, "failure": 0, "avg_time": 0}
                        if p["success"] == 0:  # never answered (or only failed): last resort
                            return (0.0 if p["failure"] else 1e-12) / (1 + self.inflight[x])
                        return self.score(p) / (max(p["avg_time"], 1e-6) * (1 + self.inflight[x]))

                    t = max(cands, key=value)
            self.inflight[t] += 1
            return t

    def update(self, target, success: bool, elapsed_time: Optional[float] = None):
        """p2p:161-168 (the running mean counts successes only)."""
        with self.lock:
            self.inflight[target] = max(0, self.inflight[target] - 1)
            p = self.perf[target]
            if success:
                p["success"] += 1
                if elapsed_time:
                    p["avg_time"] = (p["avg_time"] * (p["success"] - 1) + elapsed_time) / p["success"]
            else:
                p["failure"] += 1

    def stats(self) -> Dict:
        with self.lock:
            return {t: dict(p) for t, p in self.perf.items()}


def poisson_schedule(rate: float, n: int, seed: int = 3, prompt_lo: int = 32, prompt_hi: int = 512,
                     vocab: int = 128256, bos: int = 1):
    """Config 5's synthetic stream: n requests, exponential inter-arrival times of
    mean 1/rate seconds, prompt lengths U[prompt_lo, prompt_hi], token ids U[3, vocab)."""
    rng = np.random.default_rng(seed)
    t = np.cumsum(rng.exponential(1.0 / rate, n))
    lens = rng.integers(prompt_lo, prompt_hi + 1, n)
    return [(float(t[i]), np.concatenate([[bos], rng.integers(3, vocab, lens[i] - 1)]).astype(np.int32))
            for i in range(n)]


def serve(board: PeerScoreboard, run: Callable, schedule, gen_tokens: int, time_scale: float = 1.0,
          max_workers: int = 256):
    """Replay ``schedule`` in (scaled) real time: at each arrival, place the request with the
    scoreboard and call ``run(target, prompt, gen_tokens) -> n_generated`` on a worker thread;
    the elapsed time of each request updates the scoreboard.  Returns per-request records and
    aggregate throughput / latency."""
    records: List[Dict] = []
    lock = threading.Lock()
    threads = []
    t0 = time.perf_counter()

    def one(i, prompt):
        tgt = board.select()
        ts = time.perf_counter()
        ok, n = True, 0
        try:
            n = run(tgt, prompt, gen_tokens)
        except Exception:  # a failed target counts against its score (p2p:152-154)
            ok = False
        el = time.perf_counter() - ts
        board.update(tgt, ok, el if ok else None)
        with lock:
            records.append({"i": i, "target": tgt, "ok": ok, "tokens": n, "latency": el,
                            "done": time.perf_counter() - t0})

    for i, (ta, prompt) in enumerate(schedule):
        delay = ta * time_scale - (time.perf_counter() - t0)
        if delay > 0:
            time.sleep(delay)
        while sum(th.is_alive() for th in threads) >= max_workers:
            time.sleep(0.001)
        th = threading.Thread(target=one, args=(i, prompt), daemon=True)
        th.start()
        threads.append(th)
    for th in threads:
        th.join()
    wall = time.perf_counter() - t0
    lat = np.array([r["latency"] for r in records if r["ok"]]) if records else np.zeros(1)
    toks = sum(r["tokens"] for r in records)
    per_target = defaultdict(int)
    for r in records:
        per_target[r["target"]] += 1
    return {"requests": len(records), "failed": sum(not r["ok"] for r in records), "tokens": toks,
            "wall_s": wall, "tok_s": toks / wall if wall > 0 else 0.0,
            "p50_s": float(np.percentile(lat, 50)) if len(lat) else 0.0,
            "p99_s": float(np.percentile(lat, 99)) if len(lat) else 0.0,
            "per_target": dict(per_target), "scores": board.stats(), "records": records}
