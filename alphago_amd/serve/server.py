"""Position-evaluation service: policy / value / move generation over HTTP + JSON.

``GoService`` turns a position (a move list from the empty board) into feature
planes (the native featurizer) and evaluates them through the
``BatchingEvaluator`` of each network.  Concurrent requests therefore share
batched HIP-graph replays.  ``serve`` runs it behind the standard library's
threading HTTP server, with one handler thread per connection and no
third-party dependency.

Endpoints (JSON bodies; moves are ``[x, y]`` with x the SGF column, ``null`` a pass):

  GET  /v1/health                      {"ok": true, "board": 19, "value": bool}
  GET  /v1/stats                       batcher counters (rounds, mean batch, ...)
  POST /v1/policy   {"moves": [...], "top_k": 5}
       -> {"to_play": 1|-1, "moves": [[x, y, p], ...]}  renormalised over legal moves
  POST /v1/genmove  {"moves": [...], "temperature": 0}
       -> {"move": [x, y] | null}       greedy (T = 0) or sampled at temperature T
  POST /v1/value    {"moves": [...]}    -> {"value": v}  for the player to move
"""
from __future__ import annotations

import json
import threading
from collections import OrderedDict
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Iterable, List, Optional, Sequence

import numpy as np

from .batcher import BatcherPool, BatchingEvaluator, state_eval_fn


MAX_BODY = 1 << 20  # a 19x19 move list is a few KB
DRAIN_LIMIT = 16 * MAX_BODY  # oversized bodies up to this size are read and discarded before the 413


class BadRequest(ValueError):
    pass


def position_from_moves(size: int, moves: Optional[Iterable]) -> object:
    """GameState after playing ``moves`` from the empty board (``BadRequest`` on a bad move)."""
    from .. import go

    st = go.GameState(size=size)
    _extend(st, list(moves or []), 0, size)
    return st


def _extend(st, moves, first: int, size: int) -> None:
    from .. import go

    for i, m in enumerate(moves, first):
        mv = None if m is None else tuple(int(v) for v in m)
        if mv is not None and (len(mv) != 2 or not all(0 <= v < size for v in mv)):
            raise BadRequest("move %d: %r is not a point of the %dx%d board" % (i, m, size, size))
        try:
            st.do_move(mv)
        except go.IllegalMove:
            raise BadRequest("move %d: %r is illegal" % (i, m))


def _batcher(nets, max_batch, max_wait_ms, name):
    """One batcher per network copy (one per GPU); a pool when there are several."""
    bs = [BatchingEvaluator(state_eval_fn(n), max_batch, max_wait_ms, "%s%d" % (name, i), device=n.device)
          for i, n in enumerate(nets)]
    return bs[0] if len(bs) == 1 else BatcherPool(bs)


class GoService(object):
    """Thread-safe evaluation front end over a policy (and optional value) network.
    ``policy`` / ``value`` may be lists of copies of one network on different GPUs: each
    copy gets its own batcher and requests go to the least-loaded one."""

    def __init__(self, policy, value=None, max_batch: int = 256, max_wait_ms: float = 2.0, seed: int = 0,
                 cache_size: int = 4096):
        pols = list(policy) if isinstance(policy, (list, tuple)) else [policy]
        vals = (list(value) if isinstance(value, (list, tuple)) else [value]) if value is not None else []
        self.policy = pols[0]
        self.value = vals[0] if vals else None
        self.size = self.policy.model.board
        # requests carry GameStates; each round is featurised in one batched call
        # (GPU featurizer inside the HIP graph when the engine has one)
        self.pol_batcher = _batcher(pols, max_batch, max_wait_ms, "policy")
        self.val_batcher = _batcher(vals, max_batch, max_wait_ms, "value") if vals else None
        self._rng = np.random.default_rng(seed)
        self._rng_lock = threading.Lock()
        # Positions by move list (LRU).  A client that plays a game through a stateless API
        # sends the whole move list every turn; the cached position of the list minus its
        # last move or two is copied and extended, instead of replaying the game.
        self._cache: "OrderedDict[tuple, object]" = OrderedDict()
        self._cache_lock = threading.Lock()
        self.cache_size = cache_size
        self.max_moves = 4 * self.size * self.size  # a few times S*S covers any real game
        self.cache_hits = 0

    # ------------------------------------------------------------ positions
    def position(self, moves: Optional[Iterable]) -> object:
        moves = list(moves or [])
        if len(moves) > self.max_moves:  # bounds the parse work and the cached positions' history
            raise BadRequest("%d moves: at most %d per request" % (len(moves), self.max_moves))
        key = tuple(None if m is None else tuple(int(v) for v in m) for m in moves)
        if self.cache_size <= 0:
            return position_from_moves(self.size, key)
        base, done = None, 0
        with self._cache_lock:
            for k in (0, 1, 2):
                if len(key) >= k:
                    hit = self._cache.get(key[:len(key) - k])
                    if hit is not None:
                        self._cache.move_to_end(key[:len(key) - k])
                        base, done = hit, len(key) - k
                        self.cache_hits += 1
                        break
        if base is None:
            st = position_from_moves(self.size, key)
        elif done == len(key):
            st = base  # cached states are never mutated: callers only read them
        else:
            st = base.copy()
            _extend(st, key[done:], done, self.size)
        with self._cache_lock:
            self._cache[key] = st
            self._cache.move_to_end(key)
            while len(self._cache) > self.cache_size:
                self._cache.popitem(last=False)
        return st

    def _ranked(self, probs: np.ndarray, st, top_k: Optional[int] = None):
        """[(move, p)] over the legal moves, renormalised, best first (numpy; no per-move
        Python work beyond the returned top_k)."""
        idx = np.flatnonzero(np.asarray(st.legal_mask()))
        if idx.size == 0:
            return []
        p = probs[idx].astype(np.float64)
        tot = p.sum()
        p = p / tot if tot > 0 else np.full(idx.size, 1.0 / idx.size)
        k = idx.size if not top_k else min(int(top_k), idx.size)
        sel = np.argpartition(-p, k - 1)[:k] if k < idx.size else np.arange(idx.size)
        sel = sel[np.argsort(-p[sel], kind="stable")]
        S = self.size
        return [((int(idx[j] // S), int(idx[j] % S)), float(p[j])) for j in sel]

    @staticmethod
    def _eval(batcher, st) -> np.ndarray:
        return batcher.submit_items([st]).result()[0]

    # ------------------------------------------------------------ queries
    def policy_moves(self, moves, top_k: Optional[int] = None) -> dict:
        st = self.position(moves)
        probs = self._eval(self.pol_batcher, st)
        ranked = self._ranked(probs, st, top_k)  # renormalised over the legal moves
        return {"to_play": int(st.current_player), "moves": [[m[0], m[1], float(p)] for m, p in ranked]}

    def genmove(self, moves, temperature: float = 0.0) -> dict:
        st = self.position(moves)
        if st.is_end_of_game:
            return {"move": None}
        ranked = self._ranked(self._eval(self.pol_batcher, st), st)
        if not ranked:
            return {"move": None}
        if temperature and temperature > 0:
            p = np.array([q for _, q in ranked], np.float64) ** (1.0 / float(temperature))
            p /= p.sum()
            with self._rng_lock:
                k = int(self._rng.choice(len(ranked), p=p))
        else:
            k = 0  # best first
        return {"move": list(ranked[k][0])}

    def value_of(self, moves) -> dict:
        if self.val_batcher is None:
            raise BadRequest("no value network loaded")
        st = self.position(moves)
        v = self._eval(self.val_batcher, st)
        return {"value": float(np.asarray(v).reshape(-1)[0])}

    def stats(self) -> dict:
        out = {"policy": self.pol_batcher.stats()}
        if self.val_batcher is not None:
            out["value"] = self.val_batcher.stats()
        return out

    def close(self) -> None:
        self.pol_batcher.close()
        if self.val_batcher is not None:
            self.val_batcher.close()


def _handler(service: GoService):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # quiet by default
            pass

        def _send(self, code: int, obj) -> None:
            body = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):
            if self.path == "/v1/health":
                self._send(200, {"ok": True, "board": service.size, "value": service.val_batcher is not None})
            elif self.path == "/v1/stats":
                self._send(200, service.stats())
            else:
                self._send(404, {"error": "unknown endpoint %s" % self.path})

        def do_POST(self):
            try:
                n = int(self.headers.get("Content-Length", "0"))
                if n < 0:  # rfile.read(-1) would block this handler until the client closes
                    self.close_connection = True
                    self._send(400, {"error": "negative Content-Length"})
                    return
                if n > MAX_BODY:
                    # drain a moderately oversized body (bounded, discarded in 64 KiB reads) so the
                    # client, still sending, receives the 413 instead of a reset; beyond the drain
                    # bound the connection is just closed
                    self.close_connection = True
                    if n <= DRAIN_LIMIT:
                        left = n
                        while left > 0:
                            got = self.rfile.read(min(left, 1 << 16))
                            if not got:
                                break
                            left -= len(got)
                    self._send(413, {"error": "request body over %d bytes" % MAX_BODY})
                    return
                req = json.loads(self.rfile.read(n) or b"{}")
                if not isinstance(req, dict):
                    raise BadRequest("body must be a JSON object")
                moves = req.get("moves", [])
                if self.path == "/v1/policy":
                    self._send(200, service.policy_moves(moves, req.get("top_k")))
                elif self.path == "/v1/genmove":
                    self._send(200, service.genmove(moves, float(req.get("temperature", 0.0))))
                elif self.path == "/v1/value":
                    self._send(200, service.value_of(moves))
                else:
                    self._send(404, {"error": "unknown endpoint %s" % self.path})
            except (BadRequest, ValueError, TypeError) as e:
                self._send(400, {"error": str(e)})
            except Exception as e:  # engine failure: the client sees it, the server keeps running
                self._send(500, {"error": "%s: %s" % (type(e).__name__, e)})

    return Handler


def make_server(service: GoService, host: str = "127.0.0.1", port: int = 8000) -> ThreadingHTTPServer:
    """Bound (not yet serving) HTTP server; ``port=0`` picks a free port (``server.server_address``)."""
    srv = ThreadingHTTPServer((host, port), _handler(service))
    srv.daemon_threads = True
    return srv


def serve_cli(argv: Sequence[str]) -> int:
    import argparse

    from ..models.policy import CNNPolicy, CNNValue

    p = argparse.ArgumentParser(prog="alphago_amd serve",
                                description="HTTP/JSON position evaluation with dynamic batching")
    p.add_argument("policy", help="policy model JSON (CNNPolicy.save_model)")
    p.add_argument("--value", default=None, help="value model JSON")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--max-batch", type=int, default=256)
    p.add_argument("--max-wait-ms", type=float, default=2.0)
    p.add_argument("--device", default=None, help="cuda:N or cpu (default: cuda:0 when available)")
    p.add_argument("--precision", default=None, choices=["bf16", "fp8"],
                   help="GPU engine precision (fp8: e4m3 block-scaled MFMA convs; default bf16 or "
                        "$ALPHAGO_AMD_PRECISION)")
    p.add_argument("--devices", default=None,
                   help="comma-separated devices (e.g. cuda:0,cuda:1,...): one network copy and batcher per "
                        "device, requests to the least-loaded one")
    a = p.parse_args(list(argv))
    if a.precision:
        import os

        os.environ["ALPHAGO_AMD_PRECISION"] = a.precision  # read when each engine is built
    devs = a.devices.split(",") if a.devices else [a.device]
    pol = [CNNPolicy.load_model(a.policy, device=d) for d in devs]
    val = [CNNValue.load_model(a.value, device=d) for d in devs] if a.value else None
    svc = GoService(pol, val, a.max_batch, a.max_wait_ms)
    srv = make_server(svc, a.host, a.port)
    print("serving on http://%s:%d" % srv.server_address[:2], flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    finally:
        srv.server_close()
        svc.close()
    return 0


def post_json(url: str, obj, timeout: float = 30.0) -> dict:
    """Small client helper (tests, benchmarks)."""
    import urllib.request

    req = urllib.request.Request(url, data=json.dumps(obj).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


def random_positions(size: int, n: int, max_moves: int = 120, seed: int = 0) -> List[List]:
    """``n`` random legal move lists (benchmarks and tests)."""
    from .. import go

    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        st = go.GameState(size=size)
        moves = []
        for _ in range(int(rng.integers(0, max_moves + 1))):
            legal = st.get_legal_moves()
            if not legal:
                break
            m = legal[int(rng.integers(len(legal)))]
            st.do_move(m)
            moves.append(list(m))
        out.append(moves)
    return out
