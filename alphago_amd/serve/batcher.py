"""Dynamic batching of network evaluations for serving.

Many client threads (HTTP handlers, GTP sessions, game workers) each need a few
positions evaluated.  One evaluation per request would leave the MI355X almost
idle: a 12 x 192 policy trunk at batch 1 is launch-latency bound, while at
batch 256 the same HIP-graph replay evaluates 256 boards in a few ms.  The
batcher queues requests, and a single worker thread drains them.  It runs one
batched evaluation per round, with up to ``max_batch`` boards.  The round
starts as soon as the queue holds ``max_batch`` boards or the oldest request has
waited ``max_wait_ms``.  Each request then gets its own rows back.

Only the worker thread touches the engine, so a HIP engine keeps one stream.
Its bucketed HIP graphs (``models/inference.py``) see the batched sizes.

The reference evaluates one state per call (``CNNPolicy.eval_state``,
/root/reference/AlphaGo/models/policy.py:44-79).  Serving is not a reference
feature: this is the serving path of the MI355X build.
"""
from __future__ import annotations

import threading
import time
from collections import deque
from concurrent.futures import Future
from typing import Callable, Deque, Dict, List, Optional, Tuple

import numpy as np

EvalFn = Callable[[np.ndarray, Optional[np.ndarray]], np.ndarray]


class _Request(object):
    __slots__ = ("planes", "legal", "future", "t_submit", "n")

    def __init__(self, planes, legal, future, t_submit):
        self.planes, self.legal, self.future, self.t_submit = planes, legal, future, t_submit
        self.n = len(planes)  # boards: rows of a planes array, or items of an object list


class BatchingEvaluator(object):
    """``evaluate_fn(planes (n, C, S, S) uint8, legal (n, S*S) uint8 or None) -> (n, ...) array``
    is called from the worker thread only.  ``submit`` is thread-safe and returns a Future
    whose result holds the request's rows, in order.  A request of k boards is never split
    across rounds.  A request larger than ``max_batch`` runs as a round of its own."""

    def __init__(self, evaluate_fn: EvalFn, max_batch: int = 256, max_wait_ms: float = 2.0, name: str = "eval",
                 device=None):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.fn = evaluate_fn
        self.device = device  # the engine's GPU: the worker thread makes it current before any launch
        self.max_batch = int(max_batch)
        self.max_wait = max(0.0, float(max_wait_ms)) / 1e3
        self.name = name
        self._q: Deque[_Request] = deque()
        self._rows = 0  # boards queued
        self._cv = threading.Condition()
        self._closed = False
        self._kind: Optional[str] = None  # "planes" or "items": one payload kind per batcher
        self._plane_shape: Optional[Tuple[int, int, int]] = None  # (C, S, S), pinned by the first request
        self._stats: Dict[str, float] = {"requests": 0, "boards": 0, "rounds": 0, "eval_s": 0.0, "errors": 0}
        self._worker = threading.Thread(target=self._loop, name="batcher-%s" % name, daemon=True)
        self._worker.start()

    # ---------------------------------------------------------------- client side
    def submit(self, planes, legal=None) -> Future:
        """planes: (C, S, S) or (k, C, S, S) uint8; legal: matching (S*S,) / (k, S*S) or None."""
        p = np.asarray(planes)
        single = p.ndim == 3
        if single:
            p = p[None]
        if p.ndim != 4 or p.shape[0] == 0:
            raise ValueError("planes must be (C, S, S) or (k, C, S, S) with k >= 1")
        p = np.ascontiguousarray(p, dtype=np.uint8)
        lg = None
        if legal is not None:
            lg = np.asarray(legal, dtype=np.uint8)
            lg = lg[None] if lg.ndim == 1 else lg
            if lg.ndim != 2 or lg.shape[0] != p.shape[0]:
                raise ValueError("legal mask rows do not match the planes")
            if lg.shape[1] != p.shape[2] * p.shape[3]:
                raise ValueError("legal mask width %d != S*S = %d" % (lg.shape[1], p.shape[2] * p.shape[3]))
        fut: Future = Future()
        fut._ag_single = single  # type: ignore[attr-defined]
        with self._cv:
            self._check_open("planes")
            shp = tuple(p.shape[1:])
            if self._plane_shape is None:
                self._plane_shape = shp  # type: ignore[assignment]
            elif shp != self._plane_shape:
                raise ValueError("planes %s do not match this batcher's %s" % (shp, self._plane_shape))
            self._q.append(_Request(p, lg, fut, time.perf_counter()))
            self._rows += p.shape[0]
            self._cv.notify()
        return fut

    def submit_items(self, items: list) -> Future:
        """Object payload (e.g. GameStates): ``evaluate_fn`` then receives the concatenated
        list of a round's items (and ``None`` for the mask)."""
        items = list(items)
        if not items:
            raise ValueError("empty request")
        fut: Future = Future()
        fut._ag_single = False  # type: ignore[attr-defined]
        with self._cv:
            self._check_open("items")
            self._q.append(_Request(items, None, fut, time.perf_counter()))
            self._rows += len(items)
            self._cv.notify()
        return fut

    def _check_open(self, kind: str) -> None:
        """(lock held) Refuse submissions after close() and a second payload kind."""
        if self._closed:
            raise RuntimeError("batcher %s is closed" % self.name)
        if self._kind is None:
            self._kind = kind
        elif self._kind != kind:
            raise ValueError("batcher %s takes %s requests, not %s" % (self.name, self._kind, kind))

    def evaluate(self, planes, legal=None, timeout: Optional[float] = None) -> np.ndarray:
        fut = self.submit(planes, legal)
        out = fut.result(timeout)
        return out[0] if fut._ag_single else out  # type: ignore[attr-defined]

    def stats(self) -> Dict[str, float]:
        with self._cv:
            s = dict(self._stats)
            s["queued_boards"] = self._rows
        s["mean_batch"] = s["boards"] / s["rounds"] if s["rounds"] else 0.0
        return s

    def close(self, timeout: float = 10.0) -> None:
        """Finish the queued requests, then stop the worker."""
        with self._cv:
            self._closed = True
            self._cv.notify_all()
        self._worker.join(timeout)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---------------------------------------------------------------- worker
    def _take(self) -> Optional[List[_Request]]:
        """Block until a round is due; pop its requests (None: closed and drained)."""
        with self._cv:
            while True:
                if self._q:
                    due = self._q[0].t_submit + self.max_wait
                    now = time.perf_counter()
                    if self._rows >= self.max_batch or now >= due or self._closed:
                        break
                    self._cv.wait(due - now)
                elif self._closed:
                    return None
                else:
                    self._cv.wait()
            batch, rows = [], 0
            while self._q and (not batch or rows + self._q[0].n <= self.max_batch):
                r = self._q.popleft()
                batch.append(r)
                rows += r.n
            self._rows -= rows
            return batch

    def _loop(self) -> None:
        if self.device is not None:
            import torch

            dev = torch.device(self.device)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)  # a thread's current device starts at 0
        while True:
            batch = self._take()
            if batch is None:
                return
            live = [r for r in batch if r.future.set_running_or_notify_cancel()]
            if not live:
                continue
            sizes = [r.n for r in live]
            nrows = sum(sizes)
            t0 = time.perf_counter()
            try:
                # batch assembly inside the try: a failure reaches this round's futures instead of
                # killing the worker (and with it every queued and later request)
                if isinstance(live[0].planes, list):
                    planes = [x for r in live for x in r.planes]
                else:
                    planes = live[0].planes if len(live) == 1 else np.concatenate([r.planes for r in live])
                legal = None
                if not isinstance(planes, list) and any(r.legal is not None for r in live):
                    S2 = planes.shape[2] * planes.shape[3]
                    legal = np.concatenate([r.legal if r.legal is not None
                                            else np.ones((r.planes.shape[0], S2), np.uint8) for r in live])
                out = np.asarray(self.fn(planes, legal))
                if out.shape[0] != nrows:
                    raise RuntimeError("evaluate_fn returned %d rows for %d boards" % (out.shape[0], nrows))
            except BaseException as e:  # delivered to every waiting client
                with self._cv:
                    self._stats["errors"] += 1
                for r in live:
                    r.future.set_exception(e)
                continue
            dt = time.perf_counter() - t0
            with self._cv:
                self._stats["requests"] += len(live)
                self._stats["boards"] += nrows
                self._stats["rounds"] += 1
                self._stats["eval_s"] += dt
            off = 0
            for r, k in zip(live, sizes):
                r.future.set_result(out[off:off + k].copy())
                off += k


def state_eval_fn(net, threads: int = 8) -> Callable:
    """Batched evaluation of GameStates for a CNNPolicy / CNNValue wrapper.

    GPU engines built with a feature list take the compact path.  The host encodes the
    whole round in one native multi-threaded call (board, ages, metadata, ladder bits).
    The featurizer kernel then runs inside the engine's HIP graph.  A board whose
    eye recursion overflows the kernel is recomputed from CPU planes.  Other engines
    get the round featurized in one native call (``states_to_uint8``)."""
    from .._native import engine as _native

    def fn(states, _legal):
        # the engine is built on first use, in the batcher's worker thread, whose current
        # device is the network's GPU (its weight packing and graph capture launch there)
        eng = net.engine
        if getattr(eng, "supports_encoded", False):
            b, a, m, lad = _native().encode_batch(list(states), eng.needs_ladder, threads)
            out, _, bad = eng.evaluate_encoded(b, a, m, lad)
            out = out.float().cpu().numpy()
            if bad:
                sub = [states[i] for i in bad]
                out[bad] = eng.evaluate(net.preprocessor.states_to_uint8(sub)).float().cpu().numpy()
            return out
        res = eng.evaluate(net.preprocessor.states_to_uint8(list(states)))
        return res.float().cpu().numpy() if hasattr(res, "cpu") else np.asarray(res)

    return fn


def engine_eval_fn(engine) -> EvalFn:
    """Adapter for the inference engines of ``models/inference.py`` (``evaluate`` returns a
    device tensor view of the bucket's outputs): copy the rows to host numpy."""

    def fn(planes, legal):
        out = engine.evaluate(planes, legal)
        return out.float().cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)

    return fn


def latency_summary(lat_s: List[float]) -> Tuple[float, float, float]:
    """(p50, p99, max) in milliseconds."""
    if not lat_s:
        return 0.0, 0.0, 0.0
    a = np.sort(np.asarray(lat_s)) * 1e3
    return float(np.percentile(a, 50)), float(np.percentile(a, 99)), float(a[-1])


class BatcherPool(object):
    """Several batchers (typically one per GPU of a node, each owning that GPU's engine) behind
    one ``submit``: a request goes to the batcher with the fewest queued boards, so load spreads
    over the devices while each batcher still forms its own rounds.  ``evaluate`` / ``submit`` /
    ``submit_items`` / ``stats`` / ``close`` mirror ``BatchingEvaluator``."""

    def __init__(self, batchers: List[BatchingEvaluator]):
        if not batchers:
            raise ValueError("BatcherPool needs at least one batcher")
        self.batchers = list(batchers)
        self._rr = 0
        self._lock = threading.Lock()

    def _pick(self) -> BatchingEvaluator:
        with self._lock:
            self._rr = (self._rr + 1) % len(self.batchers)
            order = self.batchers[self._rr:] + self.batchers[:self._rr]  # rotate: ties spread round-robin
        return min(order, key=lambda b: b._rows)

    def submit(self, planes, legal=None) -> Future:
        return self._pick().submit(planes, legal)

    def submit_items(self, items: list) -> Future:
        return self._pick().submit_items(items)

    def evaluate(self, planes, legal=None, timeout: Optional[float] = None) -> np.ndarray:
        return self._pick().evaluate(planes, legal, timeout)

    def stats(self) -> Dict[str, float]:
        per = [b.stats() for b in self.batchers]
        out: Dict[str, float] = {k: sum(s[k] for s in per) for k in ("requests", "boards", "rounds", "errors",
                                                                     "queued_boards")}
        out["mean_batch"] = out["boards"] / out["rounds"] if out["rounds"] else 0.0
        out["per_device_boards"] = [s["boards"] for s in per]  # type: ignore[assignment]
        return out

    def close(self, timeout: float = 10.0) -> None:
        for b in self.batchers:
            b.close(timeout)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
