"""Structured metrics (JSONL) and simple timers.

The reference only printed under --verbose and kept Keras epoch logs
(SURVEY.md §5); here every logged record is one JSON line with a timestamp,
written by rank 0 only (after the all-reduce of the values it reports).
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager
from typing import Optional


class MetricsLogger(object):
    def __init__(self, path: Optional[str] = None):
        self.path = path
        self._fh = None
        if path:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._fh = open(path, "a")

    def log(self, **kv) -> None:
        if self._fh is None:
            return
        kv.setdefault("ts", time.time())
        self._fh.write(json.dumps(kv) + "\n")
        self._fh.flush()

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None


class Timer(object):
    def __init__(self):
        self.totals = {}

    @contextmanager
    def section(self, name: str, sync_cuda: bool = False):
        import torch

        if sync_cuda and torch.cuda.is_available():
            torch.cuda.synchronize()
        t = time.perf_counter()
        yield
        if sync_cuda and torch.cuda.is_available():
            torch.cuda.synchronize()
        self.totals[name] = self.totals.get(name, 0.0) + time.perf_counter() - t
