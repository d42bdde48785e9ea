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


class StepMetrics(object):
    """Per-step training records (SURVEY.md §5 metrics row): every ``every`` steps, one JSONL
    record with the window's loss and top-1 accuracy (all-reduced over ranks), positions/s,
    model TFLOP/s, the peak HBM allocation (max over ranks) and, for the HIP trainer, the
    exposed gradient all-reduce time: how long the compute stream waited for RCCL after the
    last backward kernel, per step.  Every rank must call :meth:`on_step` for every step
    (the flush is a collective); only the logger of rank 0 writes."""

    def __init__(self, log: MetricsLogger, every: int, global_batch: int, flops_per_position: float,
                 device, trainer=None):
        import torch

        self.log, self.every, self.global_batch = log, int(every), global_batch
        self.flops = flops_per_position
        self.device = device
        self.trainer = trainer
        self.sums = torch.zeros(2, device=device, dtype=torch.float64)
        self.n = 0
        self.t0 = time.perf_counter()
        if trainer is not None and self.every > 0 and hasattr(trainer, "comm_events"):
            trainer.comm_events = []  # the trainer records (start, end) events around its all-reduce wait

    def on_step(self, gstep: int, epoch: int, loss, correct) -> None:
        if self.every <= 0:
            return
        self.sums[0] += loss.double()
        self.sums[1] += correct.double()
        self.n += 1
        if (gstep + 1) % self.every == 0:
            self.flush(gstep + 1, epoch)

    def flush(self, step: int, epoch: int) -> None:
        import torch

        from ..parallel import dist as agdist

        if self.n == 0:
            return
        stats = self.sums.clone()
        agdist.all_reduce_sum_(stats)  # also syncs the window's work
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - self.t0
        seen = self.n * self.global_batch
        hbm = torch.cuda.max_memory_allocated(self.device) / 1e9 if self.device.type == "cuda" else 0.0
        hbm = agdist.all_reduce_max(hbm)
        rec = {"step": step, "epoch": epoch, "loss": float(stats[0]) / seen, "acc": float(stats[1]) / seen,
               "positions_per_s": seen / dt, "tflops": self.flops * 3 * seen / dt / 1e12, "hbm_gb": round(hbm, 3),
               "world": agdist.env().world_size}
        comm = self.take_comm_ms()
        if comm is not None:
            rec["allreduce_exposed_ms_per_step"] = agdist.all_reduce_max(comm / self.n)
        self.log.log(**rec)
        self.sums.zero_()
        self.n = 0
        self.t0 = time.perf_counter()

    def take_comm_ms(self) -> Optional[float]:
        ev = getattr(self.trainer, "comm_events", None) if self.trainer is not None else None
        if ev is None:
            return None
        ms = sum(a.elapsed_time(b) for a, b in ev)
        ev.clear()
        return ms
