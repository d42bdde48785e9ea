"""Tracing / profiling (SURVEY.md §5 "Tracing / profiling").

The reference only ran ``cProfile`` over a converter call
(benchmarks/preprocessing_benchmark.py:2-16).  Here:

* ``trace_range(name)`` marks a region for both the torch profiler
  (``record_function``) and rocprofv3 (roctx range via ``torch.cuda.nvtx``,
  which is roctx on ROCm builds); it costs two no-op calls when neither tool
  is active.  The SL step brackets featurize/pack, forward, head, backward,
  all-reduce and optimizer with it.
* ``Profiler`` wraps ``torch.profiler`` for a ``--profile DIR`` flag: a
  wait/warmup/active schedule, a Chrome trace per active window and a
  per-kernel summary table (``summary.txt``) sorted by device time.
* Kernel-level counters come from rocprofv3 (``scripts/profile_step.sh``,
  ``scripts/pmc_conv.sh``); committed summaries live in ``profiles/``.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Optional

import torch

_ENABLED = os.environ.get("ALPHAGO_AMD_TRACE", "1") != "0"


def _roctx():
    try:
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # noqa: BLE001
        pass
    return None


_RX = None


@contextmanager
def trace_range(name: str):
    """Named region visible in torch.profiler traces and rocprofv3 marker traces."""
    global _RX
    if not _ENABLED:
        yield
        return
    if _RX is None:
        _RX = _roctx() or False
    pushed = False
    if _RX:
        try:
            _RX.range_push(name)
            pushed = True
        except Exception:  # noqa: BLE001 - roctx missing in this build
            _RX = False
    with torch.profiler.record_function(name):
        yield
    if pushed:
        _RX.range_pop()


class Profiler(object):
    """``with Profiler(dir) as prof: ... prof.step()`` — no-op when dir is None."""

    def __init__(self, out_dir: Optional[str], wait: int = 1, warmup: int = 2, active: int = 3,
                 record_shapes: bool = False):
        self.out_dir = out_dir
        self._p = None
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._p = torch.profiler.profile(
                activities=acts,
                schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=active, repeat=1),
                on_trace_ready=self._ready,
                record_shapes=record_shapes)

    def _ready(self, p):
        rank = int(os.environ.get("RANK", "0"))
        p.export_chrome_trace(os.path.join(self.out_dir, "trace_rank%d_%d.json" % (rank, p.step_num)))
        key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        try:
            table = p.key_averages().table(sort_by=key, row_limit=40)
        except Exception:  # noqa: BLE001 - older/newer key names
            table = p.key_averages().table(row_limit=40)
        with open(os.path.join(self.out_dir, "summary_rank%d.txt" % rank), "w") as f:
            f.write(table)

    def __enter__(self):
        if self._p is not None:
            self._p.__enter__()
        return self

    def __exit__(self, *exc):
        if self._p is not None:
            self._p.__exit__(*exc)
        return False

    def step(self):
        if self._p is not None:
            self._p.step()
