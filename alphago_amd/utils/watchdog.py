"""Failure detection: per-rank heartbeats and a hang watchdog.

The reference has none.  A training process calls ``Watchdog.beat(step)``
once per step.  The watchdog thread

* rewrites ``<dir>/heartbeat.rank<r>.json`` ({rank, step, time, pid}) every
  ``interval`` seconds, so an external supervisor can see which rank stalled;
* if no beat arrives for ``timeout`` seconds (a hung collective, a wedged
  kernel, a dead peer) it dumps every Python thread's stack to
  ``<dir>/hang.rank<r>.txt`` and exits the process with ``exit_code``.

Exiting makes ``torchrun --max-restarts N`` tear the group down and restart
it; the trainers then resume from their last native checkpoint
(``--resume auto``).  RCCL-side hangs are also bounded by the process-group
timeout passed to ``init_process_group`` (parallel/dist.py) with
``TORCH_NCCL_ASYNC_ERROR_HANDLING=1`` set by ``enable_collective_timeouts``.
"""
from __future__ import annotations

import faulthandler
import json
import os
import sys
import threading
import time
from typing import Optional


def enable_collective_timeouts() -> None:
    """Abort (instead of hanging) when an RCCL collective times out."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "0")


class Watchdog(object):
    def __init__(self, out_dir: Optional[str], rank: int = 0, timeout: float = 900.0, interval: float = 10.0,
                 exit_code: int = 75):
        self.out_dir, self.rank = out_dir, rank
        self.timeout, self.interval, self.exit_code = timeout, interval, exit_code
        self.step = -1
        self.last = time.monotonic()
        self.fired = False
        self._stop = threading.Event()
        self._th = None
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)

    def start(self) -> "Watchdog":
        if self._th is None and self.timeout > 0:
            self._th = threading.Thread(target=self._run, name="alphago-watchdog", daemon=True)
            self._th.start()
        return self

    def beat(self, step: int) -> None:
        self.step = step
        self.last = time.monotonic()

    def _write_heartbeat(self):
        if not self.out_dir:
            return
        path = os.path.join(self.out_dir, "heartbeat.rank%d.json" % self.rank)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"rank": self.rank, "step": self.step, "time": time.time(), "pid": os.getpid()}, f)
        os.replace(tmp, path)

    def _fire(self):
        self.fired = True
        msg = "watchdog: rank %d made no progress for %.0fs after step %d" % (self.rank, self.timeout, self.step)
        sys.stderr.write(msg + "\n")
        if self.out_dir:
            with open(os.path.join(self.out_dir, "hang.rank%d.txt" % self.rank), "w") as f:
                f.write(msg + "\n")
                faulthandler.dump_traceback(file=f, all_threads=True)
        else:
            faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(self.exit_code)

    def _run(self):
        while not self._stop.wait(min(self.interval, max(0.05, self.timeout / 4))):
            try:
                self._write_heartbeat()
            except OSError:
                pass
            if time.monotonic() - self.last > self.timeout:
                self._fire()
                return

    def stop(self) -> None:
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=5)
            self._th = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False
