"""Rank launcher: make ``--gpus N`` mean N ranks however a program is started.

The driver contract (and the reference's single-process trainers,
/root/reference/AlphaGo/training/supervised_policy_trainer.py:207-213) leaves two ways to start a
multi-GPU job here: under ``torch.distributed.run`` (one process per GPU, WORLD_SIZE set by the
launcher) or as a plain ``python bench.py --gpus N``.  Before round 6 the second form silently ran
one rank and labelled the result ``n_gpus: 1``.  ``ensure_ranks`` closes that hole:

* ``WORLD_SIZE`` unset and ``--gpus N > 1``: the calling process becomes a pure supervisor.  It never
  touches the GPU (``torch.cuda.device_count`` does not initialise HIP on this image), starts
  ``torch.distributed.run --nproc-per-node N`` as a child process (never ``exec``: replacing a process
  is forbidden once anything could have initialised the GPU, and the supervisor keeps the exit code),
  lets the ranks write to the inherited stdout / stderr (rank 0 prints the one result line), and
  returns the worst child exit code.
* ``WORLD_SIZE`` set and different from ``--gpus``, or fewer than N GPUs visible for a GPU backend:
  refuse with a clear message instead of measuring something other than what was asked for.
* otherwise (``--gpus`` equals the launched world, or N = 1): run in-process.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
from typing import List, Optional, Sequence


class LaunchError(SystemExit):
    """A launch that would measure or train something other than what was asked for (exit code 2)."""

    def __init__(self, msg: str):
        sys.stderr.write("alphago_amd launch error: %s\n" % msg)
        super().__init__(2)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """Device count without initialising the GPU runtime in this process."""
    import torch
    try:
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001 -- no usable runtime means no GPUs
        return 0


def ensure_ranks(gpus: int, target: Sequence[str], argv: Sequence[str], require_gpu: bool = True,
                 module: bool = False) -> Optional[int]:
    """Reconcile ``--gpus`` with the launch environment.

    ``target``/``module``: what each rank runs -- a script path (``module=False``) or a module name plus
    its leading arguments (``module=True``, e.g. ``["alphago_amd", "train-sl"]``); ``argv`` is the
    rest of the command line, passed unchanged to every rank (it still says ``--gpus N``, which then
    matches the launched world).  ``require_gpu``: N ranks need N visible GPUs; without it (the CPU
    ``torch`` backend) a box with no GPU runs the N ranks on gloo.

    Returns None when the caller should run in-process, else the supervisor's exit code."""
    if gpus < 1:
        raise LaunchError("--gpus must be >= 1 (got %d)" % gpus)
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise LaunchError("--gpus %d but the launcher started WORLD_SIZE=%s ranks; refusing to measure a "
                              "different world than the one asked for" % (gpus, ws))
        return None
    if gpus == 1:
        return None
    n_vis = visible_gpus()
    if n_vis < gpus and (require_gpu or n_vis > 0):
        raise LaunchError("--gpus %d but only %d GPU(s) are visible" % (gpus, n_vis))
    cmd: List[str] = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
                      "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    if module:
        cmd += ["-m", target[0]] + list(target[1:])
    else:
        cmd += list(target)
    cmd += list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = os.pathsep.join([root] + [x for x in [env.get("PYTHONPATH")] if x])
    sys.stdout.flush()
    sys.stderr.flush()
    p = subprocess.Popen(cmd, env=env)

    def forward(signum, frame):  # a supervisor stopped by its caller stops the launcher (which stops the ranks)
        if p.poll() is None:
            p.send_signal(signum)

    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        rc = p.wait()
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
    return int(rc) if rc >= 0 else 128 - int(rc)


class ExitCode(int):
    """A process exit code returned by a command (``cli.main`` returns it as the status; a command's
    other return values, e.g. a position count, are results, not exit codes)."""


def exit_status(result) -> int:
    """The process status of a command's return value: an ``ExitCode`` as is, any other result 0."""
    return int(result) if isinstance(result, ExitCode) else 0


def add_gpus_arg(p) -> None:
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                   help="ranks (one per GPU); without torchrun the command starts them itself "
                        "(alphago_amd/parallel/launch.py)")


def cli_ranks(cmd: str, args, argv: Sequence[str]) -> Optional[ExitCode]:
    """``ensure_ranks`` for an ``alphago_amd <cmd>`` command: the ranks run ``python -m alphago_amd
    <cmd> argv``.  A GPU is required only for ``--backend hip``; ``auto`` on a box without GPUs runs
    the ranks on the CPU (gloo)."""
    code = ensure_ranks(args.gpus, ["alphago_amd", cmd], list(argv),
                        require_gpu=getattr(args, "backend", "auto") == "hip", module=True)
    return None if code is None else ExitCode(code)
