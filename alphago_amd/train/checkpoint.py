"""Native training checkpoints (SURVEY.md §5 "Checkpoint / resume", Q16).

The reference saved only Keras weights per epoch (ModelCheckpoint,
supervised_policy_trainer.py:161-162) and lost the optimizer iteration count
and data position on resume.  A native checkpoint holds everything needed to
continue *bit-identically* (in a deterministic configuration):

* the flat fp32 master parameters (``trainer.fp.flat``);
* the Keras-SGD iteration count (drives ``lr/(1+decay*t)``) and the optimizer state (momentum
  velocity / Adam moments) when the optimizer keeps one;
* the data cursor, epoch and step-within-epoch, partial epoch sums;
* the augmentation RNG state;
* the run configuration (argparse namespace as a dict) for provenance.

Written by rank 0 with tmp + ``os.replace`` (atomic on POSIX); read back with
``torch.load(weights_only=True)`` — only tensors and plain containers.
The Keras-format ``weights.%05d.hdf5`` export is separate (io/keras_compat).
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch

FORMAT = "alphago_amd.ckpt.v1"


def trainer_state(trainer) -> Dict[str, Any]:
    st = {"flat": trainer.fp.flat.detach().to("cpu", copy=True),
          "names": list(trainer.fp.names),
          "iterations": int(trainer.sched.iterations)}
    sched = trainer.sched
    st["optimizer"] = sched.optimizer
    st["hyper"] = optimizer_hyper(sched)
    opt = getattr(trainer, "opt_state", None)
    if opt:  # momentum velocity / Adam moments
        st["opt_state"] = [t.detach().to("cpu", copy=True) for t in opt]
    return st


def optimizer_hyper(sched) -> Dict[str, float]:
    """The optimizer hyperparameters a resume must keep (the moments are only meaningful under them)."""
    return {"momentum": float(sched.momentum), "nesterov": float(bool(sched.nesterov)),
            "beta_1": float(sched.beta_1), "beta_2": float(sched.beta_2), "epsilon": float(sched.epsilon)}


def load_trainer_state(trainer, st: Dict[str, Any]) -> None:
    flat = st["flat"]
    if list(st["names"]) != list(trainer.fp.names) or flat.numel() != trainer.fp.flat.numel():
        raise ValueError("checkpoint parameters do not match this model")
    with torch.no_grad():
        trainer.fp.flat.copy_(flat.to(trainer.fp.flat.device))
    trainer.sched.iterations = int(st["iterations"])
    opt = getattr(trainer, "opt_state", None) or []
    saved = st.get("opt_state", [])
    if "optimizer" in st and st["optimizer"] != trainer.sched.optimizer:
        # e.g. an Adam checkpoint resumed by an SGD trainer would silently drop its moments
        raise ValueError("checkpoint optimizer %r != this trainer's %r" % (st["optimizer"], trainer.sched.optimizer))
    if len(saved) != len(opt):
        raise ValueError("checkpoint holds %d optimizer state buffers, this trainer keeps %d" % (len(saved), len(opt)))
    if "hyper" in st:
        mine = optimizer_hyper(trainer.sched)
        diff = {k: (v, mine[k]) for k, v in st["hyper"].items() if k in mine and abs(v - mine[k]) > 1e-12}
        if diff:
            raise ValueError("resume with different optimizer hyperparameters (saved, now): %s" % diff)
    if opt:
        with torch.no_grad():
            for dst, src in zip(opt, st["opt_state"]):
                dst.copy_(src.to(dst.device))
    if hasattr(trainer, "sync_schedule"):
        trainer.sync_schedule()  # graph replays read the schedule from the device
    if hasattr(trainer, "repack"):
        trainer.repack()


def save(path: str, trainer, **extra) -> None:
    state = {"format": FORMAT, "trainer": trainer_state(trainer)}
    for k, v in extra.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().to("cpu", copy=True)
        state[k] = v
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load(path: str) -> Optional[Dict[str, Any]]:
    if not os.path.exists(path):
        return None
    st = torch.load(path, map_location="cpu", weights_only=True)
    if st.get("format") != FORMAT:
        return {"legacy": st}
    return st
