"""Fault injection for recovery tests (SURVEY.md §5 "fault-injection hooks").

``ALPHAGO_AMD_FAULT="<kind>@<step>[:rank<r>][:once=<marker file>]"`` makes
``maybe_inject(step, rank)`` fail at that global step:

* ``exit``  — ``os._exit(13)`` (a crashed rank; torchrun restarts the group);
* ``raise`` — raise ``InjectedFault`` (Python-level failure);
* ``hang``  — sleep forever (exercises the watchdog / collective timeouts).

With ``once=<file>`` the fault fires only if the marker file does not exist
yet (it is created just before firing), so a restarted job runs through.
"""
from __future__ import annotations

import os
import time
from typing import Optional


class InjectedFault(RuntimeError):
    pass


def parse(spec: Optional[str]):
    if not spec:
        return None
    head, *opts = spec.split(":")
    kind, _, step = head.partition("@")
    out = {"kind": kind, "step": int(step), "rank": None, "once": None}
    for o in opts:
        if o.startswith("rank"):
            out["rank"] = int(o[4:])
        elif o.startswith("once="):
            out["once"] = o[5:]
    if out["kind"] not in ("exit", "raise", "hang"):
        raise ValueError("unknown fault kind %r" % kind)
    return out


_SPEC = parse(os.environ.get("ALPHAGO_AMD_FAULT"))


def maybe_inject(step: int, rank: int = 0) -> None:
    f = _SPEC
    if f is None or step != f["step"] or (f["rank"] is not None and rank != f["rank"]):
        return
    if f["once"]:
        if os.path.exists(f["once"]):
            return
        with open(f["once"], "w") as fh:
            fh.write("fired at step %d rank %d\n" % (step, rank))
    if f["kind"] == "exit":
        os._exit(13)
    if f["kind"] == "raise":
        raise InjectedFault("injected fault at step %d (rank %d)" % (step, rank))
    while True:  # hang
        time.sleep(3600)


def reload_from_env() -> None:
    global _SPEC
    _SPEC = parse(os.environ.get("ALPHAGO_AMD_FAULT"))
