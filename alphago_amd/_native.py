"""Loader for the in-tree native extensions (built by ``alphago_amd._build``).

The engine (`_engine`) is CPU C++ and is built on demand if missing, so a
fresh checkout works without an explicit build step.  The HIP kernel library is
loaded by :mod:`alphago_amd.ops` (it needs torch).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_engine = None


def engine():
    global _engine
    if _engine is not None:
        return _engine
    with _lock:
        if _engine is None:
            from . import _build

            if not os.path.exists(_build.engine_path()) or os.environ.get("ALPHAGO_AMD_REBUILD"):
                _build.build_engine()
            _engine = importlib.import_module("alphago_amd._engine")
    return _engine
