"""Load the reference implementation as a *test oracle* (differential tests).

The reference (/root/reference, Python 2 + Keras 1) is imported read-only from
its own files at test time, with minimal textual Python-3 shims applied in
memory (filter -> list, np.int -> int).  Nothing from it is copied into this
repository.  Tests that use it are skipped where the reference is absent
(e.g. on the GPU box).
"""
import os
import types

import numpy as np

REF = os.environ.get("ALPHAGO_REFERENCE", "/root/reference")


def available():
    return os.path.exists(os.path.join(REF, "AlphaGo", "go.py"))


def _load(name, relpath, extra_globals=None, shims=()):
    with open(os.path.join(REF, relpath)) as f:
        src = f.read()
    for a, b in shims:
        src = src.replace(a, b)
    mod = types.ModuleType(name)
    mod.__dict__.update(extra_globals or {})
    exec(compile(src, os.path.join(REF, relpath), "exec"), mod.__dict__)
    return mod


_cache = {}


def ref_go():
    if "go" not in _cache:
        _cache["go"] = _load(
            "ref_go", "AlphaGo/go.py",
            shims=[("return filter(self._on_board,", "return list(filter(self._on_board,"),
                   ("(x - 1, y + 1)])", "(x - 1, y + 1)]))"),
                   ("(x, y + 1)])", "(x, y + 1)]))"),
                   ("dtype=np.int)", "dtype=int)")])
    return _cache["go"]


def ref_preprocessing():
    if "pp" not in _cache:
        go = ref_go()
        import sys
        pkg = types.ModuleType("AlphaGo")
        pkg.go = go
        saved = {k: sys.modules.get(k) for k in ("AlphaGo", "AlphaGo.go")}
        sys.modules["AlphaGo"] = pkg
        sys.modules["AlphaGo.go"] = go
        try:
            _cache["pp"] = _load("ref_pp", "AlphaGo/preprocessing/preprocessing.py")
        finally:
            for k, v in saved.items():
                if v is None:
                    sys.modules.pop(k, None)
                else:
                    sys.modules[k] = v
    return _cache["pp"]
