"""Self-play records -> SL training data: the consumer of the MCTS visit distributions.

``selfplay-mcts`` (search/selfplay_mcts.py) writes ``states`` (the value net's 49 planes), ``pi`` (the
root visit distribution per searched position, S*S + 1 with the pass last), ``moves``, ``outcomes`` and
``game``.  ``train-value`` reads ``states`` + ``outcomes`` directly.  This module turns the same file
into the SL trainer's schema (converter output: ``states`` with the policy's 48 planes -- the value
planes minus the trailing ``color`` plane, features.VALUE_FEATURES = DEFAULT_FEATURES + ["color"] --
and ``actions`` (N, 2)), so ``train-sl`` can fit the policy to the search: the target of each
position is the most-visited move (``--target pi``, the search's improved policy) or the move the
game played (``--target played``).  Positions whose target is a pass are dropped (the SL policy has
no pass output, reference policy.py:132-154).

    python -m alphago_amd selfplay-to-sl run/selfplay.h5 sl_from_search.h5 [--target pi|played]
"""
from __future__ import annotations

import argparse
import json
import os
from typing import List, Optional

import numpy as np

from ..features import DEFAULT_FEATURES
from ..io.h5lite import H5File, H5Writer

_CHUNK = 4096


def selfplay_to_sl(src: str, dst: str, target: str = "pi") -> dict:
    """Write ``dst`` (SL schema) from the self-play file ``src``; returns counts."""
    if target not in ("pi", "played"):
        raise ValueError("target must be 'pi' or 'played'")
    with H5File(src) as f:
        feats = [x.decode() if isinstance(x, bytes) else str(x) for x in np.asarray(f.attrs["features"]).tolist()]
        size = int(np.asarray(f.attrs["board_size"]))
        ds = f["states"]
        n, C = ds.shape[0], ds.shape[1]
        n_policy = C - 1 if feats and feats[-1] == "color" else C
        if feats[:len(DEFAULT_FEATURES)] != list(DEFAULT_FEATURES) or n_policy != 48:
            raise ValueError("self-play planes %s are not the value features (policy planes + color)" % feats)
        if target == "pi":
            pi = np.asarray(f["pi"].read())
            idx = pi.argmax(1)
        else:
            idx = np.asarray(f["moves"].read()).astype(np.int64)
            idx = np.where(idx < 0, size * size, idx)
        keep = np.flatnonzero(idx < size * size)  # drop pass targets
        tmp = dst + ".tmp"
        with H5Writer(tmp) as w:
            w.attrs["features"] = np.array([x.encode() for x in DEFAULT_FEATURES])
            w.attrs["board_size"] = np.int64(size)
            w.attrs["source"] = np.array([("selfplay-to-sl:%s:%s" % (os.path.basename(src), target)).encode()])
            out = w.stream_dataset("states", (n_policy, size, size), np.uint8)
            for s in range(0, len(keep), _CHUNK):
                rows = keep[s:s + _CHUNK]
                out.append(np.ascontiguousarray(np.asarray(ds.rows(rows))[:, :n_policy]))
            out.finish()
            acts = np.stack([idx[keep] // size, idx[keep] % size], axis=1).astype(np.uint8)
            w.create_dataset("actions", data=acts)
    os.replace(tmp, dst)
    return {"positions": int(n), "written": int(len(keep)), "dropped_pass": int(n - len(keep)), "target": target}


def selfplay_to_sl_cli(argv: Optional[List[str]] = None) -> dict:
    p = argparse.ArgumentParser(prog="selfplay-to-sl", description=__doc__.split("\n\n")[0])
    p.add_argument("selfplay_h5")
    p.add_argument("out_h5")
    p.add_argument("--target", default="pi", choices=["pi", "played"])
    a = p.parse_args(argv)
    res = selfplay_to_sl(a.selfplay_h5, a.out_h5, a.target)
    print(json.dumps(res))
    return res
