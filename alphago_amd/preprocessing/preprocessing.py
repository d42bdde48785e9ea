"""Reference module path ``AlphaGo.preprocessing.preprocessing``.

``Preprocess`` / ``FEATURES`` / ``DEFAULT_FEATURES`` come from
``alphago_amd.features`` (native C++ featurizer).  The per-feature functions
(preprocessing.py:9-161) are provided with the reference signatures: each
returns the ``(planes, S, S)`` one-hot array of one feature family for one
state.  ``maximum`` (the plane count of the 8-plane families) may be 1..8;
planes at or beyond ``maximum - 1`` fold into the last one, which is what the
reference computes with a smaller ``maximum``.  The ladder planes, which the
reference leaves unimplemented (:147-152), are computed natively.
"""
import numpy as np

from ..features import DEFAULT_FEATURES, FEATURES, Preprocess
from .._native import engine as _engine


def _planes(state, name: str) -> np.ndarray:
    return np.asarray(_engine().featurize(state, [name]), dtype=np.float64)


def _capped(state, name: str, maximum: int) -> np.ndarray:
    if not 1 <= maximum <= 8:
        raise ValueError("maximum must be in 1..8 (native planes are computed with 8)")
    p = _planes(state, name)
    if maximum == 8:
        return p
    out = p[:maximum].copy()
    out[maximum - 1] = p[maximum - 1:].max(axis=0)
    return out


def get_board(state):
    return _planes(state, "board")


def get_turns_since(state, maximum=8):
    return _capped(state, "turns_since", maximum)


def get_liberties(state, maximum=8):
    return _capped(state, "liberties", maximum)


def get_capture_size(state, maximum=8):
    return _capped(state, "capture_size", maximum)


def get_self_atari_size(state, maximum=8):
    return _capped(state, "self_atari_size", maximum)


def get_liberties_after(state, maximum=8):
    return _capped(state, "liberties_after", maximum)


def get_ladder_capture(state):
    return _planes(state, "ladder_capture")


def get_ladder_escape(state):
    return _planes(state, "ladder_escape")


def get_sensibleness(state):
    return _planes(state, "sensibleness")


__all__ = ["Preprocess", "FEATURES", "DEFAULT_FEATURES", "get_board", "get_turns_since", "get_liberties",
           "get_capture_size", "get_self_atari_size", "get_liberties_after", "get_ladder_capture",
           "get_ladder_escape", "get_sensibleness"]
