"""Board featurizer: named feature planes -> one-hot tensors.

Same registry names, plane counts and ordering as the reference
(AlphaGo/preprocessing/preprocessing.py:164-214), computed natively in C++
(``csrc/engine/featurize.cpp``) instead of per-feature numpy passes, plus:

* ``ladder_capture`` / ``ladder_escape`` are implemented (ladder reading in C++);
  the reference raises ``NotImplementedError`` (preprocessing.py:147-152).
* ``color`` — the value network's 49th plane (paper "player colour"; the
  reference declares 49 inputs in value.py:16 but has no such feature, Q18).
* ``legal`` — legal-move mask (used by search/players, not by the paper nets).
* ``liberties_after_exact`` / ``self_atari_size_exact`` — capture-aware versions of
  the reference planes, CPU featurizer only; the reference names keep
  the reference semantics bit-exactly.

A GPU featurizer (``alphago_amd.ops.featurize_gpu``) produces bit-identical
planes for batches of boards on the device.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np

from ._native import engine as _engine

FEATURES = {
    "board": {"size": 3},
    "ones": {"size": 1},
    "turns_since": {"size": 8},
    "liberties": {"size": 8},
    "capture_size": {"size": 8},
    "self_atari_size": {"size": 8},
    "liberties_after": {"size": 8},
    "ladder_capture": {"size": 1},
    "ladder_escape": {"size": 1},
    "sensibleness": {"size": 1},
    "zeros": {"size": 1},
    "color": {"size": 1},
    "legal": {"size": 1},
    # capture-aware variants (CPU featurizer only): liberties gained by
    # capturing count, so a legal move never lands on the "0 liberties -> plane 7" quirk
    "self_atari_size_exact": {"size": 8},
    "liberties_after_exact": {"size": 8},
}

# 48 planes, preprocessing.py:211-214
DEFAULT_FEATURES = [
    "board", "ones", "turns_since", "liberties", "capture_size",
    "self_atari_size", "liberties_after", "ladder_capture", "ladder_escape",
    "sensibleness", "zeros"]

# 46 planes: the converter's "all" (game_converter.py:166-178; no ladders)
ALL_NO_LADDER_FEATURES = [
    "board", "ones", "turns_since", "liberties", "capture_size",
    "self_atari_size", "liberties_after", "sensibleness", "zeros"]

# 49 planes: value network input (value.py:16)
VALUE_FEATURES = DEFAULT_FEATURES + ["color"]


def num_planes(feature_list: Iterable[str]) -> int:
    total = 0
    for f in feature_list:
        key = f.lower()
        if key not in FEATURES:
            raise ValueError("unknown feature: %s" % f)
        total += FEATURES[key]["size"]
    return total


class Preprocess(object):
    """Convert GameStates into one-hot feature tensors (preprocessing.py:217-245)."""

    def __init__(self, feature_list: Sequence[str] = DEFAULT_FEATURES):
        self.feature_list = list(feature_list)
        self._names = [f.lower() for f in self.feature_list]
        self.output_dim = num_planes(self._names)
        self._E = _engine()

    def state_to_uint8(self, state) -> np.ndarray:
        """(F, S, S) uint8 planes."""
        return self._E.featurize(state, self._names)

    def state_to_tensor(self, state) -> np.ndarray:
        """(1, F, S, S) float32 planes (reference returns float64 of the same values)."""
        return self.state_to_uint8(state)[None].astype(np.float32)

    def states_to_uint8(self, states: List, threads: int = 8) -> np.ndarray:
        """(B, F, S, S) uint8, featurised in parallel native threads."""
        return self._E.featurize_batch(list(states), self._names, threads)
