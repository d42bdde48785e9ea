"""Batched board featurization on the GPU.

The reference featurizes one board at a time in numpy
(AlphaGo/preprocessing/preprocessing.py:217-245, ~265 positions/s).  Here the
C++ engine writes a ~2-byte-per-point encoding of each board (stones, move
ages, ko, side to move) and ``featurize_kernel`` expands it on the device —
chain labelling, liberty sets, legality, capture/self-atari/liberties-after
and the recursive true-eye test — into uint8 planes, or straight into the
conv trunk's padded NHWC bf16 input together with the sensible-move mask.
Ladder planes (a tree search per candidate point; NotImplementedError in the
reference, preprocessing.py:147-152) come from the host encoder by default:
its incremental-liberty reader is several times faster than the device
reader ``ladder_planes`` (csrc/kernels/ladder.hip, bit-identical), because a
ladder search is one long serial chain of dependent board updates
(profiles/r2_gpu_ladders.md).  ``gpu_ladders=True`` reads them on the device.

Boards whose eye recursion is deeper than the kernel's frame stack (only
pathological positions such as a full-board checkerboard) are flagged and
recomputed on the CPU, so results always equal ``Preprocess``'s.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from .. import ops
from .._native import engine as _engine
from ..features import FEATURES

# feature ids, same numbering as csrc/engine/featurize.h (FeatureId)
FEATURE_IDS = {name: i for i, name in enumerate(
    ["board", "ones", "turns_since", "liberties", "capture_size", "self_atari_size", "liberties_after",
     "ladder_capture", "ladder_escape", "sensibleness", "zeros", "color", "legal"])}
LADDER_FEATURES = ("ladder_capture", "ladder_escape")


class GpuFeaturizer(object):
    def __init__(self, feature_list: Sequence[str], board: int = 19, device="cuda", threads: int = 8,
                 gpu_ladders: bool = False):
        self.features = [f.lower() for f in feature_list]
        for f in self.features:
            if f not in FEATURE_IDS:
                raise ValueError("unknown feature: %s" % f if f not in FEATURES
                                 else "feature %s is computed by the CPU featurizer only" % f)
        self.fids = [FEATURE_IDS[f] for f in self.features]
        self.fplanes = [FEATURES[f]["size"] for f in self.features]
        self.nplanes = sum(self.fplanes)
        if self.nplanes > 64:
            raise ValueError("GPU featurizer supports at most 64 planes")
        self.need_ladder = any(f in LADDER_FEATURES for f in self.features)
        self.gpu_ladders = gpu_ladders
        self.S = board
        self.device = torch.device(device)
        self.threads = threads
        self._E = _engine()
        ops.load()

    @property
    def host_needs_ladder(self) -> bool:
        """Whether the host encoder must supply ladder bits (GPU ladders off)."""
        return self.need_ladder and not self.gpu_ladders

    # ------------------------------------------------------------ host side
    def encode(self, states):
        """numpy (board int8 (B,S*S), ages uint8, meta int32 (B,2), ladder uint8 or None)."""
        return self._E.encode_batch(list(states), self.host_needs_ladder, self.threads)

    def to_device(self, enc):
        b, a, m, l = enc
        dev = self.device
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev, non_blocking=True)  # noqa: E731
        return t(b), t(a), t(m), (t(l) if l is not None else None)

    # ------------------------------------------------------------ device side
    def run(self, board, ages, meta, ladder=None, planes=None, nhwc=None, P: int = 0, sensible=None, legal=None,
            overflow=None):
        """With GPU ladders, ``ladder`` (a (B, S*S) uint8 buffer, or None) is
        written on the device from ``board``/``meta`` before featurising."""
        if self.need_ladder and self.gpu_ladders:
            if ladder is None:
                ladder = torch.empty(board.shape, dtype=torch.uint8, device=board.device)
            ops.ladder_planes(board, meta, ladder, self.S)
            if overflow is not None:  # bit 2: search budget exhausted -> recompute on the CPU
                overflow |= (ladder & 4).amax(1).to(overflow.dtype)
        ops.featurize(board, ages, meta, self.fids, self.fplanes, self.S, ladder=ladder, planes=planes, nhwc=nhwc,
                      P=P, sensible=sensible, legal=legal, overflow=overflow)

    @torch.no_grad()
    def planes(self, states, with_sensible: bool = False):
        """(B, F, S, S) uint8 planes on the device (and the (B, S*S) sensible mask)."""
        states = list(states)
        B, NP = len(states), self.S * self.S
        dev = self.device
        board, ages, meta, ladder = self.to_device(self.encode(states))
        out = torch.empty((B, self.nplanes, self.S, self.S), dtype=torch.uint8, device=dev)
        sens = torch.empty((B, NP), dtype=torch.uint8, device=dev) if with_sensible else None
        ovf = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.run(board, ages, meta, ladder, planes=out, sensible=sens, overflow=ovf)
        self._fix_overflow(states, ovf, out, sens)
        return (out, sens) if with_sensible else out

    def _fix_overflow(self, states, ovf, out=None, sens=None):
        bad = torch.nonzero(ovf).flatten().tolist()
        for i in bad:
            s = states[i]
            if out is not None:
                out[i].copy_(torch.from_numpy(self._E.featurize(s, self.features)))
            if sens is not None:
                m = self._E.featurize(s, ["sensibleness"]).reshape(-1)
                sens[i].copy_(torch.from_numpy(m))
        return bad
