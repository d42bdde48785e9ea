"""Vectorised self-play: many games advanced in lock-step, one batched forward per side per ply.

``BatchedSampler.select(states)`` encodes all states compactly in native
threads and runs ONE policy forward whose graph featurises on the device and
builds the sensible-move masks (legal and not filling an own eye, ai.py:15)
that the fused head kernel applies; then samples p**(1/T) (or argmax) on the
device.  When the caller needs the planes (RL training records) or the engine
has no encoded path (CPU), planes are featurised natively on the host.  This replaces the
reference's per-state Python move lists and CPU renormalisation
(ai.py:51-68, policy.py:44-79).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from .. import go
from .._native import engine as _engine


class BatchedSampler(object):
    def __init__(self, policy, temperature: float = 1.0, greedy: bool = False, seed: int = 0, threads: int = 8):
        self.policy = policy
        self.beta = 1.0 / temperature if temperature > 0 else 1.0
        self.greedy = greedy or temperature <= 0
        self.threads = threads
        self._names = [f.lower() for f in policy.preprocessor.feature_list]
        self.gen = torch.Generator(device=policy.device)
        self._bad: List[int] = []
        self.gen.manual_seed(seed)
        # HIP engines: one fused sampling kernel per call (ops.sample_moves), its uniforms from a
        # counter-based hash of (seed, call, board)
        self._fused = None  # resolved at the first sample (the engine is built lazily)
        self._calls = int(seed) * 1000003

    def featurize(self, states) -> np.ndarray:
        return _engine().featurize_batch(list(states), self._names, self.threads)

    def masks(self, states) -> np.ndarray:
        m = _engine().featurize_batch(list(states), ["sensibleness"], self.threads)
        return m.reshape(len(states), -1)

    def _probs_encoded(self, states, eng, want_planes: bool = False):
        E = _engine()
        b, a, m, l = E.encode_batch(list(states), eng.needs_ladder, self.threads)
        probs, sens, bad = eng.evaluate_encoded(b, a, m, l)
        self._bad = list(bad)
        self._enc_planes = None
        if want_planes:
            # the featurizer's output rows; the fallback evaluation below may reuse the same bucket
            # buffers, so they are copied out first when it runs
            self._enc_planes = eng.encoded_planes_view(len(states))
            if bad:
                self._enc_planes = self._enc_planes.clone()
        if bad:  # eye recursion too deep for the kernel: recompute those rows from CPU planes
            sub = [states[i] for i in bad]
            masks = self.masks(sub)
            probs = probs.clone()
            sens = sens.clone()
            probs[bad] = eng.evaluate(self.featurize(sub), masks).to(probs.dtype)
            sens[bad] = torch.from_numpy(masks).to(sens.device)
        return probs, (sens != 0).any(1)

    def sample_device(self, probs: torch.Tensor, has: torch.Tensor) -> torch.Tensor:
        """Flat move per board on the probs' device: argmax, or a sample of p**(1/T) (ai.py:37-49);
        -1 (pass) where no sensible move exists.  No host synchronisation."""
        if self._fused is None:
            self._fused = bool(getattr(self.policy.engine, "supports_encoded", False)) and probs.is_cuda
        if self.greedy:
            idx = probs.argmax(1)
        elif self._fused and probs.dtype == torch.float32 and probs.shape[1] <= 512:
            from .. import ops
            self._calls += 1
            return ops.sample_moves(probs, has, self.beta, self._calls)
        else:
            p = probs.clamp_min(0) ** self.beta if self.beta != 1.0 else probs.clamp_min(0)
            p = torch.where(has.unsqueeze(1), p, torch.ones_like(p))
            p = p / p.sum(1, keepdim=True).clamp_min(1e-30)
            idx = torch.multinomial(p, 1, generator=self.gen).squeeze(1)
        return torch.where(has, idx, torch.full_like(idx, -1))

    def sample_device_mask(self, probs: torch.Tensor, legal: torch.Tensor) -> torch.Tensor:
        """sample_device from the (n, S*S) sensible-move mask: on the fused kernel the mask goes in as
        it is (each workgroup reduces its row), saving the two tensor kernels of ``legal.any(1)``."""
        if self._fused is None:
            self._fused = bool(getattr(self.policy.engine, "supports_encoded", False)) and probs.is_cuda
        if (not self.greedy and self._fused and probs.dtype == torch.float32 and probs.shape[1] <= 512
                and legal.dtype == torch.uint8 and legal.shape == probs.shape):
            from .. import ops
            self._calls += 1
            return ops.sample_moves(probs, legal, self.beta, self._calls)
        return self.sample_device(probs, (legal != 0).any(1))

    def device_planes_ok(self) -> bool:
        """The engine featurises on the device and can hand its uint8 planes back (HIP engines)."""
        eng = self.policy.engine
        return getattr(eng, "supports_encoded", False) and hasattr(eng, "set_encoded_planes")

    def select(self, states: Sequence, planes: Optional[np.ndarray] = None, need_planes: bool = True,
               device_planes: bool = False):
        """Returns (moves list, planes or None, flat move indices (-1 = pass)).  ``device_planes``
        (HIP engines): the planes come back as a (n, C, S, S) uint8 DEVICE tensor written by the
        GPU featurizer of the same forward -- no host featurisation, no host copy -- valid until
        the next select."""
        n = len(states)
        if n == 0:
            return [], None, np.zeros(0, np.int64)
        size = states[0].size
        eng = self.policy.engine
        dev_planes = None
        if device_planes and planes is None and self.device_planes_ok():
            eng.set_encoded_planes(True)
            probs, has = self._probs_encoded(states, eng, want_planes=True)
            dev_planes = self._enc_planes
            if self._bad:  # overflowed eye recursion: those rows from the host featurizer
                dev_planes[self._bad] = torch.from_numpy(self.featurize([states[i] for i in self._bad])).to(
                    dev_planes.device)
            planes = dev_planes
        elif planes is None and not need_planes and getattr(eng, "supports_encoded", False):
            probs, has = self._probs_encoded(states, eng)
        elif dev_planes is None:
            if planes is None:
                planes = self.featurize(states)
            masks = self.masks(states)
            probs = eng.evaluate(planes, masks)
            has = torch.from_numpy(masks.any(axis=1)).to(probs.device)
        idx = self.sample_device(probs, has).cpu().numpy()
        moves = [go.PASS_MOVE if i < 0 else (int(i) // size, int(i) % size) for i in idx]
        return moves, planes, idx

    # GreedyPolicyPlayer/ProbabilisticPolicyPlayer-compatible interface
    def get_moves(self, states):
        return self.select(states, need_planes=False)[0]

    def get_move(self, state):
        return self.select([state], need_planes=False)[0][0]


@dataclass
class GameRecords:
    planes: List[np.ndarray] = field(default_factory=list)   # per game: (n_i, F, S, S) uint8
    moves: List[np.ndarray] = field(default_factory=list)    # per game: (n_i,) flat move index
    winners: List[int] = field(default_factory=list)
    learner_colors: List[int] = field(default_factory=list)
    lengths: List[int] = field(default_factory=list)
    states: List = field(default_factory=list)               # final states


class _DeviceRecordBuffer(object):
    """Learner planes kept on the device: rows appended by device-to-device copies from the GPU
    featurizer's output, per-game row lists; grows by doubling."""

    def __init__(self, row_shape, device, capacity: int = 4096):
        self.buf = torch.empty((capacity,) + tuple(row_shape), dtype=torch.uint8, device=device)
        self.n = 0

    def append(self, rows: torch.Tensor) -> np.ndarray:
        k = rows.shape[0]
        if self.n + k > self.buf.shape[0]:
            nb = torch.empty((max(2 * self.buf.shape[0], self.n + k),) + tuple(self.buf.shape[1:]),
                             dtype=torch.uint8, device=self.buf.device)
            nb[:self.n].copy_(self.buf[:self.n])
            self.buf = nb
        self.buf[self.n:self.n + k].copy_(rows)
        self.n += k
        return np.arange(self.n - k, self.n)


def play_games(learner: BatchedSampler, opponent: BatchedSampler, n_games: int, size: int = 19,
               komi: float = 7.5, max_moves: int = 500, rng: Optional[np.random.Generator] = None,
               record: bool = True, learner_colors: Optional[Sequence[int]] = None,
               standard_two_pass: bool = False, device_records: Optional[bool] = None,
               native: Optional[bool] = None) -> GameRecords:
    """Play n_games learner-vs-opponent games in lock-step (reference
    make_training_pairs, reinforcement_policy_trainer.py:16-76).  The learner's
    colour is drawn per game and its training pairs use the state
    *before* its own move (Q6).  ``standard_two_pass`` ends a game after any two
    consecutive passes instead of the reference rule (Q9, go.py:345-348).

    ``device_records`` (default: whenever the learner's engine featurises on the GPU): the
    learner's planes are the GPU featurizer's own output of the sampling forward, copied into a
    device buffer -- no host featurisation, numpy round trip or re-upload; ``GameRecords.planes``
    then holds one device tensor per game.

    ``native`` (default: whenever both engines featurise on the GPU): the pipelined native driver
    (search/lockstep.py); False keeps this Python loop (CPU engines, and the equality tests)."""
    from .lockstep import lockstep_ok, play_games_lockstep
    if native is None:
        native = lockstep_ok(learner, opponent)
    if native:
        return play_games_lockstep(learner, opponent, n_games, size, komi, max_moves, rng, record, learner_colors,
                                   standard_two_pass, device_records)
    rng = rng or np.random.default_rng()
    states = [go.GameState(size, komi, standard_two_pass) for _ in range(n_games)]
    colors = list(learner_colors) if learner_colors is not None else \
        [int(c) for c in rng.choice([go.BLACK, go.WHITE], size=n_games)]
    device_records = record and learner.device_planes_ok() and (device_records is None or device_records)
    dbuf = None
    if record and device_records:
        C = learner.policy.preprocessor.output_dim
        dbuf = _DeviceRecordBuffer((C, size, size), learner.policy.device, capacity=max(256, n_games * 64))
    rec_p: List[List] = [[] for _ in range(n_games)]
    rec_m: List[List[int]] = [[] for _ in range(n_games)]
    for ply in range(max_moves):
        active = [i for i in range(n_games) if not states[i].is_end_of_game]
        if not active:
            break
        lturn = [i for i in active if states[i].current_player == colors[i]]
        oturn = [i for i in active if states[i].current_player != colors[i]]
        for group, sampler, is_learner in ((lturn, learner, True), (oturn, opponent, False)):
            if not group:
                continue
            want = record and is_learner
            moves, planes, idx = sampler.select([states[i] for i in group], need_planes=want,
                                                device_planes=want and dbuf is not None)
            rows = None
            if want and dbuf is not None:
                keep = [k for k in range(len(group)) if moves[k] is not go.PASS_MOVE]
                if keep:
                    sel = planes if len(keep) == len(group) else planes[torch.as_tensor(keep, device=planes.device)]
                    rows = dict(zip(keep, dbuf.append(sel)))
            for k, i in enumerate(group):
                if want and moves[k] is not go.PASS_MOVE:
                    rec_p[i].append(rows[k] if rows is not None else planes[k])
                    rec_m[i].append(int(idx[k]))
                try:
                    states[i].do_move(moves[k])
                except go.IllegalMove:  # cannot happen for masked samples; pass defensively
                    states[i].do_move(go.PASS_MOVE)
    out = GameRecords()
    for i in range(n_games):
        out.winners.append(states[i].get_winner())
        out.learner_colors.append(colors[i])
        out.lengths.append(len(states[i].history))
        out.states.append(states[i])
        if record:
            C = learner.policy.preprocessor.output_dim
            if dbuf is not None:
                out.planes.append(dbuf.buf[torch.as_tensor(np.asarray(rec_p[i], np.int64), device=dbuf.buf.device)])
            else:
                out.planes.append(np.stack(rec_p[i]) if rec_p[i] else np.zeros((0, C, size, size), np.uint8))
            out.moves.append(np.asarray(rec_m[i], dtype=np.int64))
    return out
