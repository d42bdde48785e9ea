"""Pipelined lock-step self-play on the native game driver (``_engine.Lockstep``).

Reference: ``make_training_pairs`` (AlphaGo/training/reinforcement_policy_trainer.py:16-76) plays a
batch of games in lock-step, one batched forward per colour per ply, and the value-network data
generator of the paper plays SL moves, one random move, then RL moves to the end.

Round 3 ran that loop in Python (``selfplay.play_games``): per-game ``do_move`` through pybind, a
fresh encode thread team per forward and a blocking ``.cpu()`` after every sampling, so the host held
the GPU to ~30 % of its encoded-inference rate.  Here the games are split into two fixed sets -- the
games whose learner plays black (X) and white (Y).  Every game alternates colours each ply (a pass
too), so X and Y alternate between the learner's and the opponent's network, and the two sets form a
two-deep pipeline: while the device runs one set's forward (GPU featurizer, trunk, fused masked head,
sampling), the host applies the other set's moves and encodes its next positions (one native call
each, on a persistent worker pool, GIL released).  The only device->host traffic is one small copy
of the sampled moves (and the featurizer's overflow flags) per set per ply.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .. import go
from .._native import engine as _engine


class _HostBufs(object):
    """Pinned encode buffers (inputs of the GPU featurizer) and move outputs of one in-flight set."""

    def __init__(self, n: int, np_: int, ladder: bool):
        self.board = torch.empty((n, np_), dtype=torch.int8, pin_memory=True)
        self.ages = torch.empty((n, np_), dtype=torch.uint8, pin_memory=True)
        self.meta = torch.empty((n, 2), dtype=torch.int32, pin_memory=True)
        self.ladder = torch.empty((n, np_), dtype=torch.uint8, pin_memory=True) if ladder else None
        self.moves = torch.empty(n, dtype=torch.int64, pin_memory=True)
        self.ovf = torch.empty(n, dtype=torch.int32, pin_memory=True)
        # numpy views for the native encoder and the completion event, made once (per-ply
        # conversions and event objects were a visible part of the host time per submission)
        self.np_views = (self.board.numpy(), self.ages.numpy(), self.meta.numpy(),
                         self.ladder.numpy() if ladder else None)
        self.ev = torch.cuda.Event() if torch.cuda.is_available() else None


def lockstep_ok(*samplers) -> bool:
    """Whether the native pipelined driver applies: every sampler's engine featurises on the device."""
    return all(getattr(s.policy.engine, "supports_encoded", False) for s in samplers)


class _Inflight(object):
    """One submitted set: its games, sampler, host buffers, completion event; with device records the
    record buffer and the first of its k rows (the featurizer's planes of these boards)."""
    learner = False
    dbuf = None
    row0 = 0


class LockstepPlayer(object):
    """Submits groups of ``games`` (an ``_engine.Lockstep``) to samplers' encoded engines and collects
    their sampled moves; the caller keeps two sets in flight and applies the moves."""

    def __init__(self, games, threads: int = 8):
        self.games = games
        self.threads = threads
        self._bufs = {}

    def _buf(self, key, n, ladder):
        b = self._bufs.get(key)
        if b is None or b.board.shape[0] < n or (ladder and b.ladder is None):
            b = _HostBufs(n, self.games.size ** 2, ladder)
            self._bufs[key] = b
        return b

    def submit(self, set_id: int, idx: np.ndarray, sampler, want_planes: bool = False) -> _Inflight:
        """Encode games idx on the host, run the sampler's forward + sampling on the device and start
        the copy of the sampled moves back; returns without waiting for the device."""
        eng = sampler.policy.engine
        k = len(idx)
        lad = eng.needs_ladder
        b = self._buf((id(eng), set_id), self.games.n, lad)
        nb, na, nm, nl = b.np_views
        self.games.encode(idx, nb, na, nm, nl if lad else None)
        if want_planes:
            eng.set_encoded_planes(True)
        handle = eng.submit_encoded(b.board[:k], b.ages[:k], b.meta[:k], b.ladder[:k] if lad else None, slot=set_id)
        bk = handle[0]
        probs, legal = eng.outputs(handle)
        mv = sampler.sample_device_mask(probs, legal)
        f = _Inflight()
        f.idx, f.sampler, f.bufs, f.k = idx, sampler, b, k
        f.rows = eng.encoded_planes_view(k) if want_planes else None
        b.moves[:k].copy_(mv, non_blocking=True)
        b.ovf[:k].copy_(bk.ovf[:k], non_blocking=True)
        f.ev = b.ev if b.ev is not None else torch.cuda.Event()
        f.ev.record()
        return f

    def finish(self, f: _Inflight) -> np.ndarray:
        """Wait for a submitted set's moves; boards whose eye recursion overflowed the GPU
        featurizer are re-evaluated from host planes (and their device planes rows rewritten).
        Returns the flat moves (-1 = pass); does not apply them."""
        f.ev.synchronize()
        moves = f.bufs.moves[:f.k].numpy().copy()
        bad = np.flatnonzero(f.bufs.ovf[:f.k].numpy())
        if len(bad):
            s = f.sampler
            sub = f.idx[bad].astype(np.int32)
            planes = self.games.featurize(sub, s._names)
            masks = self.games.featurize(sub, ["sensibleness"]).reshape(len(sub), -1)
            probs = s.policy.engine.evaluate(planes, masks)
            has = torch.from_numpy(masks.any(axis=1)).to(probs.device)
            moves[bad] = s.sample_device(probs, has).cpu().numpy()
            if f.dbuf is not None:  # the recorded rows of those boards: the host planes
                rows = torch.as_tensor(f.row0 + bad, device=f.dbuf.buf.device)
                f.dbuf.buf[rows] = torch.from_numpy(planes).to(f.dbuf.buf.device)
        return moves


def play_games_lockstep(learner, opponent, n_games: int, size: int = 19, komi: float = 7.5, max_moves: int = 500,
                        rng: Optional[np.random.Generator] = None, record: bool = True,
                        learner_colors: Optional[Sequence[int]] = None, standard_two_pass: bool = False,
                        device_records: Optional[bool] = None):
    """``selfplay.play_games`` on the native driver (same records, Q6/Q7/Q9 semantics): the learner's
    training pairs are the GPU featurizer's planes of the state before its own move and the sampled
    move, passes not recorded."""
    from .selfplay import GameRecords, _DeviceRecordBuffer

    rng = rng or np.random.default_rng()
    colors = np.asarray(list(learner_colors) if learner_colors is not None else
                        [int(c) for c in rng.choice([go.BLACK, go.WHITE], size=n_games)], dtype=np.int8)
    E = _engine()
    games = E.Lockstep(n_games, size, komi, standard_two_pass, learner.threads)
    player = LockstepPlayer(games, learner.threads)
    device_records = record and learner.device_planes_ok() and (device_records is None or device_records)
    dbuf = None
    C = learner.policy.preprocessor.output_dim
    if record and device_records:
        dbuf = _DeviceRecordBuffer((C, size, size), learner.policy.device, capacity=max(256, n_games * 64))
    rec_p: List[List] = [[] for _ in range(n_games)]
    rec_m: List[List[int]] = [[] for _ in range(n_games)]
    # the two game sets: learner black (moves at even plies) / learner white
    sets = [np.flatnonzero(colors == go.BLACK).astype(np.int32), np.flatnonzero(colors == go.WHITE).astype(np.int32)]
    plies = [0, 0]

    def submit(sid):
        act = games.active()
        idx = sets[sid][act[sets[sid]] != 0]
        if len(idx) == 0 or plies[sid] >= max_moves:
            return None
        to_move = games.to_move()[idx[0]]
        is_l = to_move == colors[idx[0]]
        want = record and is_l
        f = player.submit(sid, idx, learner if is_l else opponent, want_planes=want and dbuf is not None)
        f.learner = want
        if want and dbuf is not None:
            f.dbuf = dbuf
            f.row0 = int(dbuf.append(f.rows)[0])  # every row; pass moves' rows are never referenced
        return f

    inflight = [submit(0), submit(1)]
    while any(f is not None for f in inflight):
        for sid in (0, 1):
            f = inflight[sid]
            if f is None:
                continue
            moves = player.finish(f)
            if f.learner:
                if dbuf is None:
                    planes = games.featurize(f.idx, learner._names)
                for r, (i, m) in enumerate(zip(f.idx.tolist(), moves.tolist())):
                    if m >= 0:
                        rec_p[i].append(f.row0 + r if dbuf is not None else planes[r])
                        rec_m[i].append(int(m))
            games.play(f.idx, moves)
            plies[sid] += 1
            inflight[sid] = submit(sid)
    out = GameRecords()
    winners, lengths = games.winners(), games.lengths()
    for i in range(n_games):
        out.winners.append(int(winners[i]))
        out.learner_colors.append(int(colors[i]))
        out.lengths.append(int(lengths[i]))
        out.states.append(games.state(i))
        if record:
            if dbuf is not None:
                out.planes.append(dbuf.buf[torch.as_tensor(np.asarray(rec_p[i], np.int64), device=dbuf.buf.device)])
            else:
                out.planes.append(np.stack(rec_p[i]) if rec_p[i] else np.zeros((0, C, size, size), np.uint8))
            out.moves.append(np.asarray(rec_m[i], dtype=np.int64))
    return out


def generate_value_positions_lockstep(sl, rl, n_games: int, size: int, U: np.ndarray, max_moves: int,
                                      features: Sequence[str], seed: int):
    """Value-network positions on the native driver: game i plays SL moves until ply U[i] - 2, one
    uniformly random sensible move at ply U[i] - 1 (the recorded position is the state after it), then
    RL moves to the end (paper; round-3 Python loop: train/value.py generate_positions).  Games are
    pipelined in two sets (even / odd index); within a set the SL and RL subgroups of a ply are two
    forwards.  Returns (planes uint8 (N, F, S, S), outcomes int8 (N,)) for the games that reached U."""
    E = _engine()
    games = E.Lockstep(n_games, size, 7.5, False, sl.threads)
    player = LockstepPlayer(games, sl.threads)
    feats = [f.lower() for f in features]
    recorded = {}
    rec_player = {}
    sets = [np.arange(0, n_games, 2, dtype=np.int32), np.arange(1, n_games, 2, dtype=np.int32)]
    plies = [0, 0]

    def submit(sid):
        """Random moves of the set's games at U - 1 (applied now), then its SL / RL forwards."""
        ply = plies[sid]
        if ply >= max_moves:
            return None
        act = games.active()
        idx = sets[sid][act[sets[sid]] != 0]
        if len(idx) == 0:
            return None
        rnd = idx[U[idx] - 1 == ply]
        if len(rnd):
            games.play_random(rnd, seed * 1000003 + ply)
            planes = games.featurize(rnd, feats)
            tm = games.to_move()
            for r, i in enumerate(rnd.tolist()):
                recorded[i] = planes[r]
                rec_player[i] = int(tm[i])
        out = []
        for grp, s, slot in ((idx[ply < U[idx] - 1], sl, 2 * sid), (idx[ply > U[idx] - 1], rl, 2 * sid + 1)):
            grp = grp[games.active()[grp] != 0]
            if len(grp):
                out.append(player.submit(slot, grp.astype(np.int32), s))
        return out

    inflight = [submit(0), submit(1)]
    while any(f is not None for f in inflight):
        for sid in (0, 1):
            fl = inflight[sid]
            if fl is None:
                continue
            for f in fl:
                games.play(f.idx, player.finish(f))
            plies[sid] += 1
            inflight[sid] = submit(sid)
    keep = sorted(recorded)
    C = sum(E.feature_planes(f) for f in feats)
    if not keep:
        return np.zeros((0, C, size, size), np.uint8), np.zeros(0, np.int8)
    winners = games.winners()
    planes = np.stack([recorded[i] for i in keep])
    z = np.array([winners[i] * rec_player[i] for i in keep], dtype=np.int8)
    return planes, z
