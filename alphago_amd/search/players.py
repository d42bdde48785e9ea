"""Players (reference AlphaGo/ai.py) + an MCTS player.

GreedyPolicyPlayer / ProbabilisticPolicyPlayer keep the reference semantics
(ai.py:6-68): only "sensible" moves (legal and not filling an own true eye),
pass when none; probabilistic play samples p**(1/T).  ``get_moves`` evaluates
a list of states in ONE batched forward.
"""
from __future__ import annotations

import time
from typing import List, Optional

import numpy as np

from .. import go


def sensible_moves(state) -> List:
    return [m for m in state.get_legal_moves() if not state.is_eye(m, state.current_player)]


class GreedyPolicyPlayer(object):
    def __init__(self, policy_function):
        self.policy = policy_function

    def get_move(self, state):
        moves = sensible_moves(state)
        if moves:
            probs = self.policy.eval_state(state, moves)
            return max(probs, key=lambda ap: ap[1])[0]
        return go.PASS_MOVE

    def get_moves(self, states):
        lists = [sensible_moves(st) for st in states]
        dists = self.policy.batch_eval_state(states, lists)
        return [max(d, key=lambda ap: ap[1])[0] if d else go.PASS_MOVE for d in dists]


class ProbabilisticPolicyPlayer(object):
    def __init__(self, policy_function, temperature: float = 1.0, rng: Optional[np.random.Generator] = None):
        assert temperature > 0.0
        self.policy = policy_function
        self.beta = 1.0 / temperature
        self.rng = rng or np.random.default_rng()

    def _sample(self, move_probs):
        moves, p = zip(*move_probs)
        p = np.asarray(p, dtype=np.float64) ** self.beta
        s = p.sum()
        p = p / s if s > 0 else np.full(len(p), 1.0 / len(p))
        return moves[self.rng.choice(len(moves), p=p)]

    def get_move(self, state):
        moves = sensible_moves(state)
        if moves:
            return self._sample(self.policy.eval_state(state, moves))
        return go.PASS_MOVE

    def get_moves(self, states):
        lists = [sensible_moves(st) for st in states]
        dists = self.policy.batch_eval_state(states, lists)
        return [self._sample(d) if d else go.PASS_MOVE for d in dists]


class MCTSPlayer(object):
    """Plays the most visited move of a batched PUCT search (see search.mcts)."""

    def __init__(self, policy, value=None, n_playout: int = 1600, c_puct: float = 5.0, lmbda: float = 0.0,
                 leaves_per_batch: int = 16, temperature: float = 0.0, seed: int = 0, threads: Optional[int] = None):
        from .mcts import BatchedMCTS

        self.search = BatchedMCTS(policy, value, n_trees=1, c_puct=c_puct, lmbda=lmbda, seed=seed, threads=threads)
        self.n_playout = n_playout
        self.leaves_per_batch = leaves_per_batch
        self.temperature = temperature

    supports_time_budget = True

    def get_move(self, state, time_budget: Optional[float] = None):
        """``time_budget`` (seconds, GTP time control): search in growing chunks of playouts on the same
        tree (each ``search`` call adds to the root's visits) until the next chunk would overrun the
        budget or ``n_playout`` is reached; None = the fixed ``n_playout``.  The budget's end is also a
        deadline inside the search, so a chunk slowed by a loaded host stops at its next leaf batch."""
        if not sensible_moves(state):
            return go.PASS_MOVE
        if time_budget is None:
            return self.search.search([state], self.n_playout, self.leaves_per_batch, self.temperature)[0]
        t0 = time.perf_counter()
        deadline = t0 + time_budget  # a hard stop inside a chunk too: no leaf batch starts after it
        done, chunk, move = 0, max(1, self.leaves_per_batch), None
        while True:
            t1 = time.perf_counter()
            move = self.search.search([state], chunk, self.leaves_per_batch, self.temperature,
                                      deadline=deadline)[0]
            done += chunk
            now = time.perf_counter()
            per = (now - t1) / chunk  # seconds per playout of the last chunk
            left = time_budget - (now - t0)
            if done >= self.n_playout or left <= 0:
                return move
            # next chunk: double the last, capped by the playout budget and by a third of the time left
            # (the per-playout time of a loaded host varies from chunk to chunk)
            chunk = int(min(2 * chunk, self.n_playout - done, left / 3.0 / max(per, 1e-6)))
            if chunk < 1:
                return move

    def get_moves(self, states):
        self.search.resize(len(states))
        return self.search.search(states, self.n_playout, self.leaves_per_batch, self.temperature)
