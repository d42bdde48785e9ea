"""Monte-Carlo tree search.

``BatchedMCTS``: many independent trees searched together by the native
``Forest`` (csrc/engine/mcts.cpp: PUCT with virtual loss, negamax backup,
subtree reuse, optional λ-mixed random rollouts).  Each round gathers up to
``leaves_per_tree`` leaves from every tree, writes their compact encoding
(stones, move ages, ko, side to move; ~2 bytes/point) into pinned buffers,
and evaluates ALL of them in one batched policy (+ value) forward on the GPU
whose HIP graph starts with the device featurizer (ops/gpu_features.py);
priors/values are applied back natively.  Engines without the encoded path
(CPU) get uint8 planes featurised in native threads instead.  This replaces the reference's serial search that made a
batch-1 network call per tree level (mcts.py:91-161; ParallelMCTS stub
:174-175).

``MCTS``: reference-compatible API (mcts.py:67-171) — constructor takes
value/policy/rollout *callables*, ``get_move(state)`` and
``update_with_move(move)`` — running on the same native tree.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from .. import go
from .._native import engine as _engine
from ..utils.gorecords import flatten_idx


class BatchedMCTS(object):
    def __init__(self, policy, value=None, n_trees: int = 1, c_puct: float = 5.0, lmbda: float = 0.0,
                 rollout_limit: int = 500, virtual_loss: int = 3, seed: int = 0, threads: Optional[int] = None):
        self.policy, self.value = policy, value
        self.c_puct, self.lmbda, self.rollout_limit, self.vl, self.seed = c_puct, lmbda, rollout_limit, virtual_loss, seed
        # host worker threads (gather/apply/encode); a GPU box's process gets ~16 cores
        self.threads = threads or min(16, os.cpu_count() or 1)
        pf = policy.preprocessor.feature_list
        vf = value.preprocessor.feature_list if value is not None else pf
        self._same_feats = list(pf) == list(vf)
        self._n = 0
        self._roots: List[Optional[list]] = []
        self.resize(n_trees)
        self._pinned = None
        self._enc = None

    def resize(self, n_trees: int) -> None:
        if n_trees == self._n:
            return
        pf = self.policy.preprocessor.feature_list
        self.forest = _engine().Forest(n_trees, self.c_puct, self.lmbda if self.value is None or self.lmbda > 0 else 0.0,
                                       self.rollout_limit, 1000, self.vl, self.seed, [f.lower() for f in pf])
        self.forest.set_threads(self.threads)
        self._n = n_trees
        self._roots = [None] * n_trees

    def _buffer(self, L: int, planes: int, np_: int) -> torch.Tensor:
        need = L * planes * np_
        if self._pinned is None or self._pinned.numel() < need:
            pin = torch.cuda.is_available()
            self._pinned = torch.empty(max(need, 1 << 20), dtype=torch.uint8, pin_memory=pin)
        return self._pinned[:need]

    def _enc_buffers(self, L: int, np_: int):
        if self._enc is None or self._enc[0].shape[0] < L or self._enc[0].shape[1] != np_:
            pin = torch.cuda.is_available()
            cap = max(L, 256)
            self._enc = (torch.zeros((cap, np_), dtype=torch.int8, pin_memory=pin),
                         torch.zeros((cap, np_), dtype=torch.uint8, pin_memory=pin),
                         torch.zeros((cap, 2), dtype=torch.int32, pin_memory=pin),
                         torch.zeros((cap, np_), dtype=torch.uint8, pin_memory=pin))
        return self._enc

    def _encoded_engines(self):
        pe = self.policy.engine
        ve = self.value.engine if self.value is not None else None
        if getattr(pe, "supports_encoded", False) and (ve is None or getattr(ve, "supports_encoded", False)):
            return pe, ve
        return None

    def _evaluate_encoded(self, pe, ve) -> None:
        f = self.forest
        L = f.n_pending
        s0 = f.leaf_state(0)
        np_ = s0.size * s0.size
        ladder = pe.needs_ladder or (ve is not None and ve.needs_ladder)
        b, a, m, l = self._enc_buffers(L, np_)
        f.leaf_encode_into(b.data_ptr(), a.data_ptr(), m.data_ptr(), l.data_ptr() if ladder else 0, b.shape[0],
                           self.threads)
        lad = l[:L] if ladder else None
        out, sens, bad = pe.evaluate_encoded(b[:L], a[:L], m[:L], lad)
        probs = out.float().cpu().numpy()
        mask = sens.cpu().numpy()  # sensible moves from the GPU featurizer: apply() skips its own scan
        values = None
        if ve is not None:
            vout, _, vbad = ve.evaluate_encoded(b[:L], a[:L], m[:L], lad)
            values = vout.float().cpu().numpy()
            bad = sorted(set(bad) | set(vbad))
        if bad:  # eye recursion too deep for the kernel: these rows from CPU planes
            states = [f.leaf_state(i) for i in bad]
            planes = self.policy.preprocessor.states_to_uint8(states)
            masks = _engine().featurize_batch(states, ["sensibleness"], self.threads).reshape(len(bad), -1)
            probs[bad] = pe.evaluate(planes, masks).float().cpu().numpy()
            mask[bad] = masks
            if ve is not None:
                values[bad] = ve.evaluate(self.value.preprocessor.states_to_uint8(states)).float().cpu().numpy()
        f.apply(probs, values, mask)

    def _evaluate_pending(self) -> None:
        f = self.forest
        L = f.n_pending
        if L == 0:
            return
        enc = self._encoded_engines()
        if enc is not None:
            self._evaluate_encoded(*enc)
            return
        s0 = f.leaf_state(0)
        np_ = s0.size * s0.size
        buf = self._buffer(L, f.feature_planes, np_)
        f.leaf_features_into(buf.data_ptr(), buf.numel(), self.threads)
        planes = buf.view(L, f.feature_planes, s0.size, s0.size)
        masks = torch.from_numpy(f.leaf_masks())
        probs = self.policy.engine.evaluate(planes, masks).float().cpu().numpy()
        values = None
        if self.value is not None:
            if self._same_feats:
                vplanes = planes
            else:
                states = [f.leaf_state(i) for i in range(L)]
                vplanes = self.value.preprocessor.states_to_uint8(states)
            values = self.value.engine.evaluate(vplanes).float().cpu().numpy()
        f.apply(probs, values)

    def _sync_roots(self, states: Sequence) -> None:
        for i, st in enumerate(states):
            hist = st.history
            prev = self._roots[i]
            if prev is not None and len(hist) == len(prev) + 1 and hist[:-1] == prev:
                try:
                    self.forest.advance(i, hist[-1])
                    self._roots[i] = list(hist)
                    continue
                except Exception:  # noqa: BLE001 - fall back to a fresh tree
                    pass
            if prev is None or hist != prev:
                self.forest.set_root(i, st)
                self._roots[i] = list(hist)

    def search(self, states: Sequence, n_playout: int, leaves_per_tree: int = 16,
               temperature: float = 0.0, noise: Optional[float] = None) -> List:
        """Run ``n_playout`` simulations on every tree; return the chosen move per tree."""
        if len(states) != self._n:
            self.resize(len(states))
        self._sync_roots(states)
        f = self.forest
        # expand roots first (needed for root noise)
        f.gather(1)
        self._evaluate_pending()
        if noise:
            for i in range(self._n):
                f.add_root_noise(i, noise, 0.25)
        target = [f.sims(i) + n_playout for i in range(self._n)]
        while True:
            todo = [i for i in range(self._n) if f.sims(i) < target[i]]
            if not todo:
                break
            n = f.gather(leaves_per_tree, todo)
            if n == 0 and all(f.sims(i) < target[i] for i in todo):
                # only terminal/collided paths this round; they still count as sims
                continue
            self._evaluate_pending()
        return [f.best_move(i, temperature) for i in range(self._n)]

    def visit_distribution(self, tree: int, size: int) -> np.ndarray:
        moves, visits, _ = self.forest.root_stats(tree)
        d = np.zeros(size * size + 1, dtype=np.float32)
        for m, v in zip(moves, visits):
            d[size * size if m is None else flatten_idx(m, size)] = v
        s = d.sum()
        return d / s if s > 0 else d

    def update_with_move(self, tree: int, move) -> None:
        self.forest.advance(tree, move)
        if self._roots[tree] is not None:
            self._roots[tree].append(move)


class MCTS(object):
    """Reference-compatible serial API on the native tree.

    value_network(state) -> float in [-1, 1] for the player to move;
    policy_network(state) / rollout_policy(state) -> [((x, y), prob), ...].
    """

    def __init__(self, state, value_network: Callable, policy_network: Callable, rollout_policy: Callable,
                 lmbda: float = 0.5, c_puct: float = 5, rollout_limit: int = 500, playout_depth: int = 20,
                 n_search: int = 10000, seed: int = 0):
        self._value, self._policy, self._rollout = value_network, policy_network, rollout_policy
        self._lmbda, self._c_puct = lmbda, c_puct
        self._rollout_limit, self._L, self._n_search = rollout_limit, playout_depth, n_search
        self.forest = _engine().Forest(1, c_puct, 0.0, rollout_limit, playout_depth, 1, seed, [])
        self._root_hist = None
        if state is not None:
            self.forest.set_root(0, state)
            self._root_hist = list(state.history)

    def _rollout_value(self, state) -> float:
        s = state.copy()
        me = s.current_player
        for _ in range(self._rollout_limit):
            ap = self._rollout(s)
            if not ap or s.is_end_of_game:
                break
            s.do_move(max(ap, key=lambda x: x[1])[0])
        return float(s.get_winner() * me)

    def _evaluate(self) -> None:
        f = self.forest
        L = f.n_pending
        if L == 0:
            return
        leaf = f.leaf_state(0)
        n2 = leaf.size * leaf.size
        pri = np.zeros((1, n2), dtype=np.float32)
        for (x, y), p in self._policy(leaf):
            pri[0, x * leaf.size + y] = p
        v = float(self._value(leaf)) if self._value is not None else 0.0
        if self._lmbda > 0 and self._rollout is not None:
            v = (1 - self._lmbda) * v + self._lmbda * self._rollout_value(leaf)
        f.apply(pri, np.array([v], dtype=np.float32))

    def get_move(self, state):
        if self._root_hist is None or list(state.history) != self._root_hist:
            self.forest.set_root(0, state)
            self._root_hist = list(state.history)
        f = self.forest
        target = f.sims(0) + self._n_search + 1
        guard = 0
        while f.sims(0) < target and guard < 4 * self._n_search + 8:
            guard += 1
            f.gather(1)
            self._evaluate()
        return f.best_move(0, 0.0)

    def root_visits(self):
        moves, visits, q = self.forest.root_stats(0)
        return dict(zip(moves, visits))

    def update_with_move(self, last_move) -> None:
        try:
            self.forest.advance(0, last_move)
            if self._root_hist is not None:
                self._root_hist.append(last_move)
        except Exception:  # noqa: BLE001
            self._root_hist = None


class ParallelMCTS(BatchedMCTS):
    """The reference's ParallelMCTS placeholder (mcts.py:174-175), realised as the batched forest."""
