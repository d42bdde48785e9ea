"""Monte-Carlo tree search.

``BatchedMCTS``: many independent trees searched together by the native
``Forest`` (csrc/engine/mcts.cpp: PUCT with virtual loss, negamax backup,
subtree reuse, optional λ-mixed random rollouts).  Each round gathers up to
``leaves_per_tree`` leaves from every tree, writes their compact encoding
(stones, move ages, ko, side to move; ~2 bytes/point) into pinned buffers,
and evaluates ALL of them in one batched policy (+ value) forward on the GPU
whose HIP graph starts with the device featurizer (ops/gpu_features.py);
priors/values are applied back natively.  Engines without the encoded path
(CPU) get uint8 planes featurised in native threads instead.

With ``pipeline=True`` (default on a GPU) the trees are split into two
forests whose rounds interleave: while the GPU evaluates one group's leaves
(asynchronous graph replay into its own buffer slot), the host threads apply
the other group's results and gather + encode its next leaves.  This replaces the reference's serial search that made a
batch-1 network call per tree level (mcts.py:91-161; ParallelMCTS stub
:174-175).

``MCTS``: reference-compatible API (mcts.py:67-171) — constructor takes
value/policy/rollout *callables*, ``get_move(state)`` and
``update_with_move(move)`` — running on the same native tree.
"""
from __future__ import annotations

import os
import time
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from .. import go
from .._native import engine as _engine
from ..utils.gorecords import flatten_idx


# bucket slot of the overflow fallback (slots 0 / 1 hold the pipelined search's in-flight batches)
FALLBACK_SLOT = 2


def _fallback_eval(engine, planes, masks=None) -> np.ndarray:
    return engine.evaluate(planes, masks, slot=FALLBACK_SLOT).float().cpu().numpy()


class _ForestGroup(object):
    """Several native Forests presented as one (tree t -> (forest, local index))."""

    def __init__(self, forests):
        self.forests = forests
        self.map = [(fi, j) for fi, f in enumerate(forests) for j in range(f.n_trees)]

    def _at(self, t):
        fi, j = self.map[t]
        return self.forests[fi], j

    def set_root(self, t, st):
        f, j = self._at(t)
        f.set_root(j, st)

    def advance(self, t, move):
        f, j = self._at(t)
        f.advance(j, move)

    def root_stats(self, t):
        f, j = self._at(t)
        return f.root_stats(j)

    def best_move(self, t, temperature=0.0):
        f, j = self._at(t)
        return f.best_move(j, temperature)

    def sims(self, t):
        f, j = self._at(t)
        return f.sims(j)

    def add_root_noise(self, t, alpha=0.03, eps=0.25):
        f, j = self._at(t)
        f.add_root_noise(j, alpha, eps)

    def root_state(self, t):
        f, j = self._at(t)
        return f.root_state(j)

    @property
    def total_evals(self):
        return sum(f.total_evals for f in self.forests)

    @property
    def n_trees(self):
        return len(self.map)


class BatchedMCTS(object):
    ROLLOUT_POLICIES = {"random": 0, "heuristic": 1}

    def __init__(self, policy, value=None, n_trees: int = 1, c_puct: float = 5.0, lmbda: float = 0.0,
                 rollout_limit: int = 500, virtual_loss: int = 3, seed: int = 0, threads: Optional[int] = None,
                 pipeline: Optional[bool] = None, rollout_policy: str = "random", playout_depth: int = 1000):
        """``rollout_policy`` (λ > 0): "random" = uniform over sensible moves, "heuristic" = capture /
        atari escape at the last move, else a local answer half the time, else uniform (the native
        stand-in for the reference's ``rollout_fn``, mcts.py:128-140).  Rollouts run in parallel
        over trees (one random stream per tree)."""
        if rollout_policy not in self.ROLLOUT_POLICIES:
            raise ValueError("rollout_policy must be one of %s" % sorted(self.ROLLOUT_POLICIES))
        self.policy, self.value = policy, value
        self.rollout_policy = rollout_policy
        self.playout_depth = playout_depth
        self.pipeline = pipeline
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
        pf = [f.lower() for f in self.policy.preprocessor.feature_list]
        lm = self.lmbda if self.value is None or self.lmbda > 0 else 0.0
        pipe = self.pipeline
        if pipe is None:
            pipe = self._encoded_engines() is not None and n_trees >= 8
        sizes = [n_trees - n_trees // 2, n_trees // 2] if pipe and n_trees >= 2 else [n_trees]
        forests = []
        for k, n in enumerate(sizes):
            f = _engine().Forest(n, self.c_puct, lm, self.rollout_limit, self.playout_depth, self.vl,
                                 self.seed + 7919 * k, pf)
            f.set_threads(self.threads)
            f.rollout_policy = self.ROLLOUT_POLICIES[self.rollout_policy]
            forests.append(f)
        self._forests = forests
        self.forest = forests[0] if len(forests) == 1 else _ForestGroup(forests)
        self._n = n_trees
        self._roots = [None] * n_trees

    def _buffer(self, L: int, planes: int, np_: int) -> torch.Tensor:
        need = L * planes * np_
        if self._pinned is None or self._pinned.numel() < need:
            pin = torch.cuda.is_available()
            self._pinned = torch.empty(max(need, 1 << 20), dtype=torch.uint8, pin_memory=pin)
        return self._pinned[:need]

    def _enc_buffers(self, L: int, np_: int, slot: int = 0):
        if self._enc is None:
            self._enc = {}
        e = self._enc.get(slot)
        if e is None or e[0].shape[0] < L or e[0].shape[1] != np_:
            pin = torch.cuda.is_available()
            cap = max(L, 256)
            e = (torch.zeros((cap, np_), dtype=torch.int8, pin_memory=pin),
                 torch.zeros((cap, np_), dtype=torch.uint8, pin_memory=pin),
                 torch.zeros((cap, 2), dtype=torch.int32, pin_memory=pin),
                 torch.zeros((cap, np_), dtype=torch.uint8, pin_memory=pin))
            self._enc[slot] = e
        return e

    def _encoded_engines(self):
        pe = self.policy.engine
        ve = self.value.engine if self.value is not None else None
        if getattr(pe, "supports_encoded", False) and (ve is None or getattr(ve, "supports_encoded", False)):
            return pe, ve
        return None

    def _submit(self, f, slot: int, pe, ve):
        """Encode f's pending leaves into pinned buffers and launch the GPU evaluation (async)."""
        L = f.n_pending
        s0 = f.leaf_state(0)
        np_ = s0.size * s0.size
        ladder = pe.needs_ladder or (ve is not None and ve.needs_ladder)
        b, a, m, l = self._enc_buffers(L, np_, slot)
        f.leaf_encode_into(b.data_ptr(), a.data_ptr(), m.data_ptr(), l.data_ptr() if ladder else 0, b.shape[0],
                           self.threads)
        lad = l[:L] if ladder else None
        hp = pe.submit_encoded(b[:L], a[:L], m[:L], lad, slot=slot, to_host=True)
        hv = None
        if ve is not None:
            side = self._value_stream(L, pe)
            if side is not None:
                # small leaf batches leave most CUs idle in each net's forward: the value net runs
                # beside the policy net on a second stream (both read only the pinned encodings, and
                # collect() waits on each one's own event)
                with torch.cuda.stream(side):
                    hv = ve.submit_encoded(b[:L], a[:L], m[:L], lad, slot=slot, to_host=True)
            else:
                hv = ve.submit_encoded(b[:L], a[:L], m[:L], lad, slot=slot, to_host=True)
        return hp, hv

    # leaf batches up to this many boards run the value forward on a side stream (ALPHAGO_AMD_MCTS_VALUE_STREAM=0:
    # never); above it one net's forward fills the GPU and a second stream only interleaves them
    VALUE_STREAM_MAX = 64

    def _value_stream(self, L: int, pe):
        if L > self.VALUE_STREAM_MAX or os.environ.get("ALPHAGO_AMD_MCTS_VALUE_STREAM", "1") == "0":
            return None
        dev = getattr(pe, "device", None)
        if dev is None or torch.device(dev).type != "cuda":
            return None
        if getattr(self, "_vstream", None) is None:
            self._vstream = torch.cuda.Stream(device=dev)
        return self._vstream

    def _finish(self, f, handles, pe, ve) -> None:
        """Collect a submitted evaluation and apply it to f."""
        hp, hv = handles
        # mask: sensible moves from the GPU featurizer, so apply() skips its own scan
        probs, mask, bad = pe.collect(hp)
        probs = np.array(probs, copy=True)
        mask = np.array(mask, copy=True)
        values = None
        if hv is not None:
            values, _, vbad = ve.collect(hv)
            values = np.array(values, copy=True)
            bad = sorted(set(bad) | set(vbad))
        if bad:  # eye recursion too deep for the kernel: these rows from CPU planes
            states = [f.leaf_state(i) for i in bad]
            planes = self.policy.preprocessor.states_to_uint8(states)
            masks = _engine().featurize_batch(states, ["sensibleness"], self.threads).reshape(len(bad), -1)
            # another batch may still be in flight (pipelined search: its value forward on the side
            # stream): the fallback runs on bucket buffers of its own slot, after the side stream
            vs = getattr(self, "_vstream", None)
            if vs is not None:
                torch.cuda.current_stream(vs.device).wait_stream(vs)
            probs[bad] = _fallback_eval(pe, planes, masks)
            mask[bad] = masks
            if ve is not None:
                values[bad] = _fallback_eval(ve, self.value.preprocessor.states_to_uint8(states))
        f.apply(probs, values, mask)

    def _evaluate_encoded(self, pe, ve, f=None, slot: int = 0) -> None:
        f = f if f is not None else self._forests[0]
        self._finish(f, self._submit(f, slot, pe, ve), pe, ve)

    def _evaluate_pending(self, f=None, slot: int = 0) -> None:
        f = f if f is not None else self._forests[0]
        L = f.n_pending
        if L == 0:
            return
        enc = self._encoded_engines()
        if enc is not None:
            self._evaluate_encoded(enc[0], enc[1], f, slot)
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

    def _sync_roots(self, states: Sequence, which: Optional[Sequence[int]] = None) -> None:
        """Bring tree i's root to states[i]: advance through the moves played since (subtree reuse,
        also across an opponent's reply), else a fresh tree."""
        for i in (range(len(states)) if which is None else which):
            st = states[i]
            hist = list(st.history)
            prev = self._roots[i]
            if prev is not None and len(hist) > len(prev) and hist[:len(prev)] == prev:
                try:
                    for mv in hist[len(prev):]:
                        self.forest.advance(i, mv)
                    self._roots[i] = hist
                    continue
                except Exception:  # noqa: BLE001 - fall back to a fresh tree
                    pass
            if prev is None or hist != prev:
                self.forest.set_root(i, st)
                self._roots[i] = hist

    def search(self, states: Sequence, n_playout: int, leaves_per_tree: int = 16,
               temperature=0.0, noise: Optional[float] = None, active: Optional[Sequence[int]] = None,
               deadline: Optional[float] = None) -> List:
        """Run ``n_playout`` simulations on every tree (or only the trees in ``active``; the others
        keep their roots and statistics); return the chosen move per tree (None for inactive trees).
        ``temperature``: one value, or one per tree.  ``deadline`` (a ``time.perf_counter()`` value,
        GTP time control): no new leaf batch is gathered after it; the batches in flight finish."""
        if len(states) != self._n:
            self.resize(len(states))
        act = list(range(self._n)) if active is None else sorted(set(int(i) for i in active))
        self._sync_roots(states, act)
        fg = self.forest
        offs = [0]
        for f in self._forests:
            offs.append(offs[-1] + f.n_trees)
        act_k = [[t - offs[k] for t in act if offs[k] <= t < offs[k + 1]] for k in range(len(self._forests))]
        # expand roots first (needed for root noise)
        for k, f in enumerate(self._forests):
            if act_k[k]:
                f.gather(1, act_k[k])
                self._evaluate_pending(f, k)
        if noise:
            for i in act:
                fg.add_root_noise(i, noise, 0.25)
        on = set(act)
        targets = [[fg.sims(offs[k] + j) + (n_playout if offs[k] + j in on else 0) for j in range(f.n_trees)]
                   for k, f in enumerate(self._forests)]

        def late():
            return deadline is not None and time.perf_counter() >= deadline

        def gather(k):
            """Gather the next leaves of group k; False when its trees are done."""
            f = self._forests[k]
            while True:
                if late():
                    return False
                todo = [j for j in range(f.n_trees) if f.sims(j) < targets[k][j]]
                if not todo:
                    return False
                if f.gather(leaves_per_tree, todo) > 0:
                    return True
                # only terminal/collided paths this round: they still count as sims

        def gather_once(k):
            """One gather attempt (no retry): False when the trees are done or every path ended on a
            queued leaf (a held batch's) or a terminal.  The held batch's leaves count toward the
            playout budget, so the pipelined search does the serial search's number of playouts."""
            f = self._forests[k]
            if late():
                return False
            held = f.held_counts()  # one native pass over the held batch
            todo = [j for j in range(f.n_trees) if f.sims(j) + held[j] < targets[k][j]]
            return bool(todo) and f.gather(leaves_per_tree, todo) > 0

        enc = self._encoded_engines()
        if len(self._forests) == 1 and enc is not None and self._pipeline_single():
            self._search_pipelined(self._forests[0], gather, gather_once, enc)
        elif len(self._forests) == 1 or enc is None:
            for k, f in enumerate(self._forests):
                while gather(k):
                    self._evaluate_pending(f, k)
        else:
            pe, ve = enc
            live = [gather(0), gather(1)]
            inflight = [None, None]
            if live[0]:
                inflight[0] = self._submit(self._forests[0], 0, pe, ve)
            k = 1
            while live[0] or live[1]:
                # host work for group k overlaps the GPU evaluation of group 1-k
                if live[k]:
                    if inflight[k] is not None:
                        self._finish(self._forests[k], inflight[k], pe, ve)
                        inflight[k] = None
                        live[k] = gather(k)
                    if live[k]:
                        inflight[k] = self._submit(self._forests[k], k, pe, ve)
                k ^= 1
                if inflight[k] is not None and not live[k ^ 1]:
                    # the other group is done: nothing to overlap with
                    self._finish(self._forests[k], inflight[k], pe, ve)
                    inflight[k] = None
                    live[k] = gather(k)
                    if live[k]:
                        inflight[k] = self._submit(self._forests[k], k, pe, ve)
            for k in (0, 1):
                if inflight[k] is not None:
                    self._finish(self._forests[k], inflight[k], pe, ve)
        temps = list(temperature) if isinstance(temperature, (list, tuple, np.ndarray)) else [temperature] * self._n
        return [fg.best_move(i, float(temps[i])) if i in on else None for i in range(self._n)]

    @staticmethod
    def _pipeline_single() -> bool:
        return os.environ.get("ALPHAGO_AMD_MCTS_PIPELINE", "1") != "0"

    def _search_pipelined(self, f, gather, gather_once, enc) -> None:
        """One forest (e.g. the single tree of a GTP genmove), two batches in flight: while batch A is
        evaluated on the device, the next batch B is gathered (A's leaves keep their virtual losses and
        count as collisions) and encoded and launched; then A is backed up.  The host work of each
        round overlaps the previous round's forwards instead of following them."""
        pe, ve = enc
        try:
            self._pipeline_loop(f, gather, gather_once, pe, ve)
        except BaseException:
            # a HIP error or an interrupt (e.g. a GTP session's Ctrl-C) mid-search: drop both
            # in-flight batches with their virtual losses so the forest stays usable
            f.discard()
            raise

    def _pipeline_loop(self, f, gather, gather_once, pe, ve) -> None:
        if not gather(0):
            return
        slot = 0
        cur = self._submit(f, slot, pe, ve)
        while cur is not None:
            f.hold()  # A parked with its virtual losses; pending is empty
            nxt = None
            if gather_once(0):
                nxt = self._submit(f, slot ^ 1, pe, ve)
            f.swap_held()  # pending = A, held = B (or nothing)
            self._finish(f, cur, pe, ve)  # backs up A
            f.swap_held()  # pending = B
            if nxt is None and gather(0):  # every path met A's queued leaves (a young tree): after A
                nxt = self._submit(f, slot ^ 1, pe, ve)
            cur = nxt
            slot ^= 1

    def root_value(self, tree: int) -> float:
        """Search value of the root for the player to move there: the visit-weighted mean child Q
        (each child's Q is from the perspective of the player who moved into it)."""
        _, visits, q = self.forest.root_stats(tree)
        n = float(sum(visits))
        return float(sum(v * x for v, x in zip(visits, q)) / n) if n > 0 else 0.0

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


class TreeNode(object):
    """Reference-compatible tree node (mcts.py:4-64), pure Python.

    Same fields and methods (``expansion``, ``selection``, ``isLeaf``,
    ``update``, ``toValue``) with the SURVEY Q3 fix: the exploration bonus is
    recomputed at selection time from the parent's current visit count
    (``u = c_puct * P * sqrt(N_parent) / (1 + N)``) instead of being frozen at
    the node's last update, so children of the root keep being explored.
    The production search runs on the native forest (BatchedMCTS / MCTS)."""

    def __init__(self, parent, prior_p, c_puct: float = 5.0):
        self.parent = parent
        self.nVisits = 0
        self.Q_value = 0.0
        self.u_value = prior_p
        self.children = {}
        self.P = prior_p
        self.c_puct = c_puct

    def expansion(self, actions):
        for action, prob in actions:
            if action not in self.children:
                self.children[action] = TreeNode(self, prob, self.c_puct)

    def selection(self):
        """(action, child) maximising Q + u."""
        return max(self.children.items(), key=lambda an: an[1].toValue())

    def isLeaf(self):
        return self.children == {}

    is_leaf = isLeaf

    def is_root(self):
        return self.parent is None

    def update(self, leaf_value, c_puct=None):
        """Count a visit and fold ``leaf_value`` (mover's perspective) into the running mean Q."""
        if c_puct is not None:
            self.c_puct = c_puct
        self.nVisits += 1
        self.Q_value += (leaf_value - self.Q_value) / self.nVisits
        if self.parent is not None:
            self.u_value = self.c_puct * self.P * np.sqrt(self.parent.nVisits) / (1 + self.nVisits)

    def toValue(self):
        if self.parent is not None and self.parent.nVisits > 0:
            self.u_value = self.c_puct * self.P * np.sqrt(self.parent.nVisits) / (1 + self.nVisits)
        return self.Q_value + self.u_value


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

    def _DFS(self, nDepth, treenode, state):
        """One simulation on a Python TreeNode tree (reference mcts.py:91-126):
        select/expand down to ``nDepth``, evaluate the leaf with
        V = (1 - lambda) v + lambda z, back the value up.  Fixes Q4 (no None
        nodes on early game end; negamax sign per ply) and Q3 (the root is
        counted)."""
        visited = [treenode]
        for _ in range(nDepth):
            if state.is_end_of_game:
                break
            if treenode.isLeaf():
                treenode.expansion(self._policy(state))
                if treenode.isLeaf():
                    break
            action, treenode = treenode.selection()
            state.do_move(action)
            visited.append(treenode)
        if state.is_end_of_game:
            v = float(state.get_winner() * state.current_player)
        else:
            v = float(self._value(state)) if self._value is not None else 0.0
            if self._lmbda > 0 and self._rollout is not None:
                v = (1 - self._lmbda) * v + self._lmbda * self._rollout_value(state)
        # v is for the player to move at the leaf; the node entered by the
        # opponent's move stores the mover's value -v, alternating upwards
        value = -v
        for node in reversed(visited):
            node.update(value, self._c_puct)
            value = -value

    def update_with_move(self, last_move) -> None:
        try:
            self.forest.advance(0, last_move)
            if self._root_hist is not None:
                self._root_hist.append(last_move)
        except Exception:  # noqa: BLE001
            self._root_hist = None


class ParallelMCTS(BatchedMCTS):
    """The reference's ParallelMCTS placeholder (mcts.py:174-175), realised as the batched forest."""
