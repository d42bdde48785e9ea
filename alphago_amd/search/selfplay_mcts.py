"""Full-game batched MCTS self-play and MCTS-vs-MCTS matches.

The reference searches one position at a time (``MCTS.get_move``,
/root/reference/AlphaGo/mcts.py:142-171; ``ParallelMCTS`` is an empty stub,
:174-175) and its self-play is lock-step policy sampling
(/root/reference/AlphaGo/training/reinforcement_policy_trainer.py:16-76).  Here
every GPU rank plays ``concurrent`` games at once, each with its own tree in one
``BatchedMCTS``: a search round runs ``n_playout`` simulations on every live
tree with all their leaves evaluated in batched GPU forwards (policy + value,
device featurizer inside the HIP graph), then every game plays its move.  Games
end by two passes (reference rule, go.py:345-348), by resignation (the root's
search value for the side to move stays below ``resign`` for ``resign_moves``
consecutive moves), or at ``max_moves`` (scored).  A finished game's slot starts
the next game, so the batch stays full until the last games.

Records per game: the move list, the root visit distribution of every searched
move (S*S + 1 entries, pass last), the players and the outcome.  ``SelfPlayWriter``
turns finished games into SGF files and an HDF5 dataset in the training schema:
``states`` (N, F, S, S) uint8 (chunks of 64 rows, LZF), ``pi`` (N, S*S+1) float32,
``outcomes`` (N,) int8 (z for the player to move), ``moves`` (N,) int16, ``game``
(N,) int32.  Under torchrun each rank writes its own file and rank 0 merges them
(``selfplay_cli``).
"""
from __future__ import annotations

import argparse
import json
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from .. import go
from ..features import VALUE_FEATURES, Preprocess
from ..io.h5lite import H5File, H5Writer
from ..utils.gorecords import gamestate_to_sgf, result_string
from .mcts import BatchedMCTS

STATE_CHUNK_ROWS = 64


@dataclass
class MCTSConfig:
    n_playout: int = 1600
    leaves_per_tree: int = 16
    c_puct: float = 5.0
    lmbda: float = 0.0             # value / rollout mix (reference default 0.5, mcts.py:80)
    rollout_policy: str = "random"
    rollout_limit: int = 500
    temperature: float = 1.0       # move sampling temperature for the first ``temp_moves`` moves ...
    temp_moves: int = 30           # ... then the most visited move
    noise: Optional[float] = 0.03  # Dirichlet alpha of the root noise (None: no noise)
    resign: float = -0.95          # resign below this root value ...
    resign_moves: int = 3          # ... held for this many consecutive own moves (0: never resign)
    virtual_loss: int = 3


@dataclass
class GameRecord:
    moves: List[int] = field(default_factory=list)          # flat index, -1 = pass
    pi: List[np.ndarray] = field(default_factory=list)      # (S*S+1,) visit distribution per move
    players: List[int] = field(default_factory=list)        # player to move per move
    root_values: List[float] = field(default_factory=list)  # search value for the player to move
    winner: int = 0
    resigned: int = 0                                       # colour that resigned, 0 = none
    size: int = 19
    komi: float = 7.5
    game_id: int = 0
    final_state: object = None


def _flat(mv, size: int) -> int:
    return -1 if mv is None else int(mv[0]) * size + int(mv[1])


@dataclass
class RoundStats:
    """Per search round: live games, leaf evaluations, wall time (phase tables in profiles/)."""
    round: int
    live: int
    evals: int
    seconds: float
    min_move: int
    max_move: int


def play_selfplay(policy, value, n_games: int, concurrent: int, cfg: MCTSConfig, size: int = 19,
                  komi: float = 7.5, max_moves: Optional[int] = None, seed: int = 0, threads: Optional[int] = None,
                  on_game: Optional[Callable[[GameRecord], None]] = None,
                  stats: Optional[List[RoundStats]] = None, progress_every: int = 0) -> List[GameRecord]:
    """Play ``n_games`` self-play games, ``concurrent`` at a time, to the end.  ``on_game`` gets each
    finished game (then it is not kept in the returned list)."""
    max_moves = max_moves or 2 * size * size
    conc = max(1, min(concurrent, n_games))
    search = BatchedMCTS(policy, value, n_trees=conc, c_puct=cfg.c_puct, lmbda=cfg.lmbda,
                         rollout_limit=cfg.rollout_limit, virtual_loss=cfg.virtual_loss, seed=seed,
                         threads=threads, rollout_policy=cfg.rollout_policy)
    states: List[Optional[object]] = [None] * conc
    recs: List[Optional[GameRecord]] = [None] * conc
    low: List[Dict[int, int]] = [dict() for _ in range(conc)]  # consecutive low-value moves per colour
    started = finished = 0
    out: List[GameRecord] = []

    def start(slot):
        nonlocal started
        states[slot] = go.GameState(size, komi)
        recs[slot] = GameRecord(size=size, komi=komi, game_id=started)
        low[slot] = {go.BLACK: 0, go.WHITE: 0}
        started += 1

    def finish(slot, resigned: int = 0):
        nonlocal finished
        st, r = states[slot], recs[slot]
        r.resigned = resigned
        r.winner = -resigned if resigned else st.get_winner()
        r.final_state = st
        finished += 1
        if on_game is not None:
            on_game(r)
        else:
            out.append(r)
        states[slot] = recs[slot] = None
        if started < n_games:
            start(slot)

    for s in range(conc):
        start(s)
    rnd = 0
    while True:
        live = [i for i in range(conc) if states[i] is not None]
        if not live:
            break
        temps = [0.0] * conc
        for i in live:
            temps[i] = cfg.temperature if len(states[i].history) < cfg.temp_moves else 0.0
        e0, t0 = search.forest.total_evals, time.perf_counter()
        mvs = search.search(states, cfg.n_playout, cfg.leaves_per_tree, temperature=temps, noise=cfg.noise,
                            active=live)
        if stats is not None:
            lens = [len(states[i].history) for i in live]
            stats.append(RoundStats(rnd, len(live), search.forest.total_evals - e0, time.perf_counter() - t0,
                                    min(lens), max(lens)))
        rnd += 1
        if progress_every and stats is not None and rnd % progress_every == 0:
            recent = stats[-progress_every:]
            ev, sec = sum(r.evals for r in recent), sum(r.seconds for r in recent)
            print("selfplay round %d: %d live games (moves %d-%d), %d finished, %.0f leaf evals/s" %
                  (rnd, len(live), recent[-1].min_move, recent[-1].max_move, finished, ev / max(sec, 1e-9)),
                  flush=True)
        for i in live:
            st, r = states[i], recs[i]
            me = st.current_player
            v = search.root_value(i)
            r.pi.append(search.visit_distribution(i, size))
            r.players.append(me)
            r.root_values.append(v)
            if cfg.resign_moves > 0 and v < cfg.resign:
                low[i][me] += 1
            else:
                low[i][me] = 0
            if cfg.resign_moves > 0 and low[i][me] >= cfg.resign_moves:
                r.moves.append(-1)  # the record's last row: the position at which the player resigned
                finish(i, resigned=me)
                continue
            mv = mvs[i]
            try:
                st.do_move(mv)
            except go.IllegalMove:  # a sampled move is always legal; pass defensively
                mv = go.PASS_MOVE
                st.do_move(mv)
            r.moves.append(_flat(mv, size))
            if st.is_end_of_game or len(st.history) >= max_moves:
                finish(i)
    return out


class SelfPlayWriter(object):
    """Finished games -> SGF files and the (states, pi, outcomes, moves, game) HDF5 dataset.
    ``positions_per_game`` > 0 keeps that many positions per game, drawn uniformly (the value-net
    recipe of one position per game avoids correlated samples); 0 keeps every searched position."""

    def __init__(self, h5_path: str, sgf_dir: Optional[str], features: Sequence[str] = VALUE_FEATURES,
                 size: int = 19, positions_per_game: int = 0, seed: int = 0, threads: int = 16):
        self.pre = Preprocess(list(features))
        self.size = size
        self.sgf_dir = sgf_dir
        self.ppg = positions_per_game
        self.rng = np.random.default_rng(seed)
        self.threads = threads
        self.path = h5_path
        self.tmp = h5_path + ".tmp"
        self.w = H5Writer(self.tmp)
        self.w.attrs["features"] = np.array([x.encode() for x in features])
        self.w.attrs["board_size"] = np.int64(size)
        self.st = self.w.stream_dataset("states", (self.pre.output_dim, size, size), np.uint8,
                                        chunk_rows=STATE_CHUNK_ROWS, compression="lzf")
        self.pi: List[np.ndarray] = []
        self.z: List[np.ndarray] = []
        self.mv: List[np.ndarray] = []
        self.gid: List[np.ndarray] = []
        self.games = self.positions = 0
        self.winners = {go.BLACK: 0, go.WHITE: 0, 0: 0}
        self.lengths: List[int] = []
        # how the games ended: two passes (then scored), resignation, or the move cap
        self.endings = {"two_passes": 0, "resignation": 0, "move_cap": 0}
        if sgf_dir:
            os.makedirs(sgf_dir, exist_ok=True)

    def add(self, r: GameRecord) -> None:
        n = len(r.pi)
        if r.resigned:
            self.endings["resignation"] += 1
        elif len(r.moves) >= 2 and r.moves[-1] == -1 and r.moves[-2] == -1:
            self.endings["two_passes"] += 1
        else:
            self.endings["move_cap"] += 1
        keep = np.arange(n)
        if self.ppg > 0 and n > self.ppg:
            keep = np.sort(self.rng.choice(n, self.ppg, replace=False))
        # replay the game, featurising the kept positions (the state BEFORE each searched move)
        want = set(int(k) for k in keep)
        st = go.GameState(r.size, r.komi)
        batch: List[object] = []
        for k in range(n):
            if k in want:
                batch.append(st.copy())
            if len(batch) == 64 or (k == n - 1 and batch):
                self.st.append(self.pre.states_to_uint8(batch))
                batch = []
            mv = r.moves[k]
            if k == n - 1 and r.resigned:
                break
            st.do_move(None if mv < 0 else divmod(mv, r.size))
        if batch:
            self.st.append(self.pre.states_to_uint8(batch))
        self.pi.append(np.stack([r.pi[k] for k in keep]).astype(np.float32))
        self.z.append(np.array([r.winner * r.players[k] for k in keep], np.int8))
        self.mv.append(np.array([r.moves[k] for k in keep], np.int16))
        self.gid.append(np.full(len(keep), r.game_id, np.int32))
        self.games += 1
        self.positions += len(keep)
        self.winners[r.winner] = self.winners.get(r.winner, 0) + 1
        self.lengths.append(len(r.moves))
        if self.sgf_dir:
            res = result_string(r.winner) + ("R" if r.resigned else "")
            with open(os.path.join(self.sgf_dir, "game_%06d.sgf" % r.game_id), "w") as f:
                f.write(gamestate_to_sgf(r.final_state, result=res))

    def close(self) -> int:
        S2 = self.size * self.size + 1
        self.st.finish()
        self.w.create_dataset("pi", data=np.concatenate(self.pi) if self.pi else np.zeros((0, S2), np.float32))
        self.w.create_dataset("outcomes", data=np.concatenate(self.z) if self.z else np.zeros(0, np.int8))
        self.w.create_dataset("moves", data=np.concatenate(self.mv) if self.mv else np.zeros(0, np.int16))
        self.w.create_dataset("game", data=np.concatenate(self.gid) if self.gid else np.zeros(0, np.int32))
        self.w.close()
        os.replace(self.tmp, self.path)
        return self.positions


def merge_selfplay_files(paths: List[str], outfile: str, block_rows: int = 4096) -> int:
    """Concatenate per-rank self-play files; game ids are offset so they stay unique."""
    tmp = outfile + ".tmp"
    total = 0
    with H5Writer(tmp) as w:
        with H5File(paths[0]) as first:
            shape = first["states"].shape[1:]
            for k in ("features", "board_size"):
                if k in first.attrs:
                    w.attrs[k] = first.attrs[k]
        st = w.stream_dataset("states", shape, np.uint8, chunk_rows=STATE_CHUNK_ROWS, compression="lzf")
        cols: Dict[str, List[np.ndarray]] = {"pi": [], "outcomes": [], "moves": [], "game": []}
        goff = 0
        for pth in paths:
            with H5File(pth) as f:
                ds = f["states"]
                if ds.shape[1:] != shape:
                    raise ValueError("%s: row shape %s != %s" % (pth, ds.shape[1:], shape))
                for r0 in range(0, ds.shape[0], block_rows):
                    st.append(ds.read_rows(r0, r0 + block_rows))
                for k in cols:
                    cols[k].append(np.asarray(f[k].read()))
                g = cols["game"][-1]
                cols["game"][-1] = g + goff
                goff += int(g.max()) + 1 if len(g) else 0
                total += ds.shape[0]
        st.finish()
        for k, v in cols.items():
            w.create_dataset(k, data=np.concatenate(v))
    os.replace(tmp, outfile)
    return total


def mcts_match(player1: BatchedMCTS, player2: BatchedMCTS, n_games: int, n_playout1: int, n_playout2: int,
               size: int = 19, komi: float = 7.5, max_moves: Optional[int] = None, leaves_per_tree: int = 16,
               sgf_dir: Optional[str] = None) -> Dict[str, float]:
    """``n_games`` games between two batched MCTS players, all at once: each player owns one tree
    per game (reused across the opponent's replies) and searches only the games where it is to move
    (``active``), so every round is one batched search per side.  Colours alternate by game."""
    max_moves = max_moves or 2 * size * size
    states = [go.GameState(size, komi) for _ in range(n_games)]
    p1_black = [g % 2 == 0 for g in range(n_games)]
    for p in (player1, player2):
        p.resize(n_games)
    while True:
        live = [i for i in range(n_games) if not states[i].is_end_of_game and len(states[i].history) < max_moves]
        if not live:
            break
        for p, npl, mine in ((player1, n_playout1, True), (player2, n_playout2, False)):
            turn = [i for i in live if (states[i].current_player == go.BLACK) == (p1_black[i] == mine)]
            if not turn:
                continue
            mvs = p.search(states, npl, leaves_per_tree, temperature=0.0, active=turn)
            for i in turn:
                try:
                    states[i].do_move(mvs[i])
                except go.IllegalMove:
                    states[i].do_move(go.PASS_MOVE)
            live = [i for i in live if not states[i].is_end_of_game and len(states[i].history) < max_moves]
    w1 = d = 0
    for g, st in enumerate(states):
        w = st.get_winner()
        if w == 0:
            d += 1
        elif (w == go.BLACK) == p1_black[g]:
            w1 += 1
        if sgf_dir:
            os.makedirs(sgf_dir, exist_ok=True)
            with open(os.path.join(sgf_dir, "match_%04d.sgf" % g), "w") as f:
                f.write(gamestate_to_sgf(st, result=result_string(w)))
    return {"player1_wins": w1, "player2_wins": n_games - w1 - d, "draws": d,
            "player1_win_rate": w1 / max(1, n_games),
            "mean_length": float(np.mean([len(s.history) for s in states]))}


def mcts_vs_sampler(search: BatchedMCTS, sampler, n_games: int, n_playout: int, size: int = 19,
                    komi: float = 7.5, max_moves: Optional[int] = None, leaves_per_tree: int = 16,
                    seed: int = 0) -> Dict[str, float]:
    """``n_games`` games of a batched MCTS player against a batched policy sampler
    (``selfplay.BatchedSampler``), all at once; colours alternate by game."""
    max_moves = max_moves or 2 * size * size
    states = [go.GameState(size, komi) for _ in range(n_games)]
    m_black = [g % 2 == 0 for g in range(n_games)]
    search.resize(n_games)
    while True:
        live = [i for i in range(n_games) if not states[i].is_end_of_game and len(states[i].history) < max_moves]
        if not live:
            break
        mine = [i for i in live if (states[i].current_player == go.BLACK) == m_black[i]]
        theirs = [i for i in live if i not in set(mine)]
        if mine:
            mvs = search.search(states, n_playout, leaves_per_tree, temperature=0.0, active=mine)
            for i in mine:
                states[i].do_move(mvs[i])
        if theirs:
            mvs2 = sampler.get_moves([states[i] for i in theirs])
            for k, i in enumerate(theirs):
                try:
                    states[i].do_move(mvs2[k])
                except go.IllegalMove:
                    states[i].do_move(go.PASS_MOVE)
    wins = draws = 0
    for g, st in enumerate(states):
        w = st.get_winner()
        draws += w == 0
        wins += w != 0 and (w == go.BLACK) == m_black[g]
    return {"mcts_wins": int(wins), "sampler_wins": int(n_games - wins - draws), "draws": int(draws),
            "mcts_win_rate": wins / max(1, n_games),
            "mean_length": float(np.mean([len(s.history) for s in states]))}


def phase_table(stats: List[RoundStats], width: int = 50) -> List[Dict[str, float]]:
    """Leaf evaluations per second by game phase (rounds grouped by the live games' move number)."""
    rows: Dict[int, List[RoundStats]] = {}
    for s in stats:
        rows.setdefault(s.min_move // width, []).append(s)
    out = []
    for b in sorted(rows):
        rs = rows[b]
        ev, sec = sum(r.evals for r in rs), sum(r.seconds for r in rs)
        out.append({"moves": "%d-%d" % (b * width, b * width + width - 1), "rounds": len(rs),
                    "mean_live_games": round(float(np.mean([r.live for r in rs])), 1), "leaf_evals": ev,
                    "seconds": round(sec, 2), "leaf_evals_per_s": round(ev / sec, 1) if sec > 0 else 0.0})
    return out


def selfplay_cli(argv=None):
    """``selfplay-mcts``: full-game batched MCTS self-play on every rank (torchrun), SGFs + HDF5."""
    from ..models.policy import CNNPolicy, CNNValue
    from ..parallel import dist as agdist

    p = argparse.ArgumentParser(description="Full-game batched MCTS self-play (SGF + HDF5 training records)")
    p.add_argument("policy_json")
    p.add_argument("out_directory")
    p.add_argument("--value-json", default=None)
    p.add_argument("--games", type=int, default=256, help="games per rank")
    p.add_argument("--concurrent", type=int, default=256, help="games searched together per rank")
    p.add_argument("--playouts", type=int, default=1600)
    p.add_argument("--leaves-per-tree", type=int, default=16)
    p.add_argument("--c-puct", type=float, default=5.0)
    p.add_argument("--lmbda", type=float, default=None,
                   help="value/rollout mix (default 0 with a value net, 1 without: rollouts only)")
    p.add_argument("--rollout-policy", default="heuristic", choices=sorted(BatchedMCTS.ROLLOUT_POLICIES))
    p.add_argument("--rollout-limit", type=int, default=500)
    p.add_argument("--temperature", type=float, default=1.0)
    p.add_argument("--temp-moves", type=int, default=30)
    p.add_argument("--noise", type=float, default=0.03, help="root Dirichlet alpha (0: off)")
    p.add_argument("--resign", type=float, default=-0.95)
    p.add_argument("--resign-moves", type=int, default=3)
    p.add_argument("--max-moves", type=int, default=0)
    p.add_argument("--komi", type=float, default=7.5)
    p.add_argument("--positions-per-game", type=int, default=0)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-sgf", action="store_true")
    p.add_argument("--progress-every", type=int, default=0, help="print a progress line every N search rounds")
    p.add_argument("--keep-shards", action="store_true")
    a = p.parse_args(argv)
    env = agdist.init_from_env()
    policy = CNNPolicy.load_model(a.policy_json, device=env.device)
    value = CNNValue.load_model(a.value_json, device=env.device) if a.value_json else None
    lm = a.lmbda if a.lmbda is not None else (0.0 if value is not None else 1.0)
    cfg = MCTSConfig(n_playout=a.playouts, leaves_per_tree=a.leaves_per_tree, c_puct=a.c_puct, lmbda=lm,
                     rollout_policy=a.rollout_policy, rollout_limit=a.rollout_limit, temperature=a.temperature,
                     temp_moves=a.temp_moves, noise=a.noise or None, resign=a.resign, resign_moves=a.resign_moves)
    S = policy.model.board
    os.makedirs(a.out_directory, exist_ok=True)
    h5 = os.path.join(a.out_directory, "selfplay.h5" if env.world_size == 1 else "selfplay.h5.rank%d" % env.rank)
    sgf = None if a.no_sgf else os.path.join(a.out_directory, "sgf", "rank%d" % env.rank)
    writer = SelfPlayWriter(h5, sgf, size=S, positions_per_game=a.positions_per_game,
                            seed=a.seed * 1009 + env.rank)
    stats: List[RoundStats] = []
    t0 = time.perf_counter()
    play_selfplay(policy, value, a.games, a.concurrent, cfg, size=S, komi=a.komi, max_moves=a.max_moves or None,
                  seed=a.seed * 100003 + env.rank * 7919, on_game=writer.add, stats=stats,
                  progress_every=a.progress_every if env.is_main else 0)
    dt = time.perf_counter() - t0
    n = writer.close()
    evals = sum(s.evals for s in stats)
    local = {"rank": env.rank, "games": writer.games, "positions": n, "seconds": round(dt, 2),
             "leaf_evals": evals, "winners": {"B": writer.winners.get(go.BLACK, 0), "W": writer.winners.get(go.WHITE, 0),
                                               "draw": writer.winners.get(0, 0)},
             "mean_length": round(float(np.mean(writer.lengths)), 1) if writer.lengths else 0.0,
             "endings": dict(writer.endings)}
    every = agdist.all_gather_object(local)
    if env.world_size > 1:
        agdist.barrier()
        if env.is_main:
            shards = ["%s.rank%d" % (os.path.join(a.out_directory, "selfplay.h5"), r) for r in range(env.world_size)]
            merge_selfplay_files(shards, os.path.join(a.out_directory, "selfplay.h5"))
            if not a.keep_shards:
                for sh in shards:
                    os.remove(sh)
        agdist.barrier()
    summary = {"games": sum(e["games"] for e in every), "positions": sum(e["positions"] for e in every),
               "leaf_evals": sum(e["leaf_evals"] for e in every), "seconds": max(e["seconds"] for e in every),
               "ranks": every, "phases_rank0": phase_table(stats),
               "endings": {k: sum(e["endings"][k] for e in every) for k in every[0]["endings"]}}
    summary["leaf_evals_per_s"] = round(summary["leaf_evals"] / max(summary["seconds"], 1e-9), 1)
    if env.is_main:
        with open(os.path.join(a.out_directory, "selfplay_summary.json"), "w") as f:
            json.dump(summary, f, indent=1)
        print(json.dumps({k: v for k, v in summary.items() if k != "ranks"}), flush=True)
    return summary
