"""Matches between players (reference interface/Play.py, which played a single
turn and was marked "This is incorrect.", Play.py:33).

``play_match`` plays complete games between any two objects with
``get_move(state)`` (policy players, MCTS players, external GTP engines),
alternating colours, and returns the score.  ``batched_match`` runs many
games at once for two BatchedSamplers (one GPU forward per side per ply).
"""
from __future__ import annotations

import random
from typing import Dict, List, Optional

from .. import go
from ..utils.gorecords import gamestate_to_sgf, result_string


class RandomPlayer(object):
    """Uniformly random sensible move (baseline / test opponent)."""

    def __init__(self, seed: Optional[int] = None):
        self.rng = random.Random(seed)

    def get_move(self, state):
        moves = [m for m in state.get_legal_moves() if not state.is_eye(m, state.current_player)]
        return self.rng.choice(moves) if moves else go.PASS_MOVE


def play_game(black, white, size: int = 19, komi: float = 7.5, max_moves: int = 722):
    state = go.GameState(size, komi)
    players = {go.BLACK: black, go.WHITE: white}
    while not state.is_end_of_game and len(state.history) < max_moves:
        mv = players[state.current_player].get_move(state)
        try:
            state.do_move(mv)
        except go.IllegalMove:
            state.do_move(go.PASS_MOVE)
    return state.get_winner(), state


def play_match(player1, player2, n_games: int = 2, size: int = 19, komi: float = 7.5, max_moves: int = 722,
               sgf_dir: Optional[str] = None) -> Dict[str, float]:
    wins = [0, 0]
    draws = 0
    for g in range(n_games):
        swap = g % 2 == 1
        black, white = (player2, player1) if swap else (player1, player2)
        winner, state = play_game(black, white, size, komi, max_moves)
        if winner == 0:
            draws += 1
        else:
            p1_won = (winner == go.BLACK) != swap
            wins[0 if p1_won else 1] += 1
        if sgf_dir:
            import os
            os.makedirs(sgf_dir, exist_ok=True)
            with open(os.path.join(sgf_dir, "game_%04d.sgf" % g), "w") as f:
                f.write(gamestate_to_sgf(state, result=result_string(winner)))
    return {"player1_wins": wins[0], "player2_wins": wins[1], "draws": draws,
            "player1_win_rate": wins[0] / max(1, n_games)}


def batched_match(sampler1, sampler2, n_games: int, size: int = 19, komi: float = 7.5, max_moves: int = 722,
                  seed: int = 0, standard_two_pass: bool = False) -> Dict[str, float]:
    import numpy as np

    from .selfplay import play_games

    colors = [go.BLACK if i % 2 == 0 else go.WHITE for i in range(n_games)]
    rec = play_games(sampler1, sampler2, n_games, size=size, komi=komi, max_moves=max_moves,
                     rng=np.random.default_rng(seed), record=False, learner_colors=colors,
                     standard_two_pass=standard_two_pass)
    w1 = sum(1 for w, c in zip(rec.winners, rec.learner_colors) if w == c)
    d = sum(1 for w in rec.winners if w == 0)
    return {"player1_wins": w1, "player2_wins": n_games - w1 - d, "draws": d,
            "player1_win_rate": w1 / max(1, n_games), "mean_length": float(np.mean(rec.lengths))}


class play_match_compat(object):
    """Reference-shaped class (Play.py:5-34) whose play() plays a whole game."""

    def __init__(self, player1, player2, save_dir=None, size=19):
        self.player1, self.player2, self.size = player1, player2, size
        self.state = go.GameState(size=size)

    def play(self):
        winner, self.state = play_game(self.player1, self.player2, self.size)
        return True
