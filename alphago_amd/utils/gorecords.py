"""Game-record utilities (reference AlphaGo/util.py).

``flatten_idx``/``unflatten_idx`` (util.py:6-13), ``sgf_iter_states`` and
``sgf_to_gamestate`` (util.py:50-83) with the same yield contract: the *same*
GameState object is yielded before each move and mutated in place.

Kept from the reference for dataset parity: setup stones (AB/AW) are placed
through ``do_move`` so they enter history/turn counters.
Fixed: nodes without a B/W move are skipped instead of re-yielding the previous
move (Q12), and KM sets komi.
"""
from __future__ import annotations

import string
from typing import Iterator, List, Optional, Tuple

from .. import go
from ..io import sgf as sgflib

LETTERS = string.ascii_lowercase + string.ascii_uppercase  # py2 string.letters order


def flatten_idx(position: Tuple[int, int], size: int) -> int:
    (x, y) = position
    return x * size + y


def unflatten_idx(idx: int, size: int) -> Tuple[int, int]:
    x, y = divmod(idx, size)
    return (x, y)


def parse_sgf_move(value: str, size: int = 19):
    """'' or 'tt' (on boards <= 19) is a pass; otherwise (col, row) -> (x, y)."""
    if value == "" or (value == "tt" and size <= 19):
        return go.PASS_MOVE
    return (LETTERS.index(value[0]), LETTERS.index(value[1]))


def move_to_sgf(move, size: int = 19) -> str:
    if move is go.PASS_MOVE:
        return "" if size > 19 else "tt"
    return LETTERS[move[0]] + LETTERS[move[1]]


def _init_state(root: sgflib.Node) -> go.GameState:
    props = root.properties
    size = int(props.get("SZ", ["19"])[0].split(":")[0])
    komi = 7.5
    if "KM" in props:
        try:
            komi = float(props["KM"][0])
        except ValueError:
            pass
    gs = go.GameState(size, komi)
    for stone in props.get("AB", []):
        gs.do_move(parse_sgf_move(stone, size), go.BLACK)
    for stone in props.get("AW", []):
        gs.do_move(parse_sgf_move(stone, size), go.WHITE)
    pl = props.get("PL", ["B"])[0]
    gs.current_player = go.BLACK if pl.upper().startswith("B") else go.WHITE
    return gs


def sgf_iter_states(sgf_string: str, include_end: bool = False) -> Iterator[Tuple[go.GameState, object, int]]:
    """Yield (state, move, player) for the main line of the first game."""
    game = sgflib.parse(sgf_string)[0]
    gs = _init_state(game.root)
    size = gs.size
    for node in game.rest:
        props = node.properties
        if "W" in props:
            move, player = parse_sgf_move(props["W"][0], size), go.WHITE
        elif "B" in props:
            move, player = parse_sgf_move(props["B"][0], size), go.BLACK
        else:
            continue
        yield (gs, move, player)
        gs.do_move(move, player)
    if include_end:
        yield (gs, None, None)


def sgf_to_gamestate(sgf_string: str) -> go.GameState:
    gs = None
    for gs, _, _ in sgf_iter_states(sgf_string, include_end=True):
        pass
    return gs


def gamestate_to_sgf(state: go.GameState, black: str = "alphago_amd", white: str = "alphago_amd",
                     result: Optional[str] = None) -> str:
    root = {"GM": ["1"], "FF": ["4"], "SZ": [str(state.size)], "KM": [str(state.komi)],
            "PB": [black], "PW": [white], "AP": ["alphago_amd"]}
    if result:
        root["RE"] = [result]
    nodes: List[dict] = []
    color = go.BLACK
    for mv in state.history:
        nodes.append({"B" if color == go.BLACK else "W": [move_to_sgf(mv, state.size)]})
        color = -color
    return sgflib.dumps(root, nodes)


def result_string(winner: int) -> str:
    return "B+" if winner == go.BLACK else "W+" if winner == go.WHITE else "0"
