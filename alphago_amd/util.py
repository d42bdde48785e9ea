"""Reference module path ``AlphaGo.util`` (AlphaGo/util.py:6-83): flat indices and SGF replay.

Backed by ``alphago_amd.utils.gorecords`` (own SGF parser, no ``sgf`` package)."""
from .utils.gorecords import _init_state as _sgf_init_gamestate
from .utils.gorecords import flatten_idx, parse_sgf_move, sgf_iter_states, sgf_to_gamestate, unflatten_idx


def _parse_sgf_move(node_value, size: int = 19):
    """SGF coordinate string -> (x, y), or ``None`` for a pass (util.py:16-25)."""
    return parse_sgf_move(node_value, size)


__all__ = ["flatten_idx", "unflatten_idx", "sgf_to_gamestate", "sgf_iter_states", "_parse_sgf_move",
           "_sgf_init_gamestate"]
