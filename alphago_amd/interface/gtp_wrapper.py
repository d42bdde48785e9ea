"""Reference module path ``interface.gtp_wrapper`` (gtp_wrapper.py:6-65).

``run_gtp(player_obj, inpt_fn=None)`` runs the repo's own GTP v2 engine
(``alphago_amd.gtp.engine``; the reference depends on the external ``pygtp``).
``GTPGameConnector`` keeps the reference's "game object" API with 1-based
``(x, y)`` vertices; it fixes Q13 (a pass is recorded for the given colour)."""
from .. import go
from ..gtp.engine import GTPEngine, run_gtp

PASS = (0, 0)  # pygtp's pass vertex


class GTPGameConnector(object):
    def __init__(self, player):
        self._state = go.GameState()
        self._player = player

    def clear(self):
        self._state = go.GameState(self._state.size)

    def make_move(self, color, vertex):
        try:
            if vertex == PASS or vertex is None:
                self._state.do_move(go.PASS_MOVE, color)
            else:
                self._state.do_move((vertex[0] - 1, vertex[1] - 1), color)
            return True
        except go.IllegalMove:
            return False

    def set_size(self, n):
        self._state = go.GameState(n)

    def set_komi(self, k):
        self._state.komi = k

    def get_move(self, color):
        self._state.current_player = color
        move = self._player.get_move(self._state)
        return PASS if move is go.PASS_MOVE else (move[0] + 1, move[1] + 1)


__all__ = ["GTPGameConnector", "GTPEngine", "run_gtp", "PASS"]
