"""Go rules engine (native C++).

Drop-in for the reference ``AlphaGo.go`` module (AlphaGo/go.py): same
constants, ``GameState`` method names and ``IllegalMove`` exception, backed by
the C++ engine in ``csrc/engine/go.cpp``.  Moves are ``(x, y)`` tuples with
``x`` the SGF column; ``None`` is a pass.
"""
from ._native import engine as _engine

_E = _engine()

WHITE = -1
BLACK = +1
EMPTY = 0
PASS_MOVE = None

GameState = _E.GameState
IllegalMove = _E.IllegalMove

__all__ = ["WHITE", "BLACK", "EMPTY", "PASS_MOVE", "GameState", "IllegalMove"]
