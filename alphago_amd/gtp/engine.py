"""Go Text Protocol (GTP v2) front-end.

Replaces the reference's pygtp-based wrapper (interface/gtp_wrapper.py:6-65)
with a self-contained implementation: ``GTPEngine`` parses commands and
produces ``= ...\\n\\n`` / ``? ...\\n\\n`` replies; ``run_gtp(player,
inpt_fn)`` drives it from stdin (or an injectable input function) like the
reference.

Coordinates: GTP vertex ``<letter><number>`` (letters A..Z without I, numbers
from 1) maps to (x, y) = (column index, number - 1), i.e. the reference's
1-based -> 0-based mapping (gtp_wrapper.py:18-28).  Fixed vs the reference:
``play <color> pass`` passes for the given colour.
"""
from __future__ import annotations

import sys
from typing import Callable, List, Optional

from .. import go
from ..utils.gorecords import gamestate_to_sgf

COLUMNS = "ABCDEFGHJKLMNOPQRSTUVWXYZ"


def parse_vertex(s: str, size: int):
    s = s.strip().upper()
    if s == "PASS":
        return go.PASS_MOVE
    if len(s) < 2 or s[0] not in COLUMNS:
        raise ValueError("invalid vertex")
    x = COLUMNS.index(s[0])
    y = int(s[1:]) - 1
    if not (0 <= x < size and 0 <= y < size):
        raise ValueError("vertex off board")
    return (x, y)


def format_vertex(move) -> str:
    if move is go.PASS_MOVE:
        return "pass"
    x, y = move
    return "%s%d" % (COLUMNS[x], y + 1)


def parse_color(s: str) -> int:
    s = s.strip().lower()
    if s in ("b", "black"):
        return go.BLACK
    if s in ("w", "white"):
        return go.WHITE
    raise ValueError("invalid color")


class GTPEngine(object):
    NAME = "alphago_amd"
    VERSION = "0.1"

    def __init__(self, player, size: int = 19, komi: float = 7.5):
        self.player = player
        self.size, self.komi = size, komi
        self.state = go.GameState(size, komi)
        self.disconnect = False
        self._undo: List[go.GameState] = []
        self.commands = {
            "protocol_version": lambda a: "2",
            "name": lambda a: self.NAME,
            "version": lambda a: self.VERSION,
            "known_command": lambda a: "true" if a and a[0] in self.commands else "false",
            "list_commands": lambda a: "\n".join(sorted(self.commands)),
            "quit": self._quit,
            "boardsize": self._boardsize,
            "clear_board": self._clear,
            "komi": self._komi,
            "play": self._play,
            "genmove": self._genmove,
            "undo": self._undo_cmd,
            "showboard": self._showboard,
            "final_score": self._final_score,
            "time_settings": lambda a: "",
            "time_left": lambda a: "",
            "printsgf": lambda a: gamestate_to_sgf(self.state),
        }

    # ------------------------------------------------------------- commands
    def _quit(self, a):
        self.disconnect = True
        return ""

    def _boardsize(self, a):
        n = int(a[0])
        if not 1 <= n <= 19:
            raise ValueError("unacceptable size")
        self.size = n
        self.state = go.GameState(n, self.komi)
        self._undo = []
        return ""

    def _clear(self, a):
        self.state = go.GameState(self.size, self.komi)
        self._undo = []
        return ""

    def _komi(self, a):
        self.komi = float(a[0])
        self.state.komi = self.komi
        return ""

    def _play(self, a):
        color = parse_color(a[0])
        move = parse_vertex(a[1], self.size)
        prev = self.state.copy()
        try:
            self.state.do_move(move, color)
        except go.IllegalMove:
            raise ValueError("illegal move")
        self._undo.append(prev)
        return ""

    def _genmove(self, a):
        color = parse_color(a[0])
        self.state.current_player = color
        move = self.player.get_move(self.state)
        prev = self.state.copy()
        try:
            self.state.do_move(move, color)
        except go.IllegalMove:
            move = go.PASS_MOVE
            self.state.do_move(move, color)
        self._undo.append(prev)
        return format_vertex(move)

    def _undo_cmd(self, a):
        if not self._undo:
            raise ValueError("cannot undo")
        self.state = self._undo.pop()
        return ""

    def _showboard(self, a):
        rows = []
        b = self.state.board
        for y in reversed(range(self.size)):
            row = "".join(".XO"[int(b[x, y])] + " " for x in range(self.size))
            rows.append("%2d %s" % (y + 1, row))
        rows.append("   " + " ".join(COLUMNS[:self.size]))
        return "\n" + "\n".join(rows)

    def _final_score(self, a):
        w = self.state.get_winner()
        return "B+" if w == go.BLACK else ("W+" if w == go.WHITE else "0")

    # ------------------------------------------------------------- protocol
    def send(self, line: str) -> str:
        line = line.split("#", 1)[0].strip()
        if not line:
            return ""
        parts = line.split()
        cid = ""
        if parts[0].isdigit():
            cid, parts = parts[0], parts[1:]
        if not parts:
            return ""
        cmd, args = parts[0].lower(), parts[1:]
        fn = self.commands.get(cmd)
        if fn is None:
            return "?%s unknown command\n\n" % cid
        try:
            res = fn(args)
        except (ValueError, IndexError) as e:
            return "?%s %s\n\n" % (cid, e)
        return "=%s %s\n\n" % (cid, res) if res != "" else "=%s\n\n" % cid


def run_gtp(player, inpt_fn: Optional[Callable[[], str]] = None, out=None, size: int = 19) -> GTPEngine:
    engine = GTPEngine(player, size=size)
    out = out or sys.stdout
    inpt_fn = inpt_fn or input
    sys.stderr.write("GTP engine ready\n")
    sys.stderr.flush()
    while not engine.disconnect:
        try:
            inpt = inpt_fn()
        except EOFError:
            break
        for cmd in str(inpt).split("\n"):
            reply = engine.send(cmd)
            if reply:
                out.write(reply)
                out.flush()
            if engine.disconnect:
                break
    return engine
