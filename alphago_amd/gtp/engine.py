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

Time control (beyond the reference, whose wrapper has no clock: gtp_wrapper.py:46-65):
``time_settings main byo_time byo_stones`` and ``time_left color time stones`` keep a clock per colour
(also advanced by the engine's own genmove times between ``time_left`` updates), and ``genmove`` hands a
player that supports it (``MCTSPlayer``) a per-move time budget: in byo-yomi the period's time over its
stones, in main time the remaining time over the expected moves left, minus a safety margin.
"""
from __future__ import annotations

import sys
import time
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
        self.time_settings = None  # (main, byo_time, byo_stones) seconds / stones
        self.clock = {}  # colour -> [seconds left in the current period, stones left (0: main time)]
        self.last_budget = None
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
            "time_settings": self._time_settings,
            "time_left": self._time_left,
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

    # ------------------------------------------------------------- clock
    SAFETY_S = 0.15  # per-move reserve for the reply, host jitter and the last search chunk's overshoot
    SAFETY_FRAC = 0.1

    def _time_settings(self, a):
        main, byo, stones = float(a[0]), float(a[1]), int(a[2])
        if main < 0 or byo < 0 or stones < 0:
            raise ValueError("syntax error")
        # byo_yomi_time > 0 with 0 stones means no time limit (GTP 2 spec, time_settings)
        self.time_settings = None if (byo > 0 and stones == 0) else (main, byo, stones)
        self.clock = {c: self._fresh_clock() for c in (go.BLACK, go.WHITE)} if self.time_settings else {}
        return ""

    def _fresh_clock(self):
        main, byo, stones = self.time_settings
        return [main, 0] if main > 0 else [byo, stones]

    def _time_left(self, a):
        color = parse_color(a[0])
        t, stones = float(a[1]), int(a[2])
        if self.time_settings is not None:
            self.clock[color] = [t, stones]
        return ""

    def move_budget(self, color) -> Optional[float]:
        """Seconds this genmove may spend (None: no time limit)."""
        if self.time_settings is None:
            return None
        t, stones = self.clock.get(color) or self._fresh_clock()
        if stones > 0:  # byo-yomi: the period's time over its stones
            per = t / stones
        else:  # main time: the remaining time over the moves still expected (at least 20)
            empties = int((self.state.board == go.EMPTY).sum())
            per = t / max(20.0, empties / 3.0)
            _, byo, bst = self.time_settings
            if bst > 0 and byo > 0:  # main time nearly used up: byo-yomi follows, use its per-stone pace
                per = max(per, min(t, byo / bst) if t > 0 else byo / bst)
        return max(0.0, per * (1.0 - self.SAFETY_FRAC) - self.SAFETY_S)

    def _charge(self, color, spent: float) -> None:
        """Advance the colour's clock by a genmove's wall time (until the next time_left)."""
        if self.time_settings is None:
            return
        c = self.clock.setdefault(color, self._fresh_clock())
        main, byo, bst = self.time_settings
        c[0] -= spent
        if c[1] == 0 and c[0] <= 0 and bst > 0:  # main time ran out: enter byo-yomi
            c[0], c[1] = byo + min(0.0, c[0]), bst
        elif c[1] > 0:
            c[1] -= 1
            if c[1] == 0:  # period completed: a fresh one
                c[0], c[1] = byo, bst

    def _genmove(self, a):
        color = parse_color(a[0])
        self.state.current_player = color
        t0 = time.perf_counter()
        budget = self.move_budget(color)
        self.last_budget = budget
        if budget is not None and getattr(self.player, "supports_time_budget", False):
            move = self.player.get_move(self.state, time_budget=budget)
        else:
            move = self.player.get_move(self.state)
        self._charge(color, time.perf_counter() - t0)
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
