"""Drive an external GTP engine (e.g. Pachi, GNU Go, or another alphago_amd) as a player.

The reference wires Pachi as a git submodule with an empty wrapper
(.gitmodules:1-3, interface/opponents/pachi/pachi.py is 0 bytes); here any
GTP v2 engine started as a subprocess can be an opponent in matches or RL
evaluation.  The engine's board is kept in sync incrementally with ``play``
commands (full resync with ``clear_board`` when histories diverge).
"""
from __future__ import annotations

import shlex
import subprocess
from typing import List, Optional

from .. import go
from .engine import format_vertex, parse_vertex


class GTPError(RuntimeError):
    pass


class GTPClientPlayer(object):
    def __init__(self, command, name: Optional[str] = None, timeout: float = 60.0):
        self.cmd = shlex.split(command) if isinstance(command, str) else list(command)
        self.proc = subprocess.Popen(self.cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     stderr=subprocess.DEVNULL, text=True, bufsize=1)
        self.name = name or self.send("name")
        self._synced: Optional[List] = None
        self._size = None
        self._komi = None

    def send(self, command: str) -> str:
        if self.proc.poll() is not None:
            raise GTPError("engine exited")
        self.proc.stdin.write(command + "\n")
        self.proc.stdin.flush()
        lines = []
        while True:
            line = self.proc.stdout.readline()
            if line == "":
                raise GTPError("engine closed its output")
            line = line.rstrip("\n")
            if line == "" and lines:
                break
            if line == "" and not lines:
                continue
            lines.append(line)
        head = lines[0]
        body = "\n".join([head[1:].strip()] + lines[1:]).strip()
        if head.startswith("?"):
            raise GTPError("%s -> %s" % (command, body))
        return body

    def _sync(self, state) -> None:
        hist = state.history
        if self._size != state.size or self._komi != state.komi or self._synced is None or \
                hist[:len(self._synced)] != self._synced:
            self.send("boardsize %d" % state.size)
            self.send("clear_board")
            self.send("komi %s" % state.komi)
            self._size, self._komi, self._synced = state.size, state.komi, []
        color = go.BLACK if len(self._synced) % 2 == 0 else go.WHITE
        for mv in hist[len(self._synced):]:
            self.send("play %s %s" % ("b" if color == go.BLACK else "w", format_vertex(mv)))
            self._synced.append(mv)
            color = -color

    def get_move(self, state):
        self._sync(state)
        color = "b" if state.current_player == go.BLACK else "w"
        reply = self.send("genmove %s" % color).lower()
        mv = go.PASS_MOVE if reply in ("pass", "resign") else parse_vertex(reply, state.size)
        self._synced.append(mv)
        if reply == "resign":
            self.resigned = True
        return mv

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.send("quit")
            except Exception:  # noqa: BLE001
                pass
            try:
                self.proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                self.proc.kill()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
