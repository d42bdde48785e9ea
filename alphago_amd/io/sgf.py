"""Minimal SGF (FF[1-4]) reader/writer.

Replaces the external ``sgf`` package the reference imports (util.py:70,
game_converter.py:10) — not installed here.  Produces a collection of game
trees; each tree has a main line of nodes (dicts: property -> list of values)
and variations.
"""
from __future__ import annotations

from typing import Dict, List, Optional


class SGFParseError(ValueError):
    pass


class Node:
    __slots__ = ("properties",)

    def __init__(self, properties: Optional[Dict[str, List[str]]] = None):
        self.properties = properties or {}

    def __repr__(self):
        return "Node(%r)" % self.properties


class GameTree:
    def __init__(self):
        self.nodes: List[Node] = []
        self.children: List["GameTree"] = []

    @property
    def root(self) -> Node:
        return self.nodes[0]

    @property
    def rest(self) -> List[Node]:
        """Main line after the root (follows the first variation)."""
        out = list(self.nodes[1:])
        t = self
        while t.children:
            t = t.children[0]
            out.extend(t.nodes)
        return out


class _Parser:
    def __init__(self, text: str):
        self.s = text
        self.i = 0
        self.n = len(text)

    def ws(self):
        while self.i < self.n and self.s[self.i].isspace():
            self.i += 1

    def collection(self) -> List[GameTree]:
        trees = []
        self.ws()
        while self.i < self.n:
            if self.s[self.i] != "(":
                raise SGFParseError("expected '(' at %d" % self.i)
            trees.append(self.tree())
            self.ws()
        if not trees:
            raise SGFParseError("empty SGF collection")
        return trees

    def tree(self) -> GameTree:
        assert self.s[self.i] == "("
        self.i += 1
        t = GameTree()
        self.ws()
        while self.i < self.n and self.s[self.i] == ";":
            self.i += 1
            t.nodes.append(self.node())
            self.ws()
        while self.i < self.n and self.s[self.i] == "(":
            t.children.append(self.tree())
            self.ws()
        if self.i >= self.n or self.s[self.i] != ")":
            raise SGFParseError("expected ')' at %d" % self.i)
        self.i += 1
        if not t.nodes and not t.children:
            raise SGFParseError("empty game tree")
        return t

    def node(self) -> Node:
        props: Dict[str, List[str]] = {}
        self.ws()
        while self.i < self.n and (self.s[self.i].isalpha()):
            j = self.i
            while self.i < self.n and self.s[self.i].isalpha():
                self.i += 1
            # FF[3] allows lowercase letters inside identifiers (e.g. "AddBlack"); keep the capitals
            ident = "".join(c for c in self.s[j:self.i] if c.isupper()) or self.s[j:self.i]
            self.ws()
            vals = []
            while self.i < self.n and self.s[self.i] == "[":
                vals.append(self.value())
                self.ws()
            if not vals:
                raise SGFParseError("property %s without value at %d" % (ident, self.i))
            props.setdefault(ident, []).extend(vals)
        return Node(props)

    def value(self) -> str:
        assert self.s[self.i] == "["
        self.i += 1
        out = []
        while self.i < self.n:
            c = self.s[self.i]
            if c == "\\":
                self.i += 1
                if self.i < self.n:
                    nxt = self.s[self.i]
                    if nxt == "\n":  # soft line break
                        pass
                    else:
                        out.append(nxt)
                self.i += 1
                continue
            if c == "]":
                self.i += 1
                return "".join(out)
            out.append(c)
            self.i += 1
        raise SGFParseError("unterminated property value")


def parse(text: str) -> List[GameTree]:
    return _Parser(text).collection()


def _esc(v: str) -> str:
    return v.replace("\\", "\\\\").replace("]", "\\]")


def dumps(root_props: Dict[str, List[str]], nodes: List[Dict[str, List[str]]]) -> str:
    """Serialise a single main line game."""
    def node(p):
        return ";" + "".join(k + "".join("[%s]" % _esc(str(v)) for v in vs) for k, vs in p.items())
    return "(" + node(root_props) + "".join("\n" + node(p) for p in nodes) + ")\n"
