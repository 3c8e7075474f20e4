"""Erlang terms in Python: atoms, exact (=:=) equality, and a reader/writer for the
subset of Erlang term text that scene files use (``file:consult/1`` compatible).

The reference's scene is an Erlang list of records (raytracer.erl:618-665); a record
``#vector{x=4, y=0, z=10}`` is the tuple ``{vector, 4, 0, 10}``.  Here a tuple is a
Python tuple, an atom an :class:`Atom` (a ``str`` subclass), an integer a Python int
and a float a Python float — keeping the int/float distinction that Erlang's exact
equality (used by shadow_factor/4's match, raytracer.erl:263) depends on.
"""
from __future__ import annotations

import math
import re

__all__ = ["Atom", "exact_eq", "parse_terms", "parse_term", "format_term", "consult", "write_terms"]


class Atom(str):
    """An Erlang atom.  Compares equal to the plain string of its name."""

    __slots__ = ()

    def __repr__(self):
        return f"Atom({str.__repr__(self)})"


def exact_eq(a, b) -> bool:
    """Erlang ``=:=``: structural equality where 4 and 4.0 differ."""
    if isinstance(a, tuple) or isinstance(b, tuple):
        return (isinstance(a, tuple) and isinstance(b, tuple) and len(a) == len(b)
                and all(exact_eq(x, y) for x, y in zip(a, b)))
    if isinstance(a, list) or isinstance(b, list):
        return (isinstance(a, list) and isinstance(b, list) and len(a) == len(b)
                and all(exact_eq(x, y) for x, y in zip(a, b)))
    if isinstance(a, bool) or isinstance(b, bool):
        return a is b
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return type(a) is type(b) and a == b
    return type(a) is type(b) and a == b


def exact_key(t):
    """A hashable key with ``exact_key(a) == exact_key(b)`` iff ``exact_eq(a, b)`` (Erlang
    ``=:=``): numbers keep their int/float type, atoms differ from strings."""
    if isinstance(t, tuple):
        return ("T",) + tuple(exact_key(x) for x in t)
    if isinstance(t, list):
        return ("L",) + tuple(exact_key(x) for x in t)
    if isinstance(t, bool):
        return ("B", t)
    if isinstance(t, float):
        return ("F", t)
    if isinstance(t, int):
        return ("I", t)
    return (type(t).__name__, t)


# ---- reader ---------------------------------------------------------------------------
_TOKEN = re.compile(r"""
    (?P<ws>\s+|%[^\n]*)
  | (?P<float>[+-]?\d+\.\d+(?:[eE][+-]?\d+)?)
  | (?P<based>[+-]?\d+\#[0-9a-zA-Z]+)
  | (?P<int>[+-]?\d+)
  | (?P<atom>[a-z][A-Za-z0-9_@]*)
  | (?P<qatom>'(?:[^'\\]|\\.)*')
  | (?P<string>"(?:[^"\\]|\\.)*")
  | (?P<punct>[{}\[\],.|])
""", re.VERBOSE)


def _tokens(text: str):
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ValueError(f"bad Erlang term text at offset {pos}: {text[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        yield kind, m.group(kind)


class _Parser:
    def __init__(self, text):
        self.toks = list(_tokens(text))
        self.i = 0

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else (None, None)

    def take(self, want=None):
        tok = self.peek()
        if tok[0] is None:
            raise ValueError("unexpected end of term text")
        if want is not None and tok[1] != want:
            raise ValueError(f"expected {want!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def term(self):
        kind, val = self.take()
        if kind == "float":
            return float(val)
        if kind == "int":
            return int(val)
        if kind == "based":
            sign = -1 if val.startswith("-") else 1
            base, digits = val.lstrip("+-").split("#")
            return sign * int(digits, int(base))
        if kind == "atom":
            return Atom(val)
        if kind == "qatom":
            return Atom(bytes(val[1:-1], "utf-8").decode("unicode_escape"))
        if kind == "string":
            return [ord(c) for c in bytes(val[1:-1], "utf-8").decode("unicode_escape")]
        if val == "{":
            items = self.seq("}")
            return tuple(items)
        if val == "[":
            items = self.seq("]", allow_tail=True)
            return items
        raise ValueError(f"unexpected token {val!r}")

    def seq(self, close, allow_tail=False):
        items = []
        if self.peek()[1] == close:
            self.take()
            return items
        while True:
            items.append(self.term())
            nxt = self.take()[1]
            if nxt == ",":
                continue
            if nxt == close:
                return items
            if nxt == "|" and allow_tail:
                tail = self.term()
                self.take(close)
                if not isinstance(tail, list):
                    raise ValueError("improper lists are not supported")
                return items + tail
            raise ValueError(f"expected ',' or {close!r}, got {nxt!r}")


def parse_terms(text: str) -> list:
    """Parse a sequence of dot-terminated terms (the format ``file:consult/1`` reads)."""
    p = _Parser(text)
    out = []
    while p.peek()[0] is not None:
        out.append(p.term())
        p.take(".")
    return out


def parse_term(text: str):
    """Parse one term; a trailing ``.`` is optional."""
    p = _Parser(text)
    t = p.term()
    if p.peek()[1] == ".":
        p.take()
    if p.peek()[0] is not None:
        raise ValueError("trailing text after term")
    return t


def consult(path: str) -> list:
    with open(path, "r", encoding="utf-8") as f:
        return parse_terms(f.read())


# ---- writer ----------------------------------------------------------------------------
_BARE_ATOM = re.compile(r"^[a-z][A-Za-z0-9_@]*$")


def _format_float(x: float) -> str:
    if not math.isfinite(x):
        raise ValueError("Erlang has no non-finite floats")
    s = repr(x)  # shortest round-trip representation, like Erlang's ~p
    mant, _, exp = s.partition("e")
    if "." not in mant:
        mant += ".0"
    if exp:
        return f"{mant}e{int(exp)}"
    return mant


def format_term(t) -> str:
    if isinstance(t, bool):
        return "true" if t else "false"
    if isinstance(t, Atom):
        return t if _BARE_ATOM.match(t) else "'" + t.replace("\\", "\\\\").replace("'", "\\'") + "'"
    if isinstance(t, int):
        return str(t)
    if isinstance(t, float):
        return _format_float(t)
    if isinstance(t, tuple):
        return "{" + ",".join(format_term(x) for x in t) + "}"
    if isinstance(t, list):
        return "[" + ",".join(format_term(x) for x in t) + "]"
    if isinstance(t, str):
        return format_term(Atom(t))
    raise TypeError(f"cannot format {type(t).__name__} as an Erlang term")


def write_terms(path: str, terms: list, header: str = "") -> None:
    with open(path, "w", encoding="utf-8") as f:
        if header:
            for line in header.splitlines():
                f.write(f"% {line}\n")
        for t in terms:
            f.write(format_term(t) + ".\n")
