"""PQL parser: a hand-written recursive-descent parser with PEG semantics
(ordered choice, backtracking at alternatives) for the grammar in
reference pql/pql.peg:8-83.  Produces pilosa_amd.pql.ast objects with the
same argument conventions as the reference AST builder (pql/ast.go:34-233):
positional ``_col``, ``_row``, ``_field``, ``_timestamp`` keys, conditional
``a < f <= b`` → ``f ><[a', b']`` with bounds made inclusive, duplicate
arguments rejected, int64 range checked.
"""
from __future__ import annotations

import re
from typing import Any, List, Optional, Tuple

from .ast import BETWEEN, EQ, GT, GTE, LT, LTE, NEQ, Call, Condition, Query


# nesting bound shared with native/pql_parser.cpp (Parser::MAX_NESTING)
MAX_NESTING = 1000

class ParseError(Exception):
    pass


DUPLICATE_ARG = "duplicate argument provided"
INT_OUT_OF_RANGE = "integer value out of range"

_IDENT = re.compile(r"[A-Za-z][A-Za-z0-9]*")
_FIELD = re.compile(r"[A-Za-z][A-Za-z0-9_\-]*")
_RESERVED = ("_row", "_col", "_start", "_end", "_timestamp", "_field")
_TS = re.compile(r"[0-9]{4}-[01][0-9]-[0-3][0-9]T[0-9]{2}:[0-9]{2}")
_NUM1 = re.compile(r"-?[0-9]+(\.[0-9]*)?")
_NUM2 = re.compile(r"-?\.[0-9]+")
_BARE = re.compile(r"[A-Za-z0-9\-_:]+")
_UINT = re.compile(r"[1-9][0-9]*|0")
_CONDINT = re.compile(r"-?[1-9][0-9]*|0")
_SP = re.compile(r"[ \t\n]*")
_CALL_AHEAD = re.compile(r"[A-Za-z][A-Za-z0-9]*\(")
_INT64_MIN, _INT64_MAX = -(1 << 63), (1 << 63) - 1


class _Fail(Exception):
    """Internal backtracking signal."""


class _Args:
    """Argument map builder with the reference's duplicate detection."""

    __slots__ = ("d",)

    def __init__(self):
        self.d = {}

    def put(self, k, v):
        if k in self.d:
            raise ParseError(f"{DUPLICATE_ARG}: {k}")
        self.d[k] = v


class Parser:
    def __init__(self, s: str):
        self.s = s
        self.n = len(s)

    # ------------------------------------------------------------ lexing helpers
    def sp(self, i: int) -> int:
        s = self.s
        if i < self.n and s[i] not in " \t\n":
            return i
        return _SP.match(s, i).end()

    def lit(self, i: int, t: str) -> int:
        if self.s.startswith(t, i):
            return i + len(t)
        raise _Fail

    def rx(self, i: int, r) -> Tuple[int, str]:
        m = r.match(self.s, i)
        if not m:
            raise _Fail
        return m.end(), m.group(0)

    def open(self, i):
        return self.sp(self.lit(i, "("))

    def close(self, i):
        return self.sp(self.lit(i, ")"))

    def comma(self, i):
        return self.sp(self.lit(self.sp(i), ","))

    # ------------------------------------------------------------ top level
    def parse(self) -> Query:
        i = self.sp(0)
        calls = []
        while i < self.n:
            try:
                i, c = self.call(i)
            except _Fail:
                raise ParseError(self._err(i))
            except RecursionError:
                # the native parser bounds nesting at MAX_NESTING levels
                raise ParseError(f"query nesting exceeds {MAX_NESTING} levels") from None
            calls.append(c)
            i = self.sp(i)
        return Query(calls)

    def _err(self, i):
        line = self.s.count("\n", 0, i) + 1
        col = i - (self.s.rfind("\n", 0, i) + 1) + 1
        near = self.s[i:i + 20]
        return f"parse error at line {line}, column {col}: unexpected {near!r}"

    def call(self, i: int) -> Tuple[int, Call]:
        j, name = self.rx(i, _IDENT)
        special = {
            "Set": self._set, "SetRowAttrs": self._set_row_attrs, "SetColumnAttrs": self._set_col_attrs,
            "Clear": self._clear, "ClearRow": self._clear_row, "Store": self._store, "TopN": self._posfield_call,
            "Rows": self._posfield_call, "Range": self._range,
        }
        # PEG ordered choice: the literal forms are tried in grammar order, a
        # literal matches any identifier PREFIX (e.g. 'Set' of 'SetBit').
        for lit in ("Set", "SetRowAttrs", "SetColumnAttrs", "Clear", "ClearRow", "Store", "TopN", "Rows", "Range"):
            if self.s.startswith(lit, i):
                try:
                    return special[lit](i + len(lit), lit)
                except _Fail:
                    continue
        return self._generic(j, name)

    # ------------------------------------------------------------ special forms
    def _set(self, i, name):
        a = _Args()
        i = self.open(i)
        i = self._col(i, a)
        i = self.comma(i)
        i = self._args(i, a)
        try:
            k = self.comma(i)
            k, ts = self._timestampfmt(k)
            a.put("_timestamp", ts)
            i = k
        except _Fail:
            pass
        i = self.close(i)
        return i, Call(name, a.d)

    def _set_row_attrs(self, i, name):
        a = _Args()
        i = self.open(i)
        i, f = self.rx(i, _FIELD)
        a.put("_field", f)
        i = self.comma(i)
        i = self._rowpos(i, a)
        i = self.comma(i)
        i = self._args(i, a)
        i = self.close(i)
        return i, Call(name, a.d)

    def _set_col_attrs(self, i, name):
        a = _Args()
        i = self.open(i)
        i = self._col(i, a)
        i = self.comma(i)
        i = self._args(i, a)
        i = self.close(i)
        return i, Call(name, a.d)

    def _clear(self, i, name):
        return self._set_col_attrs(i, name)

    def _clear_row(self, i, name):
        a = _Args()
        i = self.open(i)
        i = self._arg(i, a)
        i = self.close(i)
        return i, Call(name, a.d)

    def _store(self, i, name):
        a = _Args()
        i = self.open(i)
        i, child = self.call(i)
        i = self.comma(i)
        i = self._arg(i, a)
        i = self.close(i)
        return i, Call(name, a.d, [child])

    def _posfield_call(self, i, name):
        a = _Args()
        children: List[Call] = []
        i = self.open(i)
        i, f = self.rx(i, _FIELD)
        a.put("_field", f)
        try:
            k = self.comma(i)
            k = self._allargs(k, a, children)
            i = k
        except _Fail:
            pass
        i = self.close(i)
        return i, Call(name, a.d, children)

    def _range(self, i, name):
        a = _Args()
        i = self.open(i)
        i, f = self._field(i)
        i = self.sp(i)
        i = self.lit(i, "=")
        i = self.sp(i)
        i, v = self._value(i)
        a.put(f, v)
        i = self.comma(i)
        if self.s.startswith("from=", i):
            i += 5
        i, ts = self._timestampfmt(i)
        a.put("from", ts)
        i = self.comma(i)
        if self.s.startswith("to=", i):
            i += 3
        i = self.sp(i)
        i, ts = self._timestampfmt(i)
        a.put("to", ts)
        i = self.close(i)
        return i, Call(name, a.d)

    def _generic(self, i, name):
        a = _Args()
        children: List[Call] = []
        i = self.open(i)
        i = self._allargs(i, a, children)
        try:
            i = self.comma(i)
        except _Fail:
            pass
        i = self.close(i)
        return i, Call(name, a.d, children)

    # ------------------------------------------------------------ args
    def _allargs(self, i, a: _Args, children: List[Call]):
        # Call (comma Call)* (comma args)? / args / sp
        if not _CALL_AHEAD.match(self.s, i):
            try:
                sub = _Args()
                k = self._args(i, sub)
                for kk, vv in sub.d.items():
                    a.put(kk, vv)
                return k
            except _Fail:
                return self.sp(i)
        try:
            k, c = self.call(i)
            kids = [c]
            while True:
                try:
                    k2 = self.comma(k)
                    k2, c2 = self.call(k2)
                    kids.append(c2)
                    k = k2
                except _Fail:
                    break
            try:
                k2 = self.comma(k)
                sub = _Args()
                k2 = self._args(k2, sub)
                for kk, vv in sub.d.items():
                    a.put(kk, vv)
                k = k2
            except _Fail:
                pass
            children.extend(kids)
            return k
        except _Fail:
            pass
        try:
            sub = _Args()
            k = self._args(i, sub)
            for kk, vv in sub.d.items():
                a.put(kk, vv)
            return k
        except _Fail:
            pass
        return self.sp(i)

    def _args(self, i, a: _Args):
        i = self._arg(i, a)
        while True:
            try:
                k = self.comma(i)
                k = self._arg(k, a)
                i = k
            except _Fail:
                break
        return self.sp(i)

    def _field(self, i):
        for r in _RESERVED:
            if self.s.startswith(r, i):
                # fieldExpr is tried first but cannot start with '_'
                return i + len(r), r
        return self.rx(i, _FIELD)

    def _arg(self, i, a: _Args):
        # fast path: field '=' value
        m = _FIELD.match(self.s, i)
        if m and not self.s.startswith("_", i):
            k = self.sp(m.end())
            if self.s.startswith("=", k) and not self.s.startswith("==", k):
                k, v = self._value(self.sp(k + 1))
                a.put(m.group(0), v)
                return k
        # field sp '=' sp value
        try:
            k, f = self._field(i)
            k = self.sp(k)
            k = self.lit(k, "=")
            if self.s.startswith("=", k):  # '==' is a condition, not assignment
                raise _Fail
            k = self.sp(k)
            k, v = self._value(k)
            a.put(f, v)
            return k
        except _Fail:
            pass
        # field sp COND sp value
        try:
            k, f = self._field(i)
            k = self.sp(k)
            op = None
            for t in ("><", "<=", ">=", "==", "!=", "<", ">"):
                if self.s.startswith(t, k):
                    op = t
                    k += len(t)
                    break
            if op is None:
                raise _Fail
            k = self.sp(k)
            k, v = self._value(k)
            a.put(f, Condition(op, v))
            return k
        except _Fail:
            pass
        # conditional: int < field <= int
        k, lo = self.rx(i, _CONDINT)
        k = self.sp(k)
        k, op1 = self._condlt(k)
        k, f = self.rx(k, _FIELD)
        k = self.sp(k)
        k, op2 = self._condlt(k)
        k, hi = self.rx(k, _CONDINT)
        k = self.sp(k)
        low, high = self._int(lo), self._int(hi)
        if op1 == "<":
            low += 1
        if op2 == "<":
            high -= 1
        a.put(f, Condition(BETWEEN, [low, high]))
        return k

    def _condlt(self, i):
        if self.s.startswith("<=", i):
            return self.sp(i + 2), "<="
        if self.s.startswith("<", i):
            return self.sp(i + 1), "<"
        raise _Fail

    @staticmethod
    def _int(s: str) -> int:
        v = int(s)
        if v < _INT64_MIN or v > _INT64_MAX:
            raise ParseError(f'{INT_OUT_OF_RANGE}: strconv.ParseInt: parsing "{s}": value out of range')
        return v

    def _num(self, s: str):
        if "." in s:
            return float(s)
        return self._int(s)

    def _col(self, i, a: _Args):
        return self._posval(i, a, "_col")

    def _rowpos(self, i, a: _Args):
        return self._posval(i, a, "_row")

    def _posval(self, i, a: _Args, key):
        m = _UINT.match(self.s, i)
        if m:
            a.put(key, self._num(m.group(0)))
            return m.end()
        if self.s.startswith("'", i):
            j, v = self._single(i + 1)
            a.put(key, v)
            return self.lit(j, "'")
        if self.s.startswith('"', i):
            j, raw = self._double_raw(i + 1)
            a.put(key, raw)  # positional strings are not unquoted (ast addPosStr)
            return self.lit(j, '"')
        raise _Fail

    def _timestampfmt(self, i):
        if self.s.startswith('"', i):
            j, ts = self.rx(i + 1, _TS)
            return self.lit(j, '"'), ts
        if self.s.startswith("'", i):
            j, ts = self.rx(i + 1, _TS)
            return self.lit(j, "'"), ts
        return self.rx(i, _TS)

    def _single(self, i):
        j = i
        while j < self.n:
            if self.s.startswith("\\'", j) or self.s.startswith("\\\\", j):
                j += 2
                continue
            if self.s[j] == "'":
                break
            j += 1
        return j, self.s[i:j]

    def _double_raw(self, i):
        j = i
        while j < self.n:
            if self.s.startswith('\\"', j) or self.s.startswith("\\\\", j):
                j += 2
                continue
            if self.s[j] == '"':
                break
            j += 1
        return j, self.s[i:j]

    # ------------------------------------------------------------ values
    def _value(self, i):
        if self.s.startswith("[", i):
            k = self.sp(i + 1)
            vals = []
            k, v = self._item(k)
            vals.append(v)
            while True:
                try:
                    k2 = self.comma(k)
                    k2, v = self._item(k2)
                    vals.append(v)
                    k = k2
                except _Fail:
                    break
            k = self.sp(k)
            k = self.lit(k, "]")
            return self.sp(k), vals
        return self._item(i)

    def _peek_end(self, i) -> bool:
        # &(comma / sp close)
        j = self.sp(i)
        return j < self.n and self.s[j] in ",)"

    def _item(self, i):
        for word, val in (("null", None), ("true", True), ("false", False)):
            if self.s.startswith(word, i) and self._peek_end(i + len(word)):
                return i + len(word), val
        c0 = self.s[i:i + 1]
        if c0 in ('"', "'") or c0.isdigit():
            try:
                return self._timestampfmt(i)
            except _Fail:
                pass
        m = _NUM1.match(self.s, i) or _NUM2.match(self.s, i)
        if m:
            return m.end(), self._num(m.group(0))
        m = _IDENT.match(self.s, i)
        if m:
            try:
                k = self.open(m.end())
                a = _Args()
                kids: List[Call] = []
                k = self._allargs(k, a, kids)
                try:
                    k = self.comma(k)
                except _Fail:
                    pass
                k = self.close(k)
                return k, Call(m.group(0), a.d, kids)
            except _Fail:
                pass
        m = _BARE.match(self.s, i)
        if m:
            return m.end(), m.group(0)
        if self.s.startswith('"', i):
            j, raw = self._double_raw(i + 1)
            k = self.lit(j, '"')
            return k, _unquote(raw)
        if self.s.startswith("'", i):
            j, raw = self._single(i + 1)
            k = self.lit(j, "'")
            return k, raw
        raise _Fail


def _unquote(raw: str) -> str:
    out = []
    i = 0
    while i < len(raw):
        ch = raw[i]
        if ch == "\\" and i + 1 < len(raw):
            nx = raw[i + 1]
            mp = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'", "0": "\0"}
            if nx in mp:
                out.append(mp[nx])
                i += 2
                continue
            if nx == "x" and i + 3 < len(raw):
                out.append(chr(int(raw[i + 2:i + 4], 16)))
                i += 4
                continue
            if nx == "u" and i + 5 < len(raw):
                out.append(chr(int(raw[i + 2:i + 6], 16)))
                i += 6
                continue
        out.append(ch)
        i += 1
    return "".join(out)


def parse_string_py(s: str) -> Query:
    """Pure-Python parser (executable specification of the native one)."""
    return Parser(s).parse()


try:  # native parser (pilosa_amd/native/pql_parser.cpp)
    from pilosa_amd import _pql as _native
except ImportError:  # pragma: no cover - build() not run yet
    _native = None


def parse_string(s: str) -> Query:
    """Parse a PQL string (pql/parser.go:49 ParseString)."""
    if _native is not None:
        return Query(_native.parse_calls(s))
    return Parser(s).parse()
