"""PQL abstract syntax tree (reference: pql/ast.go, pql/token.go).

``Call.__str__`` reproduces the reference's canonical form (ast.go:423-469):
children first, then args in sorted key order, conditions as ``key OP value``,
strings double-quoted, lists as ``[a,b]`` — it is what a coordinator forwards
to remote nodes.
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Dict, List, Optional

from pilosa_amd.errors import PilosaError


class ArgError(PilosaError, ValueError):
    """A call argument of the wrong type or range (pql/ast.go Call.*Arg errors)."""

# tokens (pql/token.go)
ILLEGAL, EQ, NEQ, LT, LTE, GT, GTE, BETWEEN = "ILLEGAL", "==", "!=", "<", "<=", ">", ">=", "><"
TOKENS = (EQ, NEQ, LT, LTE, GT, GTE, BETWEEN)

TIME_FORMAT = "%Y-%m-%dT%H:%M"


class Condition:
    __slots__ = ("op", "value")

    def __init__(self, op: str, value: Any):
        self.op = op
        self.value = value

    def __eq__(self, other):
        return isinstance(other, Condition) and self.op == other.op and self.value == other.value

    def __repr__(self):
        return f"Condition({self.op!r}, {self.value!r})"

    def __str__(self):
        return f"{self.op} {format_value(self.value)}"

    def int_slice_value(self) -> List[int]:
        if not isinstance(self.value, list):
            raise ArgError(f"unexpected type {type(self.value).__name__} in IntSliceValue, val {self.value}")
        out = []
        for v in self.value:
            if isinstance(v, bool) or not isinstance(v, int):
                raise ArgError(f"unexpected value type {type(v).__name__} in IntSliceValue, val {v}")
            out.append(v)
        return out


def is_reserved_arg(name: str) -> bool:
    return name.startswith("_") or name in ("from", "to")


class Call:
    __slots__ = ("name", "args", "children")

    def __init__(self, name: str, args: Optional[Dict[str, Any]] = None, children: Optional[List["Call"]] = None):
        self.name = name
        self.args: Dict[str, Any] = args if args is not None else {}
        self.children: List[Call] = children if children is not None else []

    def __eq__(self, other):
        return (isinstance(other, Call) and self.name == other.name and self.args == other.args
                and self.children == other.children)

    def __repr__(self):
        return f"Call({self.name!r}, {self.args!r}, {self.children!r})"

    def clone(self) -> "Call":
        return Call(self.name, dict(self.args), [c.clone() for c in self.children])

    # ---- typed arg accessors (ast.go:272-392); return (value, present)
    def field_arg(self) -> str:
        for k in self.args:
            if not is_reserved_arg(k):
                return k
        raise ArgError("no field argument specified")

    def bool_arg(self, key):
        if key not in self.args:
            return False, False
        v = self.args[key]
        if not isinstance(v, bool):
            raise ArgError(f"could not convert {v} of type {type(v).__name__} to bool in Call.BoolArg")
        return v, True

    def uint_arg(self, key):
        if key not in self.args:
            return 0, False
        v = self.args[key]
        if isinstance(v, bool) or not isinstance(v, int):
            raise ArgError(f"could not convert {v} of type {type(v).__name__} to uint64 in Call.UintArg")
        if v < 0:
            raise ArgError(f"value for '{key}' must be positive, but got {v}")
        return v, True

    def int_arg(self, key):
        if key not in self.args:
            return 0, False
        v = self.args[key]
        if isinstance(v, bool) or not isinstance(v, int):
            raise ArgError(f"could not convert {v} of type {type(v).__name__} to int64 in Call.IntArg")
        return v, True

    def uint_slice_arg(self, key):
        if key not in self.args:
            return None, False
        v = self.args[key]
        if not isinstance(v, list) or not all(isinstance(x, int) and not isinstance(x, bool) for x in v):
            raise ArgError(f"unexpected type {type(v).__name__} in UintSliceArg, val {v}")
        return [int(x) for x in v], True

    def call_arg(self, key):
        if key not in self.args:
            return None, False
        v = self.args[key]
        if not isinstance(v, Call):
            raise ArgError(f"could not convert {v} of type {type(v).__name__} to Call in Call.CallArg")
        return v, True

    def has_condition_arg(self) -> bool:
        return any(isinstance(v, Condition) for v in self.args.values())

    def __str__(self):
        parts = [str(c) for c in self.children]
        for k in sorted(self.args):
            v = self.args[k]
            if isinstance(v, Condition):
                parts.append(f"{k} {v}")
            else:
                parts.append(f"{k}={format_value(v)}")
        return f"{self.name or '!UNNAMED'}({', '.join(parts)})"


def _go_quote(s: str) -> str:
    out = ['"']
    for ch in s:
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\r":
            out.append("\\r")
        elif ord(ch) < 0x20:
            out.append("\\x%02x" % ord(ch))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def format_value(v: Any) -> str:
    if isinstance(v, str):
        return _go_quote(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    if v is None:
        # the reference prints Go's "<nil>", which its own grammar cannot
        # re-parse when a call is forwarded to a remote node; emit PQL null.
        return "null"
    if isinstance(v, list):
        return "[" + ",".join(_go_quote(x) if isinstance(x, str) else format_value(x) for x in v) + "]"
    if isinstance(v, _dt.datetime):
        return '"' + v.strftime(TIME_FORMAT) + '"'
    if isinstance(v, float):
        r = repr(v)
        if r.endswith(".0"):
            r = r[:-2]
        return r
    return str(v)


class Query:
    __slots__ = ("calls", "source")

    def __init__(self, calls: Optional[List[Call]] = None, source: Optional[str] = None):
        self.calls: List[Call] = calls or []
        # the PQL text it was parsed from (the mesh forwards it as is, so
        # the ranks parse one request once instead of per re-printed call)
        self.source = source

    def write_call_n(self) -> int:
        return sum(1 for c in self.calls if c.name in ("Set", "Clear", "SetRowAttrs", "SetColumnAttrs"))

    def __str__(self):
        return "\n".join(str(c) for c in self.calls)

    def __repr__(self):
        return f"Query({self.calls!r})"
