"""PQL call tree -> device expression planner.

Bitmap calls (Row/Intersect/Union/Difference/Xor/Not) become ``Leaf``/``Op``
trees evaluated by the batched HIP kernels (reference evaluation tree:
executor.go:585-680, 1444-1533, 1668-1790).  The full executor
(pilosa_amd/executor.py) uses :class:`GpuPlanner` with its own view resolver;
``BenchPlanner`` is the same planner over a fixed ``{field: DeviceView}`` map.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

from pilosa_amd.pql import Call

from .device import Leaf, Op


class Unsupported(Exception):
    """The call cannot run on the device path (caller falls back to the host)."""


class GpuPlanner:
    def __init__(self, resolve: Callable[[str, str], object], exists_view: Optional[Callable[[], object]] = None):
        # resolve(field, view_name) -> DeviceView
        self.resolve = resolve
        self.exists_view = exists_view

    def plan(self, c: Call):
        if c.name == "Count":
            if len(c.children) != 1:
                raise Unsupported("Count needs one child")
            return self.plan(c.children[0])
        return self.bitmap(c)

    def bitmap(self, c: Call):
        n = c.name
        if n == "Row" or n == "Bitmap":
            args = c.args
            if len(args) == 1:
                # fast path: Row(field=<int>)
                for f, row in args.items():
                    t = type(row)
                    if t is int and not f.startswith("_") and f not in ("from", "to"):
                        return Leaf(self.resolve(f, "standard"), row)
            if c.has_condition_arg():
                raise Unsupported("BSI row")
            if any(k in args for k in ("from", "to", "_start", "_end")):
                raise Unsupported("time range")
            f = c.field_arg()
            row = args[f]
            if isinstance(row, bool):
                row = 1 if row else 0
            if not isinstance(row, int):
                raise Unsupported("untranslated row key")
            return Leaf(self.resolve(f, "standard"), int(row))
        if n in ("Intersect", "Union", "Difference", "Xor"):
            if not c.children:
                raise Unsupported("empty set op")
            op = _SETOPS[n]
            kids = tuple([self.bitmap(k) for k in c.children])
            if len(kids) == 1:
                return kids[0]
            return Op(op, kids)
        if n == "Not":
            if self.exists_view is None or len(c.children) != 1:
                raise Unsupported("Not without existence tracking")
            return Op("andnot", (Leaf(self.exists_view(), 0), self.bitmap(c.children[0])))
        raise Unsupported(n)


_SETOPS = {"Intersect": "and", "Union": "or", "Difference": "andnot", "Xor": "xor"}


class BenchPlanner(GpuPlanner):
    def __init__(self, views: Dict[str, object]):
        super().__init__(lambda f, v: views[f])
