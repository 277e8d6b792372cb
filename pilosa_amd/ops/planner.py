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


class NativeCountCompiler:
    """Batch compiler for ``Count(<bitmap tree>)`` PQL text over a fixed
    ``{field: DeviceView}`` map.

    The common shapes (Row(field=id) leaves under Intersect/Union/Difference/
    Xor) are compiled by the native scanner in pilosa_amd/native/pql_compile.cpp
    straight to QueryProg records (~0.3 us/query); anything else goes through
    the general parser + :class:`GpuPlanner` + ``compile_expr`` with the same
    view slots, so results never depend on which path compiled a query.
    """

    def __init__(self, views: Dict[str, object], exists_view=None):
        from pilosa_amd import _pql

        self._pql = _pql
        self.fields = {f: i for i, f in enumerate(views)}
        self.views = list(views.values())
        self.dirs = [v.rows for v in self.views]
        self.planner = GpuPlanner(lambda f, v: views[f], exists_view)
        self.native_hits = 0
        self.fallbacks = 0

    def compile(self, queries):
        """-> (progs QPROG_DTYPE[Q], views, S)."""
        import numpy as np

        from pilosa_amd.pql import parse_string

        from .device import QPROG_DTYPE, CompileError, compile_expr, pack_programs

        raw, ok = self._pql.compile_counts(list(queries), self.fields, self.dirs)
        progs = raw.view(QPROG_DTYPE)
        views = list(self.views)
        bad = np.nonzero(~ok)[0]
        self.native_hits += len(queries) - len(bad)
        if len(bad):
            self.fallbacks += len(bad)
            view_index = {id(v): i for i, v in enumerate(views)}
            comp = []
            for i in bad:
                calls = parse_string(queries[i]).calls
                if len(calls) != 1 or calls[0].name != "Count":
                    raise Unsupported("not a single Count query")
                try:
                    comp.append(compile_expr(self.planner.plan(calls[0]), view_index))
                except CompileError as e:
                    raise Unsupported(str(e)) from e
            progs[bad] = pack_programs(comp)
            if len(view_index) > len(views):
                extra = sorted((slot, vid) for vid, slot in view_index.items() if slot >= len(views))
                raise Unsupported(f"query referenced {len(extra)} view(s) outside the compiler's map")
        S = views[0].S if views else 0
        return progs, views, S
