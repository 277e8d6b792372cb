"""Random PQL generator (reference internal/test/querygenerator.go).

Builds random, valid bitmap-query trees over a given schema: Row over set /
time fields (with optional from/to), BSI conditions on int fields, and
Intersect / Union / Difference / Xor / Not nesting, wrapped in Count(),
TopN(), Sum(), Min() / Max(), GroupBy() or returned as rows.  Used by the
differential fuzz tests (host vs GPU executor, native vs Python parser)."""
from __future__ import annotations

import random
from typing import Dict, List, Optional, Sequence

from pilosa_amd.pql.ast import Call, Query


# ------------------------------------------------------------ call builders
def PQL(*calls: Call) -> Query:
    return Query(list(calls))


def Row(field: str, row: int) -> Call:
    return Call("Row", {field: int(row)})


def _nest(name: str, kids: Sequence[Call]) -> Call:
    return Call(name, {}, list(kids))


def Count(*kids: Call) -> Call:
    return _nest("Count", kids)


def Union(*kids: Call) -> Call:
    return _nest("Union", kids)


def Intersect(*kids: Call) -> Call:
    return _nest("Intersect", kids)


def Difference(*kids: Call) -> Call:
    return _nest("Difference", kids)


def Xor(*kids: Call) -> Call:
    return _nest("Xor", kids)


def Not(*kids: Call) -> Call:
    return _nest("Not", kids)


def Set(col: int, field: str, row: int) -> Call:
    return Call("Set", {"_col": int(col), field: int(row)})


def Clear(col: int, field: str, row: int) -> Call:
    return Call("Clear", {"_col": int(col), field: int(row)})



class QueryGenerator:
    def __init__(self, seed: int = 0, set_fields: Sequence[str] = ("f",), int_fields: Sequence[str] = (),
                 time_fields: Sequence[str] = (), max_row: int = 10, int_range=(-100, 100),
                 time_range=("2019-01-01T00:00", "2021-01-01T00:00"), exists: bool = True):
        self.r = random.Random(seed)
        self.set_fields = list(set_fields)
        self.int_fields = list(int_fields)
        self.time_fields = list(time_fields)
        self.max_row = max_row
        self.int_range = int_range
        self.time_range = time_range
        self.exists = exists

    # ------------------------------------------------------------ leaves
    def row(self) -> str:
        r = self.r
        kinds = ["set"] * 4 + (["int"] * 2 if self.int_fields else []) + (["time"] if self.time_fields else [])
        k = r.choice(kinds)
        if k == "set":
            return f"Row({r.choice(self.set_fields)}={r.randrange(self.max_row)})"
        if k == "time":
            f = r.choice(self.time_fields)
            y0, y1 = sorted(r.sample(range(2019, 2022), 2))
            m0, m1 = r.randrange(1, 13), r.randrange(1, 13)
            return f"Row({f}={r.randrange(self.max_row)}, from='{y0}-{m0:02d}-01T00:00', to='{y1}-{m1:02d}-01T00:00')"
        f = r.choice(self.int_fields)
        lo, hi = self.int_range
        op = r.choice(["<", "<=", ">", ">=", "==", "!=", "><", "null"])
        if op == "><":
            a, b = sorted((r.randint(lo, hi), r.randint(lo, hi)))
            return f"Row({f} >< [{a}, {b}])"
        if op == "null":
            return f"Row({f} != null)"
        return f"Row({f} {op} {r.randint(lo - 10, hi + 10)})"

    # ------------------------------------------------------------ trees
    def bitmap(self, depth: int = 3) -> str:
        r = self.r
        if depth <= 0 or r.random() < 0.35:
            return self.row()
        op = r.choice(["Intersect", "Union", "Difference", "Xor"] + (["Not"] if self.exists else []))
        if op == "Not":
            return f"Not({self.bitmap(depth - 1)})"
        n = r.randint(1, 3)
        return f"{op}({', '.join(self.bitmap(depth - 1) for _ in range(n))})"

    def query(self, depth: int = 3) -> str:
        r = self.r
        kinds = ["count"] * 4 + ["row", "topn", "groupby"] + (["sum", "min", "max"] if self.int_fields else [])
        k = r.choice(kinds)
        b = self.bitmap(depth)
        if k == "count":
            return f"Count({b})"
        if k == "row":
            return b
        if k == "topn":
            return f"TopN({r.choice(self.set_fields)}, {b}, n={r.randint(1, 5)})"
        if k == "groupby":
            f = r.choice(self.set_fields)
            return f"GroupBy(Rows({f}), filter={b}, limit={r.randint(1, 20)})"
        f = r.choice(self.int_fields)
        name = {"sum": "Sum", "min": "Min", "max": "Max"}[k]
        return f"{name}({b}, field={f})"

    def queries(self, n: int, depth: int = 3) -> List[str]:
        return [self.query(depth) for _ in range(n)]
