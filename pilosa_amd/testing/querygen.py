"""PQL call builders and a random query generator for tests and load
generation (reference internal/test/querygenerator.go): ``PQL(Union(Row(
"aaa", 10), Row("bbb", 9)))`` builds the same AST as parsing the text, and
``QueryGenerator`` draws random Count/bitmap queries over given fields."""
from __future__ import annotations

import random
from typing import List, Optional, Sequence

from pilosa_amd.pql.ast import Call, Query


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
    """Random PQL over ``fields`` with rows in [0, rows): nested set
    operations up to ``depth`` levels, optionally wrapped in Count."""

    OPS = (Union, Intersect, Difference, Xor)

    def __init__(self, fields: Sequence[str], rows: int, seed: Optional[int] = None, depth: int = 2):
        self.fields, self.rows, self.depth = list(fields), int(rows), int(depth)
        self.rng = random.Random(seed)

    def bitmap(self, depth: Optional[int] = None) -> Call:
        depth = self.depth if depth is None else depth
        if depth <= 0 or self.rng.random() < 0.3:
            return Row(self.rng.choice(self.fields), self.rng.randrange(self.rows))
        op = self.rng.choice(self.OPS)
        return op(*[self.bitmap(depth - 1) for _ in range(self.rng.randint(2, 3))])

    def count(self) -> Call:
        return Count(self.bitmap())

    def queries(self, n: int, count: bool = True) -> List[str]:
        return [str(self.count() if count else self.bitmap()) for _ in range(n)]
