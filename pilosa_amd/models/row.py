"""Row: a query result made of per-shard segments (reference: row.go).

Each segment is a host roaring ``Bitmap`` of absolute column ids
(``shard * ShardWidth + col``).  Segments of different shards are disjoint, so
``merge`` (the map/reduce reduce step, row.go:67-88) is a dict update — the
same property the multi-GPU path relies on (per-GPU results concatenate).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import numpy as np

from pilosa_amd import _roaring

from pilosa_amd.shardwidth import EXPONENT as _EXP
from pilosa_amd.shardwidth import SHARD_WIDTH
Bitmap = _roaring.Bitmap


class Row:
    __slots__ = ("segments", "keys", "attrs")

    def __init__(self, columns: Iterable[int] = (), segments: Optional[Dict[int, Bitmap]] = None):
        self.segments: Dict[int, Bitmap] = segments if segments is not None else {}
        self.keys: Optional[List[str]] = None
        self.attrs: Optional[dict] = None
        cols = np.fromiter(columns, dtype=np.uint64) if not isinstance(columns, np.ndarray) else columns
        if len(cols):
            self.add_columns(cols)

    # ------------------------------------------------------------ construction
    @classmethod
    def from_segment(cls, shard: int, bm: Bitmap) -> "Row":
        r = cls()
        if bm is not None and bm.any():
            r.segments[shard] = bm
        return r

    def add_columns(self, cols: np.ndarray):
        cols = np.asarray(cols, dtype=np.uint64)
        if len(cols) == 0:
            return
        shards = cols >> np.uint64(_EXP)
        for s in np.unique(shards):
            part = cols[shards == s]
            bm = self.segments.get(int(s))
            if bm is None:
                bm = self.segments[int(s)] = Bitmap()
            bm.add_many(part)

    def set_bit(self, col: int) -> bool:
        s = col >> _EXP
        bm = self.segments.get(s)
        if bm is None:
            bm = self.segments[s] = Bitmap()
        return bm.add(col)

    def segment(self, shard: int) -> Optional[Bitmap]:
        return self.segments.get(shard)

    def shards(self) -> List[int]:
        return sorted(self.segments)

    # ------------------------------------------------------------ algebra
    def _binary(self, other: "Row", fn, keep_left: bool, keep_right: bool) -> "Row":
        out = Row()
        for s in set(self.segments) | set(other.segments):
            a, b = self.segments.get(s), other.segments.get(s)
            if a is not None and b is not None:
                r = fn(a, b)
            elif a is not None:
                r = a.clone() if keep_left else None
            else:
                r = b.clone() if keep_right else None
            if r is not None and r.any():
                out.segments[s] = r
        return out

    def intersect(self, other: "Row") -> "Row":
        return self._binary(other, lambda a, b: a.intersect(b), False, False)

    def union(self, *others: "Row") -> "Row":
        out = Row()
        shards = set(self.segments)
        for o in others:
            shards |= set(o.segments)
        for s in shards:
            parts = [r.segments[s] for r in (self, *others) if s in r.segments]
            if len(parts) == 1:
                out.segments[s] = parts[0].clone()
            else:
                bm = Bitmap()
                bm.union_in_place(parts)
                if bm.any():
                    out.segments[s] = bm
        return out

    def difference(self, other: "Row") -> "Row":
        return self._binary(other, lambda a, b: a.difference(b), True, False)

    def xor(self, other: "Row") -> "Row":
        return self._binary(other, lambda a, b: a.xor(b), True, True)

    def shift(self, n: int = 1) -> "Row":
        """Shift columns up by n within each shard; bits shifted past a shard
        boundary move to the next shard's segment (row.go Shift)."""
        if n == 0:
            return self.clone()
        out = Row()
        for s in sorted(self.segments):
            shifted = self.segments[s].shift(n)
            # split by shard (at most two shards touched for n < ShardWidth)
            lo = s * SHARD_WIDTH
            cur = shifted.offset_range(lo, lo, lo + SHARD_WIDTH) if shifted.any() else None
            nxt = shifted.offset_range(lo + SHARD_WIDTH, lo + SHARD_WIDTH, lo + 2 * SHARD_WIDTH) \
                if shifted.any() else None
            for shard, part in ((s, cur), (s + 1, nxt)):
                if part is not None and part.any():
                    if shard in out.segments:
                        out.segments[shard] = out.segments[shard].union(part)
                    else:
                        out.segments[shard] = part
        return out

    def merge(self, other: "Row") -> None:
        for s, bm in other.segments.items():
            if s in self.segments:
                self.segments[s] = self.segments[s].union(bm)
            else:
                self.segments[s] = bm

    def intersection_count(self, other: "Row") -> int:
        n = 0
        for s, a in self.segments.items():
            b = other.segments.get(s)
            if b is not None:
                n += a.intersection_count(b)
        return n

    def clone(self) -> "Row":
        r = Row(segments={s: b.clone() for s, b in self.segments.items()})
        r.keys = list(self.keys) if self.keys is not None else None
        r.attrs = dict(self.attrs) if self.attrs is not None else None
        return r

    # ------------------------------------------------------------ inspection
    def count(self) -> int:
        return sum(b.count() for b in self.segments.values())

    def is_empty(self) -> bool:
        return not any(b.any() for b in self.segments.values())

    def any(self) -> bool:
        return not self.is_empty()

    def columns(self) -> np.ndarray:
        if not self.segments:
            return np.zeros(0, dtype=np.uint64)
        parts = [self.segments[s].slice() for s in sorted(self.segments)]
        return np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint64)

    def includes(self, col: int) -> bool:
        bm = self.segments.get(col >> _EXP)
        return bm is not None and bm.contains(col)

    def __eq__(self, other):
        if not isinstance(other, Row):
            return NotImplemented
        return np.array_equal(self.columns(), other.columns())

    def to_json(self) -> dict:
        out = {"attrs": self.attrs or {}, "columns": [int(c) for c in self.columns()]}
        if self.keys:
            out["keys"] = list(self.keys)
            out["columns"] = []
        return out

    def __repr__(self):
        cols = self.columns()
        return f"Row({cols[:10].tolist()}{'...' if len(cols) > 10 else ''}, n={len(cols)})"
