"""(row, column) pair iterators (reference iterator.go:24-194), used by the
anti-entropy block merge (``Fragment.merge_block``) to walk replica pair sets
in order.

The reference drives them one pair at a time through Go interfaces.  Here
every iterator is backed by a sorted uint64 *position* array (row * W +
column, W = the shard width) so seeks are binary searches and whole runs can
be drained as numpy slices (``drain``); the pair-at-a-time ``next`` /
``peek`` / ``unread`` API is kept for callers and tests that want the
reference's semantics.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np

from pilosa_amd.errors import PilosaError
from pilosa_amd.shardwidth import SHARD_WIDTH

EOF = (0, 0, True)


class SliceIterator:
    """Pairs from two equal-length slices, already sorted by (row, column)
    (iterator.go newSliceIterator)."""

    def __init__(self, row_ids: Optional[Sequence[int]], column_ids: Optional[Sequence[int]],
                 width: int = SHARD_WIDTH):
        r = np.asarray(row_ids if row_ids is not None else [], dtype=np.uint64)
        c = np.asarray(column_ids if column_ids is not None else [], dtype=np.uint64)
        if len(r) != len(c):
            raise PilosaError(f"pilosa.SliceIterator: pair length mismatch: {len(r)} != {len(c)}")
        self.rows, self.cols = r, c
        self.width = int(width)
        self.i = 0

    def seek(self, row: int, col: int):
        """Position at the first pair >= (row, col)."""
        key = (row, col)
        lo, hi = 0, len(self.rows)
        while lo < hi:
            mid = (lo + hi) // 2
            if (int(self.rows[mid]), int(self.cols[mid])) < key:
                lo = mid + 1
            else:
                hi = mid
        self.i = lo

    def next(self) -> Tuple[int, int, bool]:
        if self.i >= len(self.rows):
            return EOF
        r, c = int(self.rows[self.i]), int(self.cols[self.i])
        self.i += 1
        return r, c, False

    def drain(self) -> Tuple[np.ndarray, np.ndarray]:
        """Every remaining pair at once (rows, columns)."""
        r, c = self.rows[self.i:], self.cols[self.i:]
        self.i = len(self.rows)
        return r, c


class RoaringIterator:
    """Pairs of a fragment bitmap's positions (row * width + column),
    iterator.go newRoaringIterator."""

    def __init__(self, positions: np.ndarray, width: int = SHARD_WIDTH):
        self.pos = np.asarray(positions, dtype=np.uint64)
        self.width = np.uint64(width)
        self.i = 0

    def seek(self, row: int, col: int):
        self.i = int(np.searchsorted(self.pos, np.uint64(row) * self.width + np.uint64(col)))

    def next(self) -> Tuple[int, int, bool]:
        if self.i >= len(self.pos):
            return EOF
        p = self.pos[self.i]
        self.i += 1
        return int(p // self.width), int(p % self.width), False

    def drain(self) -> Tuple[np.ndarray, np.ndarray]:
        p = self.pos[self.i:]
        self.i = len(self.pos)
        return p // self.width, p % self.width


class BufIterator:
    """One pair of push-back on top of another iterator (iterator.go
    newBufIterator): ``unread`` returns the last pair to the stream."""

    def __init__(self, itr):
        self.itr = itr
        self.buf: Optional[Tuple[int, int, bool]] = None
        self.full = False
        self.last: Tuple[int, int, bool] = EOF

    def seek(self, row: int, col: int):
        self.full = False
        self.itr.seek(row, col)

    def next(self) -> Tuple[int, int, bool]:
        if self.full:
            self.full = False
            return self.last
        self.last = self.itr.next()
        return self.last

    def peek(self) -> Tuple[int, int, bool]:
        p = self.next()
        self.unread()
        return p

    def unread(self):
        if self.full:
            raise PilosaError("pilosa.BufIterator: buffer full")
        self.full = True


class LimitIterator:
    """Stops at the first pair beyond (max_row, max_column) and stays at EOF
    (iterator.go newLimitIterator)."""

    def __init__(self, itr, max_row: int, max_col: int):
        self.itr = itr
        self.max_row, self.max_col = int(max_row), int(max_col)
        self.eof = False

    def seek(self, row: int, col: int):
        self.itr.seek(row, col)

    def next(self) -> Tuple[int, int, bool]:
        if self.eof:
            return EOF
        r, c, eof = self.itr.next()
        if eof or r > self.max_row or (r == self.max_row and c > self.max_col):
            self.eof = True
            return EOF
        return r, c, False


def pairs_to_positions(rows, cols, width: int = SHARD_WIDTH) -> np.ndarray:
    """Sorted unique uint64 positions row * width + column."""
    r = np.asarray(rows, dtype=np.uint64)
    c = np.asarray(cols, dtype=np.uint64)
    return np.unique(r * np.uint64(width) + c)
