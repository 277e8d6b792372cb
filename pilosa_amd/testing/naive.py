"""Slice-based roaring oracle and differential fuzzer (reference:
roaring/naive.go:27-321, roaring/fuzzer.go:28-323).

``NaiveBitmap`` keeps a sorted Python list of uint64 values and implements
the same operations as the native ``_roaring.Bitmap`` in the most obvious
way, so that every native result can be diffed against it.  ``fuzz_ops``
drives both with the same random operation stream (the ``FuzzRoaringOps``
analog) and ``fuzz_unmarshal`` feeds mutated serialized bitmaps to the
loader, which must either reject them with an exception or produce a bitmap
that is safe to walk (the ``FuzzBitmapUnmarshalBinary`` analog).
"""
from __future__ import annotations

import bisect
from typing import Iterable, List, Optional

import numpy as np


# ---- slice helpers (roaring/naive.go): the oracle's operations on plain
# lists of uint64 values; inputs may be unsorted and hold duplicates, every
# set result comes back sorted and distinct
def sort_slice(a: List[int]) -> List[int]:
    a.sort()
    return a


def remove_slice_duplicates(a: Iterable[int]) -> List[int]:
    return sorted(set(a))


def intersect_slice(a: Iterable[int], b: Iterable[int]) -> List[int]:
    return sorted(set(a) & set(b))


def union_slice(a: Iterable[int], b: Iterable[int]) -> List[int]:
    return sorted(set(a) | set(b))


def difference_slice(a: Iterable[int], b: Iterable[int]) -> List[int]:
    return sorted(set(a) - set(b))


def xor_slice(a: Iterable[int], b: Iterable[int]) -> List[int]:
    return sorted(set(a) ^ set(b))


def max_in_slice(a: Iterable[int]) -> int:
    return max(a, default=0)


def shift_slice(a: Iterable[int], n: int) -> List[int]:
    return sorted(int(x) + n for x in set(a))


def for_each_in_slice(a: Iterable[int], fn) -> None:
    for x in a:           # in the slice's own order
        fn(x)


def for_each_in_range_slice(a: Iterable[int], start: int, end: int, fn) -> None:
    for x in a:           # values in [start, end), in the slice's own order
        if start <= x < end:
            fn(x)


def contained_in_slice(a: List[int], v: int):
    """(index of v in the slice as given, found)"""
    for i, x in enumerate(a):
        if x == v:
            return i, True
    return -1, False


def add_n_to_slice(a: Iterable[int], *b: int):
    """(sorted union, number of values of b that were not in a)"""
    s = set(a)
    n = len(s)
    s.update(b)
    return sorted(s), len(s) - n


def remove_n_from_slice(a: Iterable[int], *b: int):
    """(sorted difference, number of values removed)"""
    s = set(a)
    n = len(s)
    s.difference_update(b)
    return sorted(s), n - len(s)


def count_range_slice(a: Iterable[int], start: int, end: int) -> int:
    return sum(1 for x in set(a) if start <= x < end)


def range_slice(a: Iterable[int], start: int, end: int) -> List[int]:
    return sorted(x for x in set(a) if start <= x < end)


def flip_slice(a: Iterable[int], start: int, end: int) -> List[int]:
    """Flip [start, end] inclusive (Bitmap.Flip); start > end flips nothing."""
    s = set(a)
    if start <= end:
        s ^= set(range(start, end + 1))
    return sorted(s)


class NaiveBitmap:
    def __init__(self, values: Iterable[int] = ()):
        self.v: List[int] = sorted(set(int(x) for x in values))

    # mutation
    def add(self, x: int) -> bool:
        i = bisect.bisect_left(self.v, x)
        if i < len(self.v) and self.v[i] == x:
            return False
        self.v.insert(i, x)
        return True

    def remove(self, x: int) -> bool:
        i = bisect.bisect_left(self.v, x)
        if i < len(self.v) and self.v[i] == x:
            del self.v[i]
            return True
        return False

    # queries
    def contains(self, x: int) -> bool:
        i = bisect.bisect_left(self.v, x)
        return i < len(self.v) and self.v[i] == x

    def count(self) -> int:
        return len(self.v)

    def count_range(self, lo: int, hi: int) -> int:
        return bisect.bisect_left(self.v, hi) - bisect.bisect_left(self.v, lo)

    def max(self) -> int:
        return self.v[-1] if self.v else 0

    def min(self) -> int:
        return self.v[0] if self.v else 0

    def slice(self) -> List[int]:
        return list(self.v)

    def offset_range(self, offset: int, lo: int, hi: int) -> "NaiveBitmap":
        a, b = bisect.bisect_left(self.v, lo), bisect.bisect_left(self.v, hi)
        return NaiveBitmap(offset + x - lo for x in self.v[a:b])

    # set algebra
    def intersect(self, o: "NaiveBitmap") -> "NaiveBitmap":
        return NaiveBitmap(set(self.v) & set(o.v))

    def union(self, o: "NaiveBitmap") -> "NaiveBitmap":
        return NaiveBitmap(set(self.v) | set(o.v))

    def difference(self, o: "NaiveBitmap") -> "NaiveBitmap":
        return NaiveBitmap(set(self.v) - set(o.v))

    def xor(self, o: "NaiveBitmap") -> "NaiveBitmap":
        return NaiveBitmap(set(self.v) ^ set(o.v))

    def intersection_count(self, o: "NaiveBitmap") -> int:
        return len(set(self.v) & set(o.v))

    def shift(self, n: int) -> "NaiveBitmap":
        return NaiveBitmap(x + n for x in self.v if x + n < (1 << 64))

    def flip(self, lo: int, hi: int) -> "NaiveBitmap":
        """Flip [lo, hi] inclusive (reference Bitmap.Flip)."""
        return NaiveBitmap(set(self.v) ^ set(range(lo, hi + 1)))

    def seek_next(self, x: int) -> Optional[int]:
        i = bisect.bisect_left(self.v, x)
        return self.v[i] if i < len(self.v) else None


def _rand_values(rng: np.random.Generator, n: int, span: int) -> np.ndarray:
    """Clustered values so that array, bitmap and run containers all appear."""
    kind = rng.integers(0, 3)
    if kind == 0:
        return rng.integers(0, span, n, dtype=np.uint64)
    if kind == 1:  # dense block -> bitmap container
        base = int(rng.integers(0, max(1, span - 70000)))
        return (base + rng.integers(0, 65536, max(n, 5000))).astype(np.uint64)
    base = int(rng.integers(0, max(1, span - 5000)))  # contiguous runs
    return np.arange(base, base + int(rng.integers(1, 4000)), dtype=np.uint64)


def fuzz_ops(seed: int, steps: int = 200, span: int = 1 << 22) -> int:
    """Apply one random op stream to a native bitmap and the naive oracle and
    assert that they agree after every step.  Returns the number of checks."""
    from pilosa_amd import _roaring as R

    rng = np.random.default_rng(seed)
    nb, ob = R.Bitmap(), NaiveBitmap()
    checks = 0
    for _ in range(steps):
        op = int(rng.integers(0, 11))
        if op <= 1:
            vals = _rand_values(rng, int(rng.integers(1, 300)), span)
            if op == 0:
                nb.add_many(vals)
                for x in vals.tolist():
                    ob.add(x)
            else:
                nb.remove_many(vals)
                for x in vals.tolist():
                    ob.remove(x)
        elif op == 2:
            x = int(rng.integers(0, span))
            assert nb.add(x) == ob.add(x)
        elif op == 3:
            nb.optimize()
        elif op in (4, 5, 6, 7):
            other = _rand_values(rng, int(rng.integers(1, 2000)), span)
            no, oo = R.Bitmap(other), NaiveBitmap(other.tolist())
            if rng.integers(0, 2):
                no.optimize()
            fn = {4: "intersect", 5: "union", 6: "difference", 7: "xor"}[op]
            assert getattr(nb, fn)(no).slice().tolist() == getattr(ob, fn)(oo).slice(), fn
            assert nb.intersection_count(no) == ob.intersection_count(oo)
        elif op == 8:
            lo, hi = sorted(int(x) for x in rng.integers(0, span, 2))
            assert nb.count_range(lo, hi) == ob.count_range(lo, hi)
        elif op == 9:
            x = int(rng.integers(0, span))
            it = nb.iterator()
            it.seek(x)
            v, eof = it.next()
            want = ob.seek_next(x)
            assert (None if eof else v) == want, (x, v, eof, want)
        else:
            data = nb.to_bytes()
            nb = R.Bitmap.from_bytes(data)
        assert nb.count() == ob.count()
        checks += 1
    assert nb.slice().tolist() == ob.slice()
    assert nb.check() == "" or nb.check() is None
    return checks


def fuzz_unmarshal(seed: int, iters: int = 100) -> int:
    """Mutate serialized bitmaps byte-wise and load them.  Loading must either
    raise or yield a bitmap that is safe to walk (count, slice, iterate,
    check); like the reference's loader, headers are trusted for cardinality,
    so ``check()`` may report the inconsistency (that is what ``pilosa check``
    is for) but nothing may read out of bounds.  Returns the number of inputs
    the loader accepted."""
    from pilosa_amd import _roaring as R

    rng = np.random.default_rng(seed)
    accepted = 0
    for _ in range(iters):
        b = R.Bitmap(_rand_values(rng, int(rng.integers(1, 3000)), 1 << 22))
        if rng.integers(0, 2):
            b.optimize()
        raw = bytearray(b.to_bytes())
        for _ in range(int(rng.integers(1, 6))):
            mode = int(rng.integers(0, 3))
            if mode == 0 and raw:
                raw[int(rng.integers(0, len(raw)))] = int(rng.integers(0, 256))
            elif mode == 1 and len(raw) > 1:
                del raw[int(rng.integers(1, len(raw))):]
            else:
                raw += bytes(rng.integers(0, 256, int(rng.integers(1, 32)), dtype=np.uint8))
        try:
            got = R.Bitmap.from_bytes(bytes(raw))
        except Exception:
            continue
        ok = not got.check()
        got.count()
        vals = got.slice()
        walked = list(got.iterator())
        if ok:  # a consistent bitmap must iterate exactly its values
            assert walked == vals.tolist()
        accepted += 1
    return accepted
