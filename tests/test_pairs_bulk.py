"""Bulk Pair construction (models/cache.pairs_from_arrays over the native
make_pairs): the objects equal the ones Pair.__init__ builds."""
import gc

import numpy as np

from pilosa_amd import _roaring
from pilosa_amd.models import cache
from pilosa_amd.models.cache import Pair, pairs_from_arrays, sort_pairs


def test_bulk_pairs_equal_init_built():
    rng = np.random.default_rng(3)
    ids = rng.integers(0, 1 << 63, 5000, dtype=np.uint64)
    cnt = rng.integers(-(1 << 40), 1 << 40, 5000)
    got = pairs_from_arrays(ids, cnt)
    want = [Pair(int(i), int(c)) for i, c in zip(ids, cnt)]
    assert got == want and all(type(p) is Pair and p.key == "" for p in got)
    assert isinstance(got, list) and sort_pairs(got) == sort_pairs(want)
    got[7].count += 1      # ordinary mutable objects
    assert got[7].count == int(cnt[7]) + 1
    del got
    gc.collect()


def test_bulk_pairs_empty_and_types():
    assert pairs_from_arrays(np.zeros(0, np.uint64), np.zeros(0, np.int64)) == []
    assert pairs_from_arrays([1, 2], [3, 4]) == [Pair(1, 3), Pair(2, 4)]


def test_native_refuses_other_layouts(monkeypatch):
    class Other:
        __slots__ = ("a",)
    assert _roaring.make_pairs(Other, np.zeros(1, np.uint64), np.zeros(1, np.int64)) is None
    # the Python fallback builds the same list
    monkeypatch.setattr(cache, "_MAKE_PAIRS", [None])
    assert pairs_from_arrays([5], [6]) == [Pair(5, 6)]
