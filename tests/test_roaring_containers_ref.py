"""Ported expectations of roaring/containers_test.go (TestContainersIterator):
containers enumerate in key order from a seek key, with "found" when that key
holds a container.  The reference walks its Containers interface; here the
same order comes from Bitmap.container_info (the native container map)."""
import bisect

import numpy as np

from pilosa_amd import _roaring


def _iterator(bm, key):
    info = bm.container_info()                       # [(key, type, n)] ascending
    keys = [k for k, _, _ in info]
    i = bisect.bisect_left(keys, key)
    found = i < len(keys) and keys[i] == key
    return iter([(k, n) for k, _, n in info[i:]]), found


def _put(bm, key, values):
    bm.add_many(np.asarray([(key << 16) | v for v in values], dtype=np.uint64))


def test_containers_iterator():
    bm = _roaring.Bitmap()
    itr, found = _iterator(bm, 0)
    assert not found and next(itr, None) is None
    _put(bm, 1, [1])
    _put(bm, 2, [1, 2])
    itr, found = _iterator(bm, 0)
    assert not found and list(itr) == [(1, 1), (2, 2)]
    _put(bm, 3, [1, 2, 3])
    _put(bm, 5, [1, 2, 3, 4, 5])
    _put(bm, 6, [1, 2, 3, 4, 5, 6])
    itr, found = _iterator(bm, 3)
    assert found and next(itr) == (3, 3) and next(itr) == (5, 5)
    itr, found = _iterator(bm, 4)
    assert not found and list(itr) == [(5, 5), (6, 6)]
