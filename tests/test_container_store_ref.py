"""Port of roaring/btree_test.go: the reference keeps a bitmap's containers
in a B+tree keyed by the high 48 bits; the native bitmap here keeps them in
an ordered map (pilosa_amd/native/roaring.hpp).  The tree's contract is
checked through the bitmap: Set/Get over many keys in random order, Delete,
Seek + Next enumeration (with the value re-set mid-walk, as
TestBtreeEnumeratorNext's verChange does), Seek over 2^13 odd keys and the
split-edge case of TestBtreePR4.  Not ported: the Prev enumerator and
Put-with-callback (the bitmap exposes neither) and the allocation
benchmarks."""
import random

import numpy as np
import pytest

from pilosa_amd import _roaring

C = 1 << 16   # one container per key: value = key << 16 (+ low bits)


def _bm(keys, low=0):
    b = _roaring.Bitmap()
    for k in keys:
        b.add(int(k) * C + low)
    return b


def _keys(b):
    return [int(k) for k in b.keys()]


def test_get_on_empty():  # TestBtreeGet0
    b = _roaring.Bitmap()
    assert not b.contains(42 * C) and b.container_count() == 0


@pytest.mark.parametrize("n", [1, 31, 1000, 20000])
def test_set_get_random_order(n):  # TestBtreeSetGet0/1/2/3
    rng = random.Random(n)
    keys = rng.sample(range(1 << 40), n)
    b = _roaring.Bitmap()
    for k in keys:
        b.add(k * C + (k & 0xffff))
    assert b.container_count() == n
    assert _keys(b) == sorted(keys)
    for k in keys:
        assert b.contains(k * C + (k & 0xffff)) and not b.contains(k * C + ((k + 1) & 0xffff))
    # setting again replaces nothing
    for k in keys[: n // 2]:
        b.add(k * C + (k & 0xffff))
    assert b.container_count() == n and b.count() == n


def test_split_on_edge():  # TestBtreeSplitXOnEdge: sequential keys across node-size boundaries
    for n in (2 * 32 + 1, 2 * 64 + 1, 3 * 128):
        b = _bm(range(n))
        assert _keys(b) == list(range(n))
        b2 = _bm(reversed(range(n)))
        assert b2.equals(b)


@pytest.mark.parametrize("n", [1, 64, 5000])
def test_delete(n):  # TestBtreeDelete0/1/2
    rng = random.Random(7 + n)
    keys = rng.sample(range(1 << 30), n)
    b = _bm(keys)
    order = keys[:]
    rng.shuffle(order)
    live = set(keys)
    for i, k in enumerate(order):
        b.remove(k * C)
        live.discard(k)
        assert not b.contains(k * C)
        if i % max(1, n // 8) == 0:
            assert _keys(b) == sorted(live)
    assert b.container_count() == 0 and b.count() == 0
    b.remove(12345 * C)   # deleting a missing key is a no-op
    assert b.count() == 0


@pytest.mark.parametrize("k,hit,keys", [
    (5, False, [10, 20, 30]), (10, True, [10, 20, 30]), (15, False, [20, 30]), (20, True, [20, 30]),
    (25, False, [30]), (30, True, [30]), (35, False, [])])
def test_seek_next(k, hit, keys):  # TestBtreeEnumeratorNext
    for ver_change in range(16):
        b = _bm([10, 20, 30])
        assert b.contains(k * C) == hit
        it = b.iterator()
        it.seek(k * C)
        got = []
        j = 0
        while True:
            if ver_change & (1 << j):
                b.add(20 * C)   # the tree changes under the enumerator
            v, eof = it.next()
            if eof:
                break
            got.append(v // C)
            j += 1
        assert got == keys, (ver_change, got)


def test_seek_first_and_last():  # TestBtreeSeekFirst0-3 / SeekLast0-3
    b = _roaring.Bitmap()
    it = b.iterator()
    assert it.next()[1] is True
    for ks in ([1], [1, 2], [1, 2, 3]):
        b = _bm(ks)
        it = b.iterator()
        assert [v // C for v in it] == ks
        assert b.max() // C == ks[-1] and b.min() // C == ks[0]


def test_seek_odd_keys():  # TestBtreeSeek
    N = 1 << 13
    b = _bm(np.arange(N) * 2 + 1)
    for i in range(0, N, 97):
        it = b.iterator()
        it.seek(2 * i * C)
        assert not b.contains(2 * i * C)
        rest = [v // C for v in it]
        assert rest == list(range(2 * i + 1, 2 * N, 2))


def test_key_survives_split_after_delete():  # TestBtreePR4
    kd = 32
    b = _bm([1000 * i for i in range(2 * kd + 1)])
    b.remove(1000 * kd * C)
    for i in range(kd):
        b.add((1000 * (kd + 1) - 1 - i) * C)
    k = 1000 * (kd + 1) - 1 - kd
    b.add(k * C)
    assert b.contains(k * C)
    assert _keys(b) == sorted(_keys(b)) and len(_keys(b)) == 2 * kd + 1 + kd
