"""Port of roaring/roaring_helpers_test.go: the reference's container
fixtures (empty, full, first/last bit set or unset, inner / outer bits,
odd / even bits) in each encoding (array, bitmap, run;
setupContainerTests).  Every pair of fixtures, in every pair of encodings,
goes through the binary set operations and their counts, checked against
numpy boolean vectors of the same 65536 bits."""
import itertools

import numpy as np
import pytest

from pilosa_amd import _roaring

W = 1 << 16
_ar = np.arange(W)
PATTERNS = {
    "empty": _ar < 0,
    "full": _ar >= 0,
    "firstBitSet": _ar == 0,
    "lastBitSet": _ar == W - 1,
    "firstBitUnset": _ar != 0,
    "lastBitUnset": _ar != W - 1,
    "innerBitsSet": (_ar != 0) & (_ar != W - 1),
    "outerBitsSet": (_ar == 0) | (_ar == W - 1),
    "oddBitsSet": (_ar & 1) == 1,
    "evenBitsSet": (_ar & 1) == 0,
}
TYPES = ("array", "bitmap", "run")


def _container(name: str, typ: str, key: int = 0):
    bits = PATTERNS[name]
    b = _roaring.Bitmap((np.flatnonzero(bits) + key * W).astype(np.uint64))
    if bits.any():
        b.convert_container(key, typ)
        assert b.container_info()[0][1] == typ
    return b


def _bits(b, key: int = 0):
    v = np.asarray(b.slice(), dtype=np.int64) - key * W
    out = np.zeros(W, bool)
    out[v] = True
    return out


@pytest.mark.parametrize("name", list(PATTERNS))
@pytest.mark.parametrize("typ", TYPES)
def test_fixture_round_trips(name, typ):
    b = _container(name, typ)
    assert b.count() == int(PATTERNS[name].sum())
    assert (_bits(b) == PATTERNS[name]).all()
    b2 = _roaring.Bitmap.from_bytes(b.to_bytes())
    assert b2.equals(b)


@pytest.mark.parametrize("ta,tb", list(itertools.product(TYPES, TYPES)))
def test_binary_ops_over_all_fixtures(ta, tb):
    names = list(PATTERNS)
    for na in names:
        a = _container(na, ta)
        pa = PATTERNS[na]
        for nb in names:
            b = _container(nb, tb)
            pb = PATTERNS[nb]
            for op, want in (("intersect", pa & pb), ("union", pa | pb), ("difference", pa & ~pb),
                             ("xor", pa ^ pb)):
                got = getattr(a, op)(b)
                assert got.count() == int(want.sum()), (op, na, ta, nb, tb)
                assert (_bits(got) == want).all(), (op, na, ta, nb, tb)
            assert a.intersection_count(b) == int((pa & pb).sum()), (na, ta, nb, tb)


@pytest.mark.parametrize("typ", TYPES)
def test_shift_and_flip_fixtures(typ):
    for name, bits in PATTERNS.items():
        a = _container(name, typ)
        s = a.shift(1)
        want = np.flatnonzero(bits) + 1
        assert np.array_equal(np.asarray(s.slice(), dtype=np.int64), want), (name, typ)
        f = a.flip(0, W - 1)
        assert (_bits(f) == ~bits).all(), (name, typ)
