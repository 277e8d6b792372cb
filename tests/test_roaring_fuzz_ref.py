"""Port of roaring/fuzz_test.go (TestUnmarshalBinary): inputs that once
crashed the reference's decoder are rejected with the reference's messages,
and random / mutated buffers either decode or raise (never crash)."""
import random

import numpy as np
import pytest

from pilosa_amd import _roaring

CRASHERS = [
    (b":0\x00\x00\x01\x00\x00\x000000",
     "reading roaring header: malformed bitmap, key-cardinality slice overruns buffer at 12"),
    (b"<0\x000\x00\x00\x00\x00000000000000" b"0",
     "unmarshaling as pilosa roaring: unknown op type: 48"),
    (b"<0\x0000000000000000000" b"\x00\x00\xec\x00\x03\x00\x00\x00\xec000",
     "unmarshaling as pilosa roaring: malformed bitmap, key-cardinality not provided for 67372036 containers"),
    (b"<0\x00\x02\x00\x00\x00\\f\x01\xb5\x8d\x009\x0b\x01\x00\x00\x00\x00" b"\x00\x00e\x04\x00\x00\x00\x04\xfd\x00\x01\x00",
     "unmarshaling as pilosa roaring: malformed bitmap, key-cardinality not provided for 128625322 containers"),
    (b"<0\x00\x02\x00\x00\x00&x.field safe",
     "unmarshaling as pilosa roaring: malformed bitmap, key-cardinality not provided for 53127850 containers"),
    (b"<0\x00\x00\x14\x00\x00\x00\x80\xffp\x05_ 4\x114089\x00\x00\xff\x000\x00\x02\x00\x00\x00\x00\xff\x7f\x00\x00"
     b"\x01\x10\x00\x00j\x02\x00\x00$\x04_\x00\xff\x7f\xff062616163\x00"
     b"0\x00\x02\x00\x01\xbf\x00\x04\x00\xfcad$\x00\x00j\x10\x00\x00\xc3",
     "unmarshaling as pilosa roaring: malformed bitmap, key-cardinality not provided for 1 containers"),
    ("<0\x00\x02\x03\x00\x00\x00쳫\x0b\x00d9\x0b\x00\x009\x0b".encode(),
     "unmarshaling as pilosa roaring: malformed bitmap, key-cardinality not provided for 0 containers"),
    (b";0\x00\x00\x0b00000",
     "reading offsets from official roaring format: offset incomplete: len=10"),
    (b":0\x00\x00\x03\x00\x00\x00000000000000" b"\x00",
     "reading offsets from official roaring format: offset incomplete: len=1"),
]


@pytest.mark.parametrize("data,expected", CRASHERS)
def test_unmarshal_confirmed_crashers(data, expected):  # TestUnmarshalBinary
    with pytest.raises(RuntimeError) as ei:
        _roaring.Bitmap.from_bytes(data)
    assert str(ei.value) == expected


def _decode(data: bytes):
    try:
        b = _roaring.Bitmap.from_bytes(data)
    except RuntimeError:
        return None
    b.count()
    return b


def test_random_buffers_never_crash():
    rng = random.Random(5)
    heads = [b"<0\x00\x00", b":0\x00\x00", b";0", b""]
    for _ in range(3000):
        h = rng.choice(heads)
        data = h + bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 64)))
        _decode(data)


def test_mutated_valid_bitmaps_never_crash():
    rng = np.random.default_rng(9)
    vals = np.unique(np.concatenate([rng.integers(0, 1 << 20, 3000), np.arange(70000, 80000)])).astype(np.uint64)
    good = _roaring.Bitmap(vals)
    good.optimize()
    base = good.to_bytes()
    assert _decode(base).count() == len(vals)
    r = random.Random(3)
    for _ in range(600):
        data = bytearray(base)
        for _ in range(r.randrange(1, 6)):
            data[r.randrange(len(data))] = r.getrandbits(8)
        if r.random() < 0.3:
            data = data[:r.randrange(len(data))]
        _decode(bytes(data))
