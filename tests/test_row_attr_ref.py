"""Ported expectations of the reference's row_test.go and attr_test.go.
Each test names the reference test it ports."""
import os
import tempfile

import numpy as np
import pytest

from pilosa_amd.models.attrs import MemAttrStore, SQLiteAttrStore
from pilosa_amd.models.row import Row
from pilosa_amd.shardwidth import SHARD_WIDTH as SW


def R(*cols):
    return Row(np.array(cols, dtype=np.uint64))


def cols(r):
    return [int(c) for c in r.columns()]


@pytest.mark.parametrize("a,b,exp", [((1, 2, 3, SW + 1, 2 * SW), (3, 4, 5), 7),
                                     ((), (2, 66000, 70000, 70001, 70002, 70003, 70004), 7)])
def test_row_merge(a, b, exp):  # TestRow_Merge
    r1 = R(*a)
    r1.merge(R(*b))
    assert r1.count() == exp and len(r1.columns()) == exp


def test_row_xor():  # TestRow_Xor
    r1, r2 = R(0, 1, SW), R(0, 2 * SW)
    exp = [1, SW, 2 * SW]
    assert r1.xor(r2).count() == 3 and cols(r1.xor(r2)) == exp
    assert r2.xor(r1).count() == 3 and cols(r2.xor(r1)) == exp


def test_row_union_segment():  # TestRow_Union_Segment
    r1, r2 = R(0, 1, SW), R(0, 2 * SW)
    exp = [0, 1, SW, 2 * SW]
    assert r1.union(r2).count() == 4 and cols(r1.union(r2)) == exp
    assert r2.union(r1).count() == 4 and cols(r2.union(r1)) == exp


def test_row_difference_segment():  # TestRow_Difference_Segment
    res = R(0, 1, SW).difference(R(0, 2 * SW))
    assert res.count() == 2 and cols(res) == [1, SW]


def test_row_is_empty():  # TestRow_IsEmpty
    r1, r2 = R(1, SW), R(0, 2 * SW)
    assert not r1.is_empty()
    assert r2.intersect(r1).is_empty()


@pytest.fixture(params=["mem", "sqlite"])
def store(request):
    if request.param == "mem":
        s = MemAttrStore()
    else:
        s = SQLiteAttrStore(os.path.join(tempfile.mkdtemp(), "attrs.db"))
    s.open()
    yield s
    s.close()


def test_attr_store_attrs(store):  # TestAttrStore_Attrs
    store.set_attrs(1, {"A": 100, "C": -27})
    store.set_attrs(2, {"A": 200})
    store.set_attrs(1, {"B": "VALUE"})
    assert store.attrs(1) == {"A": 100, "B": "VALUE", "C": -27}
    assert store.attrs(2) == {"A": 200}


def test_attr_store_attrs_empty(store):  # TestAttrStore_Attrs_Empty
    assert not store.attrs(100)


def test_attr_store_attrs_unset(store):  # TestAttrStore_Attrs_Unset
    store.set_attrs(1, {"A": "X", "B": "Y"})
    store.set_attrs(1, {"B": None})
    assert store.attrs(1) == {"A": "X"}


def test_attr_store_blocks(store):  # TestAttrStore_Blocks
    store.set_attrs(1, {"A": 100})
    store.set_attrs(2, {"A": 200})
    store.set_attrs(100, {"B": "VALUE"})
    store.set_attrs(350, {"C": "FOO"})
    b0 = store.blocks()
    assert [b for b, _ in b0] == [0, 1, 3]
    store.set_attrs(100, {"X": 12})
    b1 = store.blocks()
    assert b0[0] == b1[0] and b0[1] != b1[1] and b0[2] == b1[2]
