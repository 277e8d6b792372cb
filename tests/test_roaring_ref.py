"""Reference expectations of roaring/roaring_test.go, ported test by test to
the C++ roaring core (pilosa_amd/native/roaring.cpp via _roaring).

Every test names its reference function; the literal inputs and expected
counts / slices are the reference's.  ``NewFileBitmap(vals...)`` is
``Bitmap(np.array(vals))``; ``Optimize()`` chooses array / bitmap / run by the
reference rule.  The property tests (testBitmapQuick,
testBitmapMarshalQuick) run on seeded random inputs instead of testing/quick.
Size() (in-memory byte size of the Go container structs) has no counterpart
and is not ported."""
import numpy as np
import pytest

from pilosa_amd import _roaring as R

SW = 1 << 20
MAXU64 = (1 << 64) - 1


def bm(*vals):
    return R.Bitmap(np.array(vals, dtype=np.uint64)) if vals else R.Bitmap()


def bm_add(vals):
    b = R.Bitmap()
    for v in vals:
        b.add(int(v))
    return b


def sl(b):
    return [int(x) for x in b.slice()]


def types(b):
    return {t for _, t, n in b.container_info() if n}


def make_test_bm():
    """testBM: 3 containers -- array, bitmap, run (count 75007)."""
    b = R.Bitmap()
    b.add_many(np.array([(1 << 16) + i for i in range(0, 1024, 4)], np.uint64), True)
    b.add_many(np.array([(2 << 16) + i for i in range(0, 16384, 2)], np.uint64), True)
    b.add_many(np.array([(3 << 16) + i for i in range(1024)], np.uint64), True)
    b.add_many(np.array([(4 << 16) + i for i in range(65535)], np.uint64), True)
    b.optimize()
    return b


def test_container_count():  # TestContainerCount
    b = bm(65535)
    assert b.count() == b.count_range(0, 65546)


COUNT_RANGE = [
    ("j < 0 : 1", [0, 1, 2, 3 * 65536], 0, 65536, 3),
    ("i < 0 : 1", [0, 1, 2, 2 * 65536, 3 * 65536], 65536, 3 * 65536, 1),
    ("single-container-run", [0, 2, 3, 4, 5, 2 * 65536, 3 * 65536], 2, 5, 3),
    ("single-container-beg", [1, 2, 3, 4, 5, 2 * 65536, 3 * 65536], 1, 4, 3),
    ("partial-start", [1, 2, 3, 4, 5, 2 * 65536, 3 * 65536], 5, 3 * 65536, 2),
    ("partial-end", [1, 2 * 65536, 3 * 65536, 3 * 65536 + 1, 3 * 65536 + 2], 0, 3 * 65536 + 1, 3),
    ("partial-both", [65536, 65537, 65538, 2 * 65536, 2 * 65536 + 1, 2 * 65536 + 2], 65537, 2 * 65536 + 1, 3),
    ("partial-both-bookends", [0, 65535, 65536, 65537, 65538, 2 * 65536, 2 * 65536 + 1, 2 * 65536 + 2, 3 * 65536],
     65537, 2 * 65536 + 1, 3),
    ("empty-bookends", [1, 65535, 5 * 65536, 5 * 65536 + 1], 65536, 5 * 65536, 0),
    ("i not found, j found", [1, 65535, 5 * 65536], 2 * 65535, 5 * 65536 + 1, 1),
    ("i not found, j not found", [1, 65535, 5 * 65536, 7 * 65536], 2 * 65535, 6 * 65536, 1),
    ("start < end in different containers", [65537, 65538, 65539, 65540], 65536, 2, 0),
    ("start == end", [65537, 65538, 65539, 65540], 65537, 65537, 0),
]


@pytest.mark.parametrize("name,vals,start,end,exp", COUNT_RANGE, ids=[c[0] for c in COUNT_RANGE])
def test_count_range(name, vals, start, end, exp):  # TestCountRange
    assert bm(*vals).count_range(start, end) == exp


def test_check_bitmap():  # TestCheckBitmap
    b = bm_add(list(range(61000, 71000)) + list(range(75000, 75100)))
    assert b.check() == ""


def test_check_array():  # TestCheckArray
    assert bm(0, 1, 10, 100, 1000, 10000, 90000, 100000).check() == ""


def test_check_run():  # TestCheckRun
    b = bm(0, 1, 2, 3, 4, 5, 1000, 1001, 1002, 1003, 1004, 1005, 100000, 100001, 100002, 100003, 100004, 100005)
    b.optimize()
    assert b.check() == ""


def test_check_full_run():  # TestCheckFullRun
    b = R.Bitmap()
    for lo in range(0, 2097152, 16384):
        b.optimize()
        b.add_many(np.arange(lo, lo + 16384, dtype=np.uint64), True)
    assert b.check() == ""
    b.optimize()
    assert b.check() == ""
    assert b.count() == 2097152 and types(b) == {"run"}


def test_container_transitions():  # TestContainerTransitions
    vals = [0, 1, 2, 3, 4, 5, 1000, 1001, 1002, 1003, 1004, 1005, 100000, 100001, 100002, 132000, 132001, 132002,
            132003, 132004, 132005]
    b = bm(*vals)
    b.optimize()
    assert sl(b) == vals
    vals2 = [65531, 65532, 65533, 65534, 65535, 65536, 131071, 131072, 131073, 131074, 131075, 131076]
    b2 = bm(*vals2)
    b2.optimize()
    assert sl(b2) == vals2


def test_contains_empty():  # TestBitmap_Contains_Empty
    assert not bm().contains(1000)


def test_remove_empty():  # TestBitmap_Remove_Empty
    assert bm().remove(1000) is False


def test_slice():  # TestBitmap_Slice, TestBitmap_Slice_Empty
    assert sl(bm(1, 2, 3)) == [1, 2, 3]
    assert sl(bm()) == []


def test_slice_range():  # TestBitmap_SliceRange
    assert [int(x) for x in bm(0, 1000001, 1000002, 1000003).slice_range(1, 1000003)] == [1000001, 1000002]


def test_for_each():  # TestBitmap_ForEach, TestBitmap_ForEachRange
    assert [v for v, _ in _iter(bm(1, 2, 3))] == [1, 2, 3]
    assert [int(x) for x in bm(1, 2, 3, 4).slice_range(2, 4)] == [2, 3]


def _iter(b, seek=0):
    it = b.iterator()
    it.seek(seek)
    out = []
    while True:
        v, eof = it.next()
        if eof:
            return out
        out.append((v, eof))


def test_max():  # TestBitmap_Max
    b = R.Bitmap()
    for i in range(1000, 100001, 997):
        b.add(i)
        assert b.max() == i


def test_min():  # TestBitmap_Min
    b = R.Bitmap()
    for i in range(100000, 0, -991):
        b.add(i)
        assert b.any() and b.min() == i
    assert not R.Bitmap().any()   # Min() of an empty bitmap: ok == false


def test_bitmap_count_range_edge_case():  # TestBitmap_BitmapCountRangeEdgeCase
    s, e = 2009 * SW, 2010 * SW
    start = s + (39314024 % SW)
    vals = []
    for i in range(65536):
        start += 16384 if (i + 1) % 4096 == 0 else 2
        vals.append(start)
    b = bm_add(vals)
    assert b.count() == b.count_range(s, e)


def _bm0_big(extra=()):
    b = bm(0, 2683177)
    b.add_many(np.arange(628, 2683301, dtype=np.uint64), True)
    for v in extra:
        b.add(v)
    return b


def test_bitmap_count_range():  # TestBitmap_BitmapCountRange
    b = _bm0_big([2683307])
    assert b.count_range(1, 2683311) == 2682674
    assert b.count_range(2683177, 2683310) == 125
    assert b.count_range(2683301, 3000000) == 1
    assert b.count_range(0, 1) == 1
    assert b.count_range(10000000, 10000001) == 0
    assert b.count_range(65536, 2) == 0


def test_array_count_range():  # TestBitmap_ArrayCountRange
    b = bm(0, 2683177, 2683313)
    assert b.count_range(1, 2683313) == 1
    assert b.count_range(2621440, 2) == 0


def test_direct_add():  # TestBitmap_DirectAdd
    bits = [0, 1, 2, 3, 4, 5, 12, 13, 14, 15, 16, 17, 1000000, 1000002, 1000003, 1000004, 1000005, 1000006,
            1000010, 1000011, 1000012, 1000013, 1000014]
    b = bm_add(bits)
    assert b.count() == len(bits) and all(b.contains(x) for x in bits)


def test_run_count_range():  # TestBitmap_RunCountRange
    b0 = bm(0, 1, 2, 3, 4, 5, 12, 13, 14, 15, 16, 17, 1000000, 1000002, 1000003, 1000004, 1000005, 1000006, 1000010,
            1000011, 1000012, 1000013, 1000014)
    b0.optimize()
    assert b0.count_range(15, 1000003) == 5
    b1 = bm(*range(18))
    b1.optimize()
    assert b1.count_range(5, 12) == 7
    b2 = bm(*range(65536, 65554))
    b2.optimize()
    assert b2.count_range(3, 2) == 0


def test_intersection():  # TestBitmap_Intersection
    b1 = R.Bitmap()
    b1.add_many(np.arange(628, 2683301, dtype=np.uint64), True)
    assert bm(0, 2683177).intersect(b1).count() == 1


def test_union1():  # TestBitmap_Union1
    b0 = bm(0, 2683177)
    b1 = R.Bitmap()
    b1.add_many(np.arange(628, 2683301, dtype=np.uint64), True)
    b1.add(4000000)
    assert b0.union(b1).count() == 2682675
    t = make_test_bm()
    assert t.union(b0).count() == 75009
    assert t.union(t).count() == 75007


def test_union_in_place1():  # TestBitmap_UnionInPlace1
    b0 = bm(0, 2683177)
    b1 = R.Bitmap()
    b1.add_many(np.arange(628, 2683301, dtype=np.uint64), True)
    b1.add(4000000)
    r = R.Bitmap()
    r.union_in_place([b0, b1])
    assert r.count() == 2682675
    t = make_test_bm()
    r = R.Bitmap()
    r.union_in_place([t, b0])
    assert r.count() == 75009
    r = R.Bitmap()
    r.union_in_place([t, t])
    assert r.count() == 75007
    assert b0.count() == 2 and b1.count() == 2682674   # inputs not mutated


def test_union_in_place_prop():  # TestBitmap_UnionInPlaceProp
    rng = np.random.default_rng(551)
    for _ in range(100):
        sets, bitmaps = [], []
        for _ in range(int(rng.integers(0, 100)) + 2):
            s, b = set(), R.Bitmap()
            if rng.integers(0, 100) <= 2:   # max-range run containers
                st = int(rng.integers(0, 1000000))
                r = np.arange(st, st + 2 * 65536, dtype=np.uint64)
                s.update(r.tolist())
                b.add_many(r, True)
            vals = rng.integers(0, 1000000, int(rng.integers(0, 100))).astype(np.uint64)
            for v in vals.tolist():
                s.add(v)
                b.add(v)
            sets.append(s)
            bitmaps.append(b)
        want = set().union(*sets)
        b0 = bitmaps[0]
        b0.union_in_place(bitmaps[1:])
        assert b0.count() == len(want)
        assert sl(b0) == sorted(want)


def test_intersection_empty():  # TestBitmap_Intersection_Empty
    assert bm(0, 2683177).intersect(bm()).count() == 0


def test_intersect_array_array():  # TestBitmap_IntersectArrayArray
    b0, b1 = bm(0, 1, 7, 9, 11, 2683, 5005), bm(0, 2683, 2684, 5000)
    for r in (b0.intersect(b1), b1.intersect(b0)):
        assert r.count() == 2 and r.contains(0) and r.contains(2683)


def test_intersect_bitmap_bitmap():  # TestBitmap_IntersectBitmapBitmap
    b0 = bm(*range(0, 65536, 2))
    b1 = bm(*range(0, 65536, 3))
    assert b0.intersect(b1).count() == 10923


def test_intersect_run_run():  # TestBitmap_IntersectRunRun
    b0 = bm(0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15)
    b0.optimize()
    b1 = bm(5, 6, 7, 8, 9, 10, 11)
    b1.optimize()
    assert b0.intersect(b1).count() == 3
    vals = []
    run_len, space = 25, 8
    off = run_len // 2 + space
    for i in range(0, 65536 - run_len - off, run_len + space):
        vals += [off + i + j for j in range(run_len)]
    b2 = bm(*vals)
    b2.optimize()
    vals = []
    run_len, space = 32, 1
    for i in range(0, 65536 - run_len, run_len + space):
        vals += [i + j for j in range(run_len)]
    b3 = bm(*vals)
    b3.optimize()
    assert b2.intersect(b3).count() == 47628


def test_difference():  # TestBitmap_Difference, Difference_Empty
    b1 = R.Bitmap()
    b1.add_many(np.arange(628, 2683301, dtype=np.uint64), True)
    assert bm(0, 2683177).difference(b1).count() == 1
    assert bm(0, 2683177).difference(bm()).count() == 2


def test_difference2():  # TestBitmap_Difference2
    b0 = bm(0, 1, 2, 131072, 262144, SW + 5, SW + 7)
    b1 = bm(2, 3, 100000, 262144, 2 * SW + 1)
    assert sl(b0.difference(b1)) == [0, 1, 131072, SW + 5, SW + 7]


def test_difference_array_array_and_run():  # TestBitmap_DifferenceArrayArray, DifferenceArrayRun
    assert bm(0, 4, 8, 12, 16, 20).difference(bm(1, 3, 6, 9, 12, 15, 18)).count() == 5
    b1 = bm(1, 2, 3, 4, 5, 6, 7, 8, 9, 30, 31, 32, 33, 34, 35, 36)
    b1.optimize()
    assert bm(0, 4, 8, 12, 16, 20, 36, 40, 44).difference(b1).count() == 6


def test_union_and_in_place():  # TestBitmap_Union, TestBitmap_UnionInPlace
    b0, b1 = bm(0, 1000001, 1000002, 1000003), bm(0, 50000, 1000001, 1000002)
    assert b0.union(b1).count() == 5
    r = R.Bitmap()
    r.union_in_place([b0, b1])
    assert r.count() == 5 and b0.count() == 4 and b1.count() == 4


def test_xor():  # TestBitmap_Xor
    t, b1 = make_test_bm(), bm(0, 1, 2, 3)
    assert b1.xor(t).count() == 75011
    assert t.xor(b1).count() == 75011
    assert t.xor(t).count() == 0


def test_xor_array_array_and_empty():  # TestBitmap_Xor_ArrayArray, Xor_Empty
    r = bm(0, 1000001, 1000002, 1000003).xor(bm(0, 50000, 1000001, 1000002))
    assert r.count() == 2 and r.xor(r).count() == 0
    assert bm(0, 50000, 1000001, 1000002).xor(bm()).count() == 4


def test_xor_array_bitmap():  # TestBitmap_Xor_ArrayBitmap
    b0 = bm(1, 70, 200, 4097, 4098)
    b1 = bm(*range(0, 10000, 2))
    assert b0.xor(b1).count() == 4999
    r = b1.xor(b0)
    assert r.count() == 4999 and r.xor(r).count() == 0
    assert b1.xor(bm()).count() == 5000


def test_xor_bitmap_bitmap():  # TestBitmap_Xor_BitmapBitmap
    assert bm(*range(1, 10000, 2)).xor(bm(*range(0, 10000, 2))).count() == 10000


def test_flip():  # TestBitmap_Flip_Empty, Flip_Array, Flip_Bitmap, Flip_After
    r = bm().flip(0, 10)
    assert r.count() == 11 and r.flip(0, 10).count() == 0
    b = bm(0, 1, 2, 3, 4, 8, 16, 32, 64, 128, 256, 512, 1024)
    r = b.flip(0, 4)
    assert sl(r) == [8, 16, 32, 64, 128, 256, 512, 1024]
    assert sl(r.flip(0, 4)) == [0, 1, 2, 3, 4, 8, 16, 32, 64, 128, 256, 512, 1024]
    b = bm(*range(0, 10000, 2))
    r = b.flip(0, 9999)
    assert r.count() == 5000 and r.flip(0, 9999).count() == 5000
    r = bm(0, 2, 4, 8).flip(9, 10)
    assert sl(r) == [0, 2, 4, 8, 9, 10]
    r = r.flip(0, 1)
    assert sl(r) == [1, 2, 4, 8, 9, 10]
    assert sl(r.flip(4, 8)) == [1, 2, 5, 6, 7, 9, 10]


def _ic_both(a, b, want):
    assert a.intersection_count(b) == want and b.intersection_count(a) == want


def test_intersection_count_pairs():  # TestBitmap_IntersectionCount_{ArrayArray,ArrayRun,RunRun,BitmapRun,ArrayBitmap,BitmapBitmap}
    _ic_both(bm(0, 1000001, 1000002, 1000003), bm(0, 50000, 999998, 999999, 1000000, 1000001, 1000002), 3)
    r1 = bm(0, 1, 2, 3, 4, 5, 1000000, 1000002, 1000003, 1000004, 1000005, 1000006)
    r1.optimize()
    _ic_both(bm(0, 1000001, 1000002, 1000003), r1, 3)
    r0 = bm(3, 4, 5, 6, 7, 8, 1000001, 1000002, 1000003, 1000004)
    r0.optimize()
    _ic_both(r0, r1, 6)
    _ic_both(bm(*range(3, 1000007, 2)), r1, 4)
    _ic_both(bm(1, 70, 200, 4097, 4098), bm(*range(0, 10001, 2)), 3)
    b0 = bm(*(list(range(0, 10001, 2)) + [1000, 2000]))
    b1 = bm(*(list(range(1, 10002, 2)) + [1000, 2000]))
    _ic_both(b0, b1, 2)


def test_intersection_count_mixed():  # TestBitmap_IntersectionCount_Mixed
    t = make_test_bm()
    assert t.intersection_count(t) == t.count()
    assert t.intersection_count(bm(0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 65536)) == 1
    assert t.intersection_count(bm(131072)) == 1


def test_shift():  # TestBitmap_Shift
    b1 = bm(0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 65536, MAXU64)
    assert sl(b1.shift(1)) == [1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 65537]
    assert sl(bm(65535, 131073).shift(1)) == [65536, 131074]
    b1 = bm(65535, 131073, 65536 * 5 - 1, 65536 * 10, 65536 * 15 - 1)
    assert sl(b1.shift(1)) == [65536, 131074, 65536 * 5, 65536 * 10 + 1, 65536 * 15]


QUICK = [(1000, 1000, 2000), (10000, 0, 1000), (10000, 0, 10000), (10000, 10000, 20000), (10000, 0, (1 << 63) - 1)]


@pytest.mark.parametrize("n,lo,hi", QUICK, ids=["Array1", "Array2", "Bitmap1", "Bitmap2", "LargeValue"])
def test_bitmap_quick(n, lo, hi):  # TestBitmap_Quick_*
    rng = np.random.default_rng(n + lo)
    for _ in range(5):
        a = (lo + rng.integers(0, hi - lo, int(rng.integers(0, n)), dtype=np.uint64)).tolist()
        b, m, cnt = R.Bitmap(), set(), 0
        for v in a:
            cnt += bool(b.add(v))
            m.add(v)
        assert b.count() == cnt
        for v in a:
            assert b.contains(v)
            assert b.contains(v + 1) == ((v + 1) in m)
        assert sl(b) == sorted(m)
        for i in rng.permutation(len(a)):
            cnt -= bool(b.remove(a[i]))
            assert b.count() == cnt
        assert sl(b) == []


@pytest.mark.parametrize("n,lo,hi,srt", [(1000, 1000, 2000, False), (10000, 0, 1000, False), (10000, 0, 10000, False),
                                         (10000, 10000, 20000, False), (100, 0, (1 << 63) - 1, False),
                                         (10000, 0, 10000, True)],
                         ids=["Array1", "Array2", "Bitmap1", "Bitmap2", "LargeValue", "Bitmap_Sorted"])
def test_bitmap_marshal_quick(n, lo, hi, srt):  # TestBitmap_Marshal_Quick_*
    """Snapshot + op log: after every logged Add, unmarshalling the buffer
    (snapshot followed by the add ops) gives the same set."""
    rng = np.random.default_rng(n ^ lo)
    for _ in range(3):
        a0 = (lo + rng.integers(0, hi - lo, int(rng.integers(0, n)), dtype=np.uint64))
        a1 = (lo + rng.integers(0, hi - lo, int(rng.integers(0, 100)), dtype=np.uint64))
        if srt:
            a0, a1 = np.sort(a0), np.sort(a1)
        b = R.Bitmap(a0)
        buf = bytearray(b.to_bytes())
        want = set(a0.tolist())
        for v in a1.tolist():
            want.add(v)
            if b.add(v):
                buf += R.encode_op(0, v)
            b2 = R.Bitmap.from_bytes(bytes(buf))
            assert sl(b) == sorted(want)
            assert sl(b2) == sorted(want)


def test_iterator():  # TestIterator
    assert [v for v, _ in _iter(bm(1, 2, 3))] == [1, 2, 3]
    b1 = bm(*range(11))
    b1.optimize()
    b2 = bm(*range(12))
    b2.optimize()
    for b, exp in ((b1, list(range(11))), (b2, list(range(12))), (b1.difference(b2), []), (b2.difference(b1), [11])):
        assert [v for v, _ in _iter(b)] == exp


def test_offset_range():  # TestBitmapOffsetRange
    t = make_test_bm()
    assert t.offset_range(0, 0, 327680).count() == t.count()
    assert t.offset_range(0, 0, 131072).count() == 256


def test_contains():  # TestBitmapContains
    t = make_test_bm()
    assert t.contains(3 << 16)
    assert not t.contains((3 << 16) + 2048)


def test_intersect_self():  # TestBitmap_Intersect
    t = make_test_bm()
    assert t.intersect(t).count() == t.count()


def test_bench_data_container_types():  # getBenchData / isAllType
    rng = np.random.default_rng(7)
    mx = (1 << 24) // 64
    a1, a2 = R.Bitmap(), R.Bitmap()
    for _ in range(4096 // 3):
        a1.add(int(rng.integers(0, mx)))
        a2.add(int(rng.integers(0, mx)))
    for _ in range(4096 // 3):
        a1.add(int(rng.integers(0, mx)))
    b = bm(*range(0, 65535, 3))
    r1 = bm(*range(65535))
    r2_vals, i = [], 0
    while i < 65535:
        r2_vals.append(i)
        if i & 0xfff == 0xfff:
            i += 5
        i += 1
    r2 = bm(*r2_vals)
    for x in (a1, a2, b, r1, r2):
        x.optimize()
    assert types(a1) == {"array"} and types(a2) == {"array"}
    assert types(b) == {"bitmap"}
    assert types(r1) == {"run"} and types(r2) == {"run"}
    # the intersection counts the reference benchmarks time, against the set oracle
    bms = dict(a1=a1, a2=a2, b=b, r1=r1, r2=r2)
    sets = {k: set(sl(v)) for k, v in bms.items()}
    for x, y in (("a1", "r1"), ("r1", "r2"), ("a1", "b"), ("b", "r2"), ("a1", "a2")):
        assert bms[x].intersection_count(bms[y]) == len(sets[x] & sets[y])
