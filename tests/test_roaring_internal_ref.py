"""Ported expectations of the reference's container-level roaring tests
(/root/reference/roaring/roaring_internal_test.go).  The reference drives its
container functions directly; here each case builds one-container bitmaps of
the exact encoding the reference test uses (``convert_container`` forces
array / bitmap / run) and goes through the public Bitmap operations, which
dispatch to the same type-pair code in native/roaring.cpp.  Each test names
the reference test (and line) it ports."""
import numpy as np
import pytest

from pilosa_amd import _roaring

Bitmap = _roaring.Bitmap


def _vals_of_runs(runs):
    out = []
    for s, e in runs:
        out.extend(range(s, e + 1))
    return out


def _vals_of_words(words):
    out = []
    for i, w in enumerate(words):
        for b in range(64):
            if (w >> b) & 1:
                out.append(i * 64 + b)
    return out


def _typed(vals, kind):
    b = Bitmap(np.array(sorted(set(vals)), dtype=np.uint64))
    if len(vals):
        b.convert_container(0, kind)
    return b


def arr(vals):
    return _typed(list(vals), "array")


def bmp(words):
    return _typed(_vals_of_words(words), "bitmap")


def run(runs):
    return _typed(_vals_of_runs(runs), "run")


def vals(b):
    return b.slice().tolist()


def types(b):
    return [t for _, t, _ in b.container_info()]


def test_container_run_add():  # TestContainerRunAdd :84, TestContainerRunAdd2 :115
    steps = [(1, [(1, 1)]), (2, [(1, 2)]), (4, [(1, 2), (4, 4)]), (3, [(1, 4)]), (10, [(1, 4), (10, 10)]),
             (7, [(1, 4), (7, 7), (10, 10)]), (6, [(1, 4), (6, 7), (10, 10)]), (0, [(0, 4), (6, 7), (10, 10)]),
             (8, [(0, 4), (6, 8), (10, 10)])]
    c = run([(1, 1)])
    c.remove(1)
    for v, exp in steps:
        assert c.add(v), v
        assert vals(c) == _vals_of_runs(exp)
        c.optimize()
    c = Bitmap()
    assert c.add(0) and not c.add(0)


def test_run_count_range():  # TestRunCountRange :130
    c = run([])
    assert c.count_range(2, 9) == 0
    c = run([(5, 7)])
    assert c.count_range(2, 9) == 3
    c = run([(5, 11)])
    assert c.count_range(6, 8) == 2
    assert c.count_range(3, 9) == 4
    assert c.count_range(9, 14) == 3
    c = run([(5, 11), (17, 19)])
    assert c.count_range(1, 22) == 10
    c = run([(5, 11), (13, 14), (17, 19)])
    assert c.count_range(6, 18) == 9
    assert c.container_run_count(0) == 3


def test_run_contains():  # TestRunContains :188
    assert not run([]).contains(5)
    c = run([(5, 5)])
    assert c.contains(5)
    c = run([(5, 7), (9, 11)])
    assert c.contains(10) and not c.contains(8)


@pytest.mark.parametrize("start,end,words,exp", [
    (0, 1, [1], 1), (2, 7, [0xFFFFFFFFFFFFFF18], 2), (67, 68, [0, 0x8], 1), (1, 68, [0x3, 0x8, 0xF], 2),
    (1, 258, [0xF, 0x8, 0xA, 0x4, 0xFFFFFFFFFFFFFFFF], 9), (66, 71, [0xF, 0xFFFFFFFFFFFFFF18], 2),
    (63, 64, [0x8000000000000000], 1)])
def test_bitmap_count_range(start, end, words, exp):  # TestBitmapCountRange :210
    assert bmp(words).count_range(start, end) == exp


def test_intersection_count_full_bitmap_and_runs():  # TestIntersectionCountArrayBitmap3 :235
    full = [0xFFFFFFFFFFFFFFFF] * 1024
    a, b = bmp(full), bmp(full)
    assert a.intersect(b).count() == 65536 == a.intersection_count(b)
    r = run([(0, 65535)])
    assert b.intersect(r).count() == 65536 == b.intersection_count(r)
    r2 = run([(0, 65535)])
    assert r.intersect(r2).count() == 65536 == r.intersection_count(r2)


@pytest.mark.parametrize("array,words,exp", [
    ([0], [1], 1), ([0, 1], [3], 2), ([64, 128, 129, 2000], [932421, 2], 0),
    ([0, 65, 130, 195], [255] * 12, 4),
    ([63, 120, 543, 639, 12000], [0x8000000000000000, 0, 0, 0, 0, 0, 0, 0, 0, 0x8000000000000000], 2)])
def test_intersection_count_array_bitmap(array, words, exp):  # TestIntersectionCountArrayBitmap2 :256
    a, b = arr(array), bmp(words)
    assert a.intersection_count(b) == exp == b.intersection_count(a)


def test_run_remove():  # TestRunRemove :300
    c = run([(2, 10), (12, 13), (15, 16)])
    steps = [(2, [(3, 10), (12, 13), (15, 16)], True), (10, [(3, 9), (12, 13), (15, 16)], True),
             (12, [(3, 9), (13, 13), (15, 16)], True), (13, [(3, 9), (15, 16)], True),
             (16, [(3, 9), (15, 15)], True), (6, [(3, 5), (7, 9), (15, 15)], True),
             (8, [(3, 5), (7, 7), (9, 9), (15, 15)], True), (8, [(3, 5), (7, 7), (9, 9), (15, 15)], False),
             (1, [(3, 5), (7, 7), (9, 9), (15, 15)], False), (44, [(3, 5), (7, 7), (9, 9), (15, 15)], False)]
    for v, exp, ret in steps:
        assert c.remove(v) == ret, v
        assert vals(c) == _vals_of_runs(exp)


def test_run_max():  # TestRunMax :335
    assert run([(2, 10), (12, 13), (15, 16)]).max() == 16
    assert Bitmap().max() == 0


def test_intersection_count_array_run():  # TestIntersectionCountArrayRun :349
    a, b = arr([1, 5, 10, 11, 12]), run([(2, 10), (12, 13), (15, 16)])
    assert a.intersection_count(b) == 3 == b.intersection_count(a)


def test_intersection_count_bitmap_run():  # TestIntersectionCountBitmapRun :359
    words = [0] * 1024
    words[0] = 1 << 63
    a, b = bmp(words), run([(63, 64)])
    assert a.intersection_count(b) == 1
    a = bmp([0xF0000001, 0xFF00000000000000, 0xFF000000000000F0, 0x0F0000])
    b = run([(29, 31), (125, 134), (191, 197), (200, 300)])
    assert a.intersection_count(b) == 14 == b.intersection_count(a)


@pytest.mark.parametrize("aruns,bruns,exp", [
    ([], [(3, 8)], 0), ([(2, 10)], [(3, 8)], 6), ([(2, 10)], [(1, 11)], 9), ([(2, 10)], [(0, 2)], 1),
    ([(2, 10)], [(1, 10)], 9), ([(2, 10)], [(5, 12)], 6), ([(2, 10)], [(10, 99)], 1),
    ([(2, 10), (44, 99)], [(12, 14)], 0), ([(2, 10), (12, 13)], [(2, 10), (12, 13)], 11),
    ([(8, 12), (15, 19)], [(9, 9), (11, 17)], 6)])
def test_intersection_count_run_run(aruns, bruns, exp):  # TestIntersectionCountRunRun :379
    a, b = run(aruns), run(bruns)
    assert a.intersection_count(b) == exp == b.intersection_count(a)


@pytest.mark.parametrize("array,runs,exp", [
    ([1, 4, 5, 7, 10, 11, 12], [(5, 10)], [5, 7, 10]), ([], [(5, 10)], []),
    ([1, 4, 5, 7, 10, 11, 12], [], []), ([0, 1, 4, 5, 7, 10, 11, 12], [(0, 5), (7, 7)], [0, 1, 4, 5, 7])])
def test_intersect_array_run(array, runs, exp):  # TestIntersectArrayRun :426
    a, b = arr(array), run(runs)
    assert vals(a.intersect(b)) == exp == vals(b.intersect(a))


@pytest.mark.parametrize("aruns,bruns,exp,n", [
    ([], [(5, 10)], [], 0), ([(5, 12)], [(5, 10)], [(5, 10)], 6),
    ([(1, 3), (5, 5), (7, 8), (9, 12)], [(5, 10)], [(5, 5), (7, 10)], 5),
    ([(20, 30)], [(5, 10), (19, 21)], [(20, 21)], 2), ([(5, 10)], [(7, 12)], [(7, 10)], 4),
    ([(5, 12)], [(7, 10)], [(7, 10)], 4)])
def test_intersect_run_run(aruns, bruns, exp, n):  # TestIntersectRunRun :470
    r = run(aruns).intersect(run(bruns))
    assert r.count() == n and vals(r) == _vals_of_runs(exp)


@pytest.mark.parametrize("words,runs,exp,n", [
    ([1], [(0, 0), (2, 5), (62, 71), (77, 4096)], [1], 1),
    ([0xFFFFFFFFFFFFFFFF], [(1, 1)], [2], 1),
    ([0xFFFFFFFFFFFFFFFF], [(1, 1), (10, 12), (61, 77)], [0xe000000000001C02], 7),
    ([0xFFFFFFFFFFFFFFFF] * 2, [(1, 1), (61, 77)], [0xE000000000000002, 0x3FFF], 18),
    ([0xFFFFFFFFFFFFFFFF, 1, 1, 1, 0xA, 1, 1, 0, 1], [(63, 10000)], [0x8000000000000000, 1, 1, 1, 0xA, 1, 1, 0, 1], 9)])
def test_intersect_bitmap_run(words, runs, exp, n):  # TestIntersectBitmapRunBitmap :533, ...RunArray :591
    r = bmp(words).intersect(run(runs))
    assert r.count() == n and vals(r) == _vals_of_words(exp)
    assert vals(run(runs).intersect(bmp(words))) == _vals_of_words(exp)


def test_union_mixed():  # TestUnionMixed :645
    a = arr([1, 4, 5, 7, 10, 11, 12])
    b = bmp([0x3])
    r = run([(5, 10)])
    assert vals(r.union(a)) == vals(a.union(r)) == [1, 4, 5, 6, 7, 8, 9, 10, 11, 12]
    assert vals(r.union(r)) == [5, 6, 7, 8, 9, 10]
    assert vals(b.union(r)) == vals(r.union(b)) == [0, 1, 5, 6, 7, 8, 9, 10]
    assert vals(a.union(b)) == vals(b.union(a)) == [0, 1, 4, 5, 7, 10, 11, 12]


def test_intersect_mixed():  # TestIntersectMixed :687
    a, b, c = run([(5, 10)]), arr([1, 4, 5, 7, 10, 11, 12]), bmp([0x60])
    assert vals(a.intersect(b)) == vals(b.intersect(a)) == [5, 7, 10]
    assert vals(a.intersect(a)) == _vals_of_runs([(5, 10)])
    assert vals(c.intersect(a)) == vals(a.intersect(c)) == [5, 6]
    assert vals(b.intersect(c)) == vals(c.intersect(b)) == [5]


def test_difference_mixed():  # TestDifferenceMixed :725
    a = run([(5, 10)])
    b = arr([0, 2, 4, 6, 8, 10, 12])
    c = bmp([0x64])
    d = arr([1, 3, 5, 7, 9, 11, 12])
    assert vals(a.difference(b)) == [5, 7, 9]
    assert vals(b.difference(a)) == [0, 2, 4, 12]
    assert vals(a.difference(a)) == []
    assert vals(c.difference(a)) == [2]
    assert vals(a.difference(c)) == [7, 8, 9, 10]
    assert vals(b.difference(c)) == [0, 4, 8, 10, 12]
    assert vals(c.difference(b)) == [5]
    assert b.difference(b).count() == 0 and c.difference(c).count() == 0
    assert vals(d.difference(b)) == [1, 3, 5, 7, 9, 11]
    assert vals(b.difference(d)) == [0, 2, 4, 6, 8, 10]


@pytest.mark.parametrize("aruns,bruns,exp", [
    ([], [(5, 10)], [(5, 10)]), ([(5, 12)], [(5, 10)], [(5, 12)]),
    ([(1, 3), (5, 5), (7, 8), (9, 12)], [(5, 10)], [(1, 3), (5, 12)]),
    ([(1, 3), (5, 5), (7, 8), (9, 12)], [(2, 65535)], [(1, 65535)]),
    ([(2, 65535)], [(1, 3), (5, 5), (7, 8), (9, 12)], [(1, 65535)]),
    ([(1, 3), (5, 5), (7, 8), (9, 12)], [(0, 65535)], [(0, 65535)]),
    ([(0, 65535)], [(1, 3), (5, 5), (7, 8), (9, 12)], [(0, 65535)]),
    ([(1, 3), (5, 5), (7, 9), (12, 22)], [(2, 8), (16, 27), (33, 34)], [(1, 9), (12, 27), (33, 34)])])
def test_union_run_run(aruns, bruns, exp):  # TestUnionRunRun :792
    u = run(aruns).union(run(bruns))
    assert vals(u) == _vals_of_runs(exp)
    u.optimize()
    if u.count() > 1:   # the optimised form of these unions is the reference's run list
        assert types(u) == ["run"] and u.container_runs(0) == exp


@pytest.mark.parametrize("array,runs,exp", [
    ([1, 4, 5, 7, 10, 11, 12], [(5, 10)], [1, 4, 5, 6, 7, 8, 9, 10, 11, 12]), ([], [(5, 10)], [5, 6, 7, 8, 9, 10]),
    ([1, 4, 5, 7, 10, 11, 12], [], [1, 4, 5, 7, 10, 11, 12]),
    ([0, 1, 4, 5, 7, 10, 11, 12], [(0, 5), (7, 7)], [0, 1, 2, 3, 4, 5, 7, 10, 11, 12])])
def test_union_array_run(array, runs, exp):  # TestUnionArrayRun :851
    assert vals(arr(array).union(run(runs))) == exp == vals(run(runs).union(arr(array)))


def test_array_bitmap_conversions():  # TestArrayToBitmap :927, TestBitmapToArray :953
    b = arr([0, 1, 2, 3])
    b.convert_container(0, "bitmap")
    assert types(b) == ["bitmap"] and vals(b) == [0, 1, 2, 3]
    b = bmp([0xF])
    b.convert_container(0, "array")
    assert types(b) == ["array"] and vals(b) == [0, 1, 2, 3]


@pytest.mark.parametrize("runs,words", [
    ([(0, 0)], [1]), ([(0, 4)], [31]), ([(2, 2), (5, 7), (13, 14), (17, 17)], [155876]),
    ([(0, 3), (60, 67)], [0xF00000000000000F, 0xF])])
def test_run_to_bitmap(runs, words):  # TestRunToBitmap :977
    b = run(runs)
    b.convert_container(0, "bitmap")
    assert types(b) == ["bitmap"] and vals(b) == _vals_of_words(words)


def _tail_words():
    w = [0] * 1024
    w[1022] = w[1023] = 0xFFFFFFFFFFFFFFFF
    return w


@pytest.mark.parametrize("words,exp", [
    ([1], [(0, 0)]), ([31], [(0, 4)]), ([155876], [(2, 2), (5, 7), (13, 14), (17, 17)]),
    ([0xF00000000000000F, 0xF], [(0, 3), (60, 67)]), ([0xFFFFFFFFFFFFFFFF, 0xF], [(0, 67)]),
    ([0xF000000000000000, 0xFFFFFFFFFFFFFFFF], [(60, 127)]),
    ([0xF000000000000000, 0xFFFFFFFFFFFFFFFF, 0xF], [(60, 131)]),
    (_tail_words(), [(65408, 65535)]), ([0xFFFFFFFFFFFFFFFF] * 1024, [(0, 65535)])])
def test_bitmap_to_run_and_back(words, exp):  # TestBitmapToRun :1028
    b = bmp(words)
    before = vals(b)
    b.convert_container(0, "run")
    assert b.container_runs(0) == exp
    b.convert_container(0, "bitmap")
    assert vals(b) == before


@pytest.mark.parametrize("array,exp", [
    ([0], [(0, 0)]), ([0, 1, 2, 3, 4], [(0, 4)]), ([2, 5, 6, 7, 13, 14, 17], [(2, 2), (5, 7), (13, 14), (17, 17)])])
def test_array_run_conversions(array, exp):  # TestArrayToRun :1099, TestRunToArray :1131
    b = arr(array)
    b.convert_container(0, "run")
    assert b.container_runs(0) == exp
    b.convert_container(0, "array")
    assert types(b) == ["array"] and vals(b) == array


def test_union_bitmap_run():  # TestUnionBitmapRun :1204
    u = bmp([2]).union(run([(0, 0), (2, 5), (62, 71), (77, 78)]))
    assert u.count() == 18 and vals(u) == _vals_of_words([0xC00000000000003F, 0x60FF])


@pytest.mark.parametrize("words,exp", [
    ([0xFF00FF00], 2), ([0xFF00FF0000000000, 0x1], 2), ([0xFF00FF0000000000, 0x2, 0x100], 4),
    ([0xFF00FF0000000000, 0x1010101FF0101010, 0x100], 10)])
def test_bitmap_count_runs(words, exp):  # TestBitmapCountRuns :1238
    assert bmp(words).container_run_count(0) == exp
    at_end = [0] * (1024 - len(words)) + list(words)
    assert bmp(at_end).container_run_count(0) == exp


@pytest.mark.parametrize("array,exp", [
    ([0], 1), ([1], 1), ([1, 2, 3, 5], 2), ([0, 1, 3, 9, 2048, 4096, 4097, 65534, 65535], 6), ([0, 10, 11, 12], 2)])
def test_array_count_runs(array, exp):  # TestArrayCountRuns :1285
    assert arr(array).container_run_count(0) == exp


@pytest.mark.parametrize("words,start,last,exp,n", [
    ([0x0000000000FFF900], 9, 10, [0x0000000000FFFF00], 16),
    ([0xFF0, 0xFF, 0xFF], 60, 130, [0xF000000000000FF0, 0xFFFFFFFFFFFFFFFF, 0xFF], 84)])
def test_bitmap_set_range(words, start, last, exp, n):  # TestBitmapSetRange :891
    r = bmp(words).union(run([(start, last)]))
    assert r.count() == n and vals(r) == _vals_of_words(exp)


@pytest.mark.parametrize("words,start,last,exp,n", [
    ([0x0000000000FFFF00], 9, 10, [0x0000000000FFF900], 14),
    ([0xFF0, 0xFF, 0xFF], 60, 130, [0xFF0, 0, 0xF8], 13)])
def test_bitmap_zero_range(words, start, last, exp, n):  # TestBitmapZeroRange :1163
    r = bmp(words).difference(run([(start, last)]))
    assert r.count() == n and vals(r) == _vals_of_words(exp)


def test_difference_array_run():  # TestDifferenceArrayRun :1326
    assert vals(arr(list(range(13))).difference(run([(5, 10)]))) == [0, 1, 2, 3, 4, 11, 12]


@pytest.mark.parametrize("runs,array,exp", [
    ([(0, 12)], [5, 6, 7, 8, 9, 10], [(0, 4), (11, 12)]), ([(0, 12)], [0, 1, 2, 3], [(4, 12)]),
    ([(0, 12)], [9, 10, 11, 12, 13], [(0, 8)]), ([(1, 12)], [0, 9, 10, 11, 12, 13], [(1, 8)]),
    ([(1, 12), (14, 14), (18, 18)], [0, 9, 10, 11, 12, 13, 14, 17], [(1, 8), (18, 18)]),
    ([(1, 12), (14, 14), (18, 18)], [0, 9, 10, 11, 12, 13, 14, 17, 19], [(1, 8), (18, 18)]),
    ([(1, 12), (14, 17), (19, 28)], [0, 9, 10, 11, 12, 13, 14, 17, 19, 25, 27],
     [(1, 8), (15, 16), (20, 24), (26, 26), (28, 28)]),
    ([(0, 20), (65533, 65535)], [65533, 65534, 65535], [(0, 20)]),
    ([(0, 20), (65530, 65535)], [37, 65535], [(0, 20), (65530, 65534)])])
def test_difference_run_array(runs, array, exp):  # TestDifferenceRunArray :1348
    assert vals(run(runs).difference(arr(array))) == _vals_of_runs(exp)


def _last_bit():
    w = [0] * 1024
    w[1023] = 1 << 63
    return w


@pytest.mark.parametrize("runs,words,exp", [
    ([(0, 63)], [0x0000FFFF000000F0], [(0, 3), (8, 31), (48, 63)]), ([(0, 63)], [0x8000000000000000], [(0, 62)]),
    ([(0, 63)], [1], [(1, 63)]), ([(0, 63)], [0, 1], [(0, 63)]), ([(0, 65)], [0, 1], [(0, 63), (65, 65)]),
    ([(0, 65)], [0, 0x8000000000000000], [(0, 65)]), ([(1, 65535)], [1], [(1, 65535)]),
    ([(0, 65533), (65535, 65535)], _last_bit(), [(0, 65533)])])
def test_difference_run_bitmap(runs, words, exp):  # TestDifferenceRunBitmap :1421
    assert vals(run(runs).difference(bmp(words))) == _vals_of_runs(exp)


@pytest.mark.parametrize("words,runs,exp", [
    ([0xFFFFFFFFFFFFFFFF], [(4, 7), (32, 47)], [0xFFFF0000FFFFFF0F]),
    ([0xFFFFFFFFFFFFFFBF], [(0, 5), (7, 63)], [0]), ([0xFFFFFFFFFFFFFFBF], [(0, 5)], [0xFFFFFFFFFFFFFF80]),
    ([0xFFFFFFFFFFFFFFFF], [(60, 63)], [0x0FFFFFFFFFFFFFFF]), ([0xFFFFFFFFFFFFFFFF], [(60, 65)], [0x0FFFFFFFFFFFFFFF]),
    ([0xFFFFFFFFFFFFFFFF] * 3, [(60, 65), (67, 72), (126, 130)],
     [0x0FFFFFFFFFFFFFFF, 0x3FFFFFFFFFFFFE04, 0xFFFFFFFFFFFFFFF8]),
    ([1], [(0, 0)], [0]), ([0x8000000000000000], [(63, 63)], [0]),
    ([0xC000000000000000, 0x3], [(63, 64)], [0x4000000000000000, 0x2]), ([0], [(5, 7)], [0]),
    (_last_bit(), [(65535, 65535)], [0]), ([0xFFFFFFFFFFFFFFFF] * 1024, [(0, 65535)], [0])])
def test_difference_bitmap_run(words, runs, exp):  # TestDifferenceBitmapRun :1478
    assert vals(bmp(words).difference(run(runs))) == _vals_of_words(exp)


_ODD = [0xAAAAAAAAAAAAAAAA]


@pytest.mark.parametrize("words,array,exp", [
    ([0xFF0F], [0, 1, 2, 3, 4, 5, 6, 7, 10], [8, 9, 11, 12, 13, 14, 15]),
    ([0], [0, 1, 2, 3, 4, 5, 6, 7, 10], []), ([0xFFFF], [0, 1, 2, 3, 4, 5, 6, 7, 10], [8, 9, 11, 12, 13, 14, 15]),
    (_ODD, [0, 1, 2, 3, 4, 5, 6, 7, 10], list(range(9, 64, 2))), (_ODD, [63], list(range(1, 63, 2))),
    ([0x0000FFFF000000F0], [4, 5, 6, 7, 20, 21, 22, 23] + list(range(32, 48)), [])])
def test_difference_bitmap_array(words, array, exp):  # TestDifferenceBitmapArray :1555
    assert vals(bmp(words).difference(arr(array))) == exp


@pytest.mark.parametrize("a,b,exp", [([0xFF00FFFFFFFFFFFF], [0xFFFFFFFFFFFFF000], list(range(12))),
                                     ([0xF], [0], [0, 1, 2, 3])])
def test_difference_bitmap_bitmap(a, b, exp):  # TestDifferenceBitmapBitmap :1602
    assert vals(bmp(a).difference(bmp(b))) == exp


def test_difference_run_run():  # TestDifferenceRunRun :1629
    a = run([(3, 6), (13, 16), (24, 26), (33, 38), (43, 46), (53, 56)])
    b = run([(1, 8), (11, 14), (21, 23), (35, 37), (44, 48), (57, 59)])
    d = a.difference(b)
    assert d.count() == 13
    assert vals(d) == _vals_of_runs([(15, 16), (24, 26), (33, 34), (38, 38), (43, 43), (53, 56)])


def test_write_read_containers():  # TestWriteReadArray :1659, ...Bitmap :1678, ...FullBitmap :1701, ...Run :1734
    a = arr([1, 10, 100, 1000])
    back = Bitmap.from_bytes(a.to_bytes())
    assert types(back) == ["array"] and vals(back) == [1, 10, 100, 1000]
    b = bmp([0x5555555555555555] * 129)
    back = Bitmap.from_bytes(b.to_bytes())
    assert types(back) == ["bitmap"] and vals(back) == vals(b) and back.count() == 129 * 32
    full = bmp([0xFFFFFFFFFFFFFFFF] * 1024)
    back = Bitmap.from_bytes(full.to_bytes())   # written optimised: one run
    assert back.count() == 65536 and vals(back) == list(range(65536))
    r = run([(3, 13), (100, 109)])
    back = Bitmap.from_bytes(r.to_bytes())
    assert types(back) == ["run"] and back.container_runs(0) == [(3, 13), (100, 109)]


@pytest.mark.parametrize("a,runs,exp", [
    ([1, 5, 10, 11, 12], [(2, 10), (12, 13), (15, 16)], [1, 2, 3, 4, 6, 7, 8, 9, 11, 13, 15, 16]),
    ([1, 5, 10, 11, 12, 13, 14], [(2, 10), (12, 13), (15, 16)], [1, 2, 3, 4, 6, 7, 8, 9, 11, 14, 15, 16]),
    ([65535], [(65534, 65535)], [65534]), ([65535], [(65535, 65535)], [])])
def test_xor_array_run(a, runs, exp):  # TestXorArrayRun :1753
    assert vals(arr(a).xor(run(runs))) == exp == vals(run(runs).xor(arr(a)))


def test_xor_run_run1():  # TestXorRunRun1 :1794
    a, b = run([(4, 10)]), run([(5, 10)])
    assert vals(a.xor(b)) == [4] == vals(b.xor(a))


@pytest.mark.parametrize("aruns,bruns,exp", [
    ([], [(5, 10)], [(5, 10)]), ([(0, 4)], [(6, 10)], [(0, 4), (6, 10)]), ([(0, 6)], [(4, 10)], [(0, 3), (7, 10)]),
    ([(4, 10)], [(0, 6)], [(0, 3), (7, 10)]), ([(0, 10)], [(0, 6)], [(7, 10)]), ([(0, 6)], [(0, 10)], [(7, 10)]),
    ([(5, 12)], [(5, 10)], [(11, 12)]),
    ([(1, 3), (5, 5), (7, 12)], [(5, 10)], [(1, 3), (6, 6), (11, 12)]),
    ([(1, 3), (5, 5), (7, 12)], [(2, 65535)], [(1, 1), (4, 4), (6, 6), (13, 65535)]),
    ([(2, 65535)], [(1, 3), (5, 5), (7, 12)], [(1, 1), (4, 4), (6, 6), (13, 65535)]),
    ([(1, 3), (5, 5), (7, 12)], [(0, 65535)], [(0, 0), (4, 4), (6, 6), (13, 65535)]),
    ([(0, 65535)], [(1, 3), (5, 5), (7, 12)], [(0, 0), (4, 4), (6, 6), (13, 65535)]),
    ([(1, 3), (5, 5), (7, 9), (12, 22)], [(2, 8), (16, 27), (33, 34)],
     [(1, 1), (4, 4), (6, 6), (9, 9), (12, 15), (23, 27), (33, 34)]),
    ([(65530, 65535)], [(65532, 65535)], [(65530, 65531)])])
def test_xor_run_run(aruns, bruns, exp):  # TestXorRunRun :1807 (the run/run xor state machine)
    a, b = run(aruns), run(bruns)
    assert vals(a.xor(b)) == _vals_of_runs(exp) == vals(b.xor(a))


@pytest.mark.parametrize("words,start,last,exp,n", [
    ([0], 0, 2, [0x7], 3), ([0xF1], 4, 8, [0x101], 2), ([0xAA], 0, 7, [0x55], 4),
    ([0, 0, 0], 63, 128, [0x8000000000000000, 0xFFFFFFFFFFFFFFFF, 0x1], 66),
    ([0, 0xFF, 0], 63, 128, [0x8000000000000000, 0xFFFFFFFFFFFFFF00, 0x1], 58),
    ([0, 0, 0], 129, 131, [0, 0, 0xE], 3)])
def test_bitmap_xor_range(words, start, last, exp, n):  # TestBitmapXorRange :1905 (Flip), TestXorBitmapRun :1969
    b = bmp(words) if any(words) else Bitmap()
    f = b.flip(start, last)
    assert f.count() == n and vals(f) == _vals_of_words(exp)
    assert vals(b.xor(run([(start, last)]))) == _vals_of_words(exp)


REF_TESTDATA = "/root/reference/roaring/testdata"


@pytest.mark.parametrize("hexdata,count", [
    ("3A300000020000000000020001000000180000001E0000000100020003000100", 4),
    ("3B3001000100000900010000000100010009000100", 11)])
def test_unmarshal_official_roaring(hexdata, count):  # TestUnmarshalRoaringWithNoErrors :3359
    b = Bitmap.from_bytes(bytes.fromhex(hexdata))
    assert b.count() == count
    assert b.contains(65537)


def test_unmarshal_official_roaring_file():  # TestUnmarshalRoaringWithNoErrors :3376 (testdata file)
    import os
    p = os.path.join(REF_TESTDATA, "bitmapcontainer.roaringbitmap")
    if not os.path.exists(p):
        pytest.skip("reference testdata not present")
    with open(p, "rb") as fh:
        assert Bitmap.from_bytes(fh.read()).count() == 10000


def test_unmarshal_roaring_with_errors():  # TestUnmarshalRoaringWithErrors :3404
    for hx, at in (("3A30000000000000", 8), ("3B30000000000000", 9)):
        with pytest.raises(RuntimeError) as ei:
            Bitmap.from_bytes(bytes.fromhex(hx))
        assert str(ei.value) == f"reading roaring header: malformed bitmap, key-cardinality slice overruns buffer at {at}"
    assert Bitmap.from_bytes(bytes.fromhex("3C30000000000000")).count() == 0   # Pilosa format, no containers


@pytest.mark.parametrize("array,exp", [([1], [2]), ([], []), ([1, 2, 3, 4, 5, 11, 12], [2, 3, 4, 5, 6, 12, 13]),
                                       ([65535], [65536])])
def test_shift_array(array, exp):  # TestShiftArray :3478 (the carry lands in the next container)
    a = arr(array) if array else Bitmap()
    assert vals(a.shift(1)) == exp


def test_shift_bitmap():  # TestShiftBitmap :3520
    first = [0] * 1024
    first[0] = 1
    assert vals(bmp(first).shift(1)) == [1]
    assert vals(bmp(_last_bit()).shift(1)) == [65536]
    row_end = [0] * 1024
    row_end[0] = 1 << 63
    assert vals(bmp(row_end).shift(1)) == [64]


@pytest.mark.parametrize("runs,exp", [([(5, 10)], _vals_of_runs([(6, 11)])),
                                      ([(5, 65535)], _vals_of_runs([(6, 65536)])),
                                      ([(65535, 65535)], [65536])])
def test_shift_run(runs, exp):  # TestShiftRun :3552
    assert vals(run(runs).shift(1)) == exp


_OPS = [(0, 27, []), (1, 28, []), (2, 0, [1, 2, 6, 19]), (3, 0, [1, 2, 6, 19, 22, 44]), (2, 0, [51234567890]),
        (3, 0, [51234567890]), (0, 0, []), (1, 0, []), (2, 0, [0]), (3, 0, [0]), (2, 0, []), (3, 0, [])]


def test_op_log_write_unmarshal():  # TestOpLogWriteUnmarshal :3595
    want = set()
    data = bytearray(Bitmap().to_bytes())
    for typ, value, values in _OPS:
        v = np.array(values, np.uint64)
        enc = _roaring.encode_op(typ, len(values) if typ in (2, 3) else value, v, b"", 0)
        assert len(enc) == 13 + (8 * len(values) if typ in (2, 3) else 0)
        # each op alone replays
        one = Bitmap.from_bytes(bytes(Bitmap().to_bytes()) + enc)
        assert one.ops == 1
        data += enc
        if typ == 0:
            want.add(value)
        elif typ == 1:
            want.discard(value)
        elif typ == 2:
            want |= set(values)
        else:
            want -= set(values)
    b = Bitmap.from_bytes(bytes(data))   # all of them back to back
    assert b.ops == len(_OPS) and vals(b) == sorted(want)
    bad = bytearray(data)
    bad[-20] ^= 0xFF                     # a corrupted op fails its checksum
    with pytest.raises(Exception):
        Bitmap.from_bytes(bytes(bad))


@pytest.mark.parametrize("call1,n1,call2,n2,exp", [
    ([0], 1, [0, 1], 1, [0, 1]), ([0, 22, 55], 3, [0, 14, 22, 99, 55], 2, [0, 14, 22, 55, 99])])
def test_direct_add_n(call1, n1, call2, n2, exp):  # TestDirectAddN :3705
    b = Bitmap()
    assert b.add_many(np.array(call1, np.uint64)) == n1
    assert b.add_many(np.array(call2, np.uint64)) == n2
    assert vals(b) == exp


def test_direct_add_n_vs_add():  # TestDirectAddNVsAdd :3753
    tests = [[], [0], [0, 1, 2, 3], [0, 1, 2, 101000, 9384932], [9384932, 101000, 2, 1, 0],
             [3489, 19230, 394, 0, 893982, 890283, 14, 7]]
    ca, cd = Bitmap(), Bitmap()
    for t in tests:
        fa, fd = Bitmap(), Bitmap()
        na = any([fa.add(v) for v in t])
        nd = fd.add_many(np.array(t, np.uint64))
        assert na == (nd > 0) and vals(fa) == vals(fd)
        na = any([ca.add(v) for v in t])
        nd = cd.add_many(np.array(t, np.uint64))
        assert na == (nd > 0) and vals(ca) == vals(cd)


def test_bitmap_any():  # TestBitmapAny :3851
    b = Bitmap()
    assert not b.any()
    b.add(1)
    assert b.any()
    b.add(100000)
    assert b.any()
    assert b.remove(1) and b.any()
    b.add(1)
    b = b.difference(Bitmap(np.array([1], np.uint64)))
    assert b.any()
    b.remove(100000)
    assert not b.any()
