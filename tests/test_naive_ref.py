"""Reference roaring/naive_test.go, ported (16 tests): the slice oracle's
helpers (pilosa_amd/testing/naive.py), with the reference's expectations."""
from pilosa_amd.testing import naive as nv

A = [1, 4, 9, 5, 24, 13]
B = [2, 1, 9, 5, 12]


def test_sort_slice():
    assert nv.sort_slice([1, 3, 2, 8, 5, 21, 13]) == [1, 2, 3, 5, 8, 13, 21]


def test_remove_slice_duplicates():
    assert nv.remove_slice_duplicates([2, 3, 2, 1, 2, 5, 8, 5, 13, 3, 2, 5, 144]) == [1, 2, 3, 5, 8, 13, 144]
    assert nv.remove_slice_duplicates([2, 3, 2, 1, 2, 5, 8, 5, 13, 3, 2, 5, 144, 21, 8, 3, 3, 5, 5, 1, 34, 21, 21]) == \
        [1, 2, 3, 5, 8, 13, 21, 34, 144]


def test_intersect_slice():
    assert nv.intersect_slice(A, B) == [1, 5, 9]
    assert nv.intersect_slice(B, A) == [1, 5, 9]
    assert nv.intersect_slice(A, [1, 5, 9]) == [1, 5, 9]


def test_union_slice():
    assert nv.union_slice(A, B) == [1, 2, 4, 5, 9, 12, 13, 24]
    assert nv.union_slice(B, A) == [1, 2, 4, 5, 9, 12, 13, 24]
    assert nv.union_slice(A, [1, 5, 9]) == [1, 4, 5, 9, 13, 24]


def test_max_in_slice():
    a = list(A)
    assert nv.max_in_slice(a) == 24
    for i in range(1000, 100001, 997):
        a.append(i)
        assert nv.max_in_slice(a) == i


def test_difference_slice():
    assert nv.difference_slice(A, B) == [4, 13, 24]
    assert nv.difference_slice(B, A) == [2, 12]
    assert nv.difference_slice(A, A) == []


def test_xor_slice():
    assert nv.xor_slice(A, B) == [2, 4, 12, 13, 24]
    assert nv.xor_slice(B, A) == [2, 4, 12, 13, 24]
    assert nv.xor_slice([2, 4, 12, 13, 24], A) == [1, 2, 5, 9, 12]
    assert nv.xor_slice([2, 4, 12, 13, 24], [1, 2, 5, 9, 12]) == [1, 4, 5, 9, 13, 24]


def test_shift_slice():
    assert nv.shift_slice(A, 12) == [13, 16, 17, 21, 25, 36]
    assert nv.shift_slice(A, 0) == [1, 4, 5, 9, 13, 24]
    assert nv.shift_slice(A, 1) == [2, 5, 6, 10, 14, 25]


def test_for_each_in_slice():
    c = []
    nv.for_each_in_slice(A, lambda v: c.append(v + 1))
    assert c == [2, 5, 10, 6, 25, 14]


def test_for_each_in_range_slice():
    c = []
    nv.for_each_in_range_slice(A, 3, 12, lambda v: c.append(v + 1))
    assert c == [5, 10, 6]


def test_contained_in_slice():
    assert nv.contained_in_slice(A, 4) == (1, True)
    assert nv.contained_in_slice(A, 12) == (-1, False)


def test_add_n_to_slice():
    assert nv.add_n_to_slice(A, *B) == ([1, 2, 4, 5, 9, 12, 13, 24], 2)
    assert nv.add_n_to_slice(B, *A) == ([1, 2, 4, 5, 9, 12, 13, 24], 3)
    assert nv.add_n_to_slice(A, *A) == ([1, 4, 5, 9, 13, 24], 0)


def test_remove_n_from_slice():
    assert nv.remove_n_from_slice(A, *B) == ([4, 13, 24], 3)
    assert nv.remove_n_from_slice(B, *A) == ([2, 12], 3)
    assert nv.remove_n_from_slice(A, *A) == ([], 6)


def test_count_range_slice():
    assert nv.count_range_slice(A, 3, 12) == 3
    assert nv.count_range_slice(A, 0, 25) == 6
    assert nv.count_range_slice(A, 12, 4) == 0
    assert nv.count_range_slice(A, 4, 4) == 0


def test_range_slice():
    assert nv.range_slice(A, 3, 12) == [4, 5, 9]
    assert nv.range_slice(A, 0, 25) == [1, 4, 5, 9, 13, 24]
    assert nv.range_slice(A, 5, 5) == []


def test_flip_slice():
    assert nv.flip_slice(A, 3, 12) == [1, 3, 6, 7, 8, 10, 11, 12, 13, 24]
    assert nv.flip_slice(A, 13, 12) == [1, 4, 5, 9, 13, 24]
    assert nv.flip_slice(A, 9, 13) == [1, 4, 5, 10, 11, 12, 24]
