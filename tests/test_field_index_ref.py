"""Ported expectations of the reference's field_test.go,
field_internal_test.go, index_test.go and index_internal_test.go.  Each
test names the reference test it ports."""
import datetime as dt
import os
import shutil
import tempfile

import pytest

from pilosa_amd.errors import (ErrBSIGroupNotFound, ErrBSIGroupValueTooHigh, ErrBSIGroupValueTooLow, ErrName,
                               PilosaError)
from pilosa_amd.models.field import BSIGroup, Field, FieldOptions
from pilosa_amd.models.index import Index
from pilosa_amd.shardwidth import SHARD_WIDTH as SW

I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


@pytest.fixture
def index():
    d = tempfile.mkdtemp(prefix="idxref_")
    idx = Index(os.path.join(d, "i"), "i").open()
    yield idx
    idx.close()
    shutil.rmtree(d, ignore_errors=True)


def _reopen_index(idx):
    path, name = idx.path, idx.name
    idx.close()
    return Index(path, name).open()


def test_field_set_value_ok_and_overwrite(index):  # TestField_SetValue/OK, /Overwrite
    f = index.create_field("f", FieldOptions(type="int", min=I64_MIN, max=I64_MAX))
    assert f.set_value(100, 21)
    assert f.value(100) == (21, True)
    assert not f.set_value(100, 21)
    assert f.set_value(100, 23)
    assert f.value(100) == (23, True)


def test_field_set_value_errors(index):  # TestField_SetValue/ErrBSIGroup{NotFound,ValueTooLow,ValueTooHigh}
    f = index.create_field("f", FieldOptions())
    with pytest.raises(type(ErrBSIGroupNotFound)):
        f.set_value(100, 21)
    g = index.create_field("g", FieldOptions(type="int", min=20, max=30))
    with pytest.raises(type(ErrBSIGroupValueTooLow), match=str(ErrBSIGroupValueTooLow)):
        g.set_value(100, 15)
    with pytest.raises(type(ErrBSIGroupValueTooHigh), match=str(ErrBSIGroupValueTooHigh)):
        g.set_value(100, 31)


def test_field_name_restriction_and_validation():  # TestField_NameRestriction, TestField_NameValidation
    path = tempfile.mkdtemp()
    with pytest.raises(type(ErrName)):
        Field(path, "i", ".meta")
    for name in ("foo", "hyphen-ated", "under_score", "abc123", "trailing_"):
        Field(os.path.join(path, name), "i", name, persistent_attrs=False)
    for name in ("", "123abc", "x.y", "_foo", "-bar", "abc def", "camelCase", "UPPERCASE",
                 "a12345678901234567890123456789012345678901234567890123456789012345"):
        with pytest.raises(type(ErrName)):
            Field(os.path.join(path, "x"), "i", name, persistent_attrs=False)


def test_field_available_shards(index):  # TestField_AvailableShards
    f = index.create_field("f", FieldOptions())
    f.set_bit(0, 100)
    f.set_bit(0, SW * 2)
    assert f.available_shards() == [0, 2]
    f.add_remote_available_shards([1, 2, 4])
    assert f.available_shards() == [0, 1, 2, 4]
    for s in range(5):
        f.remove_available_shard(s)
    assert f.available_shards() == [0, 2]


B0 = BSIGroup("b0", base=-100, bit_depth=10, min=-1000, max=1000)
B1 = BSIGroup("b1", base=0, bit_depth=8, min=-255, max=255)
B2 = BSIGroup("b2", base=100, bit_depth=11, min=I64_MIN, max=I64_MAX)


@pytest.mark.parametrize("g,op,val,exp,oor", [
    (B0, "<", 5, 105, False), (B0, "<", -8, 92, False), (B0, "<", -108, -8, False), (B0, "<", 1005, 1023, False),
    (B0, "<", 0, 100, False), (B1, "<", 5, 5, False), (B1, "<", -8, -8, False), (B1, "<", 1005, 255, False),
    (B1, "<", 0, 0, False), (B2, "<", 5, -95, False), (B2, "<", -8, -108, False), (B2, "<", 105, 5, False),
    (B2, "<", 1105, 1005, False),
    (B0, ">", -5, 95, False), (B0, ">", 5, 105, False), (B0, ">", 905, 1005, False), (B0, ">", 0, 100, False),
    (B1, ">", 5, 5, False), (B1, ">", -8, -8, False), (B1, ">", 1005, 0, True), (B1, ">", 0, 0, False),
    (B2, ">", 5, -95, False), (B2, ">", -8, -108, False), (B2, ">", 105, 5, False), (B2, ">", 1105, 1005, False),
    (B0, "==", -105, -5, False), (B0, "==", 5, 105, False), (B0, "==", 905, 1005, False), (B0, "==", 0, 100, False),
    (B1, "==", 5, 5, False), (B1, "==", -8, -8, False), (B1, "==", 1005, 0, True), (B1, "==", 0, 0, False),
    (B2, "==", 5, -95, False), (B2, "==", -8, -108, False), (B2, "==", 105, 5, False),
    (B2, "==", 1105, 1005, False)])
def test_bsi_group_base_value(g, op, val, exp, oor):  # TestBSIGroup_BaseValue/Normal Condition
    assert g.base_value(op, val) == (exp, oor)


@pytest.mark.parametrize("g,lo,hi,emin,emax,oor", [
    (B0, -205, -105, -105, -5, False), (B0, -105, 80, -5, 180, False), (B0, 5, 20, 105, 120, False),
    (B0, 20, 1005, 120, 1023, False), (B0, 1005, 2000, 0, 0, True),
    (B1, -105, -5, -105, -5, False), (B1, -5, 20, -5, 20, False), (B1, 5, 20, 5, 20, False),
    (B1, 20, 1005, 20, 255, False), (B1, 1005, 2000, 0, 0, True),
    (B2, 5, 95, -95, -5, False), (B2, 95, 120, -5, 20, False), (B2, 105, 120, 5, 20, False),
    (B2, 120, 1105, 20, 1005, False), (B2, 1105, 2000, 1005, 1900, False)])
def test_bsi_group_base_value_between(g, lo, hi, emin, emax, oor):  # TestBSIGroup_BaseValue/Between Condition
    assert g.base_value_between(lo, hi) == (emin, emax, oor)


def test_field_delete_and_create_view(index):  # TestField_DeleteView, TestField_CreateViewIfNotExists
    f = index.create_field("f", FieldOptions())
    v = f.create_view_if_not_exists("standard_v")
    f.delete_view("standard_v")
    assert f.view("standard_v") is None
    assert f.create_view_if_not_exists("standard_v") is not v
    v = f.create_view_if_not_exists("v")
    assert f.create_view_if_not_exists("v") is v and f.view("v") is v


def test_field_set_time_quantum_and_row_time(index):  # TestField_SetTimeQuantum, TestField_RowTime
    f = index.create_field("f", FieldOptions(type="time", time_quantum="Y"))
    f.set_time_quantum("YMDH")
    assert f.time_quantum() == "YMDH"
    index = _reopen_index(index)
    f = index.field("f")
    assert f.time_quantum() == "YMDH"
    for col, t in ((1, dt.datetime(2010, 1, 5, 12)), (2, dt.datetime(2011, 1, 5, 12)), (3, dt.datetime(2010, 2, 5, 12)),
                   (4, dt.datetime(2010, 1, 6, 12)), (5, dt.datetime(2010, 1, 5, 13))):
        f.set_bit(1, col, t)
    cols = lambda r: [int(c) for c in r.columns()]  # noqa: E731
    assert cols(f.row_time(1, dt.datetime(2010, 11, 5, 12), "Y")) == [1, 3, 4, 5]
    assert cols(f.row_time(1, dt.datetime(2010, 2, 7, 13), "YM")) == [3]
    assert cols(f.row_time(1, dt.datetime(2010, 2, 7, 13), "M")) == [3]
    assert cols(f.row_time(1, dt.datetime(2010, 1, 5, 12), "MD")) == [1, 5]
    assert cols(f.row_time(1, dt.datetime(2010, 1, 5, 13), "MDH")) == [5]
    index.close()


def test_field_persist_available_shards(index):  # TestField_PersistAvailableShards(+Footprint)
    f = index.create_field("f", FieldOptions())
    even = list(range(0, 1204, 2))
    f.add_remote_available_shards(even)
    index = _reopen_index(index)
    assert sorted(index.field("f").remote_available_shards) == even
    odd = list(range(1, 1204, 2))
    index.field("f").add_remote_available_shards(odd)
    index = _reopen_index(index)
    assert sorted(index.field("f").remote_available_shards) == sorted(even + odd)
    index.close()


def test_index_create_field_if_not_exists(index):  # TestIndex_CreateFieldIfNotExists
    f = index.create_field_if_not_exists("f", FieldOptions())
    assert index.create_field_if_not_exists("f", FieldOptions()) is f and index.field("f") is f


def test_index_create_field_time_and_int(index):  # TestIndex_CreateField/{TimeQuantum,TimeQuantumNoStandardView,BSIFields}
    assert index.create_field("t", FieldOptions(type="time", time_quantum="YMDH")).time_quantum() == "YMDH"
    f = index.create_field("tn", FieldOptions(type="time", time_quantum="YMDH", no_standard_view=True))
    assert f.time_quantum() == "YMDH" and f.options.no_standard_view
    assert index.create_field("n", FieldOptions(type="int", min=-990, max=1000)).type == "int"
    index = _reopen_index(index)
    assert index.field("n").type == "int"
    index.close()


def test_index_delete_field(index):  # TestIndex_DeleteField
    index.create_field_if_not_exists("f", FieldOptions())
    index.delete_field("f")
    assert index.field("f") is None
    with pytest.raises(PilosaError, match="field not found"):
        index.delete_field("f")


def test_index_invalid_name():  # TestIndex_InvalidName
    with pytest.raises(type(ErrName)):
        Index(tempfile.mkdtemp(), "ABC")


def test_index_existence_delete(index):  # TestIndex_Existence_Delete (index_internal_test.go:54)
    ef = index.existence_field()
    assert ef is not None
    index.create_field("f", FieldOptions())
    index.field("f").set_bit(1, 100)
    ef.set_bit(0, 100)
    index.delete_field("f")
    assert index.existence_field() is not None and index.existence_field().row(0).count() == 1
