"""Ported expectations of the reference's holder_test.go and
holder_internal_test.go (open-time errors carry the index/field/fragment
context, HasData, DeleteIndex, the holder cleaner).  The permission cases
are skipped as root, as the reference skips them."""
import os
import shutil
import tempfile

import pytest

from pilosa_amd.errors import PilosaError
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.holder import Holder
from pilosa_amd.utils.logger import CaptureLogger


@pytest.fixture
def path():
    d = tempfile.mkdtemp(prefix="holderref_")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _reopen(h):
    h.close()
    h2 = Holder(h.path)
    h2.logger = CaptureLogger()
    return h2


def test_holder_open_err_index_name(path):  # TestHolder_Open/ErrIndexName
    h = Holder(path).open()
    os.mkdir(os.path.join(path, "!"))
    h2 = _reopen(h)
    h2.open()
    assert any("ERROR opening index: !" in m for m in h2.logger.prints)
    h2.close()


def test_holder_open_err_index_attr_store_corrupt(path):  # TestHolder_Open/ErrIndexAttrStoreCorrupt
    h = Holder(path).open()
    h.create_index("test")
    h2 = _reopen(h)
    with open(os.path.join(path, "test", ".data"), "r+b") as fh:
        fh.truncate(2)
    with pytest.raises(PilosaError, match="open index: name=test, err=opening attrstore: opening storage: invalid database"):
        h2.open()


def test_holder_open_err_field_options_corrupt(path):  # TestHolder_Open/ErrFieldOptionsCorrupt
    h = Holder(path).open()
    h.create_index("foo").create_field("bar", FieldOptions())
    h2 = _reopen(h)
    with open(os.path.join(path, "foo", "bar", ".meta"), "r+b") as fh:
        fh.truncate(2)
    with pytest.raises(PilosaError, match="open index: name=foo, err=opening fields: open field: name=bar, "
                                          "err=loading meta: unmarshaling"):
        h2.open()


def test_holder_open_err_field_attr_store_corrupt(path):  # TestHolder_Open/ErrFieldAttrStoreCorrupt
    h = Holder(path).open()
    h.create_index("foo").create_field("bar", FieldOptions())
    h2 = _reopen(h)
    with open(os.path.join(path, "foo", "bar", ".data"), "r+b") as fh:
        fh.truncate(2)
    with pytest.raises(PilosaError, match="open index: name=foo, err=opening fields: open field: name=bar, "
                                          "err=opening attrstore: opening storage: invalid database"):
        h2.open()


def test_holder_open_err_fragment_storage_corrupt(path):  # TestHolder_Open/ErrFragmentStorageCorrupt
    h = Holder(path).open()
    h.create_index("foo").create_field("bar", FieldOptions()).set_bit(0, 0)
    h2 = _reopen(h)
    with open(os.path.join(path, "foo", "bar", "views", "standard", "fragments", "0"), "r+b") as fh:
        fh.truncate(2)
    with pytest.raises(PilosaError, match="open fragment: shard=0, err=opening storage: unmarshal storage"):
        h2.open()


def test_holder_has_data(path):  # TestHolder_HasData (IndexDirectory, Peek, Peek at missing directory)
    h = Holder(path).open()
    assert not h.has_data()
    h.create_index("test")
    assert h.has_data()
    h.close()
    d2 = tempfile.mkdtemp()
    h = Holder(d2)
    assert not h.has_data()
    os.mkdir(os.path.join(d2, "test"))
    assert h.has_data()
    assert not Holder("bad-path-does-not-exist").has_data()


def test_holder_delete_index(path):  # TestHolder_DeleteIndex
    h = Holder(path).open()
    for name in ("i0", "i1"):
        h.create_index(name).create_field("f", FieldOptions()).set_bit(100, 200)
    h.delete_index("i0")
    assert not os.path.exists(os.path.join(path, "i0")) and h.index("i0") is None
    assert os.path.exists(os.path.join(path, "i1")) and h.index("i1") is not None
    h.close()
