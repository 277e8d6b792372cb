"""BoltDB attribute files of a reference data directory (boltdb/attrstore.go):
models/boltdb.py reads the ``attrs`` bucket (id u64 big endian -> AttrMap
protobuf) through branch/leaf pages and inline buckets, and SQLiteAttrStore
converts such a ``.data`` file on open.  No reference fixture holds a BoltDB
file, so files come from the format writer here (parity unpinned against
bolt itself); the byte layout follows bolt/page.go and bolt/db.go."""
import os

import pytest

from pilosa_amd.models import boltdb
from pilosa_amd.models.attrs import SQLiteAttrStore


def _attrs(n):
    out = {}
    for i in range(n):
        a = {"name": f"row{i}", "n": i * 7 - 3, "ok": i % 2 == 0}
        if i % 3 == 0:
            a["f"] = i / 4
        out[i * 3 + 1] = a
    return out


@pytest.mark.parametrize("n,inline", [(0, False), (3, True), (5, False), (500, False)])
def test_read_written_bolt_file(tmp_path, n, inline):
    want = _attrs(n)
    p = str(tmp_path / ".data")
    boltdb.write_bolt_attrs(p, want, inline=inline)
    assert boltdb.is_bolt(p)
    assert boltdb.read_bolt_attrs(p) == want


def test_meta_checksum_and_newest_meta(tmp_path):
    p = str(tmp_path / ".data")
    boltdb.write_bolt_attrs(p, _attrs(4))
    data = bytearray(open(p, "rb").read())
    # meta 1 (txid 3) corrupted: the reader falls back to meta 0 (txid 2)
    data[4096 + 16 + 40] ^= 0xFF
    open(p, "wb").write(bytes(data))
    assert boltdb.read_bolt_attrs(p) == _attrs(4)
    data[16 + 40] ^= 0xFF
    open(p, "wb").write(bytes(data))
    with pytest.raises(boltdb.BoltError):
        boltdb.read_bolt_attrs(p)


def test_attr_map_encoding_matches_reference_layout():
    """EncodeAttrs (attr.go:194): AttrMap{Attrs} with keys sorted, field 1
    repeated Attr{Key=1, Type=2, StringValue=3, IntValue=4, BoolValue=5}."""
    b = boltdb.encode_attr_map({"b": 5, "a": "x"})
    # Attr "a": key, type 1 (string), value "x"; then Attr "b": type 2 (int), 5
    assert b == bytes([0x0a, 0x08, 0x0a, 0x01, 0x61, 0x10, 0x01, 0x1a, 0x01, 0x78,
                       0x0a, 0x07, 0x0a, 0x01, 0x62, 0x10, 0x02, 0x20, 0x05])
    assert boltdb.decode_attr_map(b) == {"a": "x", "b": 5}


def test_store_converts_a_reference_data_file(tmp_path):
    want = _attrs(300)
    p = str(tmp_path / "idx" / ".data")
    os.makedirs(os.path.dirname(p))
    boltdb.write_bolt_attrs(p, want)
    s = SQLiteAttrStore(p).open()
    try:
        assert {i: s.attrs(i) for i in s.ids()} == want
        s.set_attrs(4, {"name": None, "extra": 1})
    finally:
        s.close()
    assert os.path.exists(p + ".bolt") and not boltdb.is_bolt(p)
    s = SQLiteAttrStore(p).open()   # reopened from SQLite, the write kept
    try:
        assert s.attrs(4) == {"n": 4, "ok": False, "extra": 1}
        assert s.attrs(1) == want[1]
    finally:
        s.close()
