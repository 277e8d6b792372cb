"""Translate store expectations ported from the reference's translate_test.go
(TranslateColumn/Row, the 1M-key Large cases, Reader with/without offset and
the 9012-byte TinyBuffer entry, PrimaryTranslateStore replication,
ReopenTheSameInstance), plus the log format's byte layout, torn tails and
the conversion of pre-log-format files."""
import os
import struct
import threading
import time

import pytest

from pilosa_amd.errors import ErrTranslateStoreReadOnly
from pilosa_amd.models.translate import T_COLUMN, T_ROW, TranslateFile, encode_entry


@pytest.fixture
def store(tmp_path):
    s = TranslateFile(str(tmp_path / "keys")).open()
    yield s
    s.close()


def test_translate_column(store):
    s = store
    assert s.translate_columns_to_uint64("IDX0", ["foo"]) == [1]
    assert s.translate_columns_to_uint64("IDX0", ["bar"]) == [2]
    assert s.translate_columns_to_uint64("IDX1", ["bar"]) == [1]
    assert s.translate_column_to_string("IDX0", 2) == "bar"
    assert s.translate_column_to_string("IDX0", 1000) == ""
    s.reopen()
    assert s.translate_columns_to_uint64("IDX1", ["bar"]) == [1]
    assert s.translate_column_to_string("IDX0", 2) == "bar"
    assert s.translate_columns_to_uint64("IDX0", ["baz"]) == [3]


def test_translate_row(store):
    s = store
    assert s.translate_rows_to_uint64("IDX0", "FIELD0", ["foo"]) == [1]
    assert s.translate_rows_to_uint64("IDX0", "FIELD0", ["bar"]) == [2]
    assert s.translate_rows_to_uint64("IDX1", "FIELD0", ["bar"]) == [1]
    assert s.translate_rows_to_uint64("IDX0", "FIELD1", ["bar"]) == [1]
    assert s.translate_row_to_string("IDX0", "FIELD0", 2) == "bar"
    assert s.translate_row_to_string("IDX0", "FIELD0", 1000) == ""
    s.reopen()
    assert s.translate_rows_to_uint64("IDX0", "FIELD1", ["bar"]) == [1]
    assert s.translate_row_to_string("IDX0", "FIELD0", 2) == "bar"
    assert s.translate_rows_to_uint64("IDX0", "FIELD0", ["baz"]) == [3]


@pytest.mark.parametrize("kind", ["column", "row"])
def test_translate_large(store, kind):
    s = store
    n = 1_000_000
    for i in range(0, n, 1000):
        keys = [str(i + j + 1) for j in range(1000)]
        ids = (s.translate_columns_to_uint64("IDX0", keys) if kind == "column"
               else s.translate_rows_to_uint64("IDX0", "FIELD0", keys))
        assert ids == list(range(i + 1, i + 1001))

    def check():
        ids = list(range(1, n + 1))
        got = (s.translate_columns_to_strings("IDX0", ids) if kind == "column"
               else s.translate_rows_to_strings("IDX0", "FIELD0", ids))
        assert got == [str(i) for i in ids]
        # and key -> id through the hash index
        probe = [str(i) for i in range(1, n + 1, 997)]
        assert (s.translate_columns_to_uint64("IDX0", probe) if kind == "column"
                else s.translate_rows_to_uint64("IDX0", "FIELD0", probe)) == [int(k) for k in probe]
    check()
    s.reopen()
    check()


def test_reader_entries(store):
    s = store
    s.translate_columns_to_uint64("IDX0", ["foo"])
    s.translate_rows_to_uint64("IDX0", "FIELD0", ["bar", "baz"])
    e = s.entries(0)
    # first entry: Length 13 + uvarint(13) = 14 bytes
    assert e[0] == (T_COLUMN, "IDX0", "", [1], [b"foo"], 14)
    assert e[1] == (T_ROW, "IDX0", "FIELD0", [1, 2], [b"bar", b"baz"], 25)
    s.translate_columns_to_uint64("IDX0", ["xyz"])
    assert s.entries(0)[2] == (T_COLUMN, "IDX0", "", [2], [b"xyz"], 14)
    # WithOffset: start after the first entry
    assert s.entries(14)[0][:5] == (T_ROW, "IDX0", "FIELD0", [1, 2], [b"bar", b"baz"])
    raw = s.read_from(0)
    assert raw[:14] == b"\x0d\x01\x04IDX0\x00\x01\x01\x03foo"
    assert raw[:14] == encode_entry(T_COLUMN, "IDX0", "", [1], ["foo"])


def test_reader_tiny_buffer_entry(store):
    keys = [f"KEY{i}" for i in range(1024)]
    store.translate_columns_to_uint64("IDX0", keys)
    (t, index, field, ids, got, length), = store.entries(0)
    assert (t, index, ids, [k.decode() for k in got]) == (T_COLUMN, "IDX0", list(range(1, 1025)), keys)
    assert length == 9012 + 2   # Length 9012 plus its 2-byte uvarint


def test_reopen_same_instance(store):
    s = store
    assert s.translate_columns_to_uint64("IDX0", ["foo"]) == [1]
    assert s.translate_columns_to_uint64("IDX0", ["bar"]) == [2]
    assert s.translate_columns_to_uint64("IDX1", ["bar"]) == [1]
    assert (s.translate_column_to_string("IDX0", 2), s.translate_column_to_string("IDX0", 1)) == ("bar", "foo")
    assert s.translate_column_to_string("IDX0", 1000) == ""
    s.close()
    s.open()
    assert s.translate_columns_to_uint64("IDX1", ["bar"]) == [1]
    assert s.translate_column_to_string("IDX0", 2) == "bar"
    assert s.translate_columns_to_uint64("IDX0", ["baz"]) == [3]


def test_batch_dedup_and_mixed(store):
    s = store
    assert s.translate_columns_to_uint64("i", ["a", "b", "a", "c", "b"]) == [1, 2, 1, 3, 2]
    assert s.translate_columns_to_uint64("i", ["c", "d", "a"]) == [3, 4, 1]
    assert len(s.entries(0)) == 2 and s.entries(0)[1][3] == [4]   # only the new key was logged
    assert s.column_key_id("i", "d") == 4 and s.column_key_id("i", "zz") is None


def test_primary_translate_store_replication(tmp_path):
    primary = TranslateFile(str(tmp_path / "p")).open()
    replica = TranslateFile(str(tmp_path / "r"), read_only=True).open()
    stop = threading.Event()

    def tail():   # what the server's translate-replica loop does over HTTP
        while not stop.is_set():
            data = primary.read_from(replica.size)
            if data:
                replica.apply_log(data)
            time.sleep(0.01)
    t = threading.Thread(target=tail, daemon=True)
    t.start()

    def until(fn, timeout=2.0):
        deadline = time.time() + timeout
        while time.time() < deadline:
            if fn():
                return True
            time.sleep(0.01)
        return fn()
    try:
        primary.translate_columns_to_uint64("IDX0", ["foo"])
        primary.translate_rows_to_uint64("IDX0", "FIELD0", ["bar", "baz"])
        assert until(lambda: (replica.translate_column_to_string("IDX0", 1),
                              replica.translate_row_to_string("IDX0", "FIELD0", 1),
                              replica.translate_row_to_string("IDX0", "FIELD0", 2)) == ("foo", "bar", "baz"))
        primary.reopen()
        primary.translate_columns_to_uint64("IDX0", ["baz"])
        assert until(lambda: replica.translate_column_to_string("IDX0", 2) == "baz")
        replica.reopen()
        primary.translate_columns_to_uint64("IDX0", ["foobar"])
        assert until(lambda: replica.translate_column_to_string("IDX0", 3) == "foobar")
        # the replica's log is byte-identical to the primary's
        assert until(lambda: replica.read_from(0) == primary.read_from(0))
        # a read-only store refuses new keys unless it can forward them
        with pytest.raises(type(ErrTranslateStoreReadOnly)):
            replica.translate_columns_to_uint64("IDX0", ["new"])
        replica.forward = lambda index, field, keys: primary.translate_columns_to_uint64(index, keys)
        assert replica.translate_columns_to_uint64("IDX0", ["foo", "new"]) == [1, 4]
    finally:
        stop.set()
        t.join(2)
        primary.close()
        replica.close()


def test_apply_log_keeps_partial_tail(tmp_path):
    a = TranslateFile(str(tmp_path / "a")).open()
    b = TranslateFile(str(tmp_path / "b"), read_only=True).open()
    a.translate_columns_to_uint64("i", ["x", "y"])
    a.translate_columns_to_uint64("i", ["z"])
    data = a.read_from(0)
    cut = len(encode_entry(T_COLUMN, "i", "", [1, 2], ["x", "y"])) + 3
    assert b.apply_log(data[:cut]) == cut - 3
    assert b.apply_log(data[cut - 3:]) == len(data) - cut + 3
    assert b.translate_columns_to_strings("i", [1, 2, 3]) == ["x", "y", "z"]
    a.close()
    b.close()


def test_torn_tail_truncated_on_open(tmp_path):
    p = str(tmp_path / "k")
    s = TranslateFile(p).open()
    s.translate_columns_to_uint64("i", ["a"])
    good = os.path.getsize(p)
    s.close()
    with open(p, "ab") as fh:
        fh.write(b"\x20\x01\x01i")   # an entry that claims 32 bytes but stops short
    s = TranslateFile(p).open()
    assert os.path.getsize(p) == good and s.translate_columns_to_uint64("i", ["a", "b"]) == [1, 2]
    s.close()


def test_legacy_file_converted(tmp_path):
    p = str(tmp_path / "legacy")

    def rec(t, index, field, id_, key):
        ib, fb, kb = index.encode(), field.encode(), key.encode()
        return (struct.pack("<BH", t, len(ib)) + ib + struct.pack("<H", len(fb)) + fb +
                struct.pack("<QI", id_, len(kb)) + kb)
    with open(p, "wb") as fh:
        fh.write(rec(1, "i", "", 1, "a") + rec(1, "i", "", 2, "b") + rec(2, "i", "f", 1, "r"))
    s = TranslateFile(p).open()
    assert s.translate_columns_to_strings("i", [1, 2]) == ["a", "b"]
    assert s.translate_row_to_string("i", "f", 1) == "r"
    assert [e[:5] for e in s.entries(0)] == [(1, "i", "", [1, 2], [b"a", b"b"]), (2, "i", "f", [1], [b"r"])]
    assert s.translate_columns_to_uint64("i", ["c"]) == [3]
    s.close()


def test_in_memory_store():
    s = TranslateFile(None).open()
    assert s.translate_rows_to_uint64("i", "f", ["a", "b"]) == [1, 2]
    assert s.read_from(0) == encode_entry(T_ROW, "i", "f", [1, 2], ["a", "b"])
    s.close()


def test_closed_store_raises_instead_of_reading_unmapped_log(tmp_path):
    """A translate/keys_of racing a close() gets an error, never a read
    through the unmapped log (ADVICE r02 translate.cpp:187)."""
    from pilosa_amd import _translate
    s = _translate.Store(str(tmp_path / "keys"))
    s.open()
    ids = s.translate(_translate.T_COLUMN, "i", "", ["a", "b"], True)
    assert list(ids) == [1, 2]
    s.close()
    for call in (lambda: s.translate(_translate.T_COLUMN, "i", "", ["a"], False),
                 lambda: s.keys_of(_translate.T_COLUMN, "i", "", [1]),
                 lambda: s.read_from(0), lambda: s.entries(0)):
        with pytest.raises(RuntimeError):
            call()
    s.open()
    assert list(s.keys_of(_translate.T_COLUMN, "i", "", [1, 2])) == ["a", "b"]
    s.close()


def test_reopen_races_concurrent_readers(tmp_path):
    """close/reopen swaps the native store under the lock; readers running
    concurrently (the /internal/translate/data handler, a replica's tail
    loop) see a closed store as empty and never a None store."""
    primary = TranslateFile(str(tmp_path / "p")).open()
    replica = TranslateFile(str(tmp_path / "r"), read_only=True).open()
    primary.translate_columns_to_uint64("i", [f"k{j}" for j in range(64)])
    stop = threading.Event()
    errors = []

    def reader():
        try:
            while not stop.is_set():
                data = primary.read_from(replica.size)
                if data:
                    replica.apply_log(data)
                primary.entries(0)
                _ = primary.size
                replica.read_from(replica.size)
        except Exception as e:  # pragma: no cover - the failure being tested
            errors.append(e)
    ths = [threading.Thread(target=reader, daemon=True) for _ in range(3)]
    for t in ths:
        t.start()
    try:
        for _ in range(10_000):
            primary.reopen()
            replica.reopen()
    finally:
        stop.set()
        for t in ths:
            t.join(5)
    assert not errors, errors[:3]
    assert primary.translate_column_to_string("i", 64) == "k63"
    closed = TranslateFile(str(tmp_path / "c")).open()
    closed.close()
    assert closed.read_from(0) == b"" and closed.apply_log(b"xx") == 0
    assert closed.entries() == [] and closed.size == 0
    primary.close()
    replica.close()
