"""String key <-> uint64 id translation (reference: translate.go).

IDs are assigned in order starting at 1, per index for column keys and per
(index, field) for row keys (translate.go:496-585, :675).  Storage is the
native store in ``native/translate.cpp``: the reference's on-disk log of
varint-framed ``LogEntry`` records (translate.go:716-866), memory-mapped,
with a Robin-Hood key index that points into the mapping (translate.go:
880-1037), so a Pilosa data directory's ``.keys`` file opens as is and the
replication stream (``/internal/translate/data``) is byte-compatible.

Replicas are read-only and tail the primary's log from an offset
(translate.go:423-474 ``replicate``) via :meth:`TranslateFile.read_from` /
:meth:`apply_log`; keys they do not know yet are forwarded to the primary.

Files written by earlier pilosa_amd builds (fixed-width little-endian
records) are converted to the log format on open.
"""
from __future__ import annotations

import os
import struct
import threading
from typing import Iterator, List, Optional, Sequence, Tuple

from pilosa_amd.errors import ErrTranslateStoreReadOnly

T_COLUMN, T_ROW = 1, 2


def _native():
    try:
        from pilosa_amd import _translate
    except ImportError as e:  # pragma: no cover - build() makes it
        raise ImportError("pilosa_amd._translate is not built; run __graft_entry__.build()") from e
    return _translate


# ---------------------------------------------------------------- LogEntry codec
def _uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def encode_entry(t: int, index: str, field: str, ids: Sequence[int], keys: Sequence[str]) -> bytes:
    """One LogEntry exactly as LogEntry.WriteTo (translate.go:795-850)."""
    ib, fb = index.encode(), (field.encode() if t == T_ROW else b"")
    body = bytearray([t]) + _uvarint(len(ib)) + ib + _uvarint(len(fb)) + fb + _uvarint(len(ids))
    for i, k in zip(ids, keys):
        kb = k.encode() if isinstance(k, str) else bytes(k)
        body += _uvarint(int(i)) + _uvarint(len(kb)) + kb
    return _uvarint(len(body)) + bytes(body)


# ---------------------------------------------------------------- legacy format
def _legacy_records(data: bytes) -> Iterator[Tuple[int, str, str, int, str]]:
    off, n = 0, len(data)
    while off + 3 <= n:
        t, il = struct.unpack_from("<BH", data, off)
        p = off + 3
        if t not in (T_COLUMN, T_ROW) or p + il + 2 > n:
            return
        index = data[p:p + il].decode()
        p += il
        (fl,) = struct.unpack_from("<H", data, p)
        p += 2
        if p + fl + 12 > n:
            return
        field = data[p:p + fl].decode()
        p += fl
        id_, kl = struct.unpack_from("<QI", data, p)
        p += 12
        if p + kl > n:
            return
        yield t, index, field, id_, data[p:p + kl].decode()
        off = p + kl


def _migrate_legacy(path: str) -> bool:
    """Rewrite a pre-log-format file in place; True if one was converted.

    The log format can never start with byte 1 or 2 (the smallest entry is 4
    bytes long), the legacy format always does."""
    if not os.path.exists(path) or os.path.getsize(path) == 0:
        return False
    with open(path, "rb") as fh:
        data = fh.read()
    if data[0] not in (T_COLUMN, T_ROW):
        return False
    out, run = bytearray(), None
    for t, index, field, id_, key in _legacy_records(data):
        k = (t, index, field)
        if run is None or run[0] != k:
            if run is not None:
                out += encode_entry(*run[0], run[1], run[2])
            run = (k, [], [])
        run[1].append(id_)
        run[2].append(key)
    if run is not None:
        out += encode_entry(*run[0], run[1], run[2])
    tmp = path + ".migrate"
    with open(tmp, "wb") as fh:
        fh.write(out)
        fh.flush()
        os.fsync(fh.fileno())
    os.replace(tmp, path)
    return True


class TranslateFile:
    def __init__(self, path: Optional[str] = None, read_only: bool = False, map_size: int = 0):
        self.path = path
        self._read_only = read_only
        self.map_size = map_size
        self.mu = threading.RLock()
        self._s = None
        # read-only replicas: (index, field or None, keys) -> ids resolved by
        # the primary (http translate proxy, reference http/translator.go)
        self.forward = None

    def open(self):
        with self.mu:
            if self.path:
                os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
                _migrate_legacy(self.path)
            self._s = _native().Store(self.path or "", self._read_only, int(self.map_size))
            self._s.open()
        return self

    def close(self):
        with self.mu:
            if self._s is not None:
                self._s.close()
                self._s = None

    def reopen(self):
        self.close()
        return self.open()

    @property
    def read_only(self) -> bool:
        return self._read_only

    @read_only.setter
    def read_only(self, v: bool):
        with self.mu:
            self._read_only = bool(v)
            if self._s is not None:
                self._s.read_only = self._read_only

    # Every access to the native store holds ``mu``: ``close``/``reopen`` swap
    # ``_s`` under it, and a reader that fetched ``_s`` before a close would
    # otherwise call into a closed (or None) store (translate.go:1039-1124
    # holds the store's RWMutex the same way).
    def _live(self):
        s = self._s
        if s is None:
            raise RuntimeError("translate store is closed")
        return s

    @property
    def size(self) -> int:
        with self.mu:
            return self._s.size() if self._s is not None else 0

    # ------------------------------------------------------------ replication
    def apply_log(self, data: bytes, persist: bool = True) -> int:
        """Append + index whole log entries (replica tailing); returns the
        bytes consumed (a torn trailing entry is left for the next read).
        A closed store consumes nothing."""
        data = bytes(data)
        with self.mu:
            return self._s.apply_log(data) if self._s is not None else 0

    def read_from(self, offset: int) -> bytes:
        """Log bytes from ``offset`` (served at /internal/translate/data);
        empty while the store is closed (the replica retries)."""
        with self.mu:
            return self._s.read_from(int(offset)) if self._s is not None else b""

    def entries(self, offset: int = 0) -> List[tuple]:
        """[(type, index, field, ids, keys, encoded_length)] from ``offset``."""
        with self.mu:
            return self._s.entries(int(offset)) if self._s is not None else []

    # ------------------------------------------------------------ generic
    def _translate(self, t: int, index: str, field: str, keys: Sequence[str]) -> List[int]:
        keys = [k if isinstance(k, str) else str(k) for k in keys]
        with self.mu:
            ids = self._live().translate(t, index, field, keys, not self._read_only)
        if self._read_only and 0 in ids:
            if self.forward is None:
                raise ErrTranslateStoreReadOnly
            missing = sorted({k for k, i in zip(keys, ids) if i == 0})
            got = dict(zip(missing, (int(x) for x in self.forward(index, field if t == T_ROW else None, missing))))
            ids = [i or got[k] for k, i in zip(keys, ids)]
        return list(ids)

    def _keys_of(self, t: int, index: str, field: str, ids: Sequence[int]) -> List[str]:
        ids = [int(i) for i in ids]
        with self.mu:
            return self._live().keys_of(t, index, field, ids)

    def _key_id(self, t: int, index: str, field: str, key: str) -> Optional[int]:
        with self.mu:
            return self._live().translate(t, index, field, [key], False)[0] or None

    # ------------------------------------------------------------ columns
    def translate_columns_to_uint64(self, index: str, keys: Sequence[str]) -> List[int]:
        return self._translate(T_COLUMN, index, "", keys)

    def translate_column_to_string(self, index: str, id: int) -> str:
        """The key for ``id``; "" if none (TranslateColumnToString)."""
        return self._keys_of(T_COLUMN, index, "", [id])[0]

    def translate_columns_to_strings(self, index: str, ids: Sequence[int]) -> List[str]:
        return self._keys_of(T_COLUMN, index, "", ids)

    def column_key_id(self, index: str, key: str) -> Optional[int]:
        return self._key_id(T_COLUMN, index, "", key)

    # ------------------------------------------------------------ rows
    def translate_rows_to_uint64(self, index: str, field: str, keys: Sequence[str]) -> List[int]:
        return self._translate(T_ROW, index, field, keys)

    def translate_row_to_string(self, index: str, field: str, id: int) -> str:
        return self._keys_of(T_ROW, index, field, [id])[0]

    def translate_rows_to_strings(self, index: str, field: str, ids: Sequence[int]) -> List[str]:
        return self._keys_of(T_ROW, index, field, ids)

    def row_key_id(self, index: str, field: str, key: str) -> Optional[int]:
        return self._key_id(T_ROW, index, field, key)
