"""String key <-> uint64 id translation (reference: translate.go).

IDs are assigned in order starting at 1, per index for column keys and per
(index, field) for row keys (translate.go:496-585, :675).  The store is an
append-only log replayed on open; replicas are read-only and tail the
primary's log from an offset (translate.go:423-474 ``replicate``) via
:meth:`TranslateFile.read_from` / :meth:`apply_log`.

Log record (little endian): u8 type (1 column, 2 row) | u16 len(index) |
index | u16 len(field) | field | u64 id | u32 len(key) | key.
"""
from __future__ import annotations

import os
import struct
import threading
from typing import Dict, List, Optional, Sequence, Tuple

from pilosa_amd.errors import ErrTranslateStoreReadOnly, ErrTranslatingKeyNotFound

T_COLUMN, T_ROW = 1, 2


def _encode(t: int, index: str, field: str, id: int, key: str) -> bytes:
    ib, fb, kb = index.encode(), field.encode(), key.encode()
    return (struct.pack("<BH", t, len(ib)) + ib + struct.pack("<H", len(fb)) + fb +
            struct.pack("<QI", id, len(kb)) + kb)


def _decode_all(data: bytes, off: int = 0):
    n = len(data)
    while off < n:
        if off + 3 > n:
            break
        t, il = struct.unpack_from("<BH", data, off)
        p = off + 3
        if p + il + 2 > n:
            break
        index = data[p:p + il].decode()
        p += il
        (fl,) = struct.unpack_from("<H", data, p)
        p += 2
        if p + fl + 12 > n:
            break
        field = data[p:p + fl].decode()
        p += fl
        id, kl = struct.unpack_from("<QI", data, p)
        p += 12
        if p + kl > n:
            break
        key = data[p:p + kl].decode()
        p += kl
        yield p, t, index, field, id, key
        off = p


class TranslateFile:
    def __init__(self, path: Optional[str] = None, read_only: bool = False):
        self.path = path
        self.read_only = read_only
        self.mu = threading.RLock()
        self._cols: Dict[str, Dict[str, int]] = {}
        self._col_ids: Dict[str, Dict[int, str]] = {}
        self._rows: Dict[Tuple[str, str], Dict[str, int]] = {}
        self._row_ids: Dict[Tuple[str, str], Dict[int, str]] = {}
        self._log: List[bytes] = []  # in-memory copy when no path
        self._fh = None
        self.size = 0
        self._next: Dict[Tuple[str, str], int] = {}  # (index, field or "") -> next id
        # read-only replicas: (index, field or None, keys) -> ids resolved by
        # the primary (http translate proxy, reference http/translator.go)
        self.forward = None

    def open(self):
        with self.mu:
            if self.path:
                os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
                if os.path.exists(self.path):
                    with open(self.path, "rb") as fh:
                        data = fh.read()
                    end = self.apply_log(data, persist=False)
                    if end != len(data):  # truncate a torn tail
                        with open(self.path, "r+b") as fh:
                            fh.truncate(end)
                self._fh = open(self.path, "ab", buffering=0)
        return self

    def close(self):
        with self.mu:
            if self._fh is not None:
                self._fh.close()
                self._fh = None

    # ------------------------------------------------------------ internals
    def _apply(self, t, index, field, id, key):
        if t == T_COLUMN:
            self._cols.setdefault(index, {})[key] = id
            self._col_ids.setdefault(index, {})[id] = key
            nk = (index, "")
        else:
            self._rows.setdefault((index, field), {})[key] = id
            self._row_ids.setdefault((index, field), {})[id] = key
            nk = (index, field)
        if id >= self._next.get(nk, 1):
            self._next[nk] = id + 1

    def _append(self, rec: bytes):
        if self._fh is not None:
            self._fh.write(rec)
        else:
            self._log.append(rec)
        self.size += len(rec)

    def apply_log(self, data: bytes, persist: bool = True) -> int:
        """Apply log records (replica tailing); returns bytes consumed."""
        end = 0
        with self.mu:
            start = 0
            for p, t, index, field, id, key in _decode_all(data):
                self._apply(t, index, field, id, key)
                if persist:
                    self._append(data[start:p])
                else:
                    self.size += p - start
                start = p
                end = p
        return end

    def read_from(self, offset: int) -> bytes:
        """Log bytes from ``offset`` (served at /internal/translate/data)."""
        with self.mu:
            if self.path:
                if self._fh is not None:
                    self._fh.flush()
                with open(self.path, "rb") as fh:
                    fh.seek(offset)
                    return fh.read()
            return b"".join(self._log)[offset:]

    def _next_id(self, index: str, field: str = "") -> int:
        return self._next.get((index, field), 1)

    def _forward(self, index: str, field: Optional[str], keys: List[str]) -> List[int]:
        if self.forward is None:
            raise ErrTranslateStoreReadOnly
        ids = self.forward(index, field, keys)
        with self.mu:
            for k, i in zip(keys, ids):  # visible now; the replicated log entry follows
                self._apply(T_ROW if field else T_COLUMN, index, field or "", int(i), k)
        return [int(i) for i in ids]

    # ------------------------------------------------------------ columns
    def translate_columns_to_uint64(self, index: str, keys: Sequence[str]) -> List[int]:
        out = []
        keys = list(keys)
        if self.read_only:
            with self.mu:
                cm = self._cols.get(index, {})
                missing = [k for k in keys if k not in cm]
            if missing:
                self._forward(index, None, sorted(set(missing)))
        with self.mu:
            cm = self._cols.setdefault(index, {})
            for k in keys:
                id = cm.get(k)
                if id is None:
                    if self.read_only:
                        raise ErrTranslateStoreReadOnly
                    id = self._next_id(index)
                    self._apply(T_COLUMN, index, "", id, k)
                    self._append(_encode(T_COLUMN, index, "", id, k))
                out.append(id)
        return out

    def translate_column_to_string(self, index: str, id: int) -> str:
        with self.mu:
            k = self._col_ids.get(index, {}).get(int(id))
        if k is None:
            raise ErrTranslatingKeyNotFound
        return k

    def column_key_id(self, index: str, key: str) -> Optional[int]:
        with self.mu:
            return self._cols.get(index, {}).get(key)

    # ------------------------------------------------------------ rows
    def translate_rows_to_uint64(self, index: str, field: str, keys: Sequence[str]) -> List[int]:
        out = []
        keys = list(keys)
        if self.read_only:
            with self.mu:
                rm = self._rows.get((index, field), {})
                missing = [k for k in keys if k not in rm]
            if missing:
                self._forward(index, field, sorted(set(missing)))
        with self.mu:
            rm = self._rows.setdefault((index, field), {})
            for k in keys:
                id = rm.get(k)
                if id is None:
                    if self.read_only:
                        raise ErrTranslateStoreReadOnly
                    id = self._next_id(index, field)
                    self._apply(T_ROW, index, field, id, k)
                    self._append(_encode(T_ROW, index, field, id, k))
                out.append(id)
        return out

    def translate_row_to_string(self, index: str, field: str, id: int) -> str:
        with self.mu:
            k = self._row_ids.get((index, field), {}).get(int(id))
        if k is None:
            raise ErrTranslatingKeyNotFound
        return k

    def row_key_id(self, index: str, field: str, key: str) -> Optional[int]:
        with self.mu:
            return self._rows.get((index, field), {}).get(key)
