"""Row/column attribute stores (reference: attr.go, boltdb/attrstore.go).

Attributes are string/int/bool/float key-values per id.  Setting a key to
``None`` deletes it (boltdb/attrstore.go:290-333).  Blocks of 100 ids carry
checksums for anti-entropy diffs (attrBlockSize=100).

Backed by SQLite (stdlib; one file per store), one JSON document per id.
A ``.data`` file written by a reference node (BoltDB, boltdb/attrstore.go)
is converted on open (models/boltdb.py), so its attributes carry over.
"""
from __future__ import annotations

import hashlib
import json
import os
import sqlite3
import threading
from typing import Dict, Iterable, List, Optional, Tuple

ATTR_BLOCK_SIZE = 100


def _validate(attrs: dict):
    for k, v in attrs.items():
        if v is None or isinstance(v, (str, bool, int, float)):
            continue
        raise ValueError(f"invalid attr type: {type(v).__name__}")


class MemAttrStore:
    """In-memory store (tests; reference mock/inmem)."""

    def __init__(self):
        self._d: Dict[int, dict] = {}
        self.mu = threading.Lock()

    def open(self):
        return self

    def close(self):
        pass

    def attrs(self, id: int) -> Optional[dict]:
        with self.mu:
            a = self._d.get(int(id))
            return dict(a) if a else None

    def set_attrs(self, id: int, attrs: dict):
        _validate(attrs)
        with self.mu:
            cur = dict(self._d.get(int(id), {}))
            for k, v in attrs.items():
                if v is None:
                    cur.pop(k, None)
                else:
                    cur[k] = v
            if cur:
                self._d[int(id)] = cur
            else:
                self._d.pop(int(id), None)

    def set_bulk_attrs(self, m: Dict[int, dict]):
        for id in sorted(m):
            self.set_attrs(id, m[id])

    def ids(self) -> List[int]:
        with self.mu:
            return sorted(self._d)

    def blocks(self) -> List[Tuple[int, bytes]]:
        return _blocks(self.ids(), self.attrs)

    def block_data(self, block: int) -> Dict[int, dict]:
        lo, hi = block * ATTR_BLOCK_SIZE, (block + 1) * ATTR_BLOCK_SIZE
        return {i: self.attrs(i) for i in self.ids() if lo <= i < hi}


def _blocks(ids: Iterable[int], get) -> List[Tuple[int, bytes]]:
    out: List[Tuple[int, bytes]] = []
    cur_block, h = None, None
    for i in ids:
        b = i // ATTR_BLOCK_SIZE
        if b != cur_block:
            if h is not None:
                out.append((cur_block, h.digest()))
            cur_block, h = b, hashlib.sha1()
        h.update(i.to_bytes(8, "big"))
        h.update(json.dumps(get(i), sort_keys=True).encode())
    if h is not None:
        out.append((cur_block, h.digest()))
    return out


class SQLiteAttrStore(MemAttrStore):
    """Durable attribute store (one SQLite db per field/index ``.data`` file)."""

    def __init__(self, path: str):
        super().__init__()
        self.path = path
        self._db: Optional[sqlite3.Connection] = None

    def open(self):
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        migrated = self._migrate_bolt()
        self._db = sqlite3.connect(self.path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("CREATE TABLE IF NOT EXISTS attrs (id INTEGER PRIMARY KEY, doc TEXT NOT NULL)")
        if migrated:
            self._db.execute("BEGIN")
            self._db.executemany("INSERT OR REPLACE INTO attrs (id, doc) VALUES (?, ?)",
                                 [(i, json.dumps(a)) for i, a in sorted(migrated.items())])
            self._db.execute("COMMIT")
        with self.mu:
            for id, doc in self._db.execute("SELECT id, doc FROM attrs"):
                self._d[int(id)] = json.loads(doc)
        return self

    def _migrate_bolt(self) -> Optional[Dict[int, dict]]:
        """A reference node's ``.data`` file is a BoltDB attribute store
        (boltdb/attrstore.go): read it once (models/boltdb.py), keep it as
        ``.data.bolt`` and let this store take its place with its contents."""
        from pilosa_amd.models import boltdb
        if not os.path.exists(self.path) or not boltdb.is_bolt(self.path):
            return None
        data = boltdb.read_bolt_attrs(self.path)
        os.replace(self.path, self.path + ".bolt")
        return data

    def close(self):
        if self._db is not None:
            self._db.close()
            self._db = None

    def set_attrs(self, id: int, attrs: dict):
        super().set_attrs(id, attrs)
        self._persist([int(id)])

    def set_bulk_attrs(self, m: Dict[int, dict]):
        for id in sorted(m):
            MemAttrStore.set_attrs(self, id, m[id])
        self._persist(sorted(int(i) for i in m))

    def _persist(self, ids: List[int]):
        if self._db is None:
            return
        with self.mu:
            rows = [(i, json.dumps(self._d[i])) for i in ids if i in self._d]
            gone = [(i,) for i in ids if i not in self._d]
        self._db.execute("BEGIN")
        if rows:
            self._db.executemany("INSERT OR REPLACE INTO attrs (id, doc) VALUES (?, ?)", rows)
        if gone:
            self._db.executemany("DELETE FROM attrs WHERE id = ?", gone)
        self._db.execute("COMMIT")
