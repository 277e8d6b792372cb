"""Read (and, for fixtures, write) the BoltDB attribute files of a Pilosa data
directory (reference: boltdb/attrstore.go:82-423 over github.com/boltdb/bolt).

A reference node keeps each index's column attributes and each field's row
attributes in a ``.data`` file: a BoltDB B+tree file with one bucket
``attrs`` mapping the id (8 bytes, big endian, ``u64tob``) to an
``internal.AttrMap`` protobuf (``pilosa.EncodeAttrs``, attr.go:194).  This
build stores attributes in SQLite (models/attrs.py); a ``.data`` file that is
a BoltDB file is read once on open and converted, so an existing Pilosa data
directory opens with its attributes (the file is kept as ``.data.bolt``).

BoltDB layout (bolt/page.go, bolt/db.go, bolt/bucket.go):
* every page starts with ``id u64, flags u16, count u16, overflow u32``;
  a page spans ``1 + overflow`` pages of the file's page size;
* pages 0 and 1 are meta pages: ``magic 0xED0CDAED, version 2, pageSize,
  flags, root bucket {root pgid, sequence}, freelist pgid, pgid, txid,
  checksum`` (FNV-64a of the fields before it); the valid one with the
  higher txid is current;
* a branch page holds ``count`` elements ``{pos u32, ksize u32, pgid u64}``,
  a leaf page ``{flags u32, pos u32, ksize u32, vsize u32}``; ``pos`` is the
  key's offset from the element, the value follows the key;
* a leaf element with flag 0x01 is a nested bucket whose value starts with
  ``{root pgid u64, sequence u64}``; root 0 = an inline bucket whose one leaf
  page follows that header inside the value.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Optional, Tuple

MAGIC = 0xED0CDAED
VERSION = 2
BRANCH, LEAF, META, FREELIST = 0x01, 0x02, 0x04, 0x10
BUCKET_LEAF_FLAG = 0x01
PAGE_HEADER = struct.Struct("<QHHI")          # id, flags, count, overflow
META_FMT = struct.Struct("<IIIIQQQQQQ")       # magic .. txid, then checksum
BRANCH_ELEM = struct.Struct("<IIQ")
LEAF_ELEM = struct.Struct("<IIII")
BUCKET_HDR = struct.Struct("<QQ")


class BoltError(ValueError):
    pass


def _fnv64a(data: bytes) -> int:
    h = 0xcbf29ce484222325
    for b in data:
        h ^= b
        h = (h * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def is_bolt(path: str) -> bool:
    """Is ``path`` a BoltDB file (meta page magic)?"""
    try:
        with open(path, "rb") as fh:
            head = fh.read(PAGE_HEADER.size + 8)
    except OSError:
        return False
    if len(head) < PAGE_HEADER.size + 8:
        return False
    magic, version = struct.unpack_from("<II", head, PAGE_HEADER.size)
    return magic == MAGIC and version == VERSION


class _File:
    def __init__(self, data: bytes):
        self.data = data
        metas = []
        for i in range(2):
            m = self._meta_at(i)
            if m is not None:
                metas.append(m)
        if not metas:
            raise BoltError("no valid meta page")
        self.meta = max(metas, key=lambda m: m["txid"])

    def _meta_at(self, i: int) -> Optional[dict]:
        # page 0 tells the page size; page 1 sits one page further
        ps = 4096
        if i == 1:
            m0 = self._meta_raw(0, 4096)
            ps = m0["page_size"] if m0 is not None else 4096
        m = self._meta_raw(i * ps if i else 0, ps)
        return m

    def _meta_raw(self, off: int, ps: int) -> Optional[dict]:
        o = off + PAGE_HEADER.size
        if o + META_FMT.size > len(self.data):
            return None
        (magic, version, page_size, flags, root, seq, freelist, pgid, txid, checksum) = \
            META_FMT.unpack_from(self.data, o)
        if magic != MAGIC or version != VERSION:
            return None
        if _fnv64a(self.data[o:o + META_FMT.size - 8]) != checksum:
            return None
        return {"page_size": page_size, "root": root, "freelist": freelist, "pgid": pgid, "txid": txid}

    def page(self, pgid: int) -> Tuple[int, int, int]:
        """(offset, flags, count) of page ``pgid``."""
        ps = self.meta["page_size"]
        off = pgid * ps
        if off + PAGE_HEADER.size > len(self.data):
            raise BoltError(f"page {pgid} beyond the file")
        _, flags, count, _ = PAGE_HEADER.unpack_from(self.data, off)
        return off, flags, count

    def leaf_items(self, buf: bytes, off: int, count: int) -> Iterator[Tuple[int, bytes, bytes]]:
        base = off + PAGE_HEADER.size
        for k in range(count):
            e = base + k * LEAF_ELEM.size
            flags, pos, ksize, vsize = LEAF_ELEM.unpack_from(buf, e)
            ks = e + pos
            yield flags, bytes(buf[ks:ks + ksize]), bytes(buf[ks + ksize:ks + ksize + vsize])

    def walk(self, pgid: int, depth: int = 0) -> Iterator[Tuple[int, bytes, bytes]]:
        """Every (flags, key, value) of the B+tree rooted at ``pgid``, in key order."""
        if depth > 64:
            raise BoltError("B+tree too deep (corrupt file)")
        off, flags, count = self.page(pgid)
        if flags & LEAF:
            yield from self.leaf_items(self.data, off, count)
        elif flags & BRANCH:
            base = off + PAGE_HEADER.size
            for k in range(count):
                _, _, child = BRANCH_ELEM.unpack_from(self.data, base + k * BRANCH_ELEM.size)
                yield from self.walk(child, depth + 1)
        else:
            raise BoltError(f"page {pgid}: not a branch or leaf page (flags {flags:#x})")

    def bucket(self, value: bytes) -> Iterator[Tuple[int, bytes, bytes]]:
        """The items of a nested bucket given its leaf value."""
        root, _ = BUCKET_HDR.unpack_from(value, 0)
        if root == 0:   # inline bucket: its leaf page follows the header
            _, flags, count, _ = PAGE_HEADER.unpack_from(value, BUCKET_HDR.size)
            if not flags & LEAF:
                raise BoltError("inline bucket without a leaf page")
            yield from self.leaf_items(value, BUCKET_HDR.size, count)
        else:
            yield from self.walk(root)


def decode_attr_map(data: bytes) -> dict:
    """internal.AttrMap protobuf -> {key: value} (attr.go DecodeAttrs)."""
    from pilosa_amd.server.encoding import attrs_from_pb
    from pilosa_amd.wire import pb
    m = pb.AttrMap()
    m.ParseFromString(data)
    return attrs_from_pb(m.Attrs)


def encode_attr_map(attrs: dict) -> bytes:
    """{key: value} -> internal.AttrMap protobuf, keys sorted (attr.go EncodeAttrs)."""
    from pilosa_amd.server.encoding import attrs_to_pb
    from pilosa_amd.wire import pb
    return pb.AttrMap(Attrs=attrs_to_pb(attrs)).SerializeToString()


def read_bolt_attrs(path: str) -> Dict[int, dict]:
    """{id: attrs} of the ``attrs`` bucket of a BoltDB attribute file."""
    with open(path, "rb") as fh:
        f = _File(fh.read())
    out: Dict[int, dict] = {}
    for flags, key, value in f.walk(f.meta["root"]):
        if key == b"attrs" and flags & BUCKET_LEAF_FLAG:
            for _, k, v in f.bucket(value):
                if len(k) != 8:
                    raise BoltError(f"attrs key of {len(k)} bytes")
                a = decode_attr_map(v)
                if a:
                    out[struct.unpack(">Q", k)[0]] = a
            return out
    return out   # no attrs bucket: an empty store


# ---------------------------------------------------------------- writer
def _leaf_page(pgid: int, items: List[Tuple[int, bytes, bytes]], ps: int) -> bytes:
    n = len(items)
    hdr = PAGE_HEADER.size
    body = bytearray()
    elems = bytearray()
    data_off = hdr + n * LEAF_ELEM.size
    for k, (flags, key, val) in enumerate(items):
        e = hdr + k * LEAF_ELEM.size
        pos = data_off + len(body) - e
        elems += LEAF_ELEM.pack(flags, pos, len(key), len(val))
        body += key + val
    size = data_off + len(body)
    npages = (size + ps - 1) // ps
    page = bytearray(PAGE_HEADER.pack(pgid, LEAF, n, npages - 1)) + elems + body
    return bytes(page) + b"\0" * (npages * ps - len(page))


def write_bolt_attrs(path: str, attrs: Dict[int, dict], page_size: int = 4096, per_leaf: int = 64,
                     inline: bool = False) -> None:
    """Write ``attrs`` as a BoltDB attribute file of the reference's shape:
    root bucket -> ``attrs`` bucket -> id (u64 big endian) -> AttrMap.  Leaf
    pages of ``per_leaf`` items under one branch page, or with ``inline`` one
    inline bucket (bolt keeps buckets under a quarter page inline).  For
    fixtures and export; bolt itself (not this writer) is the reference for
    the format."""
    ps = page_size
    items = [(0, struct.pack(">Q", i), encode_attr_map(attrs[i])) for i in sorted(attrs) if attrs[i]]
    pages: Dict[int, bytes] = {}
    nxt = 4                      # 0, 1 meta; 2 freelist; 3 root leaf
    if inline:
        inner = _leaf_page(0, items, 1 << 30)
        inner = inner[:PAGE_HEADER.size + len(items) * LEAF_ELEM.size + sum(len(k) + len(v) for _, k, v in items)]
        bucket_val = BUCKET_HDR.pack(0, 0) + inner
    else:
        leaves = [items[k:k + per_leaf] for k in range(0, len(items), per_leaf)] or [[]]
        leaf_ids = []
        for chunk in leaves:
            pg = _leaf_page(nxt, chunk, ps)
            pages[nxt] = pg
            leaf_ids.append((chunk[0][1] if chunk else b"", nxt))
            nxt += len(pg) // ps
        if len(leaf_ids) == 1:
            broot = leaf_ids[0][1]
        else:
            n = len(leaf_ids)
            hdr = PAGE_HEADER.size
            elems, body = bytearray(), bytearray()
            data_off = hdr + n * BRANCH_ELEM.size
            for k, (key, child) in enumerate(leaf_ids):
                e = hdr + k * BRANCH_ELEM.size
                elems += BRANCH_ELEM.pack(data_off + len(body) - e, len(key), child)
                body += key
            size = data_off + len(body)
            npages = (size + ps - 1) // ps
            page = bytearray(PAGE_HEADER.pack(nxt, BRANCH, n, npages - 1)) + elems + body
            pages[nxt] = bytes(page) + b"\0" * (npages * ps - len(page))
            broot = nxt
            nxt += npages
        bucket_val = BUCKET_HDR.pack(broot, 0)
    pages[3] = _leaf_page(3, [(BUCKET_LEAF_FLAG, b"attrs", bucket_val)], ps)
    pages[2] = PAGE_HEADER.pack(2, FREELIST, 0, 0) + b"\0" * (ps - PAGE_HEADER.size)
    high = max(p + len(b) // ps for p, b in pages.items())
    for i, txid in ((0, 2), (1, 3)):
        fields = (MAGIC, VERSION, ps, 0, 3, 0, 2, high, txid)
        raw = struct.pack("<IIIIQQQQQ", *fields)
        meta = PAGE_HEADER.pack(i, META, 0, 0) + raw + struct.pack("<Q", _fnv64a(raw))
        pages[i] = meta + b"\0" * (ps - len(meta))
    out = bytearray(high * ps)
    for p, b in pages.items():
        out[p * ps:p * ps + len(b)] = b
    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(out)
    os.replace(tmp, path)
