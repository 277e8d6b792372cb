"""Host roaring core vs a naive set oracle (reference roaring/*_test.go,
roaring/naive.go), file format, official format, op log."""
import os
import struct

import numpy as np
import pytest

from pilosa_amd import _roaring as R

SAMPLE = "/root/reference/testdata/sample_view/0"


def _rand_values(rng, kind, base=0):
    if kind == "array":
        return rng.choice(65536, size=rng.integers(1, 4000), replace=False) + base
    if kind == "bitmap":
        return rng.choice(65536, size=rng.integers(5000, 60000), replace=False) + base
    starts = rng.choice(60000, size=30, replace=False)
    return np.unique(np.concatenate([np.arange(s, s + rng.integers(1, 3000)) for s in starts]) % 65536) + base


@pytest.mark.parametrize("ka", ["array", "bitmap", "run"])
@pytest.mark.parametrize("kb", ["array", "bitmap", "run"])
def test_pairwise_ops_all_container_types(ka, kb):
    rng = np.random.default_rng(hash((ka, kb)) % 1000)
    va = _rand_values(rng, ka, 65536 * 3).astype(np.uint64)
    vb = _rand_values(rng, kb, 65536 * 3).astype(np.uint64)
    a, b = R.Bitmap(va), R.Bitmap(vb)
    a.optimize()
    b.optimize()
    sa, sb = set(va.tolist()), set(vb.tolist())
    assert a.intersection_count(b) == len(sa & sb)
    assert set(a.intersect(b).slice().tolist()) == sa & sb
    assert set(a.union(b).slice().tolist()) == sa | sb
    assert set(a.difference(b).slice().tolist()) == sa - sb
    assert set(a.xor(b).slice().tolist()) == sa ^ sb
    assert a.intersect(b).check() == ""


def test_random_mutations_vs_oracle():
    rng = np.random.default_rng(5)
    b = R.Bitmap()
    oracle = set()
    for _ in range(20000):
        v = int(rng.integers(0, 1 << 22))
        if rng.random() < 0.7:
            assert b.add(v) == (v not in oracle)
            oracle.add(v)
        else:
            assert b.remove(v) == (v in oracle)
            oracle.discard(v)
    assert b.count() == len(oracle)
    assert sorted(oracle) == b.slice().tolist()
    assert b.count_range(1000, 2000000) == sum(1 for x in oracle if 1000 <= x < 2000000)
    assert b.max() == max(oracle) and b.min() == min(oracle)
    b.optimize()
    assert b.check() == ""
    assert sorted(oracle) == R.Bitmap.from_bytes(b.to_bytes()).slice().tolist()


def test_flip_shift_offset_range():
    b = R.Bitmap(np.array([1, 2, 65535, 65536 * 2 + 5], np.uint64))
    assert b.shift(1).slice().tolist() == [2, 3, 65536, 65536 * 2 + 6]
    assert b.flip(0, 4).slice().tolist() == [0, 3, 4, 65535, 65536 * 2 + 5]
    r = b.offset_range(65536 * 10, 0, 65536 * 2)
    assert r.slice().tolist() == [65536 * 10 + 1, 65536 * 10 + 2, 65536 * 10 + 65535]
    with pytest.raises(Exception):
        b.offset_range(1, 0, 65536)


@pytest.mark.skipif(not os.path.exists(SAMPLE), reason="reference sample fragment not mounted")
def test_sample_fragment_byte_exact_roundtrip():
    data = open(SAMPLE, "rb").read()
    b = R.Bitmap.from_bytes(data)
    assert b.count() == 35001 and b.container_count() == 14207 and b.check() == ""
    assert b.to_bytes() == data


def test_pilosa_format_layout():
    b = R.Bitmap(np.array([1, 2, 3, 65536 + 7], np.uint64))
    data = b.to_bytes()
    magic, count = struct.unpack_from("<IH", data, 0)[0] & 0xFFFF, struct.unpack_from("<I", data, 4)[0]
    assert magic == 12348 and count == 2
    key0, typ0, n0 = struct.unpack_from("<QHH", data, 8)
    assert (key0, n0 + 1) == (0, 3)
    # run containers after optimize
    r = R.Bitmap(np.arange(100, 5000, dtype=np.uint64))
    data = r.to_bytes()
    _, typ, _ = struct.unpack_from("<QHH", data, 8)
    assert typ == 3
    assert R.Bitmap.from_bytes(data).slice().tolist() == list(range(100, 5000))


def _official(containers, runs=False):
    """Build an official roaring (32-bit) blob: containers = [(key, sorted values)]."""
    out = bytearray()
    n = len(containers)
    if runs:
        out += struct.pack("<I", 12347 | ((n - 1) << 16))
        out += bytes([0xFF] * ((n + 7) // 8))
    else:
        out += struct.pack("<II", 12346, n)
    for k, vals in containers:
        out += struct.pack("<HH", k, len(vals) - 1)
    payloads = []
    for k, vals in containers:
        if runs:
            rr = []
            s = p = vals[0]
            for v in vals[1:]:
                if v == p + 1:
                    p = v
                    continue
                rr.append((s, p - s))
                s = p = v
            rr.append((s, p - s))
            payloads.append(struct.pack("<H", len(rr)) + b"".join(struct.pack("<HH", a, l) for a, l in rr))
        elif len(vals) <= 4096:
            payloads.append(b"".join(struct.pack("<H", v) for v in vals))
        else:
            words = np.zeros(1024, np.uint64)
            for v in vals:
                words[v >> 6] |= np.uint64(1) << np.uint64(v & 63)
            payloads.append(words.tobytes())
    if not runs or n >= 4:
        off = len(out) + 4 * n
        for p in payloads:
            out += struct.pack("<I", off)
            off += len(p)
    for p in payloads:
        out += p
    return bytes(out)


def test_official_format_reader():
    cont = [(0, [1, 5, 9]), (3, list(range(0, 10000, 2)))]
    b = R.Bitmap.from_bytes(_official(cont))
    want = [1, 5, 9] + [3 * 65536 + v for v in range(0, 10000, 2)]
    assert b.slice().tolist() == want
    cont = [(1, list(range(10, 20)) + list(range(100, 110)))]
    b = R.Bitmap.from_bytes(_official(cont, runs=True))
    assert b.slice().tolist() == [65536 + v for v in list(range(10, 20)) + list(range(100, 110))]


def test_op_log_replay_and_checksum():
    b = R.Bitmap(np.array([1, 2], np.uint64))
    data = b.to_bytes()
    ops = R.encode_op(0, 77) + R.encode_op(1, 1) + R.encode_op(2, values=np.array([5, 6, 7], np.uint64))
    ops += R.encode_op(3, values=np.array([6], np.uint64))
    other = R.Bitmap(np.array([65536 * 4 + 1], np.uint64)).to_bytes()
    ops += R.encode_op(4, roaring=other, opn=1)
    b2 = R.Bitmap.from_bytes(data + ops)
    assert b2.slice().tolist() == [2, 5, 7, 77, 65536 * 4 + 1]
    assert b2.ops == 5
    bad = bytearray(data + ops)
    bad[len(data) + 10] ^= 0xFF
    with pytest.raises(Exception, match="checksum"):
        R.Bitmap.from_bytes(bytes(bad))
    with pytest.raises(Exception):
        R.Bitmap.from_bytes((data + ops)[:-3])


def test_import_roaring_row_deltas():
    b = R.Bitmap(np.array([(1 << 20) * 2 + 5], np.uint64))
    blob = R.Bitmap(np.array([(1 << 20) * 2 + 5, (1 << 20) * 2 + 6, (1 << 20) * 7 + 1], np.uint64)).to_bytes()
    changed, rows = b.import_roaring(blob, False, 16)
    assert changed == 2 and rows == {2: 1, 7: 1}
    changed, rows = b.import_roaring(blob, True, 16)
    assert changed == 3 and rows == {2: -2, 7: -1} and b.count() == 0


def test_arena_builder_layout():
    frag = R.Bitmap(np.array([5, 70000, (1 << 20) * 3 + 2], np.uint64))
    rows, rowptr, sb, meta, payload = R.build_arena([frag, None], 16, 2)
    assert rows.tolist() == [0, 3]
    assert rowptr.shape == (2, 3) and rowptr[0].tolist() == [0, 2, 3] and rowptr[1].tolist() == [0, 0, 0]
    assert sb.tolist() == [0, 3, 3]
    j = meta & 15
    n = (meta >> 6) & 0x1FFFF
    assert j.tolist() == [0, 1, 0] and n.tolist() == [1, 1, 1]
    back = R.arena_shard_bitmap(rows, rowptr, sb, meta, payload, 0)
    assert back.slice().tolist() == [5, 70000, (1 << 20) * 3 + 2]


def test_shift_n_one_pass_matches_repeated_shift1():
    """Bitmap.shift(n) moves every value up by n in one pass; it must equal n
    rounds of the reference's Shift(1) (row.go:217-239)."""
    rng = np.random.default_rng(7)
    vals = np.unique(np.concatenate([
        rng.integers(0, 1 << 20, 3000),                      # sparse arrays
        np.arange(65536 - 40, 65536 + 40),                   # container boundary
        np.arange(3 * 65536, 3 * 65536 + 20000),             # a run
        rng.integers(5 << 16, 6 << 16, 30000),               # a bitmap container
    ]).astype(np.uint64))
    b = R.Bitmap()
    b.add_many(vals)
    for n in (1, 2, 63, 64, 65, 1000, 65535, 65536, 65537, 200003):
        want = b
        if n <= 70:
            for _ in range(n):
                want = want.shift(1)
            assert want.slice().tolist() == b.shift(n).slice().tolist(), n
        assert b.shift(n).slice().tolist() == (vals + np.uint64(n)).tolist(), n
