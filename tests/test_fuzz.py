"""Property / differential fuzzing (reference: roaring fuzzer, internal/test
querygenerator).  CPU: native vs Python parser on generated PQL, roaring ops
vs Python sets under hypothesis, executor invariants on random trees."""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from pilosa_amd import _roaring as R
from pilosa_amd.pql import parser as P
from pilosa_amd.testing.querygen import QueryGenerator
from tests.helpers import SW, Env

vals = st.lists(st.integers(min_value=0, max_value=(1 << 22) - 1), max_size=3000)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(vals, vals, st.booleans())
def test_roaring_ops_vs_sets(a, b, optimize):
    ba, bb = R.Bitmap(np.array(a, np.uint64)), R.Bitmap(np.array(b, np.uint64))
    if optimize:
        ba.optimize()
        bb.optimize()
    sa, sb = set(a), set(b)
    assert ba.count() == len(sa)
    assert ba.intersection_count(bb) == len(sa & sb)
    assert ba.union(bb).slice().tolist() == sorted(sa | sb)
    assert ba.difference(bb).slice().tolist() == sorted(sa - sb)
    assert ba.xor(bb).slice().tolist() == sorted(sa ^ sb)
    assert R.Bitmap.from_bytes(ba.to_bytes()).slice().tolist() == sorted(sa)


@settings(max_examples=40, deadline=None)
@given(vals, st.integers(0, 1 << 22), st.integers(0, 1 << 22))
def test_roaring_ranges_vs_sets(a, x, y):
    lo, hi = min(x, y), max(x, y)
    b = R.Bitmap(np.array(a, np.uint64))
    s = set(a)
    assert b.count_range(lo, hi) == sum(1 for v in s if lo <= v < hi)
    assert b.flip(lo, hi).slice().tolist() == sorted(s ^ set(range(lo, hi + 1)))


def test_generated_queries_parse_identically():
    g = QueryGenerator(seed=3, set_fields=["f", "g"], int_fields=["v"], time_fields=["t"])
    for q in g.queries(400, depth=4):
        assert P.parse_string(q).calls == P.parse_string_py(q).calls, q
        assert P.parse_string(str(P.parse_string(q))).calls == P.parse_string(q).calls, q


def test_generated_queries_execute_consistently():
    """Every generated query runs; Count(X) == |X|; Intersect/Union laws hold."""
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "f")
        env.field("i", "g")
        env.field("i", "v", type="int", min=-100, max=100)
        env.field("i", "t", type="time", time_quantum="YMD")
        rng = np.random.default_rng(4)
        idx = env.holder.index("i")
        cols = rng.integers(0, 3 * SW, 3000).astype(np.uint64)
        idx.field("f").import_bits(rng.integers(0, 10, 3000).astype(np.uint64), cols)
        idx.field("g").import_bits(rng.integers(0, 10, 3000).astype(np.uint64), cols[::-1].copy())
        vc = np.unique(cols)[:1500]
        idx.field("v").import_values(vc, rng.integers(-100, 100, len(vc)))
        import datetime as dt
        ts = [dt.datetime(2019 + int(c % 2), 1 + int(c % 12), 1) for c in cols[:800]]
        idx.field("t").import_bits(rng.integers(0, 10, 800).astype(np.uint64), cols[:800], timestamps=ts)
        idx.existence_field().import_bits(np.zeros(len(cols), np.uint64), cols)
        g = QueryGenerator(seed=8, set_fields=["f", "g"], int_fields=["v"], time_fields=["t"])
        for _ in range(150):
            b = g.bitmap(3)
            row = env.q1("i", b)
            assert env.q1("i", f"Count({b})") == len(list(row.columns())), b
            b2 = g.bitmap(2)
            r2 = env.q1("i", b2)
            i = set(int(c) for c in env.q1("i", f"Intersect({b}, {b2})").columns())
            u = set(int(c) for c in env.q1("i", f"Union({b}, {b2})").columns())
            s1, s2 = set(int(c) for c in row.columns()), set(int(c) for c in r2.columns())
            assert i == s1 & s2 and u == s1 | s2, (b, b2)
        for q in g.queries(100):
            env.q("i", q)
    finally:
        env.close()


def test_iterator_seek_matches_naive():
    """Bitmap.iterator() with seek (reference roaring.go:1767-1982)."""
    from pilosa_amd.testing.naive import NaiveBitmap
    rng = np.random.default_rng(7)
    vals = np.concatenate([rng.integers(0, 1 << 30, 3000, dtype=np.uint64),
                           np.arange(70000, 140000, dtype=np.uint64),        # bitmap containers
                           np.arange(1 << 33, (1 << 33) + 9000, dtype=np.uint64)])
    b = R.Bitmap(vals)
    b.optimize()  # the long ranges become run containers
    nb = NaiveBitmap(vals.tolist())
    assert list(b.iterator()) == nb.slice()
    for x in rng.integers(0, (1 << 33) + 10000, 300).tolist() + [0, 70000, 139999, 140000, (1 << 40)]:
        it = b.iterator()
        it.seek(x)
        v, eof = it.next()
        assert (None if eof else v) == nb.seek_next(x)
    it = R.Bitmap().iterator()
    assert it.next() == (0, True)


def test_fuzz_roaring_ops_vs_naive():
    """FuzzRoaringOps analog: one op stream on native and naive bitmaps."""
    from pilosa_amd.testing.naive import fuzz_ops
    assert sum(fuzz_ops(seed, 120) for seed in range(8)) == 960


def test_fuzz_unmarshal_never_crashes():
    """FuzzBitmapUnmarshalBinary analog: mutated files load or raise."""
    from pilosa_amd.testing.naive import fuzz_unmarshal
    assert sum(fuzz_unmarshal(seed, 60) for seed in range(6)) > 0
