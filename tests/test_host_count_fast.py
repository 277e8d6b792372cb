"""Host Count fast paths (Executor.count_shard) against the general row path.

Count(Row), Count(time Row) and Count(Intersect(Row, Row)) are answered from
the fragments in place (Bitmap.range_intersection_count / range_union_count);
every case here is checked against ``bitmap_call_shard(...).count()``, which
extracts and intersects rows the way the reference executor does
(executor.go:728-760, fragment.go:559-580)."""
import numpy as np
import pytest

from pilosa_amd import _roaring as R
from pilosa_amd.pql import parse_string
from tests.helpers import SW, Env


@pytest.fixture
def env():
    e = Env()
    yield e
    e.close()


def _fill(env, rng):
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "g")
    env.field("i", "t", type="time", time_quantum="YMDH")
    f = env.holder.field("i", "f")
    g = env.holder.field("i", "g")
    rows, cols = [], []
    for r in range(6):
        for s in range(3):
            # dense rows -> bitmap containers, runs, sparse arrays
            if r == 0:
                c = np.arange(s * SW, s * SW + 200_000)
            elif r == 1:
                c = rng.choice(SW, 150_000, replace=False) + s * SW
            else:
                c = rng.choice(SW, 50 * (r + 1), replace=False) + s * SW
            rows.append(np.full(len(c), r))
            cols.append(c)
    rows = np.concatenate(rows).astype(np.uint64)
    cols = np.concatenate(cols).astype(np.uint64)
    f.import_bits(rows, cols)
    perm = rng.permutation(len(rows))
    g.import_bits(rows[perm][: len(rows) // 2], cols[perm][: len(rows) // 2])
    for frag in env.holder.index("i").field("f").view("standard").fragments.values():
        frag.storage.optimize()  # some containers become runs
    env.q("i", "Set(5, t=1, 2018-01-01T00:00) Set(6, t=1, 2018-01-02T10:00) "
               f"Set({SW + 7}, t=1, 2018-01-03T00:00) Set(5, t=2, 2018-01-01T00:00)")


def _both(env, pql, shard):
    call = parse_string(pql).calls[0].children[0]
    fast = env.executor.count_shard("i", call, shard)
    slow = env.executor.bitmap_call_shard("i", call, shard).count()
    return fast, slow


@pytest.mark.parametrize("pql", [
    "Count(Row(f=0))", "Count(Row(f=4))", "Count(Row(f=99))",
    "Count(Intersect(Row(f=0), Row(f=1)))", "Count(Intersect(Row(f=1), Row(g=1)))",
    "Count(Intersect(Row(f=2), Row(g=3)))", "Count(Intersect(Row(f=1), Row(f=1)))",
    "Count(Intersect(Row(f=0), Row(g=0)))", "Count(Intersect(Row(f=5), Row(nope=1)))",
    "Count(Row(t=1, from=2018-01-01T00:00, to=2018-01-04T00:00))",
    "Count(Row(t=1, from=2018-01-01T00:00, to=2018-01-02T00:00))",
    "Count(Row(t=2, from=2017-01-01T00:00, to=2019-01-02T00:00))",
    "Count(Union(Row(f=3), Row(g=2)))",
])
def test_count_shard_matches_row_path(env, pql):
    _fill(env, np.random.default_rng(3))
    for shard in range(3):
        if "nope" in pql:
            with pytest.raises(Exception):
                _both(env, pql, shard)
            continue
        fast, slow = _both(env, pql, shard)
        assert fast == slow, (pql, shard)


def test_count_query_end_to_end(env):
    _fill(env, np.random.default_rng(4))
    assert env.q1("i", "Count(Intersect(Row(f=0), Row(f=1)))") == sum(
        env.executor.bitmap_call_shard("i", parse_string("Intersect(Row(f=0), Row(f=1))").calls[0], s).count()
        for s in range(3))
    assert env.q1("i", "Count(Row(t=1, from=2018-01-01T00:00, to=2018-01-04T00:00))") == 3


def test_range_counts_native():
    rng = np.random.default_rng(0)
    a = R.Bitmap(np.sort(rng.choice(1 << 24, 300_000, replace=False)).astype(np.uint64))
    b = R.Bitmap(np.sort(rng.choice(1 << 24, 300_000, replace=False)).astype(np.uint64))
    a.optimize()
    for ra, rb in [(0, 0), (1, 3), (5, 2)]:
        want = a.offset_range(0, ra << 20, (ra + 1) << 20).intersection_count(
            b.offset_range(0, rb << 20, (rb + 1) << 20))
        assert a.range_intersection_count(ra << 20, b, rb << 20, 1 << 20) == want
        u = a.offset_range(0, ra << 20, (ra + 1) << 20).union(b.offset_range(0, rb << 20, (rb + 1) << 20))
        assert R.Bitmap.range_union_count([(a, ra << 20), (b, rb << 20)], 1 << 20) == u.count()
    with pytest.raises(ValueError):
        a.range_intersection_count(5, b, 0, 1 << 20)
