"""Executor semantics (ported expectations from reference executor_test.go)."""
import datetime as dt

import pytest

from pilosa_amd.errors import PilosaError
from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
from pilosa_amd.models.cache import Pair
from tests.helpers import SW, Env, cols


@pytest.fixture
def env():
    e = Env()
    yield e
    e.close()


def _setup_basic(env):
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "other")


def test_row(env):
    _setup_basic(env)
    env.q("i", f"Set(3, f=10) Set({SW + 1}, f=10) Set({SW + 2}, f=20)")
    assert cols(env.q1("i", "Row(f=10)")) == [3, SW + 1]
    assert cols(env.q1("i", "Row(f=20)")) == [SW + 2]
    assert cols(env.q1("i", "Row(f=99)")) == []


def test_set_ops(env):
    _setup_basic(env)
    env.q("i", f"Set(1, f=10) Set({SW + 1}, f=10) Set({SW + 2}, f=10) Set(2, f=11) Set({SW + 2}, f=11)")
    assert cols(env.q1("i", "Difference(Row(f=10), Row(f=11))")) == [1, SW + 1]
    assert cols(env.q1("i", "Intersect(Row(f=10), Row(f=11))")) == [SW + 2]
    assert cols(env.q1("i", "Union(Row(f=10), Row(f=11))")) == [1, 2, SW + 1, SW + 2]
    assert cols(env.q1("i", "Xor(Row(f=10), Row(f=11))")) == [1, 2, SW + 1]
    assert env.q1("i", "Count(Row(f=10))") == 3
    assert env.q1("i", "Count(Intersect(Row(f=10), Row(f=11)))") == 1
    with pytest.raises(PilosaError):
        env.q("i", "Intersect()")
    with pytest.raises(PilosaError):
        env.q("i", "Difference()")
    assert cols(env.q1("i", "Union()")) == []


def test_set_clear(env):
    _setup_basic(env)
    assert env.q1("i", "Set(1, f=11)") is True
    assert env.q1("i", "Set(1, f=11)") is False
    assert env.q1("i", "Clear(1, f=11)") is True
    assert env.q1("i", "Clear(1, f=11)") is False
    assert cols(env.q1("i", "Row(f=11)")) == []


def test_bool_and_mutex(env):
    env.create_index("i")
    env.field("i", "b", type="bool")
    env.field("i", "m", type="mutex")
    env.q("i", "Set(1, b=true) Set(2, b=false) Set(3, b=true)")
    assert cols(env.q1("i", "Row(b=true)")) == [1, 3]
    env.q("i", "Set(1, b=false)")
    assert cols(env.q1("i", "Row(b=true)")) == [3]
    assert cols(env.q1("i", "Row(b=false)")) == [1, 2]
    env.q("i", "Set(5, m=1) Set(5, m=2)")
    assert cols(env.q1("i", "Row(m=1)")) == []
    assert cols(env.q1("i", "Row(m=2)")) == [5]


def _setup_bsi(env):
    env.create_index("i")
    env.field("i", "x")
    env.field("i", "f", type="int", min=-1100, max=1000)
    env.q("i", f"""Set(0, x=0) Set(3, x=0) Set({SW + 1}, x=0) Set(1, x=1) Set({SW + 2}, x=2)
        Set(0, f=20) Set(1, f=-5) Set(2, f=-5) Set(3, f=10) Set({SW}, f=30) Set({SW + 2}, f=40)
        Set({5 * SW + 100}, f=50) Set({SW + 1}, f=60)""")


def test_min_max(env):
    _setup_bsi(env)
    assert env.q1("i", "Min(field=f)") == ValCount(-5, 2)
    assert env.q1("i", "Min(Row(x=0), field=f)") == ValCount(10, 1)
    assert env.q1("i", "Min(Row(x=1), field=f)") == ValCount(-5, 1)
    assert env.q1("i", "Min(Row(x=2), field=f)") == ValCount(40, 1)
    assert env.q1("i", "Max(field=f)") == ValCount(60, 1)
    assert env.q1("i", "Max(Row(x=0), field=f)") == ValCount(60, 1)
    assert env.q1("i", "Max(Row(x=1), field=f)") == ValCount(-5, 1)
    assert env.q1("i", "Max(Row(x=2), field=f)") == ValCount(40, 1)


def test_sum(env):
    env.create_index("i")
    env.field("i", "x")
    env.field("i", "foo", type="int", min=-990, max=1000)
    env.field("i", "bar", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    env.q("i", f"""Set(0, x=0) Set({SW + 1}, x=0) Set(0, foo=20) Set(0, bar=2000) Set({SW}, foo=30)
        Set({SW + 2}, foo=40) Set({5 * SW + 100}, foo=50) Set({SW + 1}, foo=60)""")
    assert env.q1("i", "Sum(field=foo)") == ValCount(200, 5)
    assert env.q1("i", "Sum(Row(x=0), field=foo)") == ValCount(80, 2)
    assert env.q1("i", "Sum(field=bar)") == ValCount(2000, 1)


def test_bsi_row_conditions(env):
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "foo", type="int", min=-990, max=1000)
    env.field("i", "other", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    env.field("i", "edge", type="int", min=-900, max=1000)
    env.q("i", f"""Set(0, f=0) Set({SW + 1}, f=0) Set(50, foo=20) Set({SW}, foo=30) Set({SW + 2}, foo=10)
        Set({5 * SW + 100}, foo=20) Set({SW + 1}, foo=60) Set(0, other=1000) Set(0, edge=100) Set(1, edge=-100)""")
    assert cols(env.q1("i", "Row(foo == 20)")) == [50, 5 * SW + 100]
    assert cols(env.q1("i", "Row(other != null)")) == [0]
    assert cols(env.q1("i", "Row(foo != 20)")) == [SW, SW + 1, SW + 2]
    assert cols(env.q1("i", "Row(other != -20)")) == [0]
    assert cols(env.q1("i", "Row(foo < 20)")) == [SW + 2]
    assert cols(env.q1("i", "Row(foo <= 20)")) == [50, SW + 2, 5 * SW + 100]
    assert cols(env.q1("i", "Row(foo > 20)")) == [SW, SW + 1]
    assert cols(env.q1("i", "Row(foo >= 20)")) == [50, SW, SW + 1, 5 * SW + 100]
    for q, exp in [("Row(0 < other < 1000)", False), ("Row(0 <= other < 1000)", False),
                   ("Row(0 <= other <= 1000)", True), ("Row(0 < other <= 1000)", True),
                   ("Row(1000 < other < 1000)", False), ("Row(1000 <= other < 1000)", False),
                   ("Row(1000 <= other <= 1000)", True), ("Row(1000 < other <= 1000)", False)]:
        assert (cols(env.q1("i", q)) == [0]) is exp, q
    assert cols(env.q1("i", "Row(edge < 0)")) == [1]
    assert cols(env.q1("i", "Row(edge > -1000)")) == [0, 1]
    assert cols(env.q1("i", "Row(edge >= -100)")) == [0, 1]
    assert cols(env.q1("i", "Row(edge == -100)")) == [1]
    assert cols(env.q1("i", "Row(-200 < edge < 200)")) == [0, 1]
    assert cols(env.q1("i", "Row(foo > 5000)")) == []
    assert cols(env.q1("i", "Row(foo < 5000)")) == [50, SW, SW + 1, SW + 2, 5 * SW + 100]


def test_topn(env):
    _setup_basic(env)
    env.q("i", f"""Set(0, f=0) Set(1, f=0) Set({SW}, f=0) Set({SW + 2}, f=0) Set({5 * SW + 100}, f=0)
        Set(0, f=10) Set({SW}, f=10) Set({SW}, f=20) Set(0, other=0)""")
    env.holder.recalculate_caches()
    assert env.q1("i", "TopN(f, n=2)") == [Pair(0, 5), Pair(10, 2)]
    assert env.q1("i", "TopN(f, Row(other=0), n=2)") == [Pair(0, 1), Pair(10, 1)]
    assert env.q1("i", "TopN(f, ids=[10, 20])") == [Pair(10, 2), Pair(20, 1)]


def test_topn_keys(env):
    env.create_index("i", keys=True)
    env.field("i", "f", keys=True, type="set", cache_type="ranked", cache_size=100)
    env.q("i", """Set("zero", f="zero") Set("one", f="zero") Set("sw", f="zero") Set("sw2", f="zero")
        Set("sw3", f="zero") Set("zero", f="ten") Set("sw", f="ten") Set("sw", f="twenty")""")
    env.holder.recalculate_caches()
    assert env.q1("i", "TopN(f, n=2)") == [Pair(0, 5, "zero"), Pair(0, 2, "ten")]
    r = env.q1("i", 'Row(f="ten")')
    assert sorted(r.keys) == ["sw", "zero"]


def test_min_max_row(env):
    _setup_basic(env)
    env.q("i", f"Set(0, f=5) Set({SW}, f=3) Set(2, f=9) Set(1, other=1) Set(2, other=1)")
    assert env.q1("i", "MinRow(field=f)") == Pair(3, 1)
    assert env.q1("i", "MaxRow(field=f)") == Pair(9, 1)
    assert env.q1("i", "MinRow(Row(other=1), field=f)") == Pair(9, 1)


def test_time_range(env):
    env.create_index("i")
    env.field("i", "f", type="time", time_quantum="YMDH")
    env.q("i", """Set(2, f=1, 1999-12-31T00:00) Set(3, f=1, 2000-01-01T00:00) Set(4, f=1, 2000-01-02T00:00)
        Set(5, f=1, 2000-02-01T00:00) Set(6, f=1, 2001-01-01T00:00) Set(7, f=1, 2002-01-01T02:00)
        Set(2, f=1, 1999-12-30T00:00) Set(2, f=1, 2002-02-01T00:00) Set(2, f=10, 2001-01-01T00:00)""")
    assert cols(env.q1("i", "Row(f=1, from=1999-12-31T00:00, to=2002-01-01T03:00)")) == [2, 3, 4, 5, 6, 7]
    assert cols(env.q1("i", "Row(f=1, from=2002-01-01T00:00, to=2002-01-01T02:00)")) == []
    assert cols(env.q1("i", "Range(f=1, 1999-12-31T00:00, 2002-01-01T03:00)")) == [2, 3, 4, 5, 6, 7]
    assert cols(env.q1("i", "Row(f=10, from=2001-01-01T00:00, to=2001-01-02T00:00)")) == [2]
    assert cols(env.q1("i", "Row(f=1)")) == [2, 3, 4, 5, 6, 7]


def test_time_clear_quantums(env):
    env.create_index("i")
    env.field("i", "f", type="time", time_quantum="YMDH")
    env.q("i", "Set(1, f=1, 2001-01-01T00:00) Set(2, f=1, 2002-01-01T00:00)")
    env.q("i", "Clear(1, f=1)")
    assert cols(env.q1("i", "Row(f=1, from=2000-01-01T00:00, to=2003-01-01T00:00)")) == [2]


def test_not_and_existence(env):
    _setup_basic(env)
    env.q("i", f"Set(3, f=10) Set({SW + 1}, f=10) Set({SW + 2}, f=20)")
    assert cols(env.q1("i", "Not(Row(f=10))")) == [SW + 2]
    assert cols(env.q1("i", "Not(Union(Row(f=10), Row(f=20)))")) == []
    env.create_index("j", track_existence=False)
    env.field("j", "f")
    with pytest.raises(PilosaError):
        env.q("j", "Not(Row(f=1))")


def test_shift(env):
    _setup_basic(env)
    env.q("i", f"Set(1, f=1) Set({SW - 1}, f=1)")
    assert cols(env.q1("i", "Shift(Row(f=1), n=1)")) == [2, SW]
    assert cols(env.q1("i", "Shift(Row(f=1), n=2)")) == [3, SW + 1]


def test_clear_row_and_store(env):
    _setup_basic(env)
    env.q("i", f"Set(1, f=1) Set({SW + 5}, f=1) Set(2, f=2)")
    assert env.q1("i", "Store(Row(f=1), f=3)") is True
    assert cols(env.q1("i", "Row(f=3)")) == [1, SW + 5]
    assert env.q1("i", "ClearRow(f=1)") is True
    assert cols(env.q1("i", "Row(f=1)")) == []
    assert env.q1("i", "ClearRow(f=1)") is False
    env.field("i", "n", type="int", min=0, max=10)
    with pytest.raises(PilosaError):
        env.q("i", "ClearRow(n=1)")


def test_rows_and_groupby(env):
    env.create_index("i")
    env.field("i", "a")
    env.field("i", "b")
    env.q("i", f"""Set(0, a=0) Set(1, a=0) Set({SW}, a=0) Set(0, a=1) Set({SW + 1}, a=2)
        Set(0, b=10) Set({SW}, b=10) Set(1, b=11) Set({SW + 1}, b=11)""")
    assert env.q1("i", "Rows(a)") == RowIdentifiers([0, 1, 2])
    assert env.q1("i", "Rows(a, previous=0)") == RowIdentifiers([1, 2])
    assert env.q1("i", "Rows(a, limit=2)") == RowIdentifiers([0, 1])
    assert env.q1("i", f"Rows(a, column={SW + 1})") == RowIdentifiers([2])
    gb = env.q1("i", "GroupBy(Rows(a), Rows(b))")
    assert gb == [GroupCount([FieldRow("a", 0), FieldRow("b", 10)], 2),
                  GroupCount([FieldRow("a", 0), FieldRow("b", 11)], 1),
                  GroupCount([FieldRow("a", 1), FieldRow("b", 10)], 1),
                  GroupCount([FieldRow("a", 2), FieldRow("b", 11)], 1)]
    assert env.q1("i", "GroupBy(Rows(a), Rows(b), limit=2)") == gb[:2]
    assert env.q1("i", "GroupBy(Rows(a), Rows(b), previous=[0, 11])") == gb[2:]
    assert env.q1("i", "GroupBy(Rows(a), Rows(b), filter=Row(b=10))") == [
        GroupCount([FieldRow("a", 0), FieldRow("b", 10)], 2), GroupCount([FieldRow("a", 1), FieldRow("b", 10)], 1)]
    assert env.q1("i", "GroupBy(Rows(a), Rows(b), offset=3)") == gb[3:]


def test_row_attrs_and_column_attrs(env):
    _setup_basic(env)
    env.q("i", 'Set(1, f=10) SetRowAttrs(f, 10, foo="bar", baz=123) SetColumnAttrs(1, name="x")')
    r = env.q1("i", "Row(f=10)")
    assert r.attrs == {"foo": "bar", "baz": 123}
    env.q("i", "SetRowAttrs(f, 10, foo=null)")
    assert env.q1("i", "Row(f=10)").attrs == {"baz": 123}
    from pilosa_amd.executor import ExecOptions
    resp = env.executor.execute("i", "Row(f=10)", opt=ExecOptions(column_attrs=True))
    assert resp.column_attr_sets == [{"id": 1, "attrs": {"name": "x"}}]


def test_options(env):
    _setup_basic(env)
    env.q("i", f"Set(1, f=10) Set({SW + 1}, f=10) SetRowAttrs(f, 10, a=1)")
    assert cols(env.q1("i", "Options(Row(f=10), shards=[1])")) == [SW + 1]
    assert cols(env.q1("i", "Options(Row(f=10), excludeColumns=true)")) == []
    assert env.q1("i", "Options(Row(f=10), excludeRowAttrs=true)").attrs == {}


def test_keys(env):
    env.create_index("i", keys=True)
    env.field("i", "f", keys=True)
    env.q("i", 'Set("c1", f="r1") Set("c2", f="r1") Set("c3", f="r2")')
    assert sorted(env.q1("i", 'Row(f="r1")').keys) == ["c1", "c2"]
    assert env.q1("i", 'Count(Row(f="r1"))') == 2
    assert env.q1("i", "Rows(f)") == RowIdentifiers(keys=["r1", "r2"])
    with pytest.raises(PilosaError):
        env.q("i", "Set(1, f=1)")


def test_max_writes(env):
    _setup_basic(env)
    env.executor.max_writes = 2
    from pilosa_amd.errors import ErrTooManyWrites
    with pytest.raises(PilosaError) as ei:
        env.q("i", "Set(1, f=1) Set(2, f=1) Set(3, f=1)")
    assert str(ei.value) == str(ErrTooManyWrites)


def test_persistence_reopen(env):
    _setup_basic(env)
    env.field("i", "n", type="int", min=-100, max=100)
    env.q("i", f"Set(1, f=1) Set({SW + 7}, f=1) Set(3, n=-42) Set(4, n=17)")
    env.reopen()
    assert cols(env.q1("i", "Row(f=1)")) == [1, SW + 7]
    assert env.q1("i", "Sum(field=n)") == ValCount(-25, 2)
    assert env.holder.field("i", "n").bsi.bit_depth == 6


def test_bsi_v1_fragment_upgrade():
    """v1 BSI files (planes at rows 0.., not-null at row bitDepth, values
    offset by min, no bitDepth in the meta) are rewritten as v2 on open
    (reference fragment.go:2717 upgradeRoaringBSIv2, field.go:500-507)."""
    import os
    import numpy as np
    from pilosa_amd import _roaring as R
    from pilosa_amd.models.field import bit_depth_int64
    from pilosa_amd.wire import pb
    env = Env()
    try:
        env.create_index("i")
        f = env.field("i", "v", type="int", min=10, max=1000)
        vals = {1: 10, 5: 17, SW + 3: 999, SW + 9: 500}
        for c, x in vals.items():
            env.q("i", f"Set({c}, v={x})")
        meta_path = f.meta_path()
        env.holder.close()
        bd = bit_depth_int64(1000 - 10)
        for shard in (0, 1):
            pos = []
            for c, x in vals.items():
                if c // SW != shard:
                    continue
                lo = c % SW
                pos.append(bd * SW + lo)  # v1 not-null row
                for i in range(bd):
                    if (x - 10) >> i & 1:
                        pos.append(i * SW + lo)
            b = R.Bitmap(np.array(sorted(pos), dtype=np.uint64))
            b.flags = 0
            path = os.path.join(env.dir, "i", "v", "views", "bsig_v", "fragments", str(shard))
            with open(path, "wb") as fh:
                fh.write(b.to_bytes())
        m = pb.FieldOptions()
        with open(meta_path, "rb") as fh:
            m.ParseFromString(fh.read())
        m.BitDepth, m.Base = 0, 0
        with open(meta_path, "wb") as fh:
            fh.write(m.SerializeToString())
        env.reopen()
        assert env.q1("i", "Sum(field=v)") == ValCount(sum(vals.values()), len(vals))
        assert env.q1("i", "Min(field=v)") == ValCount(10, 1)
        assert env.q1("i", "Max(field=v)") == ValCount(999, 1)
        assert cols(env.q1("i", "Row(v > 100)")) == [SW + 3, SW + 9]
        frag = env.holder.index("i").field("v").views["bsig_v"].fragment(0)
        assert frag.storage.flags & 1
        env.reopen()  # upgraded file is v2 on disk: a second open keeps it
        assert env.q1("i", "Sum(field=v)") == ValCount(sum(vals.values()), len(vals))
    finally:
        env.close()


def test_fresh_int_field_reopen_keeps_v2_meta():
    """A v2 int field with no writes yet has bit depth 0 on disk; reopening it
    must not take the v1 upgrade path (base := min), which would shift every
    later value by min and overflow at min = -2^63."""
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "x", type="int", min=-(1 << 63), max=(1 << 63) - 1)
        env.field("i", "y", type="int", min=10, max=1000)
        env.reopen()
        env.q("i", "Set(3, x=2000) Set(4, y=10) Set(5, y=17)")
        assert env.q1("i", "Sum(field=x)") == ValCount(2000, 1)
        assert env.q1("i", "Sum(field=y)") == ValCount(27, 2)
        env.reopen()
        assert env.q1("i", "Sum(field=x)") == ValCount(2000, 1)
        assert env.q1("i", "Min(field=y)") == ValCount(10, 1)
    finally:
        env.close()
