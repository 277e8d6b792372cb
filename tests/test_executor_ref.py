"""Expectations ported from the reference executor tests
(/root/reference/executor_test.go), one test per reference function; each
cites its source lines.  Same data, same queries, same expected results and
error texts, run through this framework's Holder + Executor on the CPU."""
import pytest

from pilosa_amd.errors import PilosaError, cause
from tests.helpers import SW, Env, cols


@pytest.fixture
def envs():
    made = []

    def make():
        e = Env()
        made.append(e)
        return e
    yield make
    for e in made:
        e.close()


def run_call(envs, write, reads, index_keys=False, **fopts):
    """runCallTest (executor_test.go:3943-3976): index ``i`` (keys option),
    field ``f`` (field options), the write query, then each read query."""
    env = envs()
    env.create_index("i", keys=index_keys)
    env.field("i", "f", **fopts)
    if write:
        env.q("i", write)
    return [env.q("i", r) for r in reads]


def set_bits(env, index, field, bits, **fopts):
    """test.Holder.SetBit: create index/field on first use, then set (row, col)."""
    if env.holder.index(index) is None:
        env.create_index(index)
    if env.holder.index(index).field(field) is None:
        env.field(index, field, **fopts)
    env.q(index, " ".join(f"Set({c}, {field}={r})" for r, c in bits))


def err_of(env, index, q):
    """The error's cause (errors.Cause in the reference tests: a top-level
    bitmap call's error arrives wrapped in "map reduce: ", executor.go:606)."""
    from pilosa_amd.errors import cause
    with pytest.raises(PilosaError) as ei:
        env.q(index, q)
    return str(cause(ei.value))


# ---------------------------------------------------------------- Row (:57-133)
def test_execute_row(envs):
    r = run_call(envs, f"Set(3, f=10)\nSet({SW + 1}, f=10)\nSet({SW + 1}, f=20)\n"
                 'SetRowAttrs(f, 10, foo="bar", baz=123)Set(1000, f=100)SetColumnAttrs(1000, foo="bar", baz=123)',
                 ["Row(f=10)", "Options(Row(f=10), excludeColumns=true)", "Options(Row(f=10), excludeRowAttrs=true)"])
    assert cols(r[0][0]) == [3, SW + 1]
    assert r[0][0].attrs == {"foo": "bar", "baz": 123}
    assert cols(r[1][0]) == [] and r[1][0].attrs == {"foo": "bar", "baz": 123}
    assert cols(r[2][0]) == [3, SW + 1] and r[2][0].attrs == {}
    # RowIDColumnKey
    r = run_call(envs, 'Set("one-hundred", f=1)\nSet("two-hundred", f=1)', ["Row(f=1)"], index_keys=True)
    assert r[0][0].keys == ["one-hundred", "two-hundred"]
    # RowKeyColumnID
    r = run_call(envs, 'Set(100, f="one")\nSet(200, f="one")', ['Row(f="one")'], keys=True)
    assert cols(r[0][0]) == [100, 200]
    # RowKeyColumnKey
    r = run_call(envs, 'Set("foo", f="bar")\nSet("foo", f="baz")\nSet("bat", f="bar")\nSet("aaa", f="bbb")\n',
                 ['Row(f="bar")'], index_keys=True, keys=True)
    assert r[0][0].keys == ["foo", "bat"] and r[0][0].attrs == {}


# ---------------------------------------------------------------- set ops (:136-447)
KEYED_WRITES = {
    "difference_ck": ('Set("one", f=10)\nSet("two", f=10)\nSet("three", f=10)\nSet("two", f=11)\nSet("four", f=11)',
                      "Difference(Row(f=10), Row(f=11))", ["one", "three"]),
    "intersect_ck": ('Set("one", f=10)\nSet("one-hundred", f=10)\nSet("two-hundred", f=10)\nSet("one", f=11)\n'
                     'Set("two", f=11)\nSet("two-hundred", f=11)', "Intersect(Row(f=10), Row(f=11))",
                     ["one", "two-hundred"]),
    "union_ck": ('Set("one", f=10)\nSet("one-hundred", f=10)\nSet("two-hundred", f=10)\nSet("one", f=11)\n'
                 'Set("two", f=11)\nSet("two-hundred", f=11)', "Union(Row(f=10), Row(f=11))",
                 ["one", "one-hundred", "two-hundred", "two"]),
    "xor_ck": ('Set("one", f=10)\nSet("one-hundred", f=10)\nSet("two-hundred", f=10)\nSet("one", f=11)\n'
               'Set("two", f=11)\nSet("two-hundred", f=11)', "Xor(Row(f=10), Row(f=11))", ["one-hundred", "two"]),
}


def _setop(envs, name, general, q, want_cols, rk_write, rk_q, rk_cols, ck_key, kk_write, kk_q, kk_keys):
    env = envs()
    set_bits(env, "i", "general", general)
    assert cols(env.q1("i", q)) == want_cols, name
    w, qq, keys = KEYED_WRITES[ck_key]
    assert run_call(envs, w, [qq], index_keys=True)[0][0].keys == keys, name
    assert cols(run_call(envs, rk_write, [rk_q], keys=True)[0][0]) == rk_cols, name
    assert run_call(envs, kk_write, [kk_q], index_keys=True, keys=True)[0][0].keys == kk_keys, name


def test_execute_difference(envs):
    _setop(envs, "Difference", [(10, 1), (10, 2), (10, 3), (11, 2), (11, 4)],
           "Difference(Row(general=10), Row(general=11))", [1, 3],
           'Set(1, f="ten")\nSet(2, f="ten")\nSet(3, f="ten")\nSet(2, f="eleven")\nSet(4, f="eleven")',
           'Difference(Row(f="ten"), Row(f="eleven"))', [1, 3], "difference_ck",
           'Set("one", f="ten")\nSet("two", f="ten")\nSet("three", f="ten")\nSet("two", f="eleven")\n'
           'Set("four", f="eleven")', 'Difference(Row(f="ten"), Row(f="eleven"))', ["one", "three"])


def test_execute_empty_difference(envs):
    """:202-211 -- Difference() is an error."""
    env = envs()
    set_bits(env, "i", "general", [(10, 1)])
    with pytest.raises(PilosaError):
        env.q("i", "Difference()")


def test_execute_intersect(envs):
    _setop(envs, "Intersect", [(10, 1), (10, SW + 1), (10, SW + 2), (11, 1), (11, 2), (11, SW + 2)],
           "Intersect(Row(general=10), Row(general=11))", [1, SW + 2],
           'Set(1, f="ten")\nSet(100, f="ten")\nSet(200, f="ten")\nSet(1, f="eleven")\nSet(2, f="eleven")\n'
           'Set(200, f="eleven")', 'Intersect(Row(f="ten"), Row(f="eleven"))', [1, 200], "intersect_ck",
           'Set("one", f="ten")\nSet("one-hundred", f="ten")\nSet("two-hundred", f="ten")\nSet("one", f="eleven")\n'
           'Set("two", f="eleven")\nSet("two-hundred", f="eleven")', 'Intersect(Row(f="ten"), Row(f="eleven"))',
           ["one", "two-hundred"])


def test_execute_empty_intersect(envs):
    """:285-292 -- Intersect() is an error."""
    env = envs()
    env.create_index("i")
    with pytest.raises(PilosaError):
        env.q("i", "Intersect()")


def test_execute_union(envs):
    _setop(envs, "Union", [(10, 0), (10, SW + 1), (10, SW + 2), (11, 2), (11, SW + 2)],
           "Union(Row(general=10), Row(general=11))", [0, 2, SW + 1, SW + 2],
           'Set(1, f="ten")\nSet(100, f="ten")\nSet(200, f="ten")\nSet(1, f="eleven")\nSet(2, f="eleven")\n'
           'Set(200, f="eleven")', 'Union(Row(f="ten"), Row(f="eleven"))', [1, 2, 100, 200], "union_ck",
           'Set("one", f="ten")\nSet("one-hundred", f="ten")\nSet("two-hundred", f="ten")\nSet("one", f="eleven")\n'
           'Set("two", f="eleven")\nSet("two-hundred", f="eleven")', 'Union(Row(f="ten"), Row(f="eleven"))',
           ["one", "one-hundred", "two-hundred", "two"])


def test_execute_empty_union(envs):
    """:365-376 -- Union() is the empty row."""
    env = envs()
    set_bits(env, "i", "general", [(10, 0)])
    assert cols(env.q1("i", "Union()")) == []


def test_execute_xor(envs):
    _setop(envs, "Xor", [(10, 0), (10, SW + 1), (10, SW + 2), (11, 2), (11, SW + 2)],
           "Xor(Row(general=10), Row(general=11))", [0, 2, SW + 1],
           'Set(1, f="ten")\nSet(100, f="ten")\nSet(200, f="ten")\nSet(1, f="eleven")\nSet(2, f="eleven")\n'
           'Set(200, f="eleven")', 'Xor(Row(f="ten"), Row(f="eleven"))', [2, 100], "xor_ck",
           'Set("one", f="ten")\nSet("one-hundred", f="ten")\nSet("two-hundred", f="ten")\nSet("one", f="eleven")\n'
           'Set("two", f="eleven")\nSet("two-hundred", f="eleven")', 'Xor(Row(f="ten"), Row(f="eleven"))',
           ["one-hundred", "two"])


# ---------------------------------------------------------------- Count (:450-507)
def test_execute_count(envs):
    env = envs()
    set_bits(env, "i", "f", [(10, 3), (10, SW + 1), (10, SW + 2)])
    assert env.q1("i", "Count(Row(f=10))") == 3
    assert run_call(envs, 'Set("three", f=10)\nSet("one-hundred", f=10)\nSet("two-hundred", f=11)',
                    ["Count(Row(f=10))"], index_keys=True)[0][0] == 2
    assert run_call(envs, 'Set(1, f="ten")\nSet(100, f="ten")\nSet(200, f="eleven")', ['Count(Row(f="ten"))'],
                    keys=True)[0][0] == 2
    assert run_call(envs, 'Set("one", f="ten")\nSet("one-hundred", f="ten")\nSet("two-hundred", f="eleven")',
                    ['Count(Row(f="ten"))'], index_keys=True, keys=True)[0][0] == 2


# ---------------------------------------------------------------- Set / Clear (:510-676)
def test_execute_set(envs):
    env = envs()
    set_bits(env, "i", "f", [(1, 0)])
    env.q("i", "Clear(1, f=11)")
    assert env.q1("i", "Count(Row(f=11))") == 0
    assert env.q1("i", "Set(1, f=11)") is True
    assert env.q1("i", "Count(Row(f=11))") == 1
    assert env.q1("i", "Set(1, f=11)") is False
    assert err_of(env, "i", 'Set("foo", f=1)') == "string 'col' value not allowed unless index 'keys' option enabled"
    assert err_of(env, "i", 'Set(2, f="bar")') == "string 'row' value not allowed unless field 'keys' option enabled"
    assert run_call(envs, "", ['Set("three", f=10)'], index_keys=True)[0][0] is True
    assert run_call(envs, "", ['Set(1, f="ten")'], keys=True)[0][0] is True
    # RowKeyColumnKey: keyed index
    env = envs()
    env.create_index("i", keys=True)
    env.field("i", "f")
    env.holder.field("i", "f").set_bit(1, 0)
    assert env.q1("i", 'Set("foo", f=11)') is True
    assert env.q1("i", "Count(Row(f=11))") == 1
    assert env.q1("i", 'Set("foo", f=11)') is False
    env.holder.index("i").delete_field("f")
    env.field("i", "f")
    assert err_of(env, "i", "Set(2, f=1)") == "column value must be a string when index 'keys' option enabled"
    env.create_index("inokey")
    env.field("inokey", "f", keys=True)
    assert err_of(env, "inokey", "Set(2, f=1)") == "row value must be a string when field 'keys' option enabled"


def test_execute_clear(envs):
    assert run_call(envs, "Set(3, f=10)", ["Clear(3, f=10)"])[0][0] is True
    assert run_call(envs, 'Set("three", f=10)', ['Clear("three", f=10)'], index_keys=True)[0][0] is True
    assert run_call(envs, 'Set(1, f="ten")', ['Clear(1, f="ten")'], keys=True)[0][0] is True
    assert run_call(envs, 'Set("one", f="ten")', ['Clear("one", f="ten")'], index_keys=True, keys=True)[0][0] is True


# ---------------------------------------------------------------- bool (:679-748)
def test_execute_set_bool(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "f", type="bool")
    assert env.q1("i", "Set(100, f=true)") is True
    assert env.q1("i", "Set(100, f=true)") is False
    assert env.q1("i", "Set(100, f=false)") is True
    assert cols(env.q1("i", "Row(f=false)")) == [100]
    assert cols(env.q1("i", "Row(f=true)")) == []
    with pytest.raises(PilosaError):
        env.q("i", 'Set(100, f="true")')
    with pytest.raises(PilosaError):
        env.q("i", "Set(100, f=1)")


# ---------------------------------------------------------------- old PQL (:751-762)
def test_execute_old_pql(envs):
    env = envs()
    set_bits(env, "i", "f", [(1, 0)])
    assert err_of(env, "i", "SetBit(frame=f, row=11, col=1)") == "unknown call: SetBit"


# ---------------------------------------------------------------- SetValue (:765-832)
def test_execute_set_value(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "f", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    env.field("i", "xxx")
    env.q("i", "Set(10, f=25)")
    env.q("i", "Set(100, f=10)")
    f = env.holder.field("i", "f")
    assert f.value(10) == (25, True)
    assert f.value(100) == (10, True)
    assert err_of(env, "i", "Set(invalid_column_name=10, f=100)") == "Set() column argument 'col' required"
    assert err_of(env, "i", 'Set("bad_column", f=100)') == \
        "string 'col' value not allowed unless index 'keys' option enabled"
    assert err_of(env, "i", 'Set(10, f="hello")') == \
        "string 'row' value not allowed unless field 'keys' option enabled"


# ---------------------------------------------------------------- SetRowAttrs (:835-892)
def test_execute_set_row_attrs(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "xxx")
    env.field("i", "kf", keys=True)
    env.q("i", 'SetRowAttrs(f, 10, foo="bar")')
    env.q("i", "SetRowAttrs(f, 200, YYY=1)")
    env.q("i", "SetRowAttrs(xxx, 10, YYY=1)")
    env.q("i", "SetRowAttrs(f, 10, baz=123, bat=true)")
    assert env.holder.field("i", "f").row_attr_store.attrs(10) == {"foo": "bar", "baz": 123, "bat": True}
    env.q("i", 'SetRowAttrs(kf, "row10", foo="bar")')
    env.q("i", 'SetRowAttrs(kf, "row200", YYY=1)')
    env.q("i", 'SetRowAttrs(kf, "row10", baz=123, bat=true)')
    assert env.q1("i", 'Row(kf="row10")').attrs == {"foo": "bar", "baz": 123, "bat": True}


# ---------------------------------------------------------------- TopN (:895-1259)
def _pairs(res):
    return [(p.id, p.count) for p in res]


def _kpairs(res):
    return [(p.key, p.count) for p in res]


def _cause(msg: str) -> str:
    return msg.split("executing: ", 1)[-1]


def test_execute_topn(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "other")
    env.q("i", f"Set(0, f=0) Set(1, f=0) Set({SW}, f=0) Set({SW + 2}, f=0) Set({5 * SW + 100}, f=0) "
               f"Set(0, f=10) Set({SW}, f=10) Set({SW}, f=20) Set(0, other=0)")
    env.holder.recalculate_caches()
    assert _pairs(env.q1("i", "TopN(f, n=2)")) == [(0, 5), (10, 2)]
    # RowIDColumnKey
    env = envs()
    env.create_index("i", keys=True)
    env.field("i", "f")
    env.field("i", "other")
    env.q("i", 'Set("zero", f=0) Set("one", f=0) Set("sw", f=0) Set("sw2", f=0) Set("sw3", f=0) '
               'Set("zero", f=10) Set("sw", f=10) Set("sw", f=20) Set("zero", other=0)')
    env.holder.recalculate_caches()
    assert _pairs(env.q1("i", "TopN(f, n=2)")) == [(0, 5), (10, 2)]
    # RowKeyColumnKey (both variants)
    for data, want in ((('Set("zero", f="zero") Set("one", f="zero") Set("sw", f="zero") Set("sw2", f="zero") '
                         'Set("sw3", f="zero") Set("zero", f="ten") Set("sw", f="ten") Set("sw", f="twenty") '
                         'Set("zero", other="zero")'), [("zero", 5), ("ten", 2)]),
                       (('Set("a", f="foo") Set("b", f="foo") Set("c", f="foo") Set("d", f="foo") Set("e", f="foo") '
                         'Set("a", f="bar") Set("b", f="bar") Set("b", f="baz") Set("a", other="foo")'),
                        [("foo", 5), ("bar", 2)])):
        env = envs()
        env.create_index("i", keys=True)
        env.field("i", "f", keys=True)
        env.field("i", "other", keys=True)
        env.q("i", data)
        env.holder.recalculate_caches()
        assert _kpairs(env.q1("i", "TopN(f, n=2)")) == want
    # ErrFieldNotFound
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.q("i", "Set(0, f=0) Set(0, f=1)")
    assert _cause(err_of(env, "i", "TopN(g, n=2)")) == 'field "g" not found'
    # ErrBSIField
    env = envs()
    env.create_index("i")
    env.field("i", "f", type="int", min=0, max=100)
    assert _cause(err_of(env, "i", "TopN(f, n=2)")).endswith('cannot compute TopN() on integer field: "f"')
    # ErrCacheNone
    env = envs()
    env.create_index("i")
    env.field("i", "f", type="set", cache_type="none", cache_size=0)
    env.q("i", "Set(0, f=0) Set(0, f=1)")
    assert _cause(err_of(env, "i", "TopN(f, n=2)")).endswith('cannot compute TopN(), field has no cache: "f"')


def test_execute_topn_fill(envs):
    """:1122-1143"""
    env = envs()
    set_bits(env, "i", "f", [(0, 0), (0, 1), (0, 2), (0, SW), (1, SW + 2), (1, SW)])
    assert _pairs(env.q1("i", "TopN(f, n=1)")) == [(0, 4)]


def test_execute_topn_fill_small(envs):
    """:1146-1177"""
    env = envs()
    set_bits(env, "i", "f", [(0, 0), (0, SW), (0, 2 * SW), (0, 3 * SW), (0, 4 * SW), (1, 0), (1, 1), (2, SW),
                             (2, SW + 1), (3, 2 * SW), (3, 2 * SW + 1), (4, 3 * SW), (4, 3 * SW + 1)])
    assert _pairs(env.q1("i", "TopN(f, n=1)")) == [(0, 5)]


def test_execute_topn_src(envs):
    """:1180-1215"""
    env = envs()
    set_bits(env, "i", "f", [(0, 0), (0, 1), (0, SW), (10, SW), (10, SW + 1), (20, SW), (20, SW + 1), (20, SW + 2)])
    set_bits(env, "i", "other", [(100, SW), (100, SW + 1), (100, SW + 2)])
    env.holder.recalculate_caches()
    assert _pairs(env.q1("i", "TopN(f, Row(other=100), n=3)")) == [(20, 3), (10, 2), (0, 1)]


def test_execute_topn_attr(envs):
    """:1218-1237"""
    env = envs()
    set_bits(env, "i", "f", [(0, 0), (0, 1), (10, SW)])
    env.holder.field("i", "f").row_attr_store.set_attrs(10, {"category": 123})
    assert _pairs(env.q1("i", 'TopN(f, n=1, attrName="category", attrValues=[123])')) == [(10, 1)]


def test_execute_topn_attr_src(envs):
    """:1240-1259"""
    env = envs()
    set_bits(env, "i", "f", [(0, 0), (0, 1), (10, SW)])
    env.holder.field("i", "f").row_attr_store.set_attrs(10, {"category": 123})
    assert _pairs(env.q1("i", 'TopN(f, Row(f=10), n=1, attrName="category", attrValues=[123])')) == [(10, 1)]


# ---------------------------------------------------------------- Min / Max (:1262-1416)
def test_execute_min_max(envs):
    for keys in (False, True):
        env = envs()
        env.create_index("i", keys=keys)
        env.field("i", "x")
        env.field("i", "f", type="int", min=-1110 if keys else -1100, max=1000)
        if keys:
            env.q("i", 'Set("zero", x=0) Set("three", x=0) Set("sw1", x=0) Set("one", x=1) Set("sw2", x=2) '
                       'Set("zero", f=20) Set("one", f=-5) Set("two", f=-5) Set("three", f=10) Set("sw", f=30) '
                       'Set("sw2", f=40) Set("sw3", f=50) Set("sw1", f=60)')
        else:
            env.q("i", f"Set(0, x=0) Set(3, x=0) Set({SW + 1}, x=0) Set(1, x=1) Set({SW + 2}, x=2) "
                       f"Set(0, f=20) Set(1, f=-5) Set(2, f=-5) Set(3, f=10) Set({SW}, f=30) Set({SW + 2}, f=40) "
                       f"Set({5 * SW + 100}, f=50) Set({SW + 1}, f=60)")
        for flt, val, cnt in (("", -5, 2), ("Row(x=0)", 10, 1), ("Row(x=1)", -5, 1), ("Row(x=2)", 40, 1)):
            r = env.q1("i", f"Min({flt + ', ' if flt else ''}field=f)")
            assert (r.val, r.count) == (val, cnt), (keys, flt)
        if keys:
            for flt, val, cnt in (("", 60, 1), ("Row(x=0)", 60, 1), ("Row(x=1)", -5, 1), ("Row(x=2)", 40, 1)):
                r = env.q1("i", f"Max({flt + ', ' if flt else ''}field=f)")
                assert (r.val, r.count) == (val, cnt), flt


def test_execute_min_max_row(envs):
    """:1419-1513"""
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.q("i", f"Set(0, f=7000) Set(3, f=50) Set({SW + 1}, f=10000) Set(1000, f=1) Set({SW + 2}, f=5000)")
    r = env.q1("i", "MinRow(field=f)")
    assert (r.id, r.count) == (1, 1)
    r = env.q1("i", "MaxRow(field=f)")
    assert (r.id, r.count) == (10000, 1)
    env = envs()
    env.create_index("i")
    env.field("i", "f", keys=True)
    env.q("i", f'Set(0, f="seven-thousand") Set(3, f="fifty") Set({SW + 1}, f="ten-thousand") Set(1000, f="one") '
               f'Set({SW + 2}, f="five-thousand")')
    r = env.q1("i", "MinRow(field=f)")
    assert (r.key, r.id, r.count) == ("seven-thousand", 1, 1)
    r = env.q1("i", "MaxRow(field=f)")
    assert (r.key, r.id, r.count) == ("five-thousand", 5, 1)


# ---------------------------------------------------------------- Sum (:1516-1632)
def test_execute_sum(envs):
    for keys in (False, True):
        env = envs()
        env.create_index("i", keys=keys)
        env.field("i", "x")
        env.field("i", "foo", type="int", min=-990, max=1000)
        env.field("i", "bar", type="int", min=-(1 << 63), max=(1 << 63) - 1)
        env.field("i", "other", type="int", min=-(1 << 63), max=(1 << 63) - 1)
        if keys:
            env.q("i", 'Set("zero", x=0) Set("sw1", x=0) Set("zero", foo=20) Set("zero", bar=2000) Set("sw", foo=30) '
                       'Set("sw2", foo=40) Set("sw3", foo=50) Set("sw1", foo=60) Set("zero", other=1000)')
        else:
            env.q("i", f"Set(0, x=0) Set({SW + 1}, x=0) Set(0, foo=20) Set(0, bar=2000) Set({SW}, foo=30) "
                       f"Set({SW + 2}, foo=40) Set({5 * SW + 100}, foo=50) Set({SW + 1}, foo=60) Set(0, other=1000)")
        r = env.q1("i", "Sum(field=foo)")
        assert (r.val, r.count) == (200, 5), keys
        r = env.q1("i", "Sum(Row(x=0), field=foo)")
        assert (r.val, r.count) == (80, 2), keys


# ---------------------------------------------------------------- time ranges (:1635-1850)
def test_execute_row_range(envs):
    import datetime
    nxt = (datetime.datetime.now() + datetime.timedelta(days=2)).strftime("%Y-%m-%dT%H:%M")
    base = ("Set({c2}, f={r1}, 1999-12-31T00:00)\nSet({c3}, f={r1}, 2000-01-01T00:00)\n"
            "Set({c4}, f={r1}, 2000-01-02T00:00)\nSet({c5}, f={r1}, 2000-02-01T00:00)\n"
            "Set({c6}, f={r1}, 2001-01-01T00:00)\nSet({c7}, f={r1}, 2002-01-01T02:00)\n"
            "Set({c2}, f={r1}, 1999-12-30T00:00)\nSet({c2}, f={r1}, 2002-02-01T00:00)\n"
            "Set({c2}, f={r10}, 2001-01-01T00:00)")
    ids = dict(c2=2, c3=3, c4=4, c5=5, c6=6, c7=7, r1=1, r10=10)
    w = base.format(**ids) + f"\nSet(8, f=1, {nxt})"
    r = run_call(envs, w, ["Row(f=1, from=1999-12-31T00:00, to=2002-01-01T03:00)", "Row(f=1, from=1999-12-31T00:00)",
                           "Row(f=1, to=2002-01-01T02:00)", "Clear( 2, f=1)",
                           "Row(f=1, from=1999-12-31T00:00, to=2002-01-01T03:00)"], type="time", time_quantum="YMDH")
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7]
    assert cols(r[1][0]) == [2, 3, 4, 5, 6, 7]
    assert cols(r[2][0]) == [2, 3, 4, 5, 6]
    assert cols(r[4][0]) == [3, 4, 5, 6, 7]
    kc = dict(c2='"two"', c3='"three"', c4='"four"', c5='"five"', c6='"six"', c7='"seven"')
    kr = dict(r1='"foo"', r10='"bar"')
    rng = "from=1999-12-31T00:00, to=2002-01-01T03:00"
    # RowIDColumnKey
    r = run_call(envs, base.format(**kc, r1=1, r10=10), [f"Row(f=1, {rng})", 'Clear("two", f=1)', f"Row(f=1, {rng})"],
                 index_keys=True, type="time", time_quantum="YMDH")
    assert r[0][0].keys == ["two", "three", "four", "five", "six", "seven"]
    assert r[2][0].keys == ["three", "four", "five", "six", "seven"]
    # RowKeyColumnID
    r = run_call(envs, base.format(c2=2, c3=3, c4=4, c5=5, c6=6, c7=7, **kr),
                 [f'Row(f="foo", {rng})', 'Clear( 2, f="foo")', f'Row(f="foo", {rng})'],
                 type="time", time_quantum="YMDH", keys=True)
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7]
    assert cols(r[2][0]) == [3, 4, 5, 6, 7]
    # RowKeyColumnKey
    r = run_call(envs, base.format(**kc, **kr), [f'Row(f="foo", {rng})', 'Clear("two", f="foo")',
                                                f'Row(f="foo", {rng})'],
                 index_keys=True, type="time", time_quantum="YMDH", keys=True)
    assert r[0][0].keys == ["two", "three", "four", "five", "six", "seven"]
    assert r[2][0].keys == ["three", "four", "five", "six", "seven"]
    # UnixTimestamp
    r = run_call(envs, base.format(**ids), ["Row(f=1, from=946598400, to=1009854000)", "Clear( 2, f=1)",
                                            "Row(f=1, from=946598400, to=1009854000)"], type="time", time_quantum="YMDH")
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7]
    assert cols(r[2][0]) == [3, 4, 5, 6, 7]


def test_execute_range_deprecated(envs):
    """:1825-1960 -- Range(f=.., from=, to=) and the positional old form."""
    base = ("Set({c2}, f={r1}, 1999-12-31T00:00)\nSet({c3}, f={r1}, 2000-01-01T00:00)\n"
            "Set({c4}, f={r1}, 2000-01-02T00:00)\nSet({c5}, f={r1}, 2000-02-01T00:00)\n"
            "Set({c6}, f={r1}, 2001-01-01T00:00)\nSet({c7}, f={r1}, 2002-01-01T02:00)\n"
            "Set({c2}, f={r1}, 1999-12-30T00:00)\nSet({c2}, f={r1}, 2002-02-01T00:00)\n"
            "Set({c2}, f={r10}, 2001-01-01T00:00)")
    ids = dict(c2=2, c3=3, c4=4, c5=5, c6=6, c7=7, r1=1, r10=10)
    rng = "from=1999-12-31T00:00, to=2002-01-01T03:00"
    tq = dict(type="time", time_quantum="YMDH")
    r = run_call(envs, base.format(**ids), [f"Range(f=1, {rng})", "Clear( 2, f=1)", f"Range(f=1, {rng})"], **tq)
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7] and cols(r[2][0]) == [3, 4, 5, 6, 7]
    r = run_call(envs, base.format(**ids), ["Range(f=1, 1999-12-31T00:00, 2002-01-01T03:00)"], **tq)
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7]
    kc = dict(c2='"two"', c3='"three"', c4='"four"', c5='"five"', c6='"six"', c7='"seven"')
    kr = dict(r1='"foo"', r10='"bar"')
    r = run_call(envs, base.format(**kc, r1=1, r10=10), [f"Range(f=1, {rng})", 'Clear("two", f=1)',
                                                         f"Range(f=1, {rng})"], index_keys=True, **tq)
    assert r[0][0].keys == ["two", "three", "four", "five", "six", "seven"]
    assert r[2][0].keys == ["three", "four", "five", "six", "seven"]
    r = run_call(envs, base.format(c2=2, c3=3, c4=4, c5=5, c6=6, c7=7, **kr),
                 [f'Range(f="foo", {rng})', 'Clear( 2, f="foo")', f'Range(f="foo", {rng})'], keys=True, **tq)
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7] and cols(r[2][0]) == [3, 4, 5, 6, 7]
    r = run_call(envs, base.format(**kc, **kr), [f'Range(f="foo", {rng})', 'Clear("two", f="foo")',
                                                f'Range(f="foo", {rng})'], index_keys=True, keys=True, **tq)
    assert r[0][0].keys == ["two", "three", "four", "five", "six", "seven"]
    assert r[2][0].keys == ["three", "four", "five", "six", "seven"]


def _bsi_env(envs, edge_min):
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "foo", type="int", min=-990, max=1000)
    env.field("i", "bar", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    env.field("i", "other", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    env.field("i", "edge", type="int", min=edge_min, max=1000)
    env.q("i", f"Set(0, f=0) Set({SW + 1}, f=0) Set(50, foo=20) Set(50, bar=2000) Set({SW}, foo=30) "
               f"Set({SW + 2}, foo=10) Set({5 * SW + 100}, foo=20) Set({SW + 1}, foo=60) Set(0, other=1000) "
               f"Set(0, edge=100) Set(1, edge=-100)")
    return env


def _bsi_checks(env, call, gt_below_min):
    from pilosa_amd.errors import ErrFieldNotFound

    def c(q):
        return cols(env.q1("i", q.replace("Row(", call + "(")))
    assert c("Row(foo == 20)") == [50, 5 * SW + 100]
    assert c("Row(other != null)") == [0]
    assert c("Row(foo != 20)") == [SW, SW + 1, SW + 2]
    assert c("Row(other != -20)") == [0]
    assert c("Row(foo < 20)") == [SW + 2]
    assert c("Row(foo <= 20)") == [50, SW + 2, 5 * SW + 100]
    assert c("Row(foo > 20)") == [SW, SW + 1]
    assert c("Row(foo >= 20)") == [50, SW, SW + 1, 5 * SW + 100]
    assert c("Row(0 <= other <= 1000)") == [0]
    assert c("Row(foo == 0)") == []
    assert c("Row(foo == 200)") == []
    assert c("Row(edge < 200)") == [0, 1]
    assert c(f"Row(edge > {gt_below_min})") == [0, 1]
    with pytest.raises(PilosaError) as ei:
        env.q("i", f"{call}(bad_field >= 20)")
    assert str(cause(ei.value)) == str(ErrFieldNotFound)   # errors.Cause


def test_execute_row_bsi_group(envs):
    """:1963-2163"""
    env = _bsi_env(envs, -900)
    _bsi_checks(env, "Row", -1000)
    for q, exp in (("Row(0 < other < 1000)", False), ("Row(0 <= other < 1000)", False),
                   ("Row(0 <= other <= 1000)", True), ("Row(0 < other <= 1000)", True),
                   ("Row(1000 < other < 1000)", False), ("Row(1000 <= other < 1000)", False),
                   ("Row(1000 <= other <= 1000)", True), ("Row(1000 < other <= 1000)", False),
                   ("Row(1000 < other < 2000)", False), ("Row(1000 <= other < 20000)", True),
                   ("Row(1000 <= other <= 2000)", True), ("Row(1000 < other <= 2000)", False)):
        assert cols(env.q1("i", q)) == ([0] if exp else []), q


def test_execute_range_bsi_group_deprecated(envs):
    """:2166-2330"""
    env = _bsi_env(envs, -1100)
    _bsi_checks(env, "Range", -1200)
    assert cols(env.q1("i", "Range(0 < other < 1000)")) == []


# ---------------------------------------------------------------- remote (:2333-2460)
def test_execute_remote_row():
    """Two nodes (node0, node1, mod hasher): node1 owns some shards, the
    coordinator's Row/Count/TopN/GroupBy/Set reach them over the wire."""
    import time as _t

    from pilosa_amd.server.client import InternalClient
    from tests.test_server import _cluster
    servers = _cluster(2)
    try:
        s0, s1 = servers
        c = InternalClient()
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set"})
        _t.sleep(0.2)
        f1 = s1.holder.field("i", "f")
        # the columns node1 owns (reference: ShardWidth+1, +2, 3*ShardWidth+4 on node1)
        remote = [SW + 1, SW + 2, 3 * SW + 4]
        assert all(s1.cluster.owns_shard("node1", "i", col // SW) for col in remote)
        for col in remote:
            f1.set_bit(10, col)
        s0.holder.field("i", "f").set_bit(10, 1)
        assert c.query(s0.uri, "i", "Row(f=10)")["results"][0]["columns"] == [1] + remote
        assert c.query(s0.uri, "i", "Count(Row(f=10))")["results"] == [4]
        c.query(s0.uri, "i", f"Set({SW + 1}, f=7)")
        assert [int(x) for x in s1.holder.field("i", "f").row(7).columns()] == [SW + 1]
        c.create_field(s0.uri, "i", "z", {"type": "time", "timeQuantum": "Y"})
        _t.sleep(0.2)
        c.query(s0.uri, "i", f"Set({SW + 1}, z=5, 2010-07-08T00:00)")
        assert [int(x) for x in s1.holder.field("i", "z").view("standard_2010").fragment(1).row(5).columns()] == \
            [SW + 1]
        c.create_field(s0.uri, "i", "fn", {"type": "set", "cacheType": "ranked", "cacheSize": 100})
        _t.sleep(0.2)
        c.query(s0.uri, "i", "Set(500001, fn=5) Set(1500001, fn=5) Set(2500001, fn=5) Set(3500001, fn=5) "
                             "Set(1500001, fn=3) Set(1500002, fn=3) Set(3500003, fn=3) Set(500001, fn=4) "
                             "Set(4500001, fn=4)")
        for s in servers:
            s.holder.recalculate_caches()
        assert c.query(s1.uri, "i", "TopN(fn, n=3)")["results"][0] == \
            [{"id": 5, "count": 4}, {"id": 3, "count": 3}, {"id": 4, "count": 2}]
        c.query(s1.uri, "i", 'SetRowAttrs(_field="f", _row=10, bat=true, baz=123)')
        a = s0.holder.field("i", "f").row_attr_store.attrs(10)
        assert a["bat"] is True and a["baz"] == 123
        got = c.query(s1.uri, "i", "GroupBy(Rows(f))")["results"][0]
        assert got == [{"group": [{"field": "f", "rowID": 7}], "count": 1},
                       {"group": [{"field": "f", "rowID": 10}], "count": 4}]
    finally:
        for s in servers:
            s.close()


# ---------------------------------------------------------------- misc (:2463-2700)
def test_execute_err_max_writes_per_request(envs):
    from pilosa_amd.errors import ErrTooManyWrites
    env = envs()
    env.create_index("i")
    env.executor.max_writes = 3
    assert err_of(env, "i", "Set() Clear() Set() Set()") == str(ErrTooManyWrites)


def test_set_column_attrs_exclude_field(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.q("i", "Set(10, f=1)")
    env.q("i", "SetColumnAttrs(10, foo='bar')")
    idx = env.holder.index("i")
    assert idx.column_attr_store.attrs(10) == {"foo": "bar"}
    env.q("i", "Set(20, f=10)")
    env.q("i", "SetColumnAttrs(20, foo='bar')")
    assert idx.column_attr_store.attrs(20) == {"foo": "bar"}


def test_time_clear_quantums(envs):
    env = envs()
    populate = ("Set(2, f=1, 1999-12-31T00:00) Set(3, f=1, 2000-01-01T00:00) Set(4, f=1, 2000-01-02T00:00) "
                "Set(5, f=1, 2000-02-01T00:00) Set(6, f=1, 2001-01-01T00:00) Set(7, f=1, 2002-01-01T02:00) "
                "Set(2, f=1, 1999-12-30T00:00) Set(2, f=1, 2002-02-01T00:00) Set(2, f=10, 2001-01-01T00:00)")
    for quantum, want in (("Y", [3, 4, 5, 6]), ("M", [3, 4, 5, 6]), ("D", [3, 4, 5, 6]), ("H", [3, 4, 5, 6, 7]),
                          ("YM", [3, 4, 5, 6]), ("YMD", [3, 4, 5, 6]), ("YMDH", [3, 4, 5, 6, 7]),
                          ("MD", [3, 4, 5, 6]), ("MDH", [3, 4, 5, 6, 7]), ("DH", [3, 4, 5, 6, 7])):
        name = quantum.lower()
        env.create_index(name)
        env.field(name, "f", type="time", time_quantum=quantum)
        env.q(name, populate)
        env.q(name, "Clear( 2, f=1)")
        assert cols(env.q1(name, "Row(f=1, from=1999-12-31T00:00, to=2002-01-01T03:00)")) == want, quantum


def test_execute_options(envs):
    r = run_call(envs, 'Set(100, f=10)\nSetRowAttrs(f, 10, foo="bar")', ["Options(Row(f=10), excludeRowAttrs=true)"])
    assert cols(r[0][0]) == [100] and r[0][0].attrs == {}
    r = run_call(envs, 'Set(100, f=10)\nSetRowAttrs(f, 10, foo="bar")', ["Options(Row(f=10), excludeColumns=true)"])
    assert cols(r[0][0]) == [] and r[0][0].attrs == {"foo": "bar"}
    # columnAttrs: the response's column attribute sets and their JSON
    import json

    from pilosa_amd.server.encoding import response_to_json
    env = envs()
    env.create_index("i")
    env.field("i", "f")
    env.q("i", 'Set(0, f=10)\nSetColumnAttrs(0, foo="baz")\nSet(100, f=10)\nSetColumnAttrs(100, foo="bar")')
    resp = env.executor.execute("i", "Options(Row(f=10), columnAttrs=true)")
    assert cols(resp.results[0]) == [0, 100]
    assert json.dumps(response_to_json(resp)["columnAttrs"], separators=(",", ":")) == \
        '[{"id":0,"attrs":{"foo":"baz"}},{"id":100,"attrs":{"foo":"bar"}}]'
    env = envs()
    env.create_index("i", keys=True)
    env.field("i", "f", keys=True)
    env.q("i", 'Set("one-hundred", f="ten")\nSetColumnAttrs("one-hundred", foo="bar")')
    resp = env.executor.execute("i", 'Options(Row(f="ten"), columnAttrs=true)')
    assert resp.results[0].keys == ["one-hundred"]
    assert json.dumps(response_to_json(resp)["columnAttrs"], separators=(",", ":")) == \
        '[{"key":"one-hundred","attrs":{"foo":"bar"}}]'
    r = run_call(envs, f"Set(100, f=10)\nSet({SW}, f=10)\nSet({SW * 2}, f=10)", ["Options(Row(f=10), shards=[0, 2])"])
    assert cols(r[0][0]) == [100, SW * 2]
    r = run_call(envs, 'Set(100, f=10)\nSetRowAttrs(f, 10, foo="bar")',
                 ["Options(Row(f=10), excludeColumns=true)\nOptions(Row(f=10), excludeRowAttrs=true)"])
    assert cols(r[0][0]) == [] and r[0][0].attrs == {"foo": "bar"}
    assert cols(r[0][1]) == [100] and r[0][1].attrs == {}


# ---------------------------------------------------------------- existence / Not (:2706-2830)
def test_execute_existence(envs):
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f")
    env.q("i", f"Set(3, f=10)\nSet({SW + 1}, f=10)\nSet({SW + 2}, f=20)\n")
    assert cols(env.q1("i", "Row(f=10)")) == [3, SW + 1]
    assert cols(env.q1("i", "Not(Row(f=10))")) == [SW + 2]
    env.reopen()
    assert cols(env.q1("i", "Not(Row(f=10))")) == [SW + 2]


def test_execute_not(envs):
    r = run_call(envs, f"Set(3, f=10)\nSet({SW + 1}, f=10)\nSet({SW + 2}, f=20)\n",
                 ["Not(Row(f=20))", "Not(Row(f=0))", "Not(Union(Row(f=10), Row(f=20)))"])
    assert cols(r[0][0]) == [3, SW + 1]
    assert cols(r[1][0]) == [3, SW + 1, SW + 2]
    assert cols(r[2][0]) == []
    r = run_call(envs, 'Set("three", f=10)\nSet("sw1", f=10)\nSet("sw2", f=20)', ["Not(Row(f=20))"], index_keys=True)
    assert r[0][0].keys == ["three", "sw1"]
    r = run_call(envs, f'Set(3, f="ten")\nSet({SW + 1}, f="ten")\nSet({SW + 2}, f="twenty")',
                 ['Not(Row(f="twenty"))'], keys=True)
    assert cols(r[0][0]) == [3, SW + 1]
    r = run_call(envs, 'Set("three", f="ten")\nSet("sw1", f="ten")\nSet("sw2", f="twenty")', ['Not(Row(f="twenty"))'],
                 index_keys=True, keys=True)
    assert r[0][0].keys == ["three", "sw1"]


# ---------------------------------------------------------------- ClearRow (:2833-3030)
def test_execute_clear_row(envs):
    w = f"Set(3, f=10)\nSet({SW - 1}, f=10)\nSet({SW + 1}, f=10)\nSet(1, f=20)\nSet({SW + 1}, f=20)\n"
    reads = ["Row(f=10)", "ClearRow(f=10)", "ClearRow(f=10)", "Row(f=10)", "Row(f=20)"]
    r = run_call(envs, w, reads)
    assert cols(r[0][0]) == [3, SW - 1, SW + 1]
    assert r[1][0] is True and r[2][0] is False
    assert cols(r[3][0]) == [] and cols(r[4][0]) == [1, SW + 1]
    r = run_call(envs, w, reads, type="mutex", cache_type="none", cache_size=0)
    assert cols(r[0][0]) == [3, SW - 1]
    assert r[1][0] is True and r[2][0] is False
    assert cols(r[3][0]) == [] and cols(r[4][0]) == [1, SW + 1]
    # Time
    r = run_call(envs, "Set(2, f=1, 1999-12-31T00:00)\nSet(3, f=1, 2000-01-01T00:00)\nSet(4, f=1, 2000-01-02T00:00)\n"
                       "Set(5, f=1, 2000-02-01T00:00)\nSet(6, f=1, 2001-01-01T00:00)\nSet(7, f=1, 2002-01-01T02:00)\n"
                       "Set(2, f=1, 1999-12-30T00:00)\nSet(2, f=1, 2002-02-01T00:00)\nSet(2, f=10, 2001-01-01T00:00)",
                 ["Row(f=1, from=1999-12-31T00:00, to=2003-01-01T03:00)",
                  "Row(f=1, from=2002-01-01T00:00, to=2002-01-02T00:00)", "ClearRow(f=1)",
                  "Row(f=1, from=1999-12-31T00:00, to=2003-01-01T03:00)",
                  "Row(f=10, from=1999-12-31T00:00, to=2003-01-01T03:00)"], type="time", time_quantum="YMD")
    assert cols(r[0][0]) == [2, 3, 4, 5, 6, 7]
    assert cols(r[1][0]) == [7]
    assert r[2][0] is True
    assert cols(r[3][0]) == [] and cols(r[4][0]) == [2]
    # Int: ClearRow is an error
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f", type="int", min=-(1 << 63), max=(1 << 63) - 1)
    with pytest.raises(PilosaError):
        env.q("i", "ClearRow(f=1)")
    # TopN: the cleared row leaves the cache
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f")
    env.q("i", " ".join([f"Set({c}, f=1)" for c in range(2, 9)] + [f"Set({c}, f=2)" for c in range(2, 8)]
                        + [f"Set({c}, f=3)" for c in range(2, 7)]))
    env.holder.recalculate_caches()
    assert _pairs(env.q1("i", "TopN(f, n=5)")) == [(1, 7), (2, 6), (3, 5)]
    assert env.q1("i", "ClearRow(f=2)") is True
    assert _pairs(env.q1("i", "TopN(f, n=5)")) == [(1, 7), (3, 5)]
    # WithKeys: an unknown key clears nothing
    assert run_call(envs, "", ['ClearRow(f="bar")'], keys=True)[0][0] is False


# ---------------------------------------------------------------- Store (:3042-3180)
def test_execute_set_row(envs):
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f")
    env.field("i", "tmp")
    env.q("i", f"Set(3, f=10)\nSet({SW - 1}, f=10)\nSet({SW + 1}, f=10)\n")
    assert cols(env.q1("i", "Row(f=10)")) == [3, SW - 1, SW + 1]
    assert env.q1("i", "Store(Row(f=10), tmp=20)") is True
    assert cols(env.q1("i", "Row(tmp=20)")) == [3, SW - 1, SW + 1]
    # Set_NoSource
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f")
    env.q("i", f"Set(3, f=10)\nSet({SW - 1}, f=10)\nSet({SW + 1}, f=10)\n")
    assert env.q1("i", "Store(Row(f=9), f=20)") is True
    assert cols(env.q1("i", "Row(f=20)")) == []
    assert env.q1("i", "Store(Row(f=9), f=10)") is True
    assert cols(env.q1("i", "Row(f=10)")) == []
    # Set_ExistingDestination
    env = envs()
    env.create_index("i", track_existence=True)
    env.field("i", "f")
    env.q("i", f"Set(3, f=10)\nSet({SW - 1}, f=10)\nSet({SW + 1}, f=10)\nSet(1, f=20)\nSet({SW + 1}, f=20)\n")
    assert cols(env.q1("i", "Row(f=20)")) == [1, SW + 1]
    assert env.q1("i", "Store(Row(f=10), f=20)") is True
    assert cols(env.q1("i", "Row(f=20)")) == [3, SW - 1, SW + 1]


# ---------------------------------------------------------------- Rows (:3226-3300)
def test_execute_rows():
    """3-node cluster (reference MustRunCluster(t, 3))."""
    import time as _t

    from pilosa_amd.server.client import InternalClient
    from tests.test_server import _cluster
    servers = _cluster(3)
    try:
        c = InternalClient()
        s0 = servers[0]
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "general", {"type": "set"})
        _t.sleep(0.2)
        bits = [(10, 0), (10, SW + 1), (11, 2), (11, SW + 2), (12, 2), (12, SW + 2), (13, 3)]
        c.query(s0.uri, "i", " ".join(f"Set({col}, general={r})" for r, col in bits))
        for q, want in (("Rows(general)", [10, 11, 12, 13]), ("Rows(field=general)", [10, 11, 12, 13]),
                        ("Rows(general, limit=2)", [10, 11]), ("Rows(general, previous=10,limit=2)", [11, 12]),
                        ("Rows(general, column=2)", [11, 12])):
            assert c.query(s0.uri, "i", q)["results"][0] == {"rows": want, "keys": None} or \
                c.query(s0.uri, "i", q)["results"][0].get("rows") == want, q
    finally:
        for s in servers:
            s.close()


def test_execute_rows_time(envs):
    """:3302-3345 -- time field without a standard view."""
    r = run_call(envs, f"Set(9, f=1, 2001-01-01T00:00)\nSet(9, f=2, 2002-01-01T00:00)\nSet(9, f=3, 2003-01-01T00:00)\n"
                       f"Set(9, f=4, 2004-01-01T00:00)\nSet({SW + 9}, f=13, 2003-02-02T00:00)\n",
                 ["Rows(f, from=1999-12-31T00:00, to=2002-01-01T03:00)",
                  "Rows(f, from=2002-01-01T00:00, to=2004-01-01T00:00)",
                  "Rows(f, from=1990-01-01T00:00, to=1999-01-01T00:00)", "Rows(f)", "Rows(f, from=2002-01-01T00:00)",
                  "Rows(f, to=2003-02-03T00:00)", "Rows(f, from=2002-01-01T00:00, to=2002-01-02T00:00)"],
                 type="time", time_quantum="YMD", no_standard_view=True)
    want = [[1], [2, 3, 13], [], [1, 2, 3, 4, 13], [2, 3, 4, 13], [1, 2, 3, 13], [2]]
    assert [list(x[0].rows) for x in r] == want


def test_execute_rows_time_empty(envs):
    env = envs()
    env.create_index("i")
    env.field("i", "x", type="time", time_quantum="YMD", no_standard_view=True)
    assert list(env.q1("i", "Rows(x, from=1999-12-31T00:00, to=2002-01-01T03:00)").rows) == []


def test_execute_query_error(envs):
    """:3355-3400 -- each error text contains the reference's substring."""
    from pilosa_amd.pql import ParseError
    env = envs()
    env.create_index("i")
    env.field("i", "general")
    for q, sub in (("GroupBy(Rows())", "Rows call must have field"), ('GroupBy(Rows("true"))', "parsing:"),
                   ("GroupBy(Rows(1))", "parsing:"), ("GroupBy(Rows(general, limit=-1))", "must be positive, but got"),
                   ("GroupBy(Rows(general), limit=-1)", "must be positive, but got"),
                   ("GroupBy(Rows(general), filter=Rows(general))", "parsing:")):
        with pytest.raises((PilosaError, ParseError)) as ei:
            env.q("i", q)
        msg = str(ei.value)
        assert sub in msg or (sub == "parsing:" and isinstance(ei.value, ParseError)), (q, msg)


def _groups(res):
    return [([(g.field, g.row_id, g.row_key or "") for g in gc.group], gc.count) for gc in res]


def test_group_by_strings(envs):
    env = envs()
    env.create_index("istring", keys=True)
    env.field("istring", "generals", keys=True)
    rk = ["r1", "r2"] * 5
    ck = [f"c{i}" for i in range(1, 11)]
    env.q("istring", " ".join(f'Set("{c}", generals="{r}")' for r, c in zip(rk, ck)))
    assert _groups(env.q1("istring", "GroupBy(Rows(generals))")) == \
        [([("generals", 1, "r1")], 5), ([("generals", 2, "r2")], 5)]
    assert _groups(env.q1("istring", 'GroupBy(Rows(generals), filter=Row(generals="r2"))')) == \
        [([("generals", 2, "r2")], 5)]


def test_execute_rows_keys(envs):
    """:3424-3560"""
    env = envs()
    env.create_index("i", keys=True)
    env.field("i", "f", keys=True)
    parts = []
    for shard in range(10):
        for i in range(shard, shard + 10):
            row = i
            while row >= 0 and row > i - 3:
                parts.append(f'Set("{shard * SW + i}", f="{row}")')
                row -= 1
    env.q("i", "".join(parts))
    allk = [str(i) for i in range(19)]
    cases = [("Rows(f)", allk), ("Rows(field=f)", allk), ("Rows(f, limit=2)", ["0", "1"]),
             ("Rows(field=f, limit=2)", ["0", "1"]), ('Rows(f, previous="15")', ["16", "17", "18"]),
             ('Rows(f, previous="11", limit=2)', ["12", "13"]), ('Rows(f, previous="17", limit=5)', ["18"]),
             ('Rows(f, previous="18")', []), ('Rows(f, previous="1", limit=0)', []),
             ('Rows(f, column="1")', ["0", "1"]), ('Rows(f, column="2")', ["0", "1", "2"]),
             ('Rows(f, column="3")', ["1", "2", "3"]), ('Rows(f, limit=2, column="3")', ["1", "2"]),
             (f'Rows(f, previous="15", column="{SW * 9 + 17}")', ["16", "17"]),
             (f'Rows(f, previous="11", limit=2, column="{SW * 5 + 14}")', ["12", "13"]),
             (f'Rows(f, previous="17", limit=5, column="{SW * 9 + 18}")', ["18"]),
             ('Rows(f, previous="18", column="19")', []), ('Rows(f, previous="1", limit=0, column="0")', [])]
    for q, want in cases:
        assert list(env.q1("i", q).keys or []) == want, q


# ---------------------------------------------------------------- GroupBy (:3563-3840)
def test_execute_group_by(envs):
    env = envs()
    env.create_index("i")
    for f in ("general", "sub", "a", "b", "wa", "wb", "wc", "ma", "mb", "na", "nb", "ppa", "ppb", "ppc"):
        env.field("i", f)

    def imp(field, bits):
        env.q("i", " ".join(f"Set({c}, {field}={r})" for r, c in bits))
    imp("general", [(10, 0), (10, 1), (10, SW + 1), (11, 2), (11, SW + 2), (12, 2), (12, SW + 2)])
    imp("sub", [(100, 0), (100, 1), (100, 3), (100, SW + 1), (110, 2), (110, 0)])
    with pytest.raises(PilosaError) as ei:
        env.q("i", "GroupBy()")
    assert "need at least one child call" in str(ei.value)
    from pilosa_amd.errors import ErrFieldNotFound
    with pytest.raises(PilosaError) as ei:
        env.q("i", "GroupBy(Rows(missing))")
    assert str(cause(ei.value)) == str(ErrFieldNotFound)

    def g(q):
        return [([(fr[0], fr[1]) for fr in grp], n) for grp, n in _groups(env.q1("i", q))]
    basic = [([("general", 10), ("sub", 100)], 3), ([("general", 10), ("sub", 110)], 1),
             ([("general", 11), ("sub", 110)], 1), ([("general", 12), ("sub", 110)], 1)]
    assert g("GroupBy(Rows(field=general), Rows(sub))") == basic
    assert g("GroupBy(Rows(general), Rows(sub))") == basic
    assert g("GroupBy(Rows(general), Rows(sub), filter=Row(general=10))") == basic[:2]
    assert g("GroupBy(Rows(general, previous=10))") == [([("general", 11)], 2), ([("general", 12)], 2)]
    assert g("GroupBy(Rows(general, previous=10), limit=1)") == [([("general", 11)], 2)]
    imp("a", [(0, 1), (1, SW + 1)])
    imp("b", [(0, SW + 1), (1, 1)])
    assert g("GroupBy(Rows(a), Rows(b), limit=1)") == [([("a", 0), ("b", 1)], 1)]
    for f in ("wa", "wb", "wc"):
        imp(f, [(0, 0), (0, 1), (0, 2), (1, 1), (2, 0), (2, 2), (3, 3)])
    assert g("GroupBy(Rows(wa), Rows(wb), Rows(wc, previous=1), limit=3)") == [
        ([("wa", 0), ("wb", 0), ("wc", 2)], 2), ([("wa", 0), ("wb", 1), ("wc", 0)], 1),
        ([("wa", 0), ("wb", 1), ("wc", 1)], 1)]
    assert g("GroupBy(Rows(wa, previous=3), Rows(wb, previous=3), Rows(wc, previous=3), limit=3)") == []
    assert g("GroupBy(Rows(wa), Rows(wb, previous=2), Rows(wc, previous=2), limit=1)") == [
        ([("wa", 1), ("wb", 0), ("wc", 0)], 1)]
    for f in ("ma", "mb"):
        imp(f, [(0, 0), (1, SW), (2, 0), (3, SW)])
    assert g("GroupBy(Rows(ma), Rows(mb), limit=5)") == [
        ([("ma", 0), ("mb", 0)], 1), ([("ma", 0), ("mb", 2)], 1), ([("ma", 1), ("mb", 1)], 1),
        ([("ma", 1), ("mb", 3)], 1), ([("ma", 2), ("mb", 0)], 1)]
    assert g("GroupBy(Rows(ma), Rows(mb, limit=2), limit=5)") == [
        ([("ma", 0), ("mb", 0)], 1), ([("ma", 1), ("mb", 1)], 1), ([("ma", 2), ("mb", 0)], 1),
        ([("ma", 3), ("mb", 1)], 1)]
    assert g(f"GroupBy(Rows(ma), Rows(mb, column={SW}), limit=5)") == [
        ([("ma", 1), ("mb", 1)], 1), ([("ma", 1), ("mb", 3)], 1), ([("ma", 3), ("mb", 1)], 1),
        ([("ma", 3), ("mb", 3)], 1)]
    for f in ("na", "nb"):
        imp(f, [(0, 0), (0, SW), (1, 0), (1, SW)])
    assert g("GroupBy(Rows(na), Rows(nb))") == [
        ([("na", 0), ("nb", 0)], 2), ([("na", 0), ("nb", 1)], 2), ([("na", 1), ("nb", 0)], 2),
        ([("na", 1), ("nb", 1)], 2)]
    for f in ("ppa", "ppb", "ppc"):
        imp(f, [(0, 0), (1, 0), (2, 0), (3, 0), (3, 91000), (3, SW), (3, SW * 2), (3, SW * 3)])
    total = []
    res = g("GroupBy(Rows(ppa), Rows(ppb), Rows(ppc), limit=3)")
    total += res
    while len(total) < 64:
        last = res[-1][0]
        res = g(f"GroupBy(Rows(ppa, previous={last[0][1]}), Rows(ppb, previous={last[1][1]}), "
                f"Rows(ppc, previous={last[2][1]}), limit=3)")
        total += res
    want = [([("ppa", i // 16), ("ppb", (i % 16) // 4), ("ppc", i % 4)], 1) for i in range(64)]
    want[63] = (want[63][0], 5)
    assert total == want
    env.field("i", "generalk", keys=True)
    env.field("i", "subk", keys=True)
    env.q("i", 'Set(0, generalk="ten") Set(1, generalk="ten") Set(1001, generalk="ten") Set(2, generalk="eleven") '
               'Set(1002, generalk="eleven") Set(2, generalk="twelve") Set(1002, generalk="twelve") '
               'Set(0, subk="one-hundred") Set(1, subk="one-hundred") Set(3, subk="one-hundred") '
               'Set(1001, subk="one-hundred") Set(2, subk="one-hundred-ten") Set(0, subk="one-hundred-ten")')
    assert _groups(env.q1("i", "GroupBy(Rows(generalk), Rows(subk))")) == [
        ([("generalk", 1, "ten"), ("subk", 1, "one-hundred")], 3),
        ([("generalk", 1, "ten"), ("subk", 2, "one-hundred-ten")], 1),
        ([("generalk", 2, "eleven"), ("subk", 2, "one-hundred-ten")], 1),
        ([("generalk", 3, "twelve"), ("subk", 2, "one-hundred-ten")], 1)]


# ---------------------------------------------------------------- Shift (:3999-4085)
def test_execute_shift(envs):
    env = envs()
    set_bits(env, "i", "general", [(10, 0)])
    assert cols(env.q1("i", "Shift(Row(general=10), n=1)")) == [1]
    assert cols(env.q1("i", "Shift(Shift(Row(general=10), n=1), n=1)")) == [2]
    env = envs()
    set_bits(env, "i", "general", [(10, 65535)])
    assert cols(env.q1("i", "Shift(Row(general=10), n=1)")) == [65536]
    env = envs()
    set_bits(env, "i", "general", [(10, 1), (10, SW - 1), (10, SW + 1)])
    assert cols(env.q1("i", "Shift(Row(general=10), n=1)")) == [2, SW, SW + 2]
    assert cols(env.q1("i", "Shift(Row(general=10), n=2)")) == [3, SW + 1, SW + 3]
    assert cols(env.q1("i", "Shift(Shift(Row(general=10)))")) == [1, SW - 1, SW + 1]
    env = envs()
    set_bits(env, "i", "general", [(10, SW - 2), (10, SW - 1), (10, SW), (10, SW + 2)])
    assert cols(env.q1("i", "Shift(Row(general=10), n=1)")) == [SW - 1, SW, SW + 1, SW + 3]
    assert cols(env.q1("i", "Shift(Shift(Row(general=10), n=1), n=1)")) == [SW, SW + 1, SW + 2, SW + 4]
