"""Native PQL -> QueryProg compiler (pilosa_amd/native/pql_compile.cpp) must
produce exactly the programs of the Python parser + planner + compile_expr."""
import numpy as np
import pytest

from pilosa_amd import _roaring as R
from pilosa_amd.ops.device import QPROG_DTYPE, DeviceView, compile_expr, pack_programs
from pilosa_amd.ops.planner import GpuPlanner, NativeCountCompiler, Unsupported
from pilosa_amd.pql import parse_string


@pytest.fixture(scope="module")
def views():
    rng = np.random.default_rng(3)
    def frag(rows):
        vals = np.concatenate([np.uint64(r) * np.uint64(1 << 20) + rng.choice(1 << 20, 50, replace=False).astype(np.uint64)
                               for r in rows])
        return R.Bitmap(vals)
    f = DeviceView.from_bitmaps([frag(range(0, 40))], "cpu")            # identity directory
    g = DeviceView.from_bitmaps([frag([3, 9, 27, 81, 243])], "cpu")      # sparse directory
    return {"f": f, "g": g}


def _python(views, q):
    planner = GpuPlanner(lambda f, v: views[f])
    vi = {id(v): i for i, v in enumerate(views.values())}
    return pack_programs([compile_expr(planner.plan(parse_string(q).calls[0]), vi)])[0]


def _gen(rng, d=0):
    if d >= 2 or rng.random() < 0.35:
        fld = "f" if rng.random() < 0.7 else "g"
        return f"Row({fld}={int(rng.integers(0, 300))})"
    op = ["Intersect", "Union", "Difference", "Xor"][int(rng.integers(0, 4))]
    n = int(rng.integers(1, 4))
    sep = "," if rng.random() < 0.5 else " , "
    return f"{op}({sep.join(_gen(rng, d + 1) for _ in range(n))})"


def test_native_equals_python(views):
    rng = np.random.default_rng(9)
    qs = [f"Count({_gen(rng)})" for _ in range(400)]
    comp = NativeCountCompiler(views)
    progs, vs, S = comp.compile(qs)
    assert S == 1 and vs == list(views.values())
    for q, p in zip(qs, progs):
        try:
            want = _python(views, q)
        except Exception:
            continue
        assert p.tobytes() == want.tobytes(), q
    assert comp.native_hits > 300


@pytest.mark.parametrize("q", [
    "Count(Row(f=1, from='2019-01-01T00:00'))",  # time range
    "Count(Row(f > 3))",                          # condition
    "Count(Row(f=1))Count(Row(f=2))",             # two calls
    "Count(Bitmap(frame=f, row=1))",              # legacy arguments
    "Count(Intersect(Row(f=1), Not(Row(f=2))))",  # Not
    "Count(Row(zz=1))",                           # unknown field
    "TopN(f, n=2)",
])
def test_unsupported_shapes_fall_back(views, q):
    from pilosa_amd import _pql
    _, ok = _pql.compile_counts([q], {"f": 0, "g": 1}, [views["f"].rows, views["g"].rows])
    assert not ok[0]


def test_fallback_paths(views):
    comp = NativeCountCompiler(views)
    with pytest.raises(Unsupported):
        comp.compile(["Count(Row(f > 3))"])   # falls back, planner refuses BSI on a set view
    progs, _, _ = comp.compile(["Count(Intersect(Row(f=1)))", "Count(Union(Row(g=9), Row(f=2)))"])
    assert comp.fallbacks == 1
    assert progs[0]["nprog"] == 1 and progs[1]["nprog"] == 3
    assert progs[1]["leaf_view"][0] == 1 and progs[1]["leaf_row"][0] == 1  # g's dense index of row 9


def test_limits(views):
    from pilosa_amd import _pql
    wide = "Count(Union(" + ",".join(f"Row(f={i})" for i in range(17)) + "))"
    deep = "Count(" + "Intersect(Row(f=1), " * 5 + "Row(f=2)" + ")" * 5 + ")"
    _, ok = _pql.compile_counts([wide, deep], {"f": 0}, [views["f"].rows])
    assert not ok.any()


def test_count_text_equals_per_query(views):
    """compile_count_text over a whole request == compile_counts per call."""
    from pilosa_amd import _pql
    rng = np.random.default_rng(11)
    qs = [f"Count({_gen(rng)})" for _ in range(300)]
    fields = {"f": 0, "g": 1}
    dirs = [views["f"].rows, views["g"].rows]
    raw, ok = _pql.compile_counts(qs, fields, dirs)
    assert ok.all()
    for sep in (" ", "\n", "  \t"):
        got = _pql.compile_count_text(sep.join(qs), fields, dirs)
        assert got is not None and got[1] == len(qs)
        assert (got[0] == raw).all()
    assert _pql.count_text_fields(" ".join(qs)) == sorted(set(_pql.count_text_fields(" ".join(qs))),
                                                          key=_pql.count_text_fields(" ".join(qs)).index)
    assert set(_pql.count_text_fields("Count(Row(f=1)) Count(Intersect(Row(g=2),Row( f =3)))")) == {"f", "g"}
    for bad in ("Count(Row(f=1)) TopN(f)", "Count(Row(f=1)) Count(Row(n > 3))", "", "Count(Row(f=1)) x",
                "Count(Row(f=1)) Count(Row(zz=1))", "Count(Row(f=1)) Count(Row(f=\"a\"))"):
        assert _pql.compile_count_text(bad, fields, dirs) is None, bad


def test_plan_count_text_matches_numpy_planner(views):
    """plan_count_text (native planner) == compile_counts + the numpy route
    classification / ordering of GpuEngine.prepare_progs, up to the
    orientation of Count(Intersect(a, b)) (a count is symmetric)."""
    from pilosa_amd import _pql
    from pilosa_amd.ops.device import OP_AND, flat_mask
    rng = np.random.default_rng(5)
    qs = [f"Count({_gen(rng)})" for _ in range(2500)]
    qs += ["Count(Intersect(Row(f=3), Row(f=3)))", "Count(Row(f=7))", "Count(Union(Row(f=1), Row(g=9), Row(f=2)))"]
    # repeats of one Count(Intersect(a, b)), either order: planned once
    qs += ["Count(Intersect(Row(f=1), Row(g=2)))", "Count(Intersect(Row(g=2), Row(f=1)))",
           "Count(Intersect(Row(f=1), Row(g=2)))"]
    fields = {"f": 0, "g": 1}
    dirs = [views["f"].rows, views["g"].rows]
    Q, segs, buf = _pql.plan_count_text("\n".join(qs), fields, dirs, True, True, 4)
    assert Q == len(qs)
    raw, ok = _pql.compile_counts(qs, fields, dirs)
    want = raw.view(QPROG_DTYPE)
    seen = np.zeros(Q, bool)
    leaves = lambda w: sorted([(int(w["leaf_view"][i]), int(w["leaf_row"][i])) for i in range(int(w["nleaf"]))])  # noqa: E731
    assert segs[-1][0] == 5, "the repeated calls form a K_ALIAS segment"
    for kind, n, po, oo in segs:
        if kind == 5:   # (from, to): to's answer is from's, the same unordered pair
            frm, to = buf[po:po + n * 8].view(np.int64), buf[oo:oo + n * 8].view(np.int64)
            assert seen[frm].all() and not seen[to].any()
            seen[to] = True
            for a, b in zip(frm, to):
                assert leaves(want[a]) == leaves(want[b])
            assert {len(qs) - 2, len(qs) - 1} <= set(int(t) for t in to) or \
                {len(qs) - 3, len(qs) - 1} <= set(int(t) for t in to) or {len(qs) - 3, len(qs) - 2} <= set(int(t) for t in to)
            continue
        progs = buf[po:po + n * 256].view(QPROG_DTYPE)
        order = buf[oo:oo + n * 8].view(np.int64)
        assert not seen[order].any()
        seen[order] = True
        lr = progs["leaf_row"]
        key = [(int(a), int(b)) for a, b in zip(lr[:, 0], lr[:, 1])]
        assert key == sorted(key)
        for p, q in zip(progs, order):
            w = want[q]
            pg, n_ = p["prog"], int(p["nprog"])
            is_and2 = n_ == 3 and pg[0] == 0 and pg[1] == 1 and pg[2] == OP_AND
            if kind == 0:
                assert is_and2
                a = sorted([(int(p["leaf_view"][i]), int(p["leaf_row"][i])) for i in range(2)])
                wl = [(int(w["leaf_view"][i]), int(w["leaf_row"][i])) for i in range(int(w["nleaf"]))]
                assert a == sorted(wl * (2 if len(wl) == 1 else 1))
            elif kind == 1:
                assert n_ == 1 and p.tobytes() == w.tobytes()
            else:
                assert p.tobytes() == w.tobytes()
                fm = bool(flat_mask(w.reshape(1))[0])
                assert (kind in (3, 4)) == fm
                if kind == 4:
                    assert all(pg[i] == 33 for i in range(2, n_, 2))
    assert seen.all()
    assert _pql.plan_count_text("Count(Row(f=1)) TopN(f)", fields, dirs, True, True, 4) is None
    assert _pql.plan_count_text("Count(Row(f=\"a\"))", fields, dirs, True, True, 4) is None


def test_plan_count_text_time_ranges(views):
    """Time-range Row leaves compile natively into the union of the row over
    the range's covering views (the slots the caller resolved per distinct
    (field, from, to)), quoted and bare times, either bound alone, mixed
    with plain rows; an unresolved range or a malformed one is refused."""
    from pilosa_amd import _pql
    from pilosa_amd.ops.device import OP_OR
    fields = {"f": 0}
    dirs = [views["f"].rows, views["g"].rows, views["f"].rows, views["g"].rows]
    text = ("Count(Row(t=3, from='2020-01-01T00:00', to='2020-01-03T05:00')) "
            "Count(Row(t=9,to=2020-01-02T00:00)) Count(Row(f=4)) "
            "Count(Intersect(Row(f=2), Row(t=27, from=\"2020-01-01T00:00\", to='2020-01-03T05:00')))")
    assert _pql.count_text_fields(text) == ["f"]
    rs = _pql.count_text_ranges(text)
    assert rs == [("t", "2020-01-01T00:00", "2020-01-03T05:00"), ("t", None, "2020-01-02T00:00")]
    k1 = "t\x1f2020-01-01T00:00\x1f2020-01-03T05:00"
    k2 = "t\x1f\x01\x1f2020-01-02T00:00"
    ranges = {k1: [1, 2, 3], k2: [1]}
    Q, segs, buf = _pql.plan_count_text(text, fields, dirs, True, True, 1, ranges)
    assert Q == 4
    progs = {}
    for kind, n, po, oo in segs:
        for p, q in zip(buf[po:po + n * 256].view(QPROG_DTYPE), buf[oo:oo + n * 8].view(np.int64)):
            progs[int(q)] = (kind, p)
    kind, p = progs[0]
    assert kind == 4 and int(p["nleaf"]) == 3 and list(p["prog"][:5]) == [0, 1, OP_OR, 2, OP_OR]
    assert list(p["leaf_view"][:3]) == [1, 2, 3]
    assert list(p["leaf_row"][:3]) == [views["g"].dense_many(np.array([3], np.uint64))[0], 3, 0]
    kind, p = progs[1]
    assert kind == 1 and int(p["leaf_view"][0]) == 1 and int(p["leaf_row"][0]) == 1   # g row 9 -> dense 1
    kind, p = progs[3]
    assert int(p["nleaf"]) == 4 and int(p["nprog"]) == 7   # f2 AND (t27@1 OR t27@2 OR t27@3)
    assert _pql.plan_count_text(text, fields, dirs, True, True, 1, {k1: [1, 2, 3]}) is None   # k2 unresolved
    for bad in ("Count(Row(t=3, from='2020-01-01))", "Count(Row(t=3, from=1, from=2))", "Count(Row(t=3, at=1))"):
        assert _pql.plan_count_text(bad, fields, dirs, True, True, 1, ranges) is None, bad
