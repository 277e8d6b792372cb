"""PQL parser tests, modelled on reference pql/parser_test.go, pqlpeg_test.go
and ast_test.go.  Every case runs against both the native C++ parser
(pilosa_amd/native/pql_parser.cpp) and the Python spec parser, and the two
must build identical ASTs."""
import pytest

from pilosa_amd.pql import BETWEEN, EQ, GT, GTE, LT, LTE, NEQ, Call, Condition, ParseError
from pilosa_amd.pql import parser as P

PARSERS = {"python": P.parse_string_py}
try:
    from pilosa_amd import _pql  # noqa: F401
    PARSERS["native"] = P.parse_string
except ImportError:  # pragma: no cover - native module missing
    pass


@pytest.fixture(params=sorted(PARSERS))
def parse(request):
    return PARSERS[request.param]


WORKING = [
    ("", 0), ("Set(2, f=10)", 1), ("Set('foo', f=10)", 1), ('Set("foo", f=10)', 1),
    ("Set(2, f=1, 1999-12-31T00:00)", 1), ("Set(1, a=4)Set(2, a=4)", 2), ("Set(1, a=4) Set(2, a=4)", 2),
    ("Set(1, a=4) \n Set(2, a=4)", 2), ("Set(1, a=4)Blerg(z=ha)", 2), ("Set(1, a=4)Blerg(z=ha)Set(2, z=99)", 3),
    ("Arb(q=1, a=4)Set(1, z=9)Arb(z=99)", 3), ("Set(1, a=zoom)", 1), ("Set(1, a=4, b=5)", 1),
    ("Set(1, a=4, bsd=haha)", 1), ("Set(1, a=4, 2017-04-03T19:34)", 1), ("Union()", 1), ("Union(Row(a=1))", 1),
    ("Union(Row(a=1), Row(z=44))", 1), ("Union(Intersect(Row(), Union(Row(), Row())), Row())", 1),
    ("TopN(boondoggle)", 1), ("TopN(boon, doggle=9)", 1), ('B(a="zm\'\'e")', 1), ("B(a='zm\"\"e')", 1),
    ("SetRowAttrs(blah, 9, a=47)", 1), ("SetRowAttrs(blah, 9, a=47, b=bval)", 1),
    ("SetRowAttrs(blah, 'rowKey', a=47)", 1), ('SetRowAttrs(blah, "rowKey", a=47)', 1),
    ("SetColumnAttrs(9, a=47)", 1), ("SetColumnAttrs(9, a=47, b=bval)", 1), ("SetColumnAttrs('colKey', a=47)", 1),
    ('SetColumnAttrs("colKey", a=47)', 1), ("Clear(1, a=53)", 1), ("Clear(1, a=53, b=33)", 1),
    ("TopN(myfield, n=44)", 1), ("TopN(myfield, Row(a=47), n=10)", 1), ("Row(a < 4)", 1), ("Row(a > 4)", 1),
    ("Row(a <= 4)", 1), ("Row(a >= 4)", 1), ("Row(a == 4)", 1), ("Row(a != null)", 1), ("Row(4 < a < 9)", 1),
    ("Row(4 < a <= 9)", 1), ("Row(4 <= a < 9)", 1), ("Row(4 <= a <= 9)", 1),
    ("Row(a=4, from=2010-07-04T00:00, to=2010-08-04T00:00)", 1),
    ("Row(a=4, from='2010-07-04T00:00', to=\"2010-08-04T00:00\")", 1), ("Row(a=4, from='2010-07-04T00:00')", 1),
    ('Row(a=4, to="2010-08-04T00:00")', 1), ("Set(1, my-frame=9)", 1), ("Set(\n1,\nmy-frame\n=9)", 1),
    ("Range(blah=1, 2019-04-07T00:00, 2019-08-07T00:00)", 1), ("SetBit(f=11, col=1)", 1), ("C(a=falsen0)", 1),
    ('SetBit(Union(Zitmap(row==4), Intersect(Qitmap(blah>4), Ritmap(field="http://zoo9.com=\\\\\'hello\' and '
     '\\"hello\\"")), Hitmap(row=ag-bee)), a="4z", b=5) Count(Union(Witmap(row=5.73, frame=.10), '
     'Row(zztop><[2, 9]))) TopN(blah, fields=["hello", "goodbye", "zero"])', 3),
]

FAILING = [
    "Set", "Set(1, a=4, 2017-94-03T19:34)", "Set(1, 2017-04-03T19:34)", "Set(, 1, a=4)", "Zeeb(, a=4)",
    "SetRowAttrs(blah, 9)", "Clear(9)", "Row(a>4, 2010-07-04T00:00, 2010-08-04T00:00)",
    "Row(a=4, 2010-07-04T00:00)", "Row(a=9223372036854775808)", "Row(a=-9223372036854775809)",
    'SetRowAttrs(attr="http://zoo9.com=\\\\\'hello\' "and \\"hello\\"")',
    "Row(a=1, a=2)", "Row(a=1", "Count(Row(a=1)))",
]


@pytest.mark.parametrize("src,ncalls", WORKING)
def test_working(parse, src, ncalls):
    assert len(parse(src).calls) == ncalls


@pytest.mark.parametrize("src", FAILING)
def test_failing(parse, src):
    with pytest.raises(ParseError):
        parse(src)


def C(name, args=None, children=None):
    return Call(name, args or {}, children or [])


DEEP = [
    ("Bitmap()", C("Bitmap")),
    ("Union(  Bitmap()  , Count()  )", C("Union", children=[C("Bitmap"), C("Count")])),
    ("Count( Bitmap( id=100))", C("Count", children=[C("Bitmap", {"id": 100})])),
    ('MyCall( key= value, foo=\'bar\', age = 12 , bool0=true, bool1=false, x=null, escape="\\" \\\\escape\\n\\\\\\\\"  )',
     C("MyCall", {"key": "value", "foo": "bar", "age": 12, "bool0": True, "bool1": False, "x": None,
                  "escape": "\" \\escape\n\\\\"})),
    ("MyCall( key=12.25, foo= 13.167, bar=2., baz=0.9)",
     C("MyCall", {"key": 12.25, "foo": 13.167, "bar": 2.0, "baz": 0.9})),
    ("MyCall( key=-12.25, foo= -13)", C("MyCall", {"key": -12.25, "foo": -13})),
    ("TopN(f, Bitmap(id=100, field=other), n=3)",
     C("TopN", {"n": 3, "_field": "f"}, [C("Bitmap", {"id": 100, "field": "other"})])),
    ("TopN(f, ids=[0,10,30])", C("TopN", {"_field": "f", "ids": [0, 10, 30]})),
    ("MyCall(key=foo, x == 12.25, y >= 100, z >< [4,8], m != null)",
     C("MyCall", {"key": "foo", "x": Condition(EQ, 12.25), "y": Condition(GTE, 100),
                  "z": Condition(BETWEEN, [4, 8]), "m": Condition(NEQ, None)})),
    ("Set(1, a=7, 2010-07-08T14:44)", C("Set", {"a": 7, "_col": 1, "_timestamp": "2010-07-08T14:44"})),
    ("SetRowAttrs(myfield, 9, z=4)", C("SetRowAttrs", {"z": 4, "_field": "myfield", "_row": 9})),
    ("SetRowAttrs(myfield, 'rowKey', z=4)", C("SetRowAttrs", {"z": 4, "_field": "myfield", "_row": "rowKey"})),
    ('SetRowAttrs(myfield, "rowKey", z=4)', C("SetRowAttrs", {"z": 4, "_field": "myfield", "_row": "rowKey"})),
    ("SetColumnAttrs(9, z=4)", C("SetColumnAttrs", {"z": 4, "_col": 9})),
    ("SetColumnAttrs('colKey', z=4)", C("SetColumnAttrs", {"z": 4, "_col": "colKey"})),
    ("Clear(1, a=7)", C("Clear", {"a": 7, "_col": 1})),
    ("TopN(myfield, Row(), a=7)", C("TopN", {"a": 7, "_field": "myfield"}, [C("Row")])),
    ("Row(a==7)", C("Row", {"a": Condition(EQ, 7)})),
    ("Row(a<7)", C("Row", {"a": Condition(LT, 7)})),
    ("Row(a<=7)", C("Row", {"a": Condition(LTE, 7)})),
    ("Row(a>=7)", C("Row", {"a": Condition(GTE, 7)})),
    ("Row(a>7)", C("Row", {"a": Condition(GT, 7)})),
    ("Row(a!=null)", C("Row", {"a": Condition(NEQ, None)})),
    # half-open comparisons are normalised to an inclusive BETWEEN
    ("Row(4 <= a < 9)", C("Row", {"a": Condition(BETWEEN, [4, 8])})),
    ("Row(4 < a < 9)", C("Row", {"a": Condition(BETWEEN, [5, 8])})),
    ("Row(4 <= a <= 9)", C("Row", {"a": Condition(BETWEEN, [4, 9])})),
    ("Row(4 < a <= 9)", C("Row", {"a": Condition(BETWEEN, [5, 9])})),
    ("Sum(field=f)", C("Sum", {"field": "f"})),
    ("Sum(field-=f)", C("Sum", {"field-": "f"})),
    ("Sum(Row(), field=f)", C("Sum", {"field": "f"}, [C("Row")])),
    ("Min(Row(), field=f)", C("Min", {"field": "f"}, [C("Row")])),
    ("Max(Row(), field=f)", C("Max", {"field": "f"}, [C("Row")])),
    ("Options(Row(f1=123), excludeRowAttrs=true)",
     C("Options", {"excludeRowAttrs": True}, [C("Row", {"f1": 123})])),
    ("GroupBy(Rows(), filter=Row(a=1))", C("GroupBy", {"filter": C("Row", {"a": 1})}, [C("Rows")])),
    ("GroupBy(Rows(), filter=Row(4 < a < 9))",
     C("GroupBy", {"filter": C("Row", {"a": Condition(BETWEEN, [5, 8])})}, [C("Rows")])),
    ("Row(a=9223372036854775807)", C("Row", {"a": 9223372036854775807})),
    ("Row(a=-9223372036854775808)", C("Row", {"a": -9223372036854775808})),
]


@pytest.mark.parametrize("src,want", DEEP)
def test_deep_equality(parse, src, want):
    q = parse(src)
    assert len(q.calls) == 1
    assert q.calls[0] == want, f"{q.calls[0]!r} != {want!r}"


def test_value_types(parse):
    q = parse("MyCall(a=12, b=1.5, c=true, d=null, e=[1,2], f='x')")
    a = q.calls[0].args
    assert type(a["a"]) is int and type(a["b"]) is float and a["c"] is True and a["d"] is None
    assert isinstance(a["e"], list) and type(a["f"]) is str


@pytest.mark.parametrize("src,want", [
    ("TopN(blah, Bitmap(id==other), field=f, n=0)", 'TopN(Bitmap(id == "other"), _field="blah", field="f", n=0)'),
    ("Bitmap(row=4, did==other)", 'Bitmap(did == "other", row=4)'),
    ("Count(Intersect(Row(f=1), Row(g=2)))", "Count(Intersect(Row(f=1), Row(g=2)))"),
    ("Row(4 < a < 9)", "Row(a >< [5,8])"),
])
def test_canonical_string(parse, src, want):
    assert str(parse(src)) == want


def test_call_string():
    assert str(Call("Bitmap")) == "Bitmap()"
    assert str(Call("Range", {"other": "f", "field0": Condition(GTE, 10)})) == 'Range(field0 >= 10, other="f")'


@pytest.mark.parametrize("vals,want", [([4, 8], [4, 8]), ([1, 2, 3], [1, 2, 3])])
def test_condition_int_slice_value(vals, want):
    assert Condition(BETWEEN, vals).int_slice_value() == want


def test_string_roundtrip_reparses(parse):
    """String() output is itself valid PQL that parses to the same AST (the
    executor relies on this when forwarding calls to remote nodes)."""
    for src, _ in DEEP:
        q = parse(src)
        assert parse(str(q)).calls == q.calls, src


@pytest.mark.skipif("native" not in PARSERS, reason="native parser not built")
def test_native_matches_python_on_generated_queries():
    import random
    rng = random.Random(7)
    leaves = ["Row(f=1)", "Row(g='k')", "Row(b >= -3)", "Row(1 < v <= 100)", "Row(t=2, from='2019-01-01T00:00')"]

    def gen(d):
        if d == 0 or rng.random() < 0.3:
            return rng.choice(leaves)
        op = rng.choice(["Union", "Intersect", "Difference", "Xor", "Not"])
        n = 1 if op == "Not" else rng.randint(1, 3)
        return f"{op}({', '.join(gen(d - 1) for _ in range(n))})"

    for _ in range(300):
        src = f"Count({gen(4)})"
        assert P.parse_string(src).calls == P.parse_string_py(src).calls


_SEEDS = ["Count(Row(f=1))", "Count(Intersect(Row(f=1), Row(g='k')))", "Set(1, f=2, 2019-01-01T00:00)",
          "TopN(f, Row(g=1), n=5, ids=[1,2])", "Row(1 < v <= 100)", 'SetRowAttrs(f, 1, a="x\\"y", b=1.5)',
          "Rows(f, previous=10, limit=5, column=3)", "GroupBy(Rows(f), Rows(g), limit=3, filter=Row(h=1))",
          "Options(Count(Row(f=1)), shards=[0, 1], excludeColumns=true)", "Range(t=1, 2018-01-01T00:00, 2019-01-01T00:00)",
          "Clear(1, f=2) ClearRow(f=3) Store(Row(f=1), g=2)", "Not(Row(f=-1))", "Row(f != null)", "Count(Shift(Row(f=1), n=2))"]


@pytest.mark.skipif("native" not in PARSERS, reason="native parser not built")
def test_native_matches_python_on_mutated_input_fuzz():
    """Differential fuzz (hypothesis): byte-level mutations of valid queries.
    The native parser and the Python spec parser must agree on accept vs
    ParseError and, when both accept, on the AST (the reference's PEG is the
    single grammar both implement, pql/pql.peg)."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    alphabet = st.sampled_from(list("()[],=<>!\"' .-_:abfgnvxyz0123456789TRCU\n\t") + ["\\", "é", "\x00"])

    @settings(max_examples=1500, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
    @given(st.sampled_from(_SEEDS), st.lists(st.tuples(st.integers(0, 200), st.integers(0, 3), alphabet),
                                             max_size=4))
    def run(seed, edits):
        s = list(seed)
        for pos, op, ch in edits:
            pos = pos % (len(s) + 1)
            if op == 0 and pos < len(s):
                s[pos] = ch
            elif op == 1:
                s.insert(pos, ch)
            elif op == 2 and pos < len(s):
                del s[pos]
            else:
                del s[pos:]
        src = "".join(s)
        try:
            want = P.parse_string_py(src).calls
        except P.ParseError:
            want = None
        except (ValueError, OverflowError, TypeError):
            want = "error"
        try:
            got = P.parse_string(src).calls
        except P.ParseError:
            got = None
        except (ValueError, OverflowError, TypeError):
            got = "error"
        assert got == want, src
    run()


@pytest.mark.parametrize("src", ["Row(a==foo, a==bar)", "Row(a=foo, a=bar)", "Row(a>5, a>6)", "Row(a=7, a=8)",
                                 "Row(a=[7], a=[7,8])"])
def test_duplicate_arg_error(parse, src):
    """pqlpeg_test.go TestDuplicateArgError: the exact reference message."""
    with pytest.raises(ParseError) as e:
        parse(src)
    assert str(e.value) == "duplicate argument provided: a"
