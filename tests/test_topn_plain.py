"""native/pql_compile.cpp topn_plain: the serving fast path's recogniser of
requests made only of plain cache-only TopN(<field>[, n=][, threshold=])
calls (anything else -> None, the general parser runs), checked against the
general PQL parser's reading of the same text."""
import pytest

from pilosa_amd import _pql
from pilosa_amd.pql import parse_string


@pytest.mark.parametrize("text", [
    "TopN(f, n=5, threshold=3) TopN(f) TopN(g,threshold=7 ,n=1)",
    "TopN(f)", "  TopN( f_1 , n = 10 )\n TopN(f-2, threshold=0)", "TopN(f, n=0)",
])
def test_plain_requests_match_the_parser(text):
    fields, ns, ths = _pql.topn_plain(text)
    calls = parse_string(text).calls
    assert [c.args.get("_field") for c in calls] == fields
    assert [c.args.get("n", 0) for c in calls] == ns
    assert [c.args.get("threshold", 0) for c in calls] == ths


@pytest.mark.parametrize("text", [
    "", "TopN(f, Row(g=1), n=5)", "TopN(f, n=-1)", "TopN(f, ids=[1])", "TopN(f, n=5) Count(Row(f=1))",
    "TopN(f, n=5, n=6)", 'TopN("f")', "TopN(f, n=5", "TopN(f, tanimotoThreshold=3)", "TopN(f, n=1.5)",
    "TopN(f, n=99999999999999999999)", "Count(Row(f=1))", "TopN(f, attrName=x, attrValues=[1])",
])
def test_other_shapes_decline(text):
    assert _pql.topn_plain(text) is None
