"""Ported expectations of internal/test/querygenerator_test.go
(TestPQL_Generator): calls built with the generator's helpers equal the
parse of their PQL text; random queries parse and round-trip."""
import pytest

from pilosa_amd.pql import parse_string
from pilosa_amd.testing.querygen import (PQL, Count, Difference, Intersect, Not, QueryGenerator, Row, Union,
                                         Xor)


@pytest.mark.parametrize("text,built", [
    ("Union(Row(aaa=10),Row(bbb=9))", PQL(Union(Row("aaa", 10), Row("bbb", 9)))),
    ("Intersect(Row(aaa=10),Row(bbb=9))", PQL(Intersect(Row("aaa", 10), Row("bbb", 9)))),
    ("Difference(Row(aaa=10),Row(bbb=9))", PQL(Difference(Row("aaa", 10), Row("bbb", 9)))),
    ("Xor(Row(aaa=10),Row(bbb=9))", PQL(Xor(Row("aaa", 10), Row("bbb", 9)))),
    ("Count(Not(Row(aaa=1)))", PQL(Count(Not(Row("aaa", 1)))))])
def test_generator_builds_parsed_ast(text, built):
    assert parse_string(text).calls == built.calls
    assert parse_string(str(built)).calls == built.calls


def test_random_queries_parse_and_round_trip():
    g = QueryGenerator(seed=7, set_fields=["f", "g"], int_fields=["v"], time_fields=["t"], max_row=50)
    for q in g.queries(200, depth=3):
        parsed = parse_string(q)
        assert len(parsed.calls) == 1
        assert parse_string(str(parsed)).calls == parsed.calls
