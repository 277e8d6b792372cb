"""Ported expectations of the reference's executor_internal_test.go:
TestExecutor_TranslateGroupByCall (string keys in GroupBy's previous=
translated to row ids, with its error cases) and TestFieldRowMarshalJSON.
TestFilterWithLimit / TestFilterWithRows exercise the reference's streaming
row filters (fragment.go:2601-2667); rows listing here filters vectorised
(Fragment.rows), whose behaviour the Rows() executor tests pin."""
import pytest

from pilosa_amd.errors import ErrFieldNotFound, PilosaError
from pilosa_amd.executor import FieldRow
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.pql import parse_string
from tests.helpers import Env


@pytest.fixture
def env():
    e = Env()
    e.create_index("i")
    idx = e.holder.index("i")
    idx.create_field("ak", FieldOptions(keys=True))
    idx.create_field("b")
    idx.create_field("ck", FieldOptions(keys=True))
    ts = e.holder.translate
    ts.translate_rows_to_uint64("i", "ak", ["la"])
    ts.translate_rows_to_uint64("i", "ck", ["ha"])
    yield e, idx
    e.holder.close()


def test_translate_group_by_previous(env):
    e, idx = env
    c = parse_string('GroupBy(Rows(ak), Rows(b), Rows(ck), previous=["la", 0, "ha"])').calls[0]
    e.executor._translate_group_by("i", idx, c)
    prev = c.args["previous"]
    assert len(prev) == 3 and all(isinstance(v, int) for v in prev)


@pytest.mark.parametrize("pql,err", [
    ("GroupBy(Rows(notfound), previous=1)", "'previous' argument must be list"),
    ('GroupBy(Rows(ak), previous=["la", 0])', "mismatched lengths"),
    ("GroupBy(Rows(ak), previous=[1])", "prev value must be a string"),
    ("GroupBy(Rows(notfound), previous=[1])", str(ErrFieldNotFound)),
    ('GroupBy(Rows(b), previous=["la"])', "which doesn't use string keys")])
def test_translate_group_by_errors(env, pql, err):
    e, idx = env
    c = parse_string(pql).calls[0]
    with pytest.raises(PilosaError) as ei:
        e.executor._translate_group_by("i", idx, c)
    assert err in str(ei.value)


def test_field_row_json():  # TestFieldRowMarshalJSON
    from pilosa_amd.utils import gojson
    assert gojson.dumps(FieldRow("blah", 0, "ha").to_json()) == '{"field":"blah","rowKey":"ha"}'
    assert gojson.dumps(FieldRow("blah", 2).to_json()) == '{"field":"blah","rowID":2}'
