"""Ported expectations of the reference's http/handler_internal_test.go:
create-index and create-field request decoding and per-type option
validation, checked through the HTTP API (status + error message)."""
import json
import tempfile

import pytest

from pilosa_amd.models.field import DEFAULT_CACHE_SIZE, FieldOptions
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger
from tests.test_server import _req


@pytest.fixture(scope="module")
def srv():
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    yield s
    s.close()


@pytest.mark.parametrize("k,body,exp,err", [
    (0, '{"options": {}}', (False, True), ""),
    (1, '{"options": {"trackExistence": false}}', (False, False), ""),
    (2, '{"options": {"keys": true}}', (True, True), ""),
    (3, '{"options": 4}', None, "options is not map[string]interface{}"),
    (4, '{"option": {}}', None, "unknown key: option:map[]"),
    (5, '{"options": {"badKey": "test"}}', None, "unknown key: badKey:test")])
def test_post_index_request(srv, k, body, exp, err):  # TestPostIndexRequestUnmarshalJSON :13
    name = f"pidx{k}"
    st, out = _req(srv, "POST", f"/index/{name}", body.encode())
    if err:
        assert st == 400 and json.loads(out)["error"]["message"] == err
        return
    assert st == 200, out
    idx = srv.holder.index(name)
    assert (idx.keys, idx.track_existence) == exp


@pytest.mark.parametrize("k,body,exp,err", [
    (0, '{"options": {}}', {"type": "set", "cacheType": "ranked", "cacheSize": DEFAULT_CACHE_SIZE}, ""),
    (1, '{"options": 4}', None, "json: cannot unmarshal"),
    (2, '{"option": {}}', None, 'json: unknown field "option"'),
    (3, '{"options": {"badKey": "test"}}', None, 'json: unknown field "badKey"'),
    (4, '{"options": {"inverseEnabled": true}}', None, 'json: unknown field "inverseEnabled"'),
    (5, '{"options": {"inverse": true, "cacheType": "foo"}}', None, 'json: unknown field "inverse"'),
    (6, '{"options": {"type": "set"}}', {"type": "set", "cacheType": "ranked", "cacheSize": DEFAULT_CACHE_SIZE}, ""),
    (7, '{"options": {"type": "set", "cacheType": "lru"}}', {"type": "set", "cacheType": "lru"}, ""),
    (8, '{"options": {"type": "set", "min": 0}}', None, "min does not apply to field type set"),
    (9, '{"options": {"type": "set", "max": 100}}', None, "max does not apply to field type set"),
    (10, '{"options": {"type": "set", "timeQuantum": "YMD"}}', None, "timeQuantum does not apply to field type set"),
    # cases 11/12 list "min/max is required" errors, but the reference's
    # validate() never returns them (its check only fires on an error) and its
    # handler fills absent bounds with MinInt64/MaxInt64 (http/handler.go:774,
    # server/handler_test.go "Query int field unbounded" :546): unbounded here
    (11, '{"options": {"type": "int"}}', {"type": "int", "min": -2 ** 63, "max": 2 ** 63 - 1}, ""),
    (12, '{"options": {"type": "int", "min": 0}}', {"type": "int", "min": 0, "max": 2 ** 63 - 1}, ""),
    (13, '{"options": {"type": "int", "min": 0, "max": 1000}}', {"type": "int", "min": 0, "max": 1000}, ""),
    (14, '{"options": {"type": "int", "min": 0, "max": 1000, "cacheType": "ranked"}}', None,
     "cacheType does not apply to field type int"),
    (15, '{"options": {"type": "int", "min": 0, "max": 1000, "cacheSize": 1000}}', None,
     "cacheSize does not apply to field type int"),
    (16, '{"options": {"type": "int", "min": 0, "max": 1000, "timeQuantum": "YMD"}}', None,
     "timeQuantum does not apply to field type int"),
    (17, '{"options": {"type": "time"}}', None, "timeQuantum is required for field type time"),
    (18, '{"options": {"type": "time", "timeQuantum": "YMD"}}', {"type": "time", "timeQuantum": "YMD"}, ""),
    (19, '{"options": {"type": "time", "timeQuantum": "YMD", "min": 0}}', None, "min does not apply to field type time"),
    (20, '{"options": {"type": "time", "timeQuantum": "YMD", "max": 1000}}', None,
     "max does not apply to field type time"),
    (21, '{"options": {"type": "time", "timeQuantum": "YMD", "cacheType": "ranked"}}', None,
     "cacheType does not apply to field type time"),
    (22, '{"options": {"type": "time", "timeQuantum": "YMD", "cacheSize": 1000}}', None,
     "cacheSize does not apply to field type time")])
def test_post_field_request(srv, k, body, exp, err):  # TestPostFieldRequestUnmarshalJSON :48, TestFieldOptionValidation :95
    if srv.holder.index("fi") is None:
        assert _req(srv, "POST", "/index/fi", b"")[0] == 200
    st, out = _req(srv, "POST", f"/index/fi/field/f{k}", body.encode())
    if err:
        assert st == 400, out
        assert json.loads(out)["error"]["message"].startswith(err)
        return
    assert st == 200, out
    got = srv.holder.field("fi", f"f{k}").options.to_json()
    for key, v in exp.items():
        assert got[key] == v, (key, got)


def test_field_options_from_json_direct():
    with pytest.raises(Exception, match='unknown field "x"'):
        FieldOptions.from_json({"x": 1})
