"""Ported expectations of the reference's ctl/import_test.go: the CSV
import command against an in-process server (set, clear, int values, keys,
key replication over two nodes, invalid files, value overwrite, bool
fields).  Each test names the reference test it ports."""
import io
import json
import tempfile
import time
import urllib.request

import pytest

from pilosa_amd.cli.main import main
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger

pytestmark = pytest.mark.timeout(120)


@pytest.fixture
def srv():
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    yield s
    s.close()


def _host(s):
    return f"127.0.0.1:{s.uri.port}"


def _post(s, path, body=""):
    req = urllib.request.Request(f"http://{_host(s)}{path}", data=body.encode(), method="POST",
                                 headers={"Accept": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return r.read().decode()


def _csv(text):
    f = tempfile.NamedTemporaryFile("w", suffix=".csv", delete=False)
    f.write(text)
    f.close()
    return f.name


def _run(s, *args):
    out, err = io.StringIO(), io.StringIO()
    rc = main(["import", "--host", _host(s) if s else "127.0.0.1:1", *args], out, err)
    return rc, err.getvalue()


def test_import_validation():  # TestImportCommand_Validation
    rc, err = _run(None)
    assert rc != 0 and "index required" in err
    rc, err = _run(None, "-i", "i")
    assert rc != 0 and "field required" in err
    rc, err = _run(None, "-i", "i", "-f", "f")
    assert rc != 0 and "path required" in err


@pytest.mark.parametrize("clear", [False, True])
def test_import_basic(srv, clear):  # TestImportCommand_Basic (set, clear)
    rc, err = _run(srv, "-i", "i", "-f", "f", "--create-schema", *(["--clear"] if clear else []), _csv("1,2\n3,4\n5,6"))
    assert rc == 0, err
    got = json.loads(_post(srv, "/index/i/query", "Count(Row(f=1)) Count(Row(f=3))"))["results"]
    assert got == ([0, 0] if clear else [1, 1])


@pytest.mark.parametrize("clear", [False, True])
def test_import_run_value(srv, clear):  # TestImportCommand_RunValue (set, clear)
    _post(srv, "/index/i")
    _post(srv, "/index/i/field/f", '{"options":{"type": "int", "min": 0, "max": 100}}')
    rc, err = _run(srv, "-i", "i", "-f", "f", _csv("1,2\n3,4\n5,6"))
    assert rc == 0, err
    if clear:
        rc, err = _run(srv, "-i", "i", "-f", "f", "--clear", _csv("1,2\n3,4\n5,6"))
        assert rc == 0, err
    got = json.loads(_post(srv, "/index/i/query", "Sum(field=f)"))["results"][0]
    assert got == ({"value": 0, "count": 0} if clear else {"value": 12, "count": 3})


def test_import_run_keys(srv):  # TestImportCommand_RunKeys
    _post(srv, "/index/i", '{"options":{"keys": true}}')
    _post(srv, "/index/i/field/f", '{"options":{"keys": true}}')
    rc, err = _run(srv, "-i", "i", "-f", "f", _csv("foo1,bar2\nfoo3,bar4\nfoo5,bar6"))
    assert rc == 0, err
    assert json.loads(_post(srv, "/index/i/query", "Row(f=foo3)"))["results"][0]["keys"] == ["bar4"]


def test_import_key_replication():  # TestImportCommand_KeyReplication
    from tests.test_server_ref import _Cluster
    cl = _Cluster(2)
    try:
        s0 = cl.nodes[0]
        _post(s0, "/index/i", '{"options":{"keys": true}}')
        _post(s0, "/index/i/field/f", '{"options":{"keys": true}}')
        time.sleep(0.2)
        rows = "".join(f"foo{r},bar{c}\n" for r in range(100) for c in range(100)) + "fooEND,barEND"
        rc, err = _run(s0, "-i", "i", "-f", "f", _csv(rows))
        assert rc == 0, err
        for s in cl.nodes:
            assert json.loads(_post(s, "/index/i/query", "Count(Row(f=foo0))")) == {"results": [100]}
    finally:
        cl.close()


def test_import_run_value_keys(srv):  # TestImportCommand_RunValueKeys
    _post(srv, "/index/i", '{"options":{"keys": true}}')
    _post(srv, "/index/i/field/f", '{"options":{"type": "int", "min": 0, "max": 100}}')
    rc, err = _run(srv, "-i", "i", "-f", "f", _csv("foo1,2\nfoo3,4\nfoo5,6"))
    assert rc == 0, err
    assert json.loads(_post(srv, "/index/i/query", "Sum(field=f)"))["results"][0] == {"value": 12, "count": 3}


def test_import_invalid_file(srv):  # TestImportCommand_InvalidFile
    _post(srv, "/index/i")
    _post(srv, "/index/i/field/f")
    for text, msg in (("a,2\n3,5\n5,6", "invalid row id on row"), ("1,\n3,\n5,6", "invalid column id on row"),
                      ("1,2,34343\n1,3,54565,\n5,6,565", "invalid timestamp on row"),
                      ("1\n3\n5", "bad column count on row")):
        rc, err = _run(srv, "-i", "i", "-f", "f", _csv(text))
        assert rc != 0 and msg in err, (text, err)


def test_import_bug_overwrite_value(srv):  # TestImportCommand_BugOverwriteValue
    _post(srv, "/index/i")
    _post(srv, "/index/i/field/f", '{"options":{"type": "int", "min": 0, "max":2147483648 }}')
    for v in (17, 16, 19):
        rc, err = _run(srv, "-i", "i", "-f", "f", _csv(f"0,{v}\n"))
        assert rc == 0, err
        assert json.loads(_post(srv, "/index/i/query", "Sum(field=f)"))["results"][0] == {"value": v, "count": 1}


def test_import_run_bool(srv):  # TestImportCommand_RunBool (Valid, Invalid)
    _post(srv, "/index/i")
    _post(srv, "/index/i/field/f", '{"options":{"type": "bool"}}')
    rc, err = _run(srv, "-i", "i", "-f", "f", _csv("0,1\n1,2\n1,3"))
    assert rc == 0, err
    assert json.loads(_post(srv, "/index/i/query", "Count(Row(f=true))"))["results"] == [2]
    rc, err = _run(srv, "-i", "i", "-f", "f", _csv("0,1\n1,2\n1,3\n2,4"))
    assert rc != 0 and "bool field imports only support values 0 and 1" in err
