"""CLI: import / export / check / inspect / config (reference ctl/*_test.go)."""
import io
import os
import tempfile

from pilosa_amd.cli.main import main
from pilosa_amd.server.config import Config, parse_duration
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger

SAMPLE = "/root/reference/testdata/sample_view/0"


def test_generate_and_resolve_config(monkeypatch):
    out = io.StringIO()
    assert main(["generate-config"], stdout=out) == 0
    assert 'bind = ":10101"' in out.getvalue() and "[cluster]" in out.getvalue()
    d = tempfile.mkdtemp()
    p = os.path.join(d, "c.toml")
    with open(p, "w") as fh:
        fh.write('bind = ":2000"\n[cluster]\nreplicas = 2\n[gpu]\nmode = "off"\n')
    monkeypatch.setenv("PILOSA_CLUSTER_REPLICAS", "3")
    out = io.StringIO()
    assert main(["config", "-c", p, "--max-writes-per-request", "7"], stdout=out) == 0
    s = out.getvalue()
    assert 'bind = ":2000"' in s and "replicas = 3" in s and "max-writes-per-request = 7" in s
    bad = os.path.join(d, "bad.toml")
    with open(bad, "w") as fh:
        fh.write("nope = 1\n")
    try:
        Config().load_toml(bad)
        raise AssertionError("unknown key accepted")
    except ValueError:
        pass
    assert parse_duration("1m30s") == 90 and parse_duration("500ms") == 0.5 and parse_duration("10m0s") == 600


def test_check_and_inspect(tmp_path):
    out = io.StringIO()
    if os.path.exists(SAMPLE):
        assert main(["check", SAMPLE], stdout=out) == 0
        assert out.getvalue().strip().endswith(": ok")
        out = io.StringIO()
        assert main(["inspect", SAMPLE, "--limit", "3"], stdout=out) == 0
        assert "Containers: 14207" in out.getvalue()
    bad = tmp_path / "bad"
    bad.write_bytes(b"\x3c\x30\x00\x00\xff\xff\xff\x7f")
    out = io.StringIO()
    assert main(["check", str(bad)], stdout=out) == 1


def test_import_export_roundtrip(tmp_path):
    srv = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    try:
        host = srv.uri.host_port()
        csvp = tmp_path / "bits.csv"
        csvp.write_text("1,10\n1,20\n2,1048580\n3,5\n")
        err = io.StringIO()
        assert main(["import", "--host", host, "-i", "i", "-f", "f", "--create-schema", "--sort", str(csvp)],
                    stderr=err) == 0, err.getvalue()
        out = io.StringIO()
        assert main(["export", "--host", host, "-i", "i", "-f", "f"], stdout=out) == 0
        assert sorted(out.getvalue().split()) == sorted(["1,10", "1,20", "2,1048580", "3,5"])
        vals = tmp_path / "vals.csv"
        vals.write_text("1,5\n2,-7\n")
        assert main(["import", "--host", host, "-i", "i", "-f", "v", "--create-schema", "--field-type", "int",
                     "--field-min", "-100", "--field-max", "100", str(vals)], stderr=err) == 0, err.getvalue()
        from pilosa_amd.server.client import InternalClient
        r = InternalClient().query(srv.uri, "i", "Sum(field=v) Count(Row(f=1))")
        assert r["results"] == [{"value": -2, "count": 2}, 2]
    finally:
        srv.close()
