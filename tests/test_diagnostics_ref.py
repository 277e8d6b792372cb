"""Reference diagnostics_internal_test.go, ported (4 tests): the collected
document before and after a flush, version parsing and comparison, and the
version check against a release endpoint."""
import http.server
import json
import threading

from pilosa_amd.utils.diagnostics import DiagnosticsCollector, version_segments
from pilosa_amd.utils.logger import CaptureLogger


def _serve(handler_body):
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            self.send_response(200)
            self.end_headers()
            self.wfile.write(handler_body)

        def do_POST(self):
            self.rfile.read(int(self.headers.get("Content-Length", 0)))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass
    srv = http.server.HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def test_diagnostics_client():                  # TestDiagnosticsClient
    srv = _serve(b"")
    try:
        d = DiagnosticsCollector(f"http://127.0.0.1:{srv.server_port}")
        d.set("gg", 10)
        d.set("ss", "ss")
        d.set("empty", "")                      # empty strings are skipped
        assert json.loads(d.encode()) == {"gg": 10, "ss": "ss"}
        assert d.flush()
        assert json.loads(d.encode()) == {"gg": 10, "ss": "ss", "Uptime": 0}
    finally:
        srv.shutdown()


def test_diagnostics_version_parse():           # TestDiagnosticsVersion_Parse
    assert version_segments("0.1.1") == [0, 1, 1]
    assert version_segments("v1.3.0-rc2") == [1, 3, 0]


def test_diagnostics_version_compare():         # TestDiagnosticsVersion_Compare
    d = DiagnosticsCollector("localhost:10101")
    d.set_version("v0.1.1")
    assert "a newer version" in d.compare_version("v1.7.0")
    assert "a newer version" in d.compare_version("1.7.0")
    assert "the latest minor release is" in d.compare_version("0.7.0")
    assert "there is a new patch release of Pilosa" in d.compare_version("0.1.2")
    assert d.compare_version("0.1.1") is None
    d.set_version("v1.7.0")
    assert d.compare_version("0.7.2") is None   # the local version is greater


def test_diagnostics_version_check():           # TestDiagnosticsVersion_Check
    srv = _serve(json.dumps({"version": "1.1.1"}).encode())
    try:
        logs = CaptureLogger()
        d = DiagnosticsCollector("localhost:10101", logger=logs)
        d.set_version("0.1.1")
        d.version_url = f"http://127.0.0.1:{srv.server_port}/version"
        d.check_version_url()
        assert len(logs.prints) == 1 and "a newer version" in logs.prints[0]
        d.check_version_url()                   # same release again: no second message
        assert len(logs.prints) == 1
    finally:
        srv.shutdown()
