"""Auxiliary subsystems: background snapshots, translate replication + key
forwarding, TLS, diagnostics, GC notifier, system info."""
import gc
import http.server
import json
import os
import subprocess
import tempfile
import threading
import time

import numpy as np
import pytest

from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger
from tests.helpers import SW, Env


def test_background_snapshot_queue():
    env = Env(max_opn=50)
    try:
        env.create_index("i")
        env.field("i", "f")
        for c in range(400):
            env.q("i", f"Set({c}, f=1)")
        q = env.holder.snapshot_queue
        q.drain()
        frag = env.holder.fragment("i", "f", "standard", 0)
        assert q.done >= 1
        assert frag.opn <= 50
        env.reopen()
        assert env.q1("i", "Count(Row(f=1))") == 400
    finally:
        env.close()


def test_translate_ids_are_dense_and_fast():
    from pilosa_amd.models.translate import TranslateFile
    ts = TranslateFile(None).open()
    t0 = time.time()
    ids = ts.translate_columns_to_uint64("i", [f"k{i}" for i in range(50000)])
    assert ids == list(range(1, 50001))
    assert time.time() - t0 < 5
    assert ts.translate_rows_to_uint64("i", "f", ["a", "b", "a"]) == [1, 2, 1]


def test_translate_replica_tails_primary_and_forwards():
    primary = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    replica = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(),
                     translation_primary_url=str(primary.uri)).open()
    try:
        pt = primary.holder.translate
        ids = pt.translate_columns_to_uint64("i", ["a", "b", "c"])
        rt = replica.holder.translate
        deadline = time.time() + 10
        while rt.column_key_id("i", "c") is None and time.time() < deadline:
            time.sleep(0.1)
        assert [rt.column_key_id("i", k) for k in "abc"] == ids
        # unknown key on the replica: resolved by the primary, not minted locally
        got = rt.translate_columns_to_uint64("i", ["zz"])
        assert got == [pt.column_key_id("i", "zz")] == [4]
        deadline = time.time() + 10
        while rt.size < pt.size and time.time() < deadline:
            time.sleep(0.1)
        assert rt.read_from(0) == pt.read_from(0)  # byte-identical log copy
    finally:
        replica.close()
        primary.close()


def test_tls_server_and_client(tmp_path):
    key, crt = tmp_path / "k.pem", tmp_path / "c.pem"
    r = subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                        str(crt), "-days", "1", "-subj", "/CN=127.0.0.1"], capture_output=True)
    if r.returncode != 0:
        pytest.skip("openssl could not create a certificate")
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(),
               tls_certificate=str(crt), tls_key=str(key)).open()
    try:
        assert s.uri.scheme == "https"
        c = InternalClient(skip_verify=True)
        assert c.version(s.uri)
        c.create_index(s.uri, "i")
        assert [i["name"] for i in c.schema(s.uri)] == ["i"]
    finally:
        s.close()


def test_diagnostics_posts_document():
    got = []

    class H(http.server.BaseHTTPRequestHandler):
        def do_POST(self):
            got.append(json.loads(self.rfile.read(int(self.headers["Content-Length"]))))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    httpd = http.server.HTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=httpd.serve_forever, daemon=True)
    t.start()
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(),
               diagnostics_host=f"http://127.0.0.1:{httpd.server_address[1]}/", diagnostics_interval=3600).open()
    try:
        s.api.create_index("i")
        s._refresh_diagnostics()
        assert s.diagnostics.flush()
        doc = got[-1]
        assert doc["NumIndexes"] == 1 and doc["Version"].startswith("v") and doc["CPULogicalCores"] > 0
        assert s.diagnostics.check_version("v99.0.0") and not s.diagnostics.check_version("v0.1.0")
    finally:
        s.close()
        httpd.shutdown()


def test_gc_notifier_counts_collections():
    from pilosa_amd.utils.gcnotify import GCNotifier
    from pilosa_amd.utils.stats import ExpvarStatsClient
    st = ExpvarStatsClient()
    n = GCNotifier(st).start()
    try:
        gc.collect()
        assert n.collections >= 1
        assert n.flush() >= 1
        assert st.expvar()["garbage_collection"] >= 1
        # a collection triggered while the registry lock is held must not
        # deadlock (the callback takes no lock)
        with st.reg.mu:
            gc.collect()
        assert n.flush() >= 1
    finally:
        n.stop()


def test_sysinfo():
    from pilosa_amd.utils.sysinfo import SystemInfo
    d = SystemInfo().to_dict()
    assert d["cpuLogicalCores"] > 0 and d["memory"] > 0 and d["platform"] == "linux"
