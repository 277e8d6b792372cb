"""Fault injection (reference internal/clustertests: pumba pauses a node for
10 s, then counts are asserted).  Three server processes, ReplicaN=2: SIGSTOP
one node, the coordinator marks it DOWN and queries keep returning exact
results from the replicas; SIGCONT brings it back READY."""
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

import pytest

from pilosa_amd.shardwidth import SHARD_WIDTH as SW  # noqa: E402
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from tests.helpers import free_port
    return free_port()


def _req(port, method, path, body=None, timeout=30):
    data = body.encode() if isinstance(body, str) else (json.dumps(body).encode() if body is not None else None)
    r = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=data, method=method)
    with urllib.request.urlopen(r, timeout=timeout) as resp:
        return json.loads(resp.read() or b"null")


def _wait(cond, timeout=60, what=""):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if cond():
                return
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.2)
    raise TimeoutError(what)


@pytest.mark.slow
def test_paused_node_failover():
    ports = [_port() for _ in range(3)]
    procs = []
    try:
        for i, p in enumerate(ports):
            args = [sys.executable, "-m", "pilosa_amd", "server", "--data-dir", tempfile.mkdtemp(prefix=f"fault{i}_"),
                    "--bind", f"127.0.0.1:{p}", "--gpu.mode", "off", "--cluster.replicas", "2",
                    "--cluster.hosts", f"127.0.0.1:{ports[0]}", "--gossip.probe-interval", "200ms",
                    "--anti-entropy.interval", "0s"]
            if i == 0:
                args += ["--cluster.coordinator", "true"]
            procs.append(subprocess.Popen(args, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                          start_new_session=True))
            _wait(lambda p=p: _req(p, "GET", "/version"), what=f"server {i} up")
        _wait(lambda: len(_req(ports[0], "GET", "/status")["nodes"]) == 3 and
              _req(ports[0], "GET", "/status")["state"] == "NORMAL", what="cluster NORMAL")
        _req(ports[0], "POST", "/index/i", {"options": {}})
        _req(ports[0], "POST", "/index/i/field/f", {"options": {}})
        time.sleep(0.5)
        cols = [s * SW + s for s in range(12)]
        _req(ports[0], "POST", "/index/i/query", " ".join(f"Set({c}, f=1)" for c in cols))
        assert _req(ports[0], "POST", "/index/i/query", "Count(Row(f=1))")["results"] == [12]

        os.kill(procs[2].pid, signal.SIGSTOP)  # pause node 2 (like `pumba pause`)
        _wait(lambda: any(n["state"] == "DOWN" for n in _req(ports[0], "GET", "/status")["nodes"]),
              timeout=30, what="paused node marked DOWN")
        for _ in range(3):
            assert _req(ports[0], "POST", "/index/i/query", "Count(Row(f=1))")["results"] == [12]
            assert _req(ports[0], "POST", "/index/i/query", "Row(f=1)")["results"][0]["columns"] == cols

        os.kill(procs[2].pid, signal.SIGCONT)
        _wait(lambda: all(n["state"] == "READY" for n in _req(ports[0], "GET", "/status")["nodes"]),
              timeout=30, what="node READY again")
        assert _req(ports[0], "POST", "/index/i/query", "Count(Row(f=1))")["results"] == [12]
    except Exception:
        # thread dumps of every node, to tell a stall from a slow machine
        for p in ports:
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{p}/debug/pprof/goroutine?debug=1", timeout=5) as r:
                    print(f"==== node :{p}\n" + r.read().decode()[:20000])
            except Exception as e:  # noqa: BLE001
                print(f"==== node :{p}: {e}")
        raise
    finally:
        for p in procs:
            try:
                os.kill(p.pid, signal.SIGCONT)
                os.killpg(p.pid, signal.SIGTERM)
                p.wait(timeout=20)
            except Exception:  # noqa: BLE001
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except Exception:  # noqa: BLE001
                    pass
