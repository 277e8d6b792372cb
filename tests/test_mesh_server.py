"""A multi-process node: ``pilosa_amd server`` under torch.distributed.run
(rank 0 = HTTP front end, rank 1 = shard worker; gloo on the CPU).  Schema
changes, imports and queries go through the normal HTTP API and must match a
single-process server."""
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

import numpy as np
import pytest

SW = 1 << 20
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from tests.helpers import free_port
    return free_port()


def _req(base, method, path, body=None):
    data = body.encode() if isinstance(body, str) else (json.dumps(body).encode() if body is not None else None)
    r = urllib.request.Request(base + path, data=data, method=method)
    with urllib.request.urlopen(r, timeout=60) as resp:
        return json.loads(resp.read() or b"null")


def _wait(base, proc, timeout=120):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited: {proc.returncode}")
        try:
            _req(base, "GET", "/status")
            return
        except Exception:  # noqa: BLE001
            time.sleep(0.5)
    raise TimeoutError("server did not come up")


def _workload(base):
    _req(base, "POST", "/index/i", {"options": {}})
    _req(base, "POST", "/index/i/field/f", {"options": {"cacheType": "ranked", "cacheSize": 100}})
    _req(base, "POST", "/index/i/field/v", {"options": {"type": "int", "min": 0, "max": 1000}})
    rng = np.random.default_rng(2)
    sets = [f"Set({int(rng.integers(0, 4 * SW))}, f={int(rng.integers(0, 4))})" for _ in range(300)]
    sets += [f"Set({int(rng.integers(0, 4 * SW))}, v={int(rng.integers(0, 1000))})" for _ in range(100)]
    _req(base, "POST", "/index/i/query", "".join(sets))
    qs = ["Count(Row(f=1))", "Count(Intersect(Row(f=1), Row(f=2)))", "TopN(f, n=2)", "Sum(field=v)",
          "Max(field=v)", "Rows(f)", "Count(Row(f=0))Count(Row(f=3))", "Row(v > 900)"]
    return [_req(base, "POST", "/index/i/query", q) for q in qs]


def _server(args, env, data):
    cmd = [sys.executable, *args, "-m", "pilosa_amd", "server", "--data-dir", data, "--gpu.mode", "off",
           "--bind", f"127.0.0.1:{env['HTTP_PORT']}"]
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            start_new_session=True)


def _stop(p):
    try:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(timeout=30)
    except Exception:  # noqa: BLE001
        os.killpg(p.pid, signal.SIGKILL)


@pytest.mark.slow
def test_two_rank_server_matches_single():
    results = []
    for mode in ("single", "mesh"):
        env = dict(os.environ)
        env["HTTP_PORT"] = str(_port())
        env.pop("WORLD_SIZE", None)
        data = tempfile.mkdtemp(prefix=f"meshsrv_{mode}_")
        if mode == "mesh":
            args = ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
                    f"--master-port={_port()}"]
            # torch.distributed.run expects a script or -m module after its options
            cmd_args = args
        else:
            cmd_args = []
        p = _server(cmd_args, env, data)
        base = f"http://127.0.0.1:{env['HTTP_PORT']}"
        try:
            _wait(base, p)
            results.append(_workload(base))
            if mode == "mesh":
                assert os.path.isdir(os.path.join(data, ".rank1", "i")), "rank 1 holds no shards"
        finally:
            _stop(p)
    assert results[0] == results[1]
