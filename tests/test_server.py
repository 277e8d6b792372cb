"""HTTP API + multi-node clusters in-process (reference server/*_test.go,
test.MustRunCluster with ModHasher placement)."""
import json
import tempfile
import time
import urllib.request

import numpy as np
import pytest

from pilosa_amd.parallel.cluster import URI, Cluster, Node, fnv64a, jump_hash
from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger

from pilosa_amd.shardwidth import SHARD_WIDTH as SW  # noqa: E402


def _req(srv, method, path, body=b"", headers=None):
    r = urllib.request.Request(f"http://127.0.0.1:{srv.uri.port}{path}", data=body if body else None,
                               method=method, headers=headers or {})
    try:
        with urllib.request.urlopen(r, timeout=10) as resp:
            return resp.status, resp.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()


@pytest.fixture
def srv():
    d = tempfile.mkdtemp()
    s = Server(d, bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    yield s
    s.close()


def test_http_roundtrip(srv):
    assert _req(srv, "POST", "/index/i", b"")[0] == 200
    assert _req(srv, "POST", "/index/i", b"")[0] == 409
    st, body = _req(srv, "POST", "/index/i/field/f", json.dumps({"options": {"type": "set"}}).encode())
    assert st == 200, body
    st, body = _req(srv, "POST", "/index/i/field/n", json.dumps({"options": {"type": "int", "min": 0,
                                                                              "max": 100}}).encode())
    assert st == 200, body
    st, body = _req(srv, "POST", "/index/i/field/bad", json.dumps({"options": {"type": "int",
                                                                                "cacheType": "x"}}).encode())
    assert st == 400
    st, body = _req(srv, "POST", "/index/i/query", f"Set(1, f=10) Set({SW + 3}, f=10) Set(1, n=42)".encode())
    assert st == 200 and json.loads(body) == {"results": [True, True, True]}
    st, body = _req(srv, "POST", "/index/i/query", b"Row(f=10) Count(Row(f=10)) Sum(field=n) TopN(f)")
    res = json.loads(body)["results"]
    assert res[0] == {"attrs": {}, "columns": [1, SW + 3]}
    assert res[1] == 2
    assert res[2] == {"value": 42, "count": 1}
    assert res[3] == [{"id": 10, "count": 2}]
    st, body = _req(srv, "POST", "/index/i/query", b"Row(f=")
    assert st == 400 and "error" in json.loads(body)
    st, body = _req(srv, "GET", "/schema")
    sch = json.loads(body)["indexes"]
    assert sch[0]["name"] == "i" and {f["name"] for f in sch[0]["fields"]} == {"f", "n"}
    assert json.loads(_req(srv, "GET", "/status")[1])["state"] == "NORMAL"
    assert json.loads(_req(srv, "GET", "/version")[1])["version"]
    assert json.loads(_req(srv, "GET", "/internal/shards/max")[1]) == {"standard": {"i": 1}}
    assert _req(srv, "GET", "/index/nope")[0] == 404
    assert _req(srv, "GET", "/index/i/query")[0] == 405
    assert _req(srv, "GET", "/export?index=i&field=f&shard=0", headers={"Accept": "text/csv"})[1] == b"10,1\n"
    assert _req(srv, "POST", "/index/i/query?bogus=1", b"Count(Row(f=1))")[0] == 400
    assert _req(srv, "DELETE", "/index/i/field/f")[0] == 200
    assert _req(srv, "DELETE", "/index/i")[0] == 200


def test_protobuf_query_and_import(srv):
    from pilosa_amd.wire import pb
    c = InternalClient()
    c.create_index(srv.uri, "i")
    c.create_field(srv.uri, "i", "f", {"type": "set"})
    c.import_bits(srv.node, "i", "f", 0, [1, 1, 2], [5, 7, 9])
    c.import_bits(srv.node, "i", "f", 1, [1], [SW + 9])
    res = c.query_node(srv.node, "i", "Count(Row(f=1))", None)
    assert res == [3]
    out = c.query(srv.uri, "i", "Row(f=1)")
    assert out["results"][0]["columns"] == [5, 7, SW + 9]
    st, body = _req(srv, "POST", "/index/i/query", pb.QueryRequest(Query="Row(f=2)").SerializeToString(),
                    {"Content-Type": "application/x-protobuf", "Accept": "application/x-protobuf"})
    m = pb.QueryResponse()
    m.ParseFromString(body)
    assert list(m.Results[0].Row.Columns) == [9]


def test_placement_matches_reference():
    # fnv64a of "" is the offset basis; jump hash fixtures
    assert fnv64a(b"") == 0xcbf29ce484222325
    assert [jump_hash(k, 10) for k in range(5)] == [jump_hash(k, 10) for k in range(5)]
    assert all(0 <= jump_hash(k, 7) < 7 for k in range(1000))
    # partition spread
    c = Cluster(Node("a", URI()), replica_n=2)
    c.set_nodes([Node("a", URI()), Node("b", URI()), Node("c", URI())])
    owners = [tuple(n.id for n in c.shard_nodes("i", s)) for s in range(64)]
    assert all(len(o) == 2 and o[0] != o[1] for o in owners)
    assert len({o[0] for o in owners}) == 3


def _cluster(n, replicas=1):
    servers = []
    coord = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", node_id="node0", gpu="off", replica_n=replicas,
                   hosts=[], coordinator=True, probe_interval=0.2, logger=CaptureLogger(), hasher="mod")
    coord.hosts = [URI.parse("127.0.0.1:1")]  # enable membership loop
    coord.open()
    servers.append(coord)
    for i in range(1, n):
        s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", node_id=f"node{i}", gpu="off", replica_n=replicas,
                   coordinator=False, coordinator_uri=coord.uri.normalize(), probe_interval=0.2,
                   logger=CaptureLogger(), hasher="mod").open()
        servers.append(s)
    deadline = time.time() + 10
    while time.time() < deadline:
        if all(len(s.cluster.nodes) == n and s.cluster.state == "NORMAL" for s in servers):
            break
        time.sleep(0.05)
    return servers


def test_three_node_cluster_queries():
    servers = _cluster(3)
    try:
        s0 = servers[0]
        c = InternalClient()
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set"})
        time.sleep(0.2)
        assert all(s.holder.field("i", "f") is not None for s in servers)
        cols = [1, SW + 2, 2 * SW + 3, 3 * SW + 4, 4 * SW + 5]
        q = " ".join(f"Set({col}, f=7)" for col in cols)
        assert c.query(s0.uri, "i", q)["results"] == [True] * 5
        # data is spread over nodes by placement
        owners = {s.node.id: sorted(s.holder.field("i", "f").view("standard").fragments) for s in servers}
        assert sum(len(v) for v in owners.values()) == 5 and sum(1 for v in owners.values() if v) >= 2
        for s in servers:
            assert c.query(s.uri, "i", "Count(Row(f=7))")["results"] == [5]
            assert c.query(s.uri, "i", "Row(f=7)")["results"][0]["columns"] == cols
        assert c.query(servers[1].uri, "i", "TopN(f, n=1)")["results"][0] == [{"id": 7, "count": 5}]
    finally:
        for s in servers:
            s.close()


def test_replication_and_failover():
    servers = _cluster(2, replicas=2)
    try:
        s0, s1 = servers
        c = InternalClient()
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set"})
        time.sleep(0.2)
        c.query(s0.uri, "i", f"Set(1, f=3) Set({SW + 1}, f=3)")
        for s in servers:  # both replicas hold every shard
            assert sorted(s.holder.field("i", "f").view("standard").fragments) == [0, 1]
        # make a replica diverge and repair it with anti-entropy
        s1.holder.fragment("i", "f", "standard", 0).set_bit(9, 5)
        s0.sync_holder()
        assert s0.holder.fragment("i", "f", "standard", 0).bit(9, 5) in (True, False)
        assert s0.holder.fragment("i", "f", "standard", 0).row_count(9) == \
            s1.holder.fragment("i", "f", "standard", 0).row_count(9)
    finally:
        for s in servers:
            s.close()


def test_anti_entropy_pass_aborts_when_resize_begins():
    """holderSyncer stops mid-pass once the cluster leaves NORMAL
    (cluster.go:253-275,465): a diverged replica is left alone while the
    cluster is RESIZING and repaired by the next pass in NORMAL."""
    from pilosa_amd.parallel.cluster import STATE_NORMAL, STATE_RESIZING
    servers = _cluster(2, replicas=2)
    try:
        s0, s1 = servers
        c = InternalClient()
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set"})
        time.sleep(0.2)
        c.query(s0.uri, "i", "Set(1, f=3)")
        s1.holder.fragment("i", "f", "standard", 0).set_bit(9, 5)
        s0.cluster.set_state(STATE_RESIZING)
        assert s0.sync_holder() is False
        assert s0.holder.fragment("i", "f", "standard", 0).row_count(9) == 0
        s0.cluster.set_state(STATE_NORMAL)
        assert s0.sync_holder() is True
        assert s0.holder.fragment("i", "f", "standard", 0).row_count(9) == \
            s1.holder.fragment("i", "f", "standard", 0).row_count(9) == 1
    finally:
        for s in servers:
            s.close()
