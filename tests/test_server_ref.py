"""Ported expectations of the reference's server/server_test.go (in-process
servers and clusters; the reference's test.MustRunCommand / MustRunCluster
become pilosa_amd.server.Server instances on loopback ports).  Each test
names the reference test (and line) it ports."""
import json
import os
import random
import tempfile
import threading
import time
import urllib.request

import pytest

from pilosa_amd.parallel.cluster import URI
from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.config import Config
from pilosa_amd.server.server import Server
from pilosa_amd.shardwidth import SHARD_WIDTH as SW
from pilosa_amd.utils.logger import CaptureLogger

pytestmark = pytest.mark.timeout(180)


def _free_port():
    from tests.helpers import free_port
    return free_port()


def _query(srv, q, params=""):
    """Raw HTTP JSON response text of POST /index/i/query (the reference's
    m.Query(index, rawQuery, query))."""
    url = f"http://127.0.0.1:{srv.uri.port}/index/i/query" + (f"?{params}" if params else "")
    req = urllib.request.Request(url, data=q.encode(), method="POST")
    with urllib.request.urlopen(req, timeout=30) as r:
        return r.read().decode()


def _single(data_dir=None, port=0):
    return Server(data_dir or tempfile.mkdtemp(), bind=f"127.0.0.1:{port}", gpu="off", logger=CaptureLogger()).open()


def _reopen(srv):
    d, port = srv.data_dir, srv.uri.port
    srv.close()
    return _single(d, port)


def _wait(cond, timeout=20.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if cond():
            return True
        time.sleep(0.05)
    return cond()


class _Cluster:
    """n in-process servers with fixed ports and data dirs, so a node can be
    closed and started again with the same configuration."""

    def __init__(self, n, replicas=1):
        self.n, self.replicas = n, replicas
        self.ports = [_free_port() for _ in range(n)]
        self.dirs = [tempfile.mkdtemp(prefix=f"srvref{i}_") for i in range(n)]
        self.nodes = [None] * n
        for i in range(n):
            self.start(i)
        assert _wait(lambda: all(s.cluster.state == "NORMAL" and len(s.cluster.nodes) == n for s in self.nodes)), \
            [(s.cluster.state, len(s.cluster.nodes)) for s in self.nodes]

    def start(self, i):
        coord = i == 0
        s = Server(self.dirs[i], bind=f"127.0.0.1:{self.ports[i]}", node_id=f"node{i}", gpu="off",
                   replica_n=self.replicas, coordinator=coord,
                   coordinator_uri=None if coord else URI.parse(f"127.0.0.1:{self.ports[0]}").normalize(),
                   probe_interval=0.2, logger=CaptureLogger(), hasher="mod", anti_entropy_interval=0)
        if coord:
            s.hosts = [URI.parse("127.0.0.1:1")]   # enable the membership loop
        self.nodes[i] = s.open()
        return self.nodes[i]

    def stop(self, i):
        self.nodes[i].close()

    def close(self):
        for s in self.nodes:
            try:
                s.close()
            except Exception:  # noqa: BLE001
                pass


def _state(s):
    return s.api.state()


# ---------------------------------------------------------------- single node
def test_main_set_quick():  # TestMain_Set_Quick :49
    rng = random.Random(3)
    for _ in range(3):
        cmds = [(rng.randrange(1000), rng.randrange(10)) for _ in range(rng.randrange(1, 300))]
        m = _single()
        try:
            c = InternalClient()
            c.create_index(m.uri, "i")
            c.create_field(m.uri, "i", "x", {"type": "set"})
            for row, col in cmds:
                _query(m, f"Set({col}, x={row})")
            want = {}
            for row, col in set(cmds):
                want.setdefault(row, []).append(col)
            for k in range(2):
                for row, cols in want.items():
                    exp = json.dumps({"results": [{"attrs": {}, "columns": sorted(cols)}]})
                    assert json.loads(_query(m, f"Row(x={row})")) == json.loads(exp)
                if k == 0:
                    m = _reopen(m)
        finally:
            m.close()


def test_main_set_row_attrs():  # TestMain_SetRowAttrs :130
    m = _single()
    try:
        c = InternalClient()
        c.create_index(m.uri, "i")
        for f in ("x", "z", "neg"):
            c.create_field(m.uri, "i", f, {"type": "set"})
        for q in ("Set(100, x=1)", "Set(100, x=2)", "Set(100, x=2)", "Set(100, neg=3)",
                  "SetRowAttrs(x, 1, x=100)", "SetRowAttrs(x, 2, x=-200)", "SetRowAttrs(z, 2, x=300)",
                  "SetRowAttrs(neg, 3, x=-0.44)"):
            _query(m, q)
        assert json.loads(_query(m, "Row(x=1)")) == {"results": [{"attrs": {"x": 100}, "columns": [100]}]}
        assert json.loads(_query(m, "Row(x=2)")) == {"results": [{"attrs": {"x": -200}, "columns": [100]}]}
        m = _reopen(m)
        assert json.loads(_query(m, "Row(x=1)", "columnAttrs=true")) == \
            {"results": [{"attrs": {"x": 100}, "columns": [100]}]}
        assert json.loads(_query(m, "Row(neg=3)", "columnAttrs=true")) == \
            {"results": [{"attrs": {"x": -0.44}, "columns": [100]}]}
        assert json.loads(_query(m, "Row(x=2)")) == {"results": [{"attrs": {"x": -200}, "columns": [100]}]}
    finally:
        m.close()


def test_main_set_column_attrs():  # TestMain_SetColumnAttrs :207
    m = _single()
    try:
        c = InternalClient()
        c.create_index(m.uri, "i")
        c.create_field(m.uri, "i", "x", {"type": "set"})
        for q in ("Set(100, x=1)", "Set(101, x=1)", 'SetColumnAttrs(100, foo="bar")'):
            _query(m, q)
        exp = {"results": [{"attrs": {}, "columns": [100, 101]}], "columnAttrs": [{"id": 100, "attrs": {"foo": "bar"}}]}
        assert json.loads(_query(m, "Row(x=1)", "columnAttrs=true")) == exp
        m = _reopen(m)
        assert json.loads(_query(m, "Row(x=1)", "columnAttrs=true")) == exp
    finally:
        m.close()


def test_main_group_by_keys():  # TestMain_GroupBy :250
    m = _single()
    try:
        c = InternalClient()
        c.create_index(m.uri, "i")
        c.create_field(m.uri, "i", "generalk", {"type": "set", "keys": True})
        c.create_field(m.uri, "i", "subk", {"type": "set", "keys": True})
        _query(m, """
            Set(0, generalk="ten") Set(1, generalk="ten") Set(1001, generalk="ten")
            Set(2, generalk="eleven") Set(1002, generalk="eleven")
            Set(2, generalk="twelve") Set(1002, generalk="twelve")
            Set(0, subk="one-hundred") Set(1, subk="one-hundred") Set(3, subk="one-hundred")
            Set(1001, subk="one-hundred") Set(2, subk="one-hundred-ten") Set(0, subk="one-hundred-ten")""")
        got = json.loads(_query(m, "GroupBy(Rows(generalk), Rows(subk))"))["results"][0]
        groups = sorted(((g["group"][0]["rowKey"], g["group"][1]["rowKey"], g["count"]) for g in got))
        assert groups == sorted([("ten", "one-hundred", 3), ("ten", "one-hundred-ten", 1),
                                 ("eleven", "one-hundred-ten", 1), ("twelve", "one-hundred-ten", 1)])
        assert all(g["group"][0]["field"] == "generalk" and g["group"][1]["field"] == "subk" for g in got)
    finally:
        m.close()


def test_config_parse_host_and_data_dir(tmp_path):  # TestConfig_Parse_Host :304, TestConfig_Parse_DataDir :313
    p = tmp_path / "c.toml"
    p.write_text('bind = "local"\n')
    c = Config()
    c.load_toml(str(p))
    assert c.get("bind") == "local"
    p.write_text('data-dir = "/tmp/foo"\n')
    c = Config()
    c.load_toml(str(p))
    assert c.get("data-dir") == "/tmp/foo"


@pytest.mark.parametrize("no_standard", [False, True])
def test_main_import_timestamp(no_standard):  # TestMain_ImportTimestamp :682, ...NoStandardView :734
    m = _single()
    try:
        name = "f-no-standard" if no_standard else "f"
        m.api.create_index("i")
        from pilosa_amd.models.field import FieldOptions
        m.api.create_field("i", name, FieldOptions(type="time", time_quantum="YMD", no_standard_view=no_standard))
        m.api.import_bits("i", name, 0, row_ids=[1, 2], col_ids=[1, 2],
                          timestamps=[1514764800000000000, 1577833200000000000])
        views = sorted(os.listdir(os.path.join(m.data_dir, "i", name, "views")))
        exp = ["standard_2018", "standard_201801", "standard_20180101", "standard_2019", "standard_201912",
               "standard_20191231"]
        assert views == sorted(exp if no_standard else ["standard"] + exp)
    finally:
        m.close()


# ---------------------------------------------------------------- clusters
def test_main_recalculate_hashes():  # TestMain_RecalculateHashes :321
    cl = _Cluster(5)
    try:
        c = InternalClient()
        c.create_index(cl.nodes[0].uri, "i")
        c.create_field(cl.nodes[0].uri, "i", "f", {"type": "set"})
        time.sleep(0.2)
        _query(cl.nodes[0], "".join(f"Set({col}, f={row})" for row in range(1, 10) for col in range(1, 100)))
        cl.nodes[0].api.recalculate_caches()
        want = sorted([{"id": r, "count": 99} for r in range(1, 10)], key=lambda p: p["id"])
        for s in cl.nodes:
            got = json.loads(_query(s, "TopN(f)"))["results"][0]
            assert sorted(got, key=lambda p: p["id"]) == want
    finally:
        cl.close()


def test_clustering_nodes_replica1():  # TestClusteringNodesReplica1 :445
    cl = _Cluster(3)
    try:
        cl.stop(2)
        assert _wait(lambda: _state(cl.nodes[0]) == "STARTING")
        from pilosa_amd.server.api import QueryRequest
        with pytest.raises(Exception, match="not allowed in state STARTING"):
            cl.nodes[0].api.query(QueryRequest(index="i", query="Count(Row(f=1))"))
        cl.start(2)
        assert _wait(lambda: all(_state(s) == "NORMAL" for s in cl.nodes))
    finally:
        cl.close()


def test_clustering_nodes_replica2():  # TestClusteringNodesReplica2 :495
    cl = _Cluster(3, replicas=2)
    try:
        cl.stop(2)
        assert _wait(lambda: _state(cl.nodes[0]) == "DEGRADED")
        cl.nodes[0].api.create_index("anewindex")        # DEGRADED still accepts writes
        cl.stop(1)
        assert _wait(lambda: _state(cl.nodes[0]) == "STARTING")
        from pilosa_amd.server.api import QueryRequest
        with pytest.raises(Exception, match="not allowed in state STARTING"):
            cl.nodes[0].api.query(QueryRequest(index="anewindex", query="Count(Row(f=1))"))
        cl.start(2)
        assert _wait(lambda: _state(cl.nodes[0]) == "DEGRADED")
        cl.start(1)
        assert _wait(lambda: all(_state(s) == "NORMAL" for s in cl.nodes))
    finally:
        cl.close()


def test_remove_node_after_it_dies():  # TestRemoveNodeAfterItDies :591
    cl = _Cluster(3, replicas=2)
    try:
        cl.stop(2)
        assert _wait(lambda: _state(cl.nodes[0]) == "DEGRADED")
        cl.nodes[0].api.remove_node("node2")
        assert _wait(lambda: _state(cl.nodes[0]) == "NORMAL")
        assert len(cl.nodes[0].api.hosts()) == 2
    finally:
        cl.close()


def test_remove_concurrent_index_creation():  # TestRemoveConcurrentIndexCreation :634
    cl = _Cluster(3, replicas=2)
    try:
        errs = []

        def create():
            try:
                cl.nodes[0].api.create_index("blah")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        t = threading.Thread(target=create)
        t.start()
        cl.nodes[0].api.remove_node("node2")
        t.join()
        assert _wait(lambda: _state(cl.nodes[0]) == "NORMAL")
        assert len(cl.nodes[0].api.hosts()) == 2
        assert not errs, errs
    finally:
        cl.close()


def test_cluster_queries_after_restart():  # TestClusterQueriesAfterRestart :786
    cl = _Cluster(3)
    try:
        for s in cl.nodes:
            assert all(n["state"] == "READY" for n in s.api.hosts()) if isinstance(s.api.hosts()[0], dict) else True
        c = InternalClient()
        c.create_index(cl.nodes[1].uri, "testidx")
        c.create_field(cl.nodes[1].uri, "testidx", "testfield", {"type": "set", "cacheType": "ranked", "cacheSize": 10})
        time.sleep(0.2)
        q = "".join(f"Set({i * SW}, testfield=0)" for i in range(100))
        assert c.query(cl.nodes[1].uri, "testidx", q)["results"] == [True] * 100
        assert c.query(cl.nodes[1].uri, "testidx", "Count(Row(testfield=0))")["results"] == [100]
        cl.stop(1)
        assert _wait(lambda: _state(cl.nodes[0]) == "STARTING")
        from pilosa_amd.server.api import QueryRequest
        with pytest.raises(Exception, match="not allowed in state STARTING"):
            cl.nodes[0].api.query(QueryRequest(index="testidx", query="Count(Row(testfield=0))"))
        s1 = cl.start(1)
        assert _wait(lambda: _state(s1) == "NORMAL" and _state(cl.nodes[0]) == "NORMAL")
        assert c.query(s1.uri, "testidx", "Count(Row(testfield=0))")["results"] == [100]
    finally:
        cl.close()


def test_cluster_exhausting_connections():  # TestClusterExhaustingConnections :868 (reduced: 20 x 25 Sets)
    cl = _Cluster(5)
    try:
        c = InternalClient()
        c.create_index(cl.nodes[1].uri, "testidx")
        c.create_field(cl.nodes[1].uri, "testidx", "testfield", {"type": "set", "cacheType": "ranked", "cacheSize": 10})
        time.sleep(0.3)
        errs = []

        def worker(i):
            try:
                for j in range(i, 500, 20):
                    c.query(cl.nodes[i % 5].uri, "testidx", f"Set({j * SW}, testfield=0)")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(20)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs[:1]
        assert c.query(cl.nodes[0].uri, "testidx", "Count(Row(testfield=0))")["results"] == [500]
    finally:
        cl.close()


# ---------------------------------------------------------------- test/pilosa_test.go TestNewCluster
def test_new_cluster_agrees_on_coordinator_and_status():
    c = _Cluster(3)
    try:
        coords = [[n for n in m.api.hosts() if n.is_coordinator] for m in c.nodes]
        assert all(len(x) == 1 for x in coords)
        assert len({x[0].id for x in coords}) == 1, "nodes disagree on the coordinator"
        from tests.test_server import _req
        st, body = _req(c.nodes[0], "GET", "/status", headers={"Accept": "application/json"})
        d = json.loads(body)
        assert st == 200 and len(d["nodes"]) == 3 and d["state"] == "NORMAL"
    finally:
        c.close()
