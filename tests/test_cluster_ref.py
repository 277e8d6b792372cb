"""Cluster placement / resize-planning / membership expectations ported from
the reference's cluster_internal_test.go (TestFragCombos, TestFragSources,
TestResizeJob, TestCluster_Owners, TestCluster_Partition, TestHasher,
TestCluster_ContainsShards, TestCluster_Nodes, TestCluster_PreviousNode,
TestCluster_Coordinator, TestCluster_Topology, TestCluster_ResizeStates,
TestCluster_UpdateCoordinator, TestCluster_confirmNodeDown*).

The server-level cases run real in-process nodes over loopback HTTP (the
reference's in-memory cluster harness, utils_internal_test.go's
NewTestCluster / ClusterCluster with a mod hasher, is the in-process
``Cluster.from_nodes(..., hasher=ModHasher())`` here)."""
import http.server
import os
import random
import socket
import tempfile
import threading
import time

import pytest

from pilosa_amd.errors import PilosaError
from pilosa_amd.parallel.cluster import (RESIZE_ACTION_ADD, RESIZE_ACTION_REMOVE, Cluster, ModHasher, Node, Topology,
                                         URI, clone_nodes, confirm_node_down, contains_node, filter_nodes,
                                         filter_nodes_uri, jump_hash, node_ids, ResizeJob)
from pilosa_amd.models.fragment import SHARD_WIDTH as SW
from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.server import Server
from pilosa_amd.utils.logger import CaptureLogger


def _n(i, port=10101):
    return Node(f"node{i}", URI("http", f"host{i}", port))


def _c(ids, replica_n=1, hasher=None):
    return Cluster.from_nodes([_n(i) for i in ids], replica_n=replica_n, hasher=hasher)


def test_frag_combos():
    c = _c([0, 1])
    assert c.frag_combos("i", [0, 1, 2], {"f": ["v1", "v2"]}) == {
        "node0": [("f", "v1", 0), ("f", "v2", 0)],
        "node1": [("f", "v1", 1), ("f", "v2", 1), ("f", "v1", 2), ("f", "v2", 2)]}
    assert c.frag_combos("foo", [0, 1, 2, 3], {"f": ["v0"]}) == {
        "node0": [("f", "v0", 1), ("f", "v0", 2)],
        "node1": [("f", "v0", 0), ("f", "v0", 3)]}


SCHEMA = {"i": {"f": ["standard"]}}
AVAIL = {"i": [0, 1, 2, 3]}   # bits at columns 101, SW+1, 2SW+1, 3SW+1


def _sources(frm, to):
    out = frm.frag_sources(to, SCHEMA, AVAIL)
    return {nid: [(s["node"]["id"], s["node"]["uri"]["host"], s["index"], s["field"], s["view"], s["shard"])
                  for s in srcs] for nid, srcs in out.items()}


def test_frag_sources():
    c1, c2 = _c([0, 1]), _c([0, 1, 2])
    c3, c4, c5 = _c([0, 1], 2), _c([0, 1, 2], 2), _c([0, 1, 2, 3], 2)
    assert _sources(c1, c2) == {
        "node0": [], "node1": [],
        "node2": [("node0", "host0", "i", "f", "standard", 0), ("node1", "host1", "i", "f", "standard", 2)]}
    assert _sources(c4, c3) == {
        "node0": [("node1", "host1", "i", "f", "standard", 1)],
        "node1": [("node0", "host0", "i", "f", "standard", 0), ("node0", "host0", "i", "f", "standard", 2)]}
    assert _sources(c5, c4) == {
        "node0": [("node2", "host2", "i", "f", "standard", 0), ("node2", "host2", "i", "f", "standard", 2)],
        "node1": [("node0", "host0", "i", "f", "standard", 3)],
        "node2": []}
    for frm, to, msg in [(c2, c4, "clusters are the same size"),
                         (c1, c5, "adding more than one node at a time is not supported"),
                         (c5, c1, "removing more than one node at a time is not supported")]:
        with pytest.raises(PilosaError, match=msg):
            frm.frag_sources(to, SCHEMA, AVAIL)


def test_frag_sources_insufficient_replicas():
    # replica 1: the leaving node's fragments exist nowhere else
    c2, c1 = _c([0, 1, 2]), _c([0, 1])
    with pytest.raises(PilosaError, match="not enough data to perform resize"):
        c2.frag_sources(c1, SCHEMA, AVAIL)


def test_resize_job():
    n0, n1, n2 = _n(0), _n(1), _n(2)
    j = ResizeJob([n0, n1], n2, RESIZE_ACTION_ADD)
    assert j.ids == {"node0": False, "node1": False, "node2": False}
    j = ResizeJob([n0, n1, n2], n2, RESIZE_ACTION_REMOVE)
    assert j.ids == {"node0": False, "node1": False}
    assert not j.mark("node0")
    assert j.pending == {"node1"} and j.leaving == "node2"
    assert j.mark("node1", "boom") and j.errors == ["boom"]


def test_owners_mod_hasher():
    c = Cluster.from_nodes([Node(f"n{x}", URI("http", f"server{x}", 1000)) for x in "ABC"], replica_n=2,
                           hasher=ModHasher())
    assert c.partition_nodes(0) == [c.nodes[0], c.nodes[1]]
    assert c.partition_nodes(2) == [c.nodes[2], c.nodes[0]]


def test_partition_in_range():
    rng = random.Random(7)
    for _ in range(500):
        pn = rng.randint(1, 1000)
        c = Cluster(Node("x", URI()), partition_n=pn)
        name = "".join(chr(rng.randint(32, 0x2fff)) for _ in range(rng.randint(0, 12)))
        assert 0 <= c.partition(name, rng.getrandbits(32)) < pn


def test_hasher_golden():
    # generated from the reference jump-hash C++ code (cluster_internal_test.go:377)
    for key, buckets in [(0, [0] * 20),
                         (1, [0, 0, 0, 0, 0, 0, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 17, 17]),
                         (0xdeadbeef, [0, 1, 2, 3, 3, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 16, 16, 16]),
                         (0x0ddc0ffeebadf00d, [0, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 15, 15, 15, 15])]:
        assert [jump_hash(key, i + 1) for i in range(len(buckets))] == buckets


def test_contains_shards():
    c = Cluster.from_nodes([Node(f"node{i}", URI("http", f"host{i}", 0)) for i in range(5)], replica_n=3,
                           hasher=ModHasher())
    assert c.contains_shards("test", range(11), c.nodes[2]) == [0, 2, 3, 5, 6, 9, 10]


def test_nodes_helpers():
    nodes = [Node(f"node{i}", URI("http", f"node{i}", 0)) for i in range(3)]
    n3 = Node("node3", URI("http", "node3", 0))
    assert node_ids(nodes) == ["node0", "node1", "node2"]
    assert [n.uri for n in filter_nodes(nodes, nodes[1])] == [nodes[0].uri, nodes[2].uri]
    assert [n.uri for n in filter_nodes_uri(nodes, nodes[1].uri)] == [nodes[0].uri, nodes[2].uri]
    assert contains_node(nodes, nodes[1]) and not contains_node(nodes, n3)
    clone = clone_nodes(nodes)
    assert [n.uri for n in clone] == [n.uri for n in nodes] and clone[0] is not nodes[0]


def test_previous_node():
    n0, n1, n2 = Node("node0", URI()), Node("node1", URI()), Node("node2", URI())
    c = Cluster.from_nodes([n0])
    assert c.previous_node() is None
    c = Cluster.from_nodes([n0, n1], local=n0)
    assert c.previous_node() is n1
    c.node = n1
    assert c.previous_node() is n0
    c = Cluster.from_nodes([n0, n1, n2], local=n0)
    assert c.previous_node() is n2
    c.node = n1
    assert c.previous_node() is n0
    c.node = n2
    assert c.previous_node() is n1


def test_coordinator():
    n1, n2 = Node("node1", URI("http", "node1", 0)), Node("node2", URI("http", "node2", 0))
    c1 = Cluster.from_nodes([n1, n2], local=n1)
    c1.set_coordinator("node1")
    c2 = Cluster.from_nodes([n1, n2], local=n2)
    c2.set_coordinator("node1")
    assert c1.is_coordinator() and not c2.is_coordinator()


def test_update_coordinator():
    c = _c([0, 1])
    old, new = c.nodes
    c.set_coordinator(old.id)
    assert not c.update_coordinator(old) and c.coordinator_id == old.id
    assert c.update_coordinator(new) and c.coordinator_id == new.id
    assert new.is_coordinator and not old.is_coordinator


def test_topology_add_node(tmp_path):
    c = Cluster(Node("node0", URI("http", "host0", 0)), path=str(tmp_path))
    n1, n2 = Node("node1", URI("http", "host1", 0)), Node("node2", URI("http", "host2", 0))
    c.add_node(n1)
    c.add_node(n1)
    c.add_node(n2)
    assert c.node_ids() == ["node0", "node1", "node2"]
    assert c.topology.contains_id("node1") and not c.topology.contains_id("nodeinvalid")
    # persisted: a fresh cluster over the same path loads it
    assert Topology.load(os.path.join(str(tmp_path), ".topology")).node_ids == ["node0", "node1", "node2"]


# ---------------------------------------------------------------- confirmNodeDown
class _VersionHandler(http.server.BaseHTTPRequestHandler):
    delay = 0.0

    def do_GET(self):  # noqa: N802
        time.sleep(self.delay)
        try:
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b"ignored\n")
        except OSError:
            pass

    def log_message(self, *a):
        pass


def _version_server(delay):
    h = type("H", (_VersionHandler,), {"delay": delay})
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), h)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, URI("http", "127.0.0.1", srv.server_address[1])


def test_confirm_node_down_up():
    srv, uri = _version_server(0.0)
    try:
        assert not confirm_node_down(uri, retries=3, sleep=0.05)
    finally:
        srv.shutdown()
        srv.server_close()


def test_confirm_node_down_timeout():
    srv, uri = _version_server(1.0)
    try:
        assert confirm_node_down(uri, retries=2, sleep=0.05, timeout=0.2)
    finally:
        srv.shutdown()
        srv.server_close()


def test_confirm_node_down_down():
    from tests.helpers import free_port
    port = free_port()   # nothing listens there (and bind(0) servers never get it)
    assert confirm_node_down(URI("http", "127.0.0.1", port), retries=2, sleep=0.05, timeout=0.5)


# ---------------------------------------------------------------- resize states
def _server(node_id, data_dir=None, coordinator=True, coordinator_uri=None):
    s = Server(data_dir or tempfile.mkdtemp(), bind="127.0.0.1:0", node_id=node_id, gpu="off",
               coordinator=coordinator, coordinator_uri=coordinator_uri, probe_interval=0.2,
               logger=CaptureLogger(), hasher="mod", native_http=False)
    if coordinator:
        s.hosts = [URI.parse("127.0.0.1:1")]   # enable the membership loop
    return s


def _wait(cond, timeout=15.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if cond():
            return True
        time.sleep(0.05)
    return cond()


def _write_topology(d, ids):
    os.makedirs(d, exist_ok=True)
    Topology(node_ids=ids).save(os.path.join(d, ".topology"))


pytestmark_timeout = pytest.mark.timeout(120)


@pytestmark_timeout
def test_resize_states_single_node_no_data():
    s = _server("node0").open()
    try:
        assert _wait(lambda: s.cluster.state == "NORMAL")
        assert s.cluster.topology.node_ids == ["node0"]
    finally:
        s.close()


@pytestmark_timeout
def test_resize_states_single_node_in_topology():
    d = tempfile.mkdtemp()
    _write_topology(d, ["node0"])
    s = _server("node0", d).open()
    try:
        assert _wait(lambda: s.cluster.state == "NORMAL")
    finally:
        s.close()


@pytestmark_timeout
def test_resize_states_single_node_not_in_topology():
    d = tempfile.mkdtemp()
    _write_topology(d, ["some-other-host"])
    with pytest.raises(PilosaError, match=r"^coordinator node0 is not in topology: \[some-other-host\]$"):
        _server("node0", d).open()


@pytestmark_timeout
def test_resize_states_multiple_nodes_no_data():
    s0 = _server("node0").open()
    s1 = None
    try:
        s1 = _server("node1", coordinator=False, coordinator_uri=s0.uri.normalize()).open()
        assert _wait(lambda: s0.cluster.state == "NORMAL" and s1.cluster.state == "NORMAL"
                     and len(s1.cluster.nodes) == 2)
        assert s0.cluster.topology.node_ids == ["node0", "node1"]
        assert _wait(lambda: s1.cluster.topology.node_ids == ["node0", "node1"])
    finally:
        for s in (s1, s0):
            if s is not None:
                s.close()


@pytestmark_timeout
def test_resize_states_in_and_not_in_topology():
    d = tempfile.mkdtemp()
    _write_topology(d, ["node0", "node2"])
    s0 = _server("node0", d).open()
    joined = []
    try:
        time.sleep(0.3)
        assert s0.cluster.state == "STARTING"
        s1 = _server("node1", coordinator=False, coordinator_uri=s0.uri.normalize()).open()
        joined.append(s1)
        assert s1.join_error == "host is not in topology: node1"
        s2 = _server("node2", coordinator=False, coordinator_uri=s0.uri.normalize()).open()
        joined.append(s2)
        assert _wait(lambda: s0.cluster.state == "NORMAL" and s2.cluster.state == "NORMAL")
        assert s0.cluster.node_ids() == ["node0", "node2"]
    finally:
        for s in joined + [s0]:
            s.close()


@pytestmark_timeout
def test_resize_states_multiple_nodes_with_data():
    s0 = _server("node0").open()
    s1 = None
    c = InternalClient()
    try:
        assert _wait(lambda: s0.cluster.state == "NORMAL")
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set"})
        c.query(s0.uri, "i", f"Set(101, f=1) Set({SW + 1}, f=1)")
        before = s0.holder.fragment("i", "f", "standard", 1).checksum()
        s1 = _server("node1", coordinator=False, coordinator_uri=s0.uri.normalize()).open()
        assert _wait(lambda: s0.cluster.state == "NORMAL" and s1.cluster.state == "NORMAL"
                     and len(s0.cluster.nodes) == 2 and len(s1.cluster.nodes) == 2)
        assert s0.cluster.topology.node_ids == ["node0", "node1"]
        assert _wait(lambda: s1.cluster.topology.node_ids == ["node0", "node1"])
        # mod hasher, 2 nodes: shard 1's partition maps to node1 -> fragment moved there intact
        owner = s0.cluster.shard_nodes("i", 1)[0].id
        holder = {"node0": s0, "node1": s1}[owner]
        assert _wait(lambda: holder.holder.fragment("i", "f", "standard", 1) is not None)
        assert holder.holder.fragment("i", "f", "standard", 1).checksum() == before
        for s in (s0, s1):
            assert c.query(s.uri, "i", "Count(Row(f=1))")["results"] == [2]
    finally:
        for s in (s1, s0):
            if s is not None:
                s.close()


# ---------------------------------------------------------------- server/cluster_test.go
def _join(coord, node_id, hosts=None):
    s = _server(node_id, coordinator=False, coordinator_uri=None if hosts else coord.uri.normalize())
    if hosts:
        s.hosts = [URI.parse(h) for h in hosts]
    return s.open()


def _all_normal(servers, n):
    return _wait(lambda: all(s.cluster.state == "NORMAL" and len(s.cluster.nodes) == n for s in servers))


@pytestmark_timeout
@pytest.mark.parametrize("cols", [[1, 1300000], [1, 2400000]], ids=["ContinuousShards", "SkippedShard"])
def test_cluster_resize_add_node_with_data(cols):
    m0 = _server("node0").open()
    m1 = None
    c = InternalClient()
    try:
        assert _wait(lambda: m0.cluster.state == "NORMAL")
        c.create_index(m0.uri, "i")
        c.create_field(m0.uri, "i", "f", {"type": "set"})
        c.query(m0.uri, "i", " ".join(f"Set({x}, f=1)" for x in cols))
        assert c.query(m0.uri, "i", "Row(f=1)")["results"] == [{"attrs": {}, "columns": cols}]
        m1 = _join(m0, "node1")
        assert _all_normal([m0, m1], 2)
        for m in (m0, m1):
            assert c.query(m.uri, "i", "Row(f=1)")["results"] == [{"attrs": {}, "columns": cols}]
    finally:
        for s in (m1, m0):
            if s is not None:
                s.close()


@pytestmark_timeout
def test_cluster_resize_add_node_concurrent_index():
    m0 = _server("node0").open()
    m1 = None
    c = InternalClient()
    try:
        assert _wait(lambda: m0.cluster.state == "NORMAL")
        c.create_index(m0.uri, "i")
        c.create_field(m0.uri, "i", "f", {"type": "set"})
        c.query(m0.uri, "i", "Set(1, f=1) Set(1300000, f=1)")
        errs = []

        def create():
            try:
                deadline = time.time() + 20
                while True:   # the reference API call blocks through RESIZING; ours is retried until NORMAL
                    try:
                        m0.api.create_index("blah")
                        return
                    except PilosaError as e:
                        if "resizing" not in str(e).lower() or time.time() > deadline:
                            raise
                        time.sleep(0.05)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        m1 = _join(m0, "node1")
        t = threading.Thread(target=create)
        t.start()
        assert _all_normal([m0, m1], 2)
        t.join(30)
        assert not errs
        assert _wait(lambda: m1.holder.index("blah") is not None)
    finally:
        for s in (m1, m0):
            if s is not None:
                s.close()


@pytestmark_timeout
def test_cluster_gossip_membership_invalid_seed_first():
    m0 = _server("node0").open()
    ms = []
    try:
        assert _wait(lambda: m0.cluster.state == "NORMAL")
        from tests.helpers import free_port
        dead = f"http://127.0.0.1:{free_port()}"
        ts = [threading.Thread(target=lambda nid=nid, h=h: ms.append(_join(m0, nid, h)))
              for nid, h in [("node1", [dead, m0.uri.normalize()]), ("node2", [m0.uri.normalize(), dead])]]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert len(ms) == 2
        assert _all_normal([m0] + ms, 3)
        assert len(m0.api.hosts()) == 3
    finally:
        for s in ms + [m0]:
            s.close()


def _post(uri, path, body):
    import urllib.error
    import urllib.request
    req = urllib.request.Request(uri.normalize() + path, data=body.encode(), method="POST",
                                 headers={"Content-Type": "application/json", "Accept": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=30) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()


@pytestmark_timeout
def test_cluster_resize_remove_node_errors():
    m0 = _server("node0").open()
    m1 = m2 = None
    c = InternalClient()
    try:
        m1 = _join(m0, "node1")
        m2 = _join(m0, "node2")
        assert _all_normal([m0, m1, m2], 3)
        st, body = _post(m0.uri, "/cluster/resize/remove-node", '{"id": "invalid-node-id"}')
        assert (st, body.strip()) == (404, "removing node: finding node to remove: node with provided ID does "
                                           "not exist")
        st, body = _post(m0.uri, "/cluster/resize/remove-node", '{"id": "node0"}')
        assert (st, body.strip()) == (500, "removing node: calling node leave: coordinator cannot be removed; "
                                           "first, make a different node the new coordinator")
        st, body = _post(m1.uri, "/cluster/resize/remove-node", '{"id": "node1"}')
        assert (st, body.strip()) == (500, "removing node: calling node leave: node removal requests are only "
                                           "valid on the coordinator node: node0")
        c.create_index(m0.uri, "i")
        c.create_field(m0.uri, "i", "f", {"type": "set"})
        c.query(m0.uri, "i", " ".join(f"Set({i * SW}, f=1)" for i in range(20)))
        st, body = _post(m0.uri, "/cluster/resize/remove-node", '{"id": "node1"}')
        assert st == 500 and "not enough data to perform resize" in body
        assert m0.cluster.state == "NORMAL"
    finally:
        for s in (m2, m1, m0):
            if s is not None:
                s.close()


@pytestmark_timeout
def test_cluster_resize_remove_node_with_replicas():
    """Removing a node from a replica-2 cluster moves its fragments to the
    survivors and the data stays queryable everywhere."""
    servers = []
    c = InternalClient()
    try:
        m0 = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", node_id="node0", gpu="off", replica_n=2,
                    coordinator=True, probe_interval=0.2, logger=CaptureLogger(), hasher="mod", native_http=False)
        m0.hosts = [URI.parse("127.0.0.1:1")]
        servers.append(m0.open())
        for i in (1, 2):
            servers.append(Server(tempfile.mkdtemp(), bind="127.0.0.1:0", node_id=f"node{i}", gpu="off",
                                  replica_n=2, coordinator=False, coordinator_uri=m0.uri.normalize(),
                                  probe_interval=0.2, logger=CaptureLogger(), hasher="mod",
                                  native_http=False).open())
        assert _all_normal(servers, 3)
        c.create_index(m0.uri, "i")
        c.create_field(m0.uri, "i", "f", {"type": "set"})
        cols = [i * SW + i for i in range(8)]
        c.query(m0.uri, "i", " ".join(f"Set({x}, f=1)" for x in cols))
        st, body = _post(m0.uri, "/cluster/resize/remove-node", '{"id": "node2"}')
        assert st == 200, body
        assert _wait(lambda: all(s.cluster.state == "NORMAL" and len(s.cluster.nodes) == 2 for s in servers[:2]))
        for s in servers[:2]:
            assert c.query(s.uri, "i", "Row(f=1)")["results"][0]["columns"] == cols
            assert s.cluster.topology.node_ids == ["node0", "node1"]
    finally:
        for s in reversed(servers):
            s.close()


# ---------------------------------------------------------------- gossip (NodeStatus push-pull)
@pytestmark_timeout
def test_gossip_spreads_schema_and_detects_failure_on_non_coordinator():
    def mk(nid, coord=None, probe=0.2):
        s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", node_id=nid, gpu="off", coordinator=coord is None,
                   coordinator_uri=None if coord is None else coord.uri.normalize(), probe_interval=probe,
                   logger=CaptureLogger(), hasher="mod", native_http=False, gossip_interval=0.1)
        if coord is None:
            s.hosts = [URI.parse("127.0.0.1:1")]
        return s.open()
    # the coordinator's own prober is slowed right down: only gossip can notice the failure in time
    m0 = mk("node0", probe=3600)
    m1 = m2 = None
    try:
        m0.probe_interval = 0.2
        m1, m2 = mk("node1", m0), mk("node2", m0)
        m0.probe_interval = 3600
        assert _all_normal([m0, m1, m2], 3)
        # a schema change made on node2 alone (no broadcast) reaches everyone through gossip
        m2.api.create_index("g", remote=True)
        assert _wait(lambda: m0.holder.index("g") is not None and m1.holder.index("g") is not None)
        m2.close()
        assert _wait(lambda: m0.cluster.node_by_id("node2").state == "DOWN", timeout=30)
        assert m0.cluster.state == "DEGRADED" or m0.cluster.state == "STARTING"
    finally:
        for s in (m2, m1, m0):
            if s is not None:
                try:
                    s.close()
                except Exception:  # noqa: BLE001 - m2 closed above
                    pass
