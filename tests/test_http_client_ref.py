"""Ported expectations of the reference's http/client_test.go (InternalClient
against in-process servers).  Each test names the reference test it ports."""
import tempfile
import time

import pytest

from pilosa_amd.parallel.cluster import URI
from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.server import Server
from pilosa_amd.shardwidth import SHARD_WIDTH as SW
from pilosa_amd.utils.logger import CaptureLogger

pytestmark = pytest.mark.timeout(120)


def _single():
    return Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()


def _cluster(n, replicas=1):
    from tests.test_server_ref import _Cluster
    return _Cluster(n, replicas)


def _pairs(res):
    return [(p.get("key", p.get("id")), p["count"]) for p in res]


def test_client_multi_node_topn():  # TestClient_MultiNode (http/client_test.go:22)
    cl = _cluster(3)
    try:
        c = InternalClient()
        s0 = cl.nodes[0]
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set", "cacheType": "ranked", "cacheSize": 100})
        time.sleep(0.2)
        shard_nums = [1, 2, 6]   # owned by node0, node1, node2 under the mod hasher
        for i, s in enumerate(shard_nums):
            assert cl.nodes[i].cluster.owns_shard(f"node{i}", "i", s)
        b0, b1, b2 = (SW * s for s in shard_nums)
        sets = {0: [(100, [b0 + 10]), (4, [b0 + 10, b0 + 11, b0 + 12]),
                    (4, [b0 + 10, b0 + 11, b0 + 12, b0 + 13, b0 + 14, b0 + 15]), (2, [b0 + k for k in (1, 2, 3, 4)]),
                    (3, [b0 + k for k in (1, 2, 3, 4, 5)]), (22, [b0 + 1, b0 + 2])],
                1: [(99, [b1 + k for k in (1, 2, 3, 4)]), (100, [b1 + k for k in range(1, 11)]),
                    (98, [b1 + k for k in range(1, 7)]), (1, [b1 + 4]), (22, [b1 + k for k in range(1, 6)])],
                2: [(24, [b2 + k for k in range(10, 15)]), (20, [b2 + k for k in range(10, 14)]), (21, [b2 + 10]),
                    (100, [b2 + 10]), (99, [b2 + 10, b2 + 11, b2 + 12]), (98, [b2 + 10, b2 + 11]),
                    (22, [b2 + 10, b2 + 11, b2 + 12])]}
        for node, rows in sets.items():
            f = cl.nodes[node].holder.field("i", "f")
            for row, cols in rows:
                for col in cols:
                    f.set_bit(row, col)
        for s in cl.nodes:
            s.api.recalculate_caches()
        want = [(100, 12), (22, 10), (98, 8), (99, 7)]
        got = [_pairs(c.query(s.uri, "i", "TopN(f, n=4)")["results"][0]) for s in cl.nodes]
        assert got[0] == want and got[1] == want and got[2] == want
    finally:
        cl.close()


BITS = [(1, 100, "row1", "col100"), (1, 101, "row1", "col101"), (1, 102, "row1", "col102"),
        (1, 103, "row1", "col103"), (2, 200, "row2", "col200"), (2, 201, "row2", "col201"),
        (2, 202, "row2", "col202"), (2, 203, "row2", "col203")]


def test_client_export():  # TestClient_Export :163
    s = _single()
    try:
        c = InternalClient()
        c.create_index(s.uri, "keyed", keys=True)
        c.create_index(s.uri, "unkeyed", keys=False)
        for idx in ("keyed", "unkeyed"):
            c.create_field(s.uri, idx, "keyedf", {"type": "set", "cacheType": "ranked", "cacheSize": 1000, "keys": True})
            c.create_field(s.uri, idx, "unkeyedf", {"type": "set", "cacheType": "ranked", "cacheSize": 1000})
        for r, col, rk, ck in BITS:
            c.query(s.uri, "unkeyed", f"Set({col}, unkeyedf={r})")
            c.query(s.uri, "unkeyed", f'Set({col}, keyedf="{rk}")')
            c.query(s.uri, "keyed", f'Set("{ck}", unkeyedf={r})')
            c.query(s.uri, "keyed", f'Set("{ck}", keyedf="{rk}")')
        assert c.export_csv(s.uri, "unkeyed", "unkeyedf", 0) == "".join(f"{r},{col}\n" for r, col, _, _ in BITS)
        assert c.export_csv(s.uri, "unkeyed", "keyedf", 0) == "".join(f"{rk},{col}\n" for _, col, rk, _ in BITS)
        assert c.export_csv(s.uri, "keyed", "unkeyedf", 0) == "".join(f"{r},{ck}\n" for r, _, _, ck in BITS)
        assert c.export_csv(s.uri, "keyed", "keyedf", 0) == "".join(f"{rk},{ck}\n" for _, _, rk, ck in BITS)
    finally:
        s.close()


def test_client_import():  # TestClient_Import :346
    s = _single()
    try:
        c = InternalClient()
        c.create_index(s.uri, "i")
        c.create_field(s.uri, "i", "f", {"type": "set"})
        c.import_bits(s.node, "i", "f", 0, [0, 0, 200], [1, 5, 6])
        f = s.holder.field("i", "f")
        assert list(f.row(0).columns()) == [1, 5] and list(f.row(200).columns()) == [6]
        c.import_bits(s.node, "i", "f", 0, [0, 200], [5, 6], clear=True)
        assert list(f.row(0).columns()) == [1] and list(f.row(200).columns()) == []
    finally:
        s.close()


def test_client_import_roaring():  # TestClient_ImportRoaring :389
    cl = _cluster(2, replicas=2)
    try:
        c = InternalClient()
        s0 = cl.nodes[0]
        c.create_index(s0.uri, "i")
        c.create_field(s0.uri, "i", "f", {"type": "set", "cacheType": "ranked", "cacheSize": 100})
        time.sleep(0.2)
        c.query(s0.uri, "i", "Set(0, f=1)")

        def rows():
            return [(list(s.holder.field("i", "f").row(0).columns()), list(s.holder.field("i", "f").row(1).columns()))
                    for s in cl.nodes]
        full = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 65537]
        c.import_roaring(s0.node, "i", "f", 0, {"": bytes.fromhex("3B3001000100000900010000000100010009000100")})
        assert rows() == [(full, [0])] * 2
        c.import_roaring(s0.node, "i", "f", 0, {"": bytes.fromhex("3A30000001000000010001001000000003000400")},
                         clear=True)
        assert rows() == [(full, [0])] * 2   # clears bits of another container key only
        c.import_roaring(s0.node, "i", "f", 0,
                         {"": bytes.fromhex("3A300000020000000000010001000100180000001C0000000400060001000300")},
                         clear=True)
        assert rows() == [([1, 2, 3, 5, 7, 8, 9, 10], [0])] * 2
        c.import_roaring(s0.node, "i", "f", 0, {"": bytes.fromhex("3B3001000100000900010000000100010009000100")},
                         clear=True)
        assert rows() == [([], [0])] * 2
    finally:
        cl.close()


KEYED = [("green", "eve"), ("green", "alice"), ("green", "bob"), ("blue", "eve"), ("blue", "alice"),
         ("purple", "eve")]


def test_client_import_keys_single_node():  # TestClient_ImportKeys/SingleNode :486
    s = _single()
    try:
        c = InternalClient()
        c.create_index(s.uri, "keyed", keys=True)
        c.create_index(s.uri, "unkeyed", keys=False)
        c.create_field(s.uri, "keyed", "keyedf", {"type": "set", "cacheType": "ranked", "cacheSize": 1000, "keys": True})
        c.create_field(s.uri, "keyed", "unkeyedf", {"type": "set", "cacheType": "ranked", "cacheSize": 1000})
        c.create_field(s.uri, "unkeyed", "keyedf", {"type": "set", "cacheType": "ranked", "cacheSize": 1000,
                                                    "keys": True})
        c.import_bits(s.node, "keyed", "keyedf", 0, [], [], row_keys=[r for r, _ in KEYED],
                      col_keys=[k for _, k in KEYED])
        s.api.recalculate_caches()
        assert _pairs(c.query(s.uri, "keyed", "TopN(keyedf)")["results"][0]) == \
            [("green", 3), ("blue", 2), ("purple", 1)]
        c.import_bits(s.node, "keyed", "unkeyedf", 0, [1, 1, 1, 2, 2, 3], [], col_keys=[k for _, k in KEYED])
        s.api.recalculate_caches()
        assert _pairs(c.query(s.uri, "keyed", "TopN(unkeyedf)")["results"][0]) == [(1, 3), (2, 2), (3, 1)]
        c.import_bits(s.node, "unkeyed", "keyedf", 0, [], [1, 2, 3, 1, 2, 1], row_keys=[r for r, _ in KEYED])
        s.api.recalculate_caches()
        assert _pairs(c.query(s.uri, "unkeyed", "TopN(keyedf)")["results"][0]) == \
            [("green", 3), ("blue", 2), ("purple", 1)]
    finally:
        s.close()


def test_client_import_keys_multi_node():  # TestClient_ImportKeys/MultiNode :583
    cl = _cluster(2)
    try:
        c = InternalClient()
        c.create_index(cl.nodes[0].uri, "keyed", keys=True)
        for f in ("keyedf0", "keyedf1"):
            c.create_field(cl.nodes[0].uri, "keyed", f, {"type": "set", "cacheType": "ranked", "cacheSize": 1000,
                                                        "keys": True})
        time.sleep(0.2)
        for node, f in ((0, "keyedf0"), (1, "keyedf1")):
            s = cl.nodes[node]
            c.import_bits(s.node, "keyed", f, 0, [], [], row_keys=[r for r, _ in KEYED],
                          col_keys=[k for _, k in KEYED])
            time.sleep(0.3)
            for n in cl.nodes:
                n.api.recalculate_caches()
            assert _pairs(c.query(s.uri, "keyed", f"TopN({f})")["results"][0]) == \
                [("green", 3), ("blue", 2), ("purple", 1)]
    finally:
        cl.close()
