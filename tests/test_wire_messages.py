"""Cluster messages on the reference wire format: 1 type byte + protobuf
(broadcast.go:56-161, internal/private.proto).  Golden byte strings are
hand-derived from the proto3 encoding rules and private.proto's field
numbers (no Go toolchain here to produce them from the reference)."""
import pytest

from pilosa_amd.wire import messages as M
from pilosa_amd.wire import pb

NODE = {"id": "node1", "uri": {"scheme": "http", "host": "h1", "port": 10101}, "isCoordinator": True,
        "state": "READY", "gpus": 8}


def test_type_bytes_follow_reference_iota():
    assert M.TYPE_NAMES[:16] == ["CreateShard", "CreateIndex", "DeleteIndex", "CreateField", "DeleteField",
                                 "CreateView", "DeleteView", "ClusterStatus", "ResizeInstruction",
                                 "ResizeInstructionComplete", "SetCoordinator", "UpdateCoordinator", "NodeState",
                                 "RecalculateCaches", "NodeEvent", "NodeStatus"]


def test_golden_bytes():
    # CreateShardMessage{Index:"i"(1), Shard:3(2), Field:"f"(3)}, type 0
    assert M.encode({"type": "CreateShard", "index": "i", "field": "f", "shard": 3}) == \
        b"\x00\x0a\x01i\x10\x03\x1a\x01f"
    # DeleteIndexMessage{Index:"ab"}, type 2
    assert M.encode({"type": "DeleteIndex", "index": "ab"}) == b"\x02\x0a\x02ab"
    # RecalculateCaches{}, type 13
    assert M.encode({"type": "RecalculateCaches"}) == b"\x0d"
    # NodeEventMessage{Event:1(leave), Node{ID:"n", URI{}}} type 14: proto3 omits zero scalars, but the
    # reference's encodeNode always sets the URI pointer, so an empty URI is still emitted (12 00)
    assert M.encode({"type": "NodeLeave", "node": {"id": "n", "uri": {"scheme": "", "host": "", "port": 0}}}) == \
        b"\x0e\x08\x01\x12\x05\x0a\x01n\x12\x00"
    # NodeStateMessage{NodeID:"a", State:"READY"} type 12
    assert M.encode({"type": "NodeState", "nodeID": "a", "state": "READY"}) == b"\x0c\x0a\x01a\x12\x05READY"
    # CreateIndexMessage{Index:"i", Meta{Keys(3):true, TrackExistence(4):true}} type 1
    assert M.encode({"type": "CreateIndex", "index": "i", "options": {"keys": True, "trackExistence": True}}) == \
        b"\x01\x0a\x01i\x12\x04\x18\x01\x20\x01"


@pytest.mark.parametrize("msg", [
    {"type": "CreateShard", "index": "i", "field": "f", "shard": 12345678901},
    {"type": "CreateIndex", "index": "i", "options": {"keys": False, "trackExistence": True}},
    {"type": "DeleteIndex", "index": "i"},
    {"type": "CreateField", "index": "i", "field": "f",
     "options": {"type": "int", "base": -5, "bitDepth": 9, "min": -10, "max": 300, "keys": False}},
    {"type": "CreateField", "index": "i", "field": "t",
     "options": {"type": "time", "timeQuantum": "YMDH", "keys": True, "noStandardView": True}},
    {"type": "CreateField", "index": "i", "field": "s",
     "options": {"type": "set", "cacheType": "ranked", "cacheSize": 50000, "keys": False}},
    {"type": "DeleteField", "index": "i", "field": "f"},
    {"type": "DeleteAvailableShard", "index": "i", "field": "f", "shard": 7},
    {"type": "CreateView", "index": "i", "field": "f", "view": "standard_2019"},
    {"type": "DeleteView", "index": "i", "field": "f", "view": "standard_2019"},
    {"type": "ResizeInstructionComplete", "jobID": 99, "node": NODE, "error": "boom"},
    {"type": "SetCoordinator", "node": NODE},
    {"type": "UpdateCoordinator", "node": NODE},
    {"type": "NodeState", "nodeID": "node1", "state": "DOWN"},
    {"type": "RecalculateCaches"},
    {"type": "NodeJoin", "node": NODE},
    {"type": "NodeLeave", "node": NODE},
])
def test_roundtrip(msg):
    assert M.decode(M.encode(msg)) == msg


SCHEMA = [{"name": "i", "options": {"keys": True, "trackExistence": False},
           "fields": [{"name": "f", "options": {"type": "set", "cacheType": "ranked", "cacheSize": 100,
                                                 "keys": False},
                       "views": [{"name": "standard"}]}]}]


def test_cluster_status_roundtrip():
    st = {"clusterID": "c-1", "state": "NORMAL",
          "nodes": [dict(NODE, isCoordinator=False), dict(NODE, id="node2", isCoordinator=True)],
          "coordinator": "node2"}
    d = M.decode(M.encode({"type": "ClusterStatus", "status": st, "schema": SCHEMA}))
    assert d == {"type": "ClusterStatus", "status": st}


def test_resize_instruction_roundtrip():
    src = {"node": NODE, "index": "i", "field": "f", "view": "standard", "shard": 3}
    msg = {"type": "ResizeInstruction", "jobID": 1234567890123, "node": NODE, "coordinator": NODE,
           "sources": [src], "schema": SCHEMA,
           "status": {"clusterID": "c", "state": "RESIZING", "nodes": [NODE], "coordinator": "node1"},
           "nodeStatus": {"node": NODE, "schema": SCHEMA, "shards": {"i": {"f": [0, 3, 9]}}}}
    d = M.decode(M.encode(msg))
    assert d["sources"] == [src] and d["schema"] == SCHEMA and d["status"] == msg["status"]
    assert d["nodeStatus"]["shards"] == {"i": {"f": [0, 3, 9]}} and d["jobID"] == msg["jobID"]


def test_apply_schema_travels_as_node_status():
    data = M.encode({"type": "ApplySchema", "schema": SCHEMA}, local_node=NODE)
    assert data[0] == M.TYPE_CODES["NodeStatus"]
    d = M.decode(data)
    assert d["type"] == "NodeStatus" and d["status"]["schema"] == SCHEMA and d["status"]["node"] == NODE


def test_reference_parser_view():
    """What a reference node parses: the extension fields are unknown to
    private.proto and skipped, the rest reads back field-for-field."""
    data = M.encode({"type": "SetCoordinator", "node": NODE})
    m = pb.SetCoordinatorMessage()
    m.ParseFromString(data[1:])
    assert (m.New.ID, m.New.URI.Host, m.New.URI.Port, m.New.IsCoordinator) == ("node1", "h1", 10101, True)


def test_errors():
    with pytest.raises(M.MessageError):
        M.decode(b"")
    with pytest.raises(M.MessageError):
        M.decode(b"\x63")
    with pytest.raises(M.MessageError):
        M.encode({"type": "Bogus"})
    with pytest.raises(M.MessageError):
        M.decode(b"\x00\xff\xff")
