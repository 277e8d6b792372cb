"""Internal cluster messages on the reference's wire format.

A message is one type byte followed by the protobuf encoding of the
matching ``internal.*`` message (reference broadcast.go:56-161
MarshalInternalMessage / getMessage, encoding/proto/proto.go), POSTed to
``/internal/cluster/message`` as ``application/x-protobuf``.  The runtime
works on plain dicts (``{"type": "CreateShard", ...}``); this module is the
only place that knows the byte layout.

Type bytes 0-15 are the reference's iota order.  Three of our dict types
have no reference tag and are mapped onto reference messages instead:

* ``ApplySchema``   -> ``NodeStatus`` carrying only the schema (what the
  reference gossips schema with);
* ``NodeJoin`` / ``NodeLeave`` -> ``NodeEvent`` with Event 0 / 1;
* ``DeleteAvailableShard`` gets tag 16: the reference sends this message
  (api.go:483) but has no tag for it (getMessageType panics), so there is
  no wire behaviour to match.

Fields the reference's schema has no slot for (index options, a node's GPU
count) travel in extension field numbers >= 100, which reference nodes skip
as unknown fields.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from pilosa_amd.wire import pb

TYPE_NAMES = ["CreateShard", "CreateIndex", "DeleteIndex", "CreateField", "DeleteField", "CreateView", "DeleteView",
              "ClusterStatus", "ResizeInstruction", "ResizeInstructionComplete", "SetCoordinator",
              "UpdateCoordinator", "NodeState", "RecalculateCaches", "NodeEvent", "NodeStatus",
              "DeleteAvailableShard"]
TYPE_CODES = {n: i for i, n in enumerate(TYPE_NAMES)}
NODE_EVENTS = ["NodeJoin", "NodeLeave", "NodeUpdate"]     # cluster.go NodeEventType iota
CONTENT_TYPE = "application/x-protobuf"


class MessageError(ValueError):
    pass


# ---------------------------------------------------------------- leaves
def _node_pb(d: Optional[dict]):
    m = pb.Node()
    if not d:
        return m
    m.ID = d.get("id", "")
    u = d.get("uri") or {}
    m.URI.Scheme = u.get("scheme", "http")
    m.URI.Host = u.get("host", "")
    m.URI.Port = int(u.get("port", 0))
    m.IsCoordinator = bool(d.get("isCoordinator", False))
    m.State = d.get("state", "") or ""
    m.GPUs = int(d.get("gpus", 0) or 0)
    return m


def _node_dict(m) -> dict:
    return {"id": m.ID, "uri": {"scheme": m.URI.Scheme or "http", "host": m.URI.Host, "port": m.URI.Port},
            "isCoordinator": m.IsCoordinator, "state": m.State, "gpus": m.GPUs}


def _field_options_pb(o: dict):
    from pilosa_amd.models.field import FieldOptions
    fo = FieldOptions(type=o.get("type", "set"), cache_type=o.get("cacheType", ""),
                      cache_size=o.get("cacheSize", 0), time_quantum=o.get("timeQuantum", ""),
                      min=o.get("min", 0), max=o.get("max", 0), keys=o.get("keys", False),
                      no_standard_view=o.get("noStandardView", False), base=o.get("base", 0),
                      bit_depth=o.get("bitDepth", 0))
    return fo.to_pb()


def _field_options_dict(m) -> dict:
    from pilosa_amd.models.field import FieldOptions
    return FieldOptions.from_pb(m).to_json()


def _schema_pb(schema: List[dict], out):
    for ii in schema or []:
        im = out.Indexes.add(Name=ii["name"])
        opts = ii.get("options") or {}
        im.Meta.Keys = bool(opts.get("keys", False))
        im.Meta.TrackExistence = bool(opts.get("trackExistence", True))
        for fi in ii.get("fields", []):
            fm = im.Fields.add(Name=fi["name"])
            fm.Meta.CopyFrom(_field_options_pb(fi.get("options") or {}))
            fm.Views.extend(v["name"] if isinstance(v, dict) else v for v in fi.get("views", []))


def _schema_list(m) -> List[dict]:
    out = []
    for im in m.Indexes:
        opts = {"keys": im.Meta.Keys, "trackExistence": im.Meta.TrackExistence} if im.HasField("Meta") \
            else {"keys": False, "trackExistence": True}
        out.append({"name": im.Name, "options": opts,
                    "fields": [{"name": fm.Name, "options": _field_options_dict(fm.Meta),
                                "views": [{"name": v} for v in fm.Views]} for fm in im.Fields]})
    return out


def _node_status_pb(st: dict, out):
    if st.get("node"):
        out.Node.CopyFrom(_node_pb(st["node"]))
    _schema_pb(st.get("schema") or [], out.Schema)
    for index in sorted(st.get("shards") or {}):
        im = out.Indexes.add(Name=index)
        for fname in sorted(st["shards"][index]):
            im.Fields.add(Name=fname, AvailableShards=[int(s) for s in st["shards"][index][fname]])


def _node_status_dict(m) -> dict:
    return {"node": _node_dict(m.Node) if m.HasField("Node") else None, "schema": _schema_list(m.Schema),
            "shards": {im.Name: {fm.Name: list(fm.AvailableShards) for fm in im.Fields} for im in m.Indexes}}


def _cluster_status_pb(st: dict, out):
    out.ClusterID = st.get("clusterID", "")
    out.State = st.get("state", "")
    coord = st.get("coordinator")
    for nd in st.get("nodes", []):
        n = out.Nodes.add()
        n.CopyFrom(_node_pb(nd))
        if coord is not None:
            n.IsCoordinator = nd.get("id") == coord


def _cluster_status_dict(m) -> dict:
    nodes = [_node_dict(n) for n in m.Nodes]
    coord = next((n["id"] for n in nodes if n["isCoordinator"]), None)
    d = {"clusterID": m.ClusterID, "state": m.State, "nodes": nodes}
    if coord is not None:
        d["coordinator"] = coord
    return d


# ---------------------------------------------------------------- encode
def encode(msg: dict, local_node: Optional[dict] = None) -> bytes:
    """dict message -> type byte + protobuf (MarshalInternalMessage)."""
    t = msg["type"]
    if t == "CreateShard":
        m = pb.CreateShardMessage(Index=msg["index"], Field=msg["field"], Shard=int(msg["shard"]))
    elif t == "CreateIndex":
        o = msg.get("options") or {}
        m = pb.CreateIndexMessage(Index=msg["index"])
        m.Meta.Keys = bool(o.get("keys", False))
        m.Meta.TrackExistence = bool(o.get("trackExistence", True))
    elif t == "DeleteIndex":
        m = pb.DeleteIndexMessage(Index=msg["index"])
    elif t == "CreateField":
        m = pb.CreateFieldMessage(Index=msg["index"], Field=msg["field"])
        m.Meta.CopyFrom(_field_options_pb(msg.get("options") or {}))
    elif t == "DeleteField":
        m = pb.DeleteFieldMessage(Index=msg["index"], Field=msg["field"])
    elif t == "DeleteAvailableShard":
        m = pb.DeleteAvailableShardMessage(Index=msg["index"], Field=msg["field"], ShardID=int(msg["shard"]))
    elif t == "CreateView":
        m = pb.CreateViewMessage(Index=msg["index"], Field=msg["field"], View=msg["view"])
    elif t == "DeleteView":
        m = pb.DeleteViewMessage(Index=msg["index"], Field=msg["field"], View=msg["view"])
    elif t == "ClusterStatus":
        m = pb.ClusterStatus()
        _cluster_status_pb(msg["status"], m)
    elif t == "ResizeInstruction":
        m = pb.ResizeInstruction(JobID=int(msg["jobID"]))
        m.Node.CopyFrom(_node_pb(msg["node"]))
        m.Coordinator.CopyFrom(_node_pb(msg["coordinator"]))
        for s in msg.get("sources", []):
            sm = m.Sources.add(Index=s["index"], Field=s["field"], View=s["view"], Shard=int(s["shard"]))
            sm.Node.CopyFrom(_node_pb(s["node"]))
        st = dict(msg.get("nodeStatus") or {})
        if msg.get("schema") is not None:
            st["schema"] = msg["schema"]
        _node_status_pb(st, m.NodeStatus)
        _cluster_status_pb(msg.get("status") or {}, m.ClusterStatus)
    elif t == "ResizeInstructionComplete":
        m = pb.ResizeInstructionComplete(JobID=int(msg["jobID"]), Error=msg.get("error") or "")
        m.Node.CopyFrom(_node_pb(msg["node"]))
    elif t in ("SetCoordinator", "UpdateCoordinator"):
        m = (pb.SetCoordinatorMessage if t == "SetCoordinator" else pb.UpdateCoordinatorMessage)()
        m.New.CopyFrom(_node_pb(msg["node"]))
    elif t == "NodeState":
        m = pb.NodeStateMessage(NodeID=msg["nodeID"], State=msg["state"])
    elif t == "RecalculateCaches":
        m = pb.RecalculateCaches()
    elif t in NODE_EVENTS:
        m = pb.NodeEventMessage(Event=NODE_EVENTS.index(t))
        m.Node.CopyFrom(_node_pb(msg["node"]))
        t = "NodeEvent"
    elif t == "NodeStatus":
        m = pb.NodeStatus()
        _node_status_pb(msg.get("status") or msg, m)
    elif t == "ApplySchema":
        m = pb.NodeStatus()
        _node_status_pb({"node": local_node, "schema": msg["schema"]}, m)
        t = "NodeStatus"
    else:
        raise MessageError(f"don't have type for message {t}")
    return bytes([TYPE_CODES[t]]) + m.SerializeToString()


# ---------------------------------------------------------------- decode
def decode(data: bytes) -> dict:
    """type byte + protobuf -> dict message (getMessage + Unmarshal)."""
    if not data:
        raise MessageError("empty message")
    code = data[0]
    if code >= len(TYPE_NAMES):
        raise MessageError(f"unknown message type {code}")
    t = TYPE_NAMES[code]
    body = bytes(data[1:])
    cls = {"CreateShard": pb.CreateShardMessage, "CreateIndex": pb.CreateIndexMessage,
           "DeleteIndex": pb.DeleteIndexMessage, "CreateField": pb.CreateFieldMessage,
           "DeleteField": pb.DeleteFieldMessage, "CreateView": pb.CreateViewMessage,
           "DeleteView": pb.DeleteViewMessage, "ClusterStatus": pb.ClusterStatus,
           "ResizeInstruction": pb.ResizeInstruction, "ResizeInstructionComplete": pb.ResizeInstructionComplete,
           "SetCoordinator": pb.SetCoordinatorMessage, "UpdateCoordinator": pb.UpdateCoordinatorMessage,
           "NodeState": pb.NodeStateMessage, "RecalculateCaches": pb.RecalculateCaches,
           "NodeEvent": pb.NodeEventMessage, "NodeStatus": pb.NodeStatus,
           "DeleteAvailableShard": pb.DeleteAvailableShardMessage}[t]
    m = cls()
    try:
        m.ParseFromString(body)
    except Exception as e:  # noqa: BLE001 - DecodeError and friends
        raise MessageError(f"unmarshaling {t}: {e}") from e
    if t == "CreateShard":
        return {"type": t, "index": m.Index, "field": m.Field, "shard": m.Shard}
    if t == "CreateIndex":
        return {"type": t, "index": m.Index,
                "options": {"keys": m.Meta.Keys, "trackExistence": m.Meta.TrackExistence}}
    if t == "DeleteIndex":
        return {"type": t, "index": m.Index}
    if t == "CreateField":
        return {"type": t, "index": m.Index, "field": m.Field, "options": _field_options_dict(m.Meta)}
    if t == "DeleteField":
        return {"type": t, "index": m.Index, "field": m.Field}
    if t == "DeleteAvailableShard":
        return {"type": t, "index": m.Index, "field": m.Field, "shard": m.ShardID}
    if t in ("CreateView", "DeleteView"):
        return {"type": t, "index": m.Index, "field": m.Field, "view": m.View}
    if t == "ClusterStatus":
        return {"type": t, "status": _cluster_status_dict(m)}
    if t == "ResizeInstruction":
        ns = _node_status_dict(m.NodeStatus)
        return {"type": t, "jobID": m.JobID, "node": _node_dict(m.Node), "coordinator": _node_dict(m.Coordinator),
                "sources": [{"node": _node_dict(s.Node), "index": s.Index, "field": s.Field, "view": s.View,
                             "shard": s.Shard} for s in m.Sources],
                "schema": ns["schema"], "nodeStatus": ns, "status": _cluster_status_dict(m.ClusterStatus)}
    if t == "ResizeInstructionComplete":
        return {"type": t, "jobID": m.JobID, "node": _node_dict(m.Node), "error": m.Error}
    if t in ("SetCoordinator", "UpdateCoordinator"):
        return {"type": t, "node": _node_dict(m.New)}
    if t == "NodeState":
        return {"type": t, "nodeID": m.NodeID, "state": m.State}
    if t == "RecalculateCaches":
        return {"type": t}
    if t == "NodeEvent":
        if m.Event >= len(NODE_EVENTS):
            raise MessageError(f"unknown node event {m.Event}")
        return {"type": NODE_EVENTS[m.Event], "node": _node_dict(m.Node)}
    # NodeStatus
    return {"type": "NodeStatus", "status": _node_status_dict(m)}
