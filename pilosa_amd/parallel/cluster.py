"""Cluster topology, shard placement and node state (reference: cluster.go).

Placement is bit-compatible with the reference so that a mixed deployment
agrees on shard ownership:

    partition = fnv64a(index || bigendian_u64(shard)) % partitionN   (256)
    primary   = jump_hash(partition, len(nodes))   over nodes sorted by ID
    replicas  = the next ReplicaN-1 nodes around the ring

Inside a node the shards a node owns are further split across its GPUs as
contiguous ranges (pilosa_amd/parallel/multi_gpu.py) — that level is ours.

Cluster states STARTING / NORMAL / DEGRADED / RESIZING and node states
READY / DOWN follow cluster.go:40-60 and determineClusterState (:547-558).
"""
from __future__ import annotations

import json
import os
import struct
import threading
import uuid
from typing import Dict, List, Optional, Sequence
from urllib.parse import urlparse

DEFAULT_PARTITION_N = 256
STATE_STARTING, STATE_DEGRADED, STATE_NORMAL, STATE_RESIZING = "STARTING", "DEGRADED", "NORMAL", "RESIZING"
NODE_READY, NODE_DOWN = "READY", "DOWN"

_FNV64_OFFSET = 0xcbf29ce484222325
_FNV64_PRIME = 0x100000001b3
_M64 = (1 << 64) - 1


def fnv64a(data: bytes, h: int = _FNV64_OFFSET) -> int:
    for b in data:
        h ^= b
        h = (h * _FNV64_PRIME) & _M64
    return h


def jump_hash(key: int, n: int) -> int:
    """Float-based jump consistent hash exactly as cluster.go:923-934."""
    b, j = -1, 0
    key &= _M64
    while j < n:
        b = j
        key = (key * 2862933555777941757 + 1) & _M64
        j = int(float(b + 1) * (float(1 << 31) / float((key >> 33) + 1)))
    return b


class ModHasher:
    """Deterministic key % n placement for tests (reference test/cluster.go)."""

    def hash(self, key: int, n: int) -> int:
        return key % n if n else 0


class JumpHasher:
    def hash(self, key: int, n: int) -> int:
        return jump_hash(key, n)


class URI:
    __slots__ = ("scheme", "host", "port")

    def __init__(self, scheme="http", host="localhost", port=10101):
        self.scheme, self.host, self.port = scheme, host, int(port)

    @classmethod
    def parse(cls, s: str) -> "URI":
        if "://" not in s:
            s = "http://" + s
        u = urlparse(s)
        return cls(u.scheme or "http", u.hostname or "localhost", u.port or 10101)

    def normalize(self) -> str:
        return f"{self.scheme}://{self.host}:{self.port}"

    def host_port(self) -> str:
        return f"{self.host}:{self.port}"

    def to_json(self):
        return {"scheme": self.scheme, "host": self.host, "port": self.port}

    @classmethod
    def from_json(cls, d):
        return cls(d.get("scheme", "http"), d.get("host", "localhost"), d.get("port", 10101))

    def __eq__(self, o):
        return isinstance(o, URI) and self.normalize() == o.normalize()

    def __hash__(self):
        return hash(self.normalize())

    def __repr__(self):
        return self.normalize()


class Node:
    __slots__ = ("id", "uri", "is_coordinator", "state", "gpus")

    def __init__(self, id: str, uri: URI, is_coordinator=False, state=NODE_DOWN, gpus=0):
        self.id, self.uri, self.is_coordinator, self.state, self.gpus = id, uri, is_coordinator, state, gpus

    def to_json(self):
        return {"id": self.id, "uri": self.uri.to_json(), "isCoordinator": self.is_coordinator,
                "state": self.state, "gpus": self.gpus}

    @classmethod
    def from_json(cls, d):
        return cls(d["id"], URI.from_json(d.get("uri", {})), d.get("isCoordinator", False),
                   d.get("state", NODE_DOWN), d.get("gpus", 0))

    def __eq__(self, o):
        return isinstance(o, Node) and self.id == o.id

    def __hash__(self):
        return hash(self.id)

    def __repr__(self):
        return f"Node({self.id}@{self.uri}, {self.state}{', coord' if self.is_coordinator else ''})"


class Topology:
    """Persisted node-id list (``.topology``, protobuf Topology)."""

    def __init__(self, cluster_id: str = "", node_ids: Optional[List[str]] = None):
        self.cluster_id = cluster_id or str(uuid.uuid4())
        self.node_ids = sorted(node_ids or [])

    def save(self, path: str):
        from pilosa_amd.wire import pb
        with open(path, "wb") as fh:
            fh.write(pb.Topology(ClusterID=self.cluster_id, NodeIDs=self.node_ids).SerializeToString())

    @classmethod
    def load(cls, path: str) -> Optional["Topology"]:
        from pilosa_amd.wire import pb
        if not os.path.exists(path):
            return None
        m = pb.Topology()
        with open(path, "rb") as fh:
            m.ParseFromString(fh.read())
        return cls(m.ClusterID, list(m.NodeIDs))


class Cluster:
    def __init__(self, node: Node, replica_n: int = 1, partition_n: int = DEFAULT_PARTITION_N, hasher=None,
                 path: Optional[str] = None):
        self.node = node
        self.nodes: List[Node] = [node]
        self.replica_n = replica_n
        self.partition_n = partition_n
        self.hasher = hasher or JumpHasher()
        self.state = STATE_STARTING
        self.path = path
        self.topology = Topology.load(os.path.join(path, ".topology")) if path else None
        if self.topology is None:
            self.topology = Topology(node_ids=[node.id])
        self.mu = threading.RLock()
        self.coordinator_id = node.id
        node.is_coordinator = True
        self.on_state_change = None

    # ------------------------------------------------------------ membership
    def set_nodes(self, nodes: Sequence[Node], coordinator_id: Optional[str] = None):
        with self.mu:
            by_id = {n.id: n for n in nodes}
            by_id[self.node.id] = by_id.get(self.node.id, self.node)
            self.nodes = sorted(by_id.values(), key=lambda n: n.id)
            if coordinator_id is not None:
                self.coordinator_id = coordinator_id
            for n in self.nodes:
                n.is_coordinator = n.id == self.coordinator_id
            self.topology.node_ids = sorted(set(self.topology.node_ids) | {n.id for n in self.nodes})
            self.save_topology()

    def add_node(self, n: Node):
        with self.mu:
            if any(x.id == n.id for x in self.nodes):
                return
            self.nodes = sorted(self.nodes + [n], key=lambda x: x.id)
            if n.id not in self.topology.node_ids:
                self.topology.node_ids = sorted(self.topology.node_ids + [n.id])
                self.save_topology()

    def remove_node(self, node_id: str):
        with self.mu:
            self.nodes = [n for n in self.nodes if n.id != node_id]
            if node_id in self.topology.node_ids:
                self.topology.node_ids.remove(node_id)
                self.save_topology()

    def save_topology(self):
        if self.path:
            os.makedirs(self.path, exist_ok=True)
            self.topology.save(os.path.join(self.path, ".topology"))

    def node_by_id(self, nid: str) -> Optional[Node]:
        for n in self.nodes:
            if n.id == nid:
                return n
        return None

    def coordinator(self) -> Optional[Node]:
        return self.node_by_id(self.coordinator_id)

    def is_coordinator(self) -> bool:
        return self.coordinator_id == self.node.id

    def set_coordinator(self, nid: str):
        with self.mu:
            self.coordinator_id = nid
            for n in self.nodes:
                n.is_coordinator = n.id == nid

    def set_node_state(self, nid: str, state: str) -> bool:
        with self.mu:
            n = self.node_by_id(nid)
            if n is None or n.state == state:
                return False
            n.state = state
            return True

    def all_nodes_ready(self) -> bool:
        return all(n.state == NODE_READY for n in self.nodes)

    def determine_state(self) -> str:
        with self.mu:
            if self.state == STATE_RESIZING:
                return STATE_RESIZING
            live = {n.id for n in self.nodes if n.state == NODE_READY}
            topo = set(self.topology.node_ids)
            if topo <= {n.id for n in self.nodes} and self.all_nodes_ready():
                return STATE_NORMAL
            if len(topo - live) < self.replica_n and live:
                return STATE_DEGRADED
            return STATE_STARTING

    def set_state(self, state: str):
        with self.mu:
            changed = state != self.state
            self.state = state
        if changed and self.on_state_change is not None:
            self.on_state_change(state)

    # ------------------------------------------------------------ placement
    def partition(self, index: str, shard: int) -> int:
        h = fnv64a(index.encode() + struct.pack(">Q", int(shard)))
        return h % self.partition_n

    def partition_nodes(self, pid: int, nodes: Optional[List[Node]] = None) -> List[Node]:
        nodes = self.nodes if nodes is None else nodes
        if not nodes:
            return []
        rn = self.replica_n
        if rn > len(nodes):
            rn = len(nodes)
        elif rn == 0:
            rn = 1
        i = self.hasher.hash(pid, len(nodes))
        return [nodes[(i + k) % len(nodes)] for k in range(rn)]

    def shard_nodes(self, index: str, shard: int) -> List[Node]:
        with self.mu:
            return self.partition_nodes(self.partition(index, shard))

    def owns_shard(self, node_id: str, index: str, shard: int) -> bool:
        return any(n.id == node_id for n in self.shard_nodes(index, shard))

    def contains_shards(self, index: str, shards: Sequence[int], node: Node) -> List[int]:
        return [s for s in shards if any(n.id == node.id for n in self.shard_nodes(index, s))]

    def frag_sources(self, to_nodes: List[Node], holder_schema: Dict[str, Dict[str, List[str]]],
                     available: Dict[str, List[int]]) -> Dict[str, List[dict]]:
        """For a resize from self.nodes to ``to_nodes``: per destination node
        id, the fragments it must fetch and from which current owner
        (cluster.go:760-844 fragSources)."""
        out: Dict[str, List[dict]] = {n.id: [] for n in to_nodes}
        from_nodes = list(self.nodes)
        for index, fields in holder_schema.items():
            for shard in available.get(index, []):
                pid = self.partition(index, shard)
                old = {n.id for n in self.partition_nodes(pid, from_nodes)}
                new = self.partition_nodes(pid, sorted(to_nodes, key=lambda n: n.id))
                src = [n for n in self.partition_nodes(pid, from_nodes) if n.state != NODE_DOWN] or \
                    self.partition_nodes(pid, from_nodes)
                for dst in new:
                    if dst.id in old:
                        continue
                    for field, views in fields.items():
                        for view in views:
                            out[dst.id].append({"node": src[0].to_json(), "index": index, "field": field,
                                                "view": view, "shard": shard})
        return out

    def status(self) -> dict:
        with self.mu:
            return {"clusterID": self.topology.cluster_id, "state": self.state,
                    "nodes": [n.to_json() for n in self.nodes]}
