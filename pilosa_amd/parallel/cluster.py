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
import random
import re
import struct
import threading
import time
import urllib.request
import uuid
from typing import Dict, List, Optional, Sequence, Tuple, Union

DEFAULT_PARTITION_N = 256
STATE_STARTING, STATE_DEGRADED, STATE_NORMAL, STATE_RESIZING = "STARTING", "DEGRADED", "NORMAL", "RESIZING"
NODE_READY, NODE_DOWN = "READY", "DOWN"
RESIZE_ACTION_ADD, RESIZE_ACTION_REMOVE = "ADD", "REMOVE"
RESIZE_JOB_RUNNING, RESIZE_JOB_DONE, RESIZE_JOB_ABORTED = "RUNNING", "DONE", "ABORTED"

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


_SCHEME_RE = re.compile(r"^[+a-z]+$")
_HOST_RE = re.compile(r"^[0-9a-z.-]+$|^\[[:0-9a-fA-F]+\]$")
_ADDRESS_RE = re.compile(r"^(([+a-z]+)://)?([0-9a-z.-]+|\[[:0-9a-fA-F]+\])?(:([0-9]+))?$")


class URI:
    """scheme://host:port of a node (reference uri.go): an address parses
    with the reference's grammar (scheme and port optional, IPv6 hosts in
    brackets, defaults http / localhost / 10101); ``normalize`` drops a
    ``+protobuf``-style scheme suffix."""
    __slots__ = ("scheme", "host", "port")

    def __init__(self, scheme="http", host="localhost", port=10101):
        self.scheme, self.host, self.port = scheme, host, int(port)

    @classmethod
    def parse(cls, s: str) -> "URI":
        """NewURIFromAddress (uri.go parseAddress); ValueError when invalid."""
        m = _ADDRESS_RE.match(s)
        if m is None:
            raise ValueError(f"invalid address: {s!r}")
        port = 10101
        if m.group(5):
            port = int(m.group(5))
            if port > 65535:
                raise ValueError("port must be in range 0 - 65535")
        return cls(m.group(2) or "http", m.group(3) or "localhost", port)

    @classmethod
    def from_host_port(cls, host: str, port: int) -> "URI":
        """NewURIFromHostPort: the default scheme with a validated host."""
        u = cls()
        u.set_host(host)
        u.set_port(port)
        return u

    def set_scheme(self, scheme: str):
        if not _SCHEME_RE.match(scheme):
            raise ValueError("invalid scheme")
        self.scheme = scheme

    def set_host(self, host: str):
        if not _HOST_RE.match(host):
            raise ValueError("invalid host")
        self.host = host

    def set_port(self, port: int):
        self.port = int(port)

    def normalize(self) -> str:
        return f"{self.scheme.split('+', 1)[0]}://{self.host}:{self.port}"

    def path(self, p: str) -> str:
        return self.normalize() + p

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


# ---------------------------------------------------------------- Nodes helpers
# (reference cluster.go Nodes: IDs / Filter / FilterURI / Contains / Clone)
def node_ids(nodes: Sequence[Node]) -> List[str]:
    return [n.id for n in nodes]


def filter_nodes(nodes: Sequence[Node], drop: Node) -> List[Node]:
    return [n for n in nodes if n.id != drop.id]


def filter_nodes_uri(nodes: Sequence[Node], uri: URI) -> List[Node]:
    return [n for n in nodes if n.uri != uri]


def contains_node(nodes: Sequence[Node], n: Node) -> bool:
    return any(x.id == n.id for x in nodes)


def clone_nodes(nodes: Sequence[Node]) -> List[Node]:
    return [Node(n.id, URI(n.uri.scheme, n.uri.host, n.uri.port), n.is_coordinator, n.state, n.gpus)
            for n in nodes]


def confirm_node_down(uri: URI, retries: int = 10, sleep: float = 1.0, timeout: float = 2.0,
                      logger=None) -> bool:
    """Guard against false leave events: a node is only DOWN when ``/version``
    fails ``retries`` times in a row (reference confirmNodeDown,
    cluster.go:1699-1726; 10 tries, 1 s apart, 2 s timeout each)."""
    url = f"{uri.scheme}://{uri.host_port()}/version"
    for i in range(retries):
        try:
            with urllib.request.urlopen(url, timeout=timeout) as resp:
                if resp.status == 200:
                    return False
        except Exception as e:  # noqa: BLE001 - any failure counts as a miss
            if logger is not None:
                logger.printf("NodeLeave confirm with %s %d. err: '%s'", uri.host_port(), i, e)
        if i + 1 < retries:
            time.sleep(sleep)
    return True


class ResizeJob:
    """One coordinator-driven resize (reference resizeJob, cluster.go:1420-1545).

    ``ids`` maps every node that must finish its ResizeInstruction to whether
    it has reported completion: on ADD the existing nodes plus the new one, on
    REMOVE every node except the one leaving."""

    def __init__(self, existing: Sequence[Node], node: Node, action: str, job_id: Optional[int] = None):
        if action == RESIZE_ACTION_REMOVE:
            self.ids = {n.id: False for n in existing if n.id != node.id}
        elif action == RESIZE_ACTION_ADD:
            self.ids = {n.id: False for n in existing}
            self.ids[node.id] = False
        else:
            raise ValueError(f"invalid resize action: {action}")
        self.id = job_id if job_id is not None else random.getrandbits(63)
        self.action = action
        self.node = node
        self.nodes: List[Node] = []       # membership once the job commits
        self.state = RESIZE_JOB_RUNNING
        self.errors: List[str] = []
        self.done = threading.Event()

    @property
    def pending(self) -> set:
        return {k for k, v in self.ids.items() if not v}

    @property
    def leaving(self) -> Optional[str]:
        return self.node.id if self.action == RESIZE_ACTION_REMOVE else None

    def mark(self, node_id: str, error: str = "") -> bool:
        """Record one node's completion; True once every node has reported."""
        if error:
            self.errors.append(error)
        if node_id in self.ids:
            self.ids[node_id] = True
        return self.is_complete()

    def is_complete(self) -> bool:
        return all(self.ids.values())

    def finish(self, state: str):
        self.state = state
        self.done.set()


class Topology:
    """Persisted node-id list (``.topology``, protobuf Topology)."""

    def __init__(self, cluster_id: str = "", node_ids: Optional[List[str]] = None):
        self.cluster_id = cluster_id or str(uuid.uuid4())
        self.node_ids = sorted(node_ids or [])

    def contains_id(self, nid: str) -> bool:
        return nid in self.node_ids

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
        # a persisted topology with nodes in it means a restarting cluster that
        # must regain agreement before it serves (cluster.go:1660-1694)
        self.topology_loaded = self.topology is not None and bool(self.topology.node_ids)
        if self.topology is None:
            self.topology = Topology(node_ids=[node.id])
        self.mu = threading.RLock()
        self.coordinator_id = node.id
        node.is_coordinator = True
        self.on_state_change = None

    @classmethod
    def from_nodes(cls, nodes: Sequence[Node], replica_n: int = 1, partition_n: int = DEFAULT_PARTITION_N,
                   hasher=None, local: Optional[Node] = None) -> "Cluster":
        """An in-memory cluster over ``nodes`` (no topology file), as a resize
        plan's from/to side or a test fixture."""
        nodes = sorted(nodes, key=lambda n: n.id)
        c = cls(local or nodes[0], replica_n=replica_n, partition_n=partition_n, hasher=hasher)
        c.nodes = list(nodes)
        c.topology.node_ids = [n.id for n in nodes]
        return c

    # ------------------------------------------------------------ membership
    def node_ids(self) -> List[str]:
        return [n.id for n in self.nodes]

    def check_coordinator_topology(self):
        """The coordinator of a restarting cluster must be in its own persisted
        topology (cluster.go:1686-1689)."""
        from pilosa_amd.errors import PilosaError
        if self.topology_loaded and not self.topology.contains_id(self.node.id):
            raise PilosaError(f"coordinator {self.node.id} is not in topology: "
                              f"[{' '.join(self.topology.node_ids)}]")

    def need_topology_agreement(self) -> bool:
        """STARTING/DEGRADED and the live node set differs from the persisted
        topology (cluster.go:1013)."""
        return self.state in (STATE_STARTING, STATE_DEGRADED) and self.topology.node_ids != self.node_ids()

    def previous_node(self) -> Optional[Node]:
        """The node before this one on the ID-sorted ring (cluster.go:1983)."""
        if len(self.nodes) <= 1:
            return None
        for i, n in enumerate(self.nodes):
            if n.id == self.node.id:
                return self.nodes[i - 1]
        return None

    def update_coordinator(self, n: Node) -> bool:
        """Point the coordinator at ``n``; True if it changed (cluster.go:356)."""
        with self.mu:
            changed = self.coordinator_id != n.id
            self.set_coordinator(n.id)
            return changed

    def set_nodes(self, nodes: Sequence[Node], coordinator_id: Optional[str] = None, exact: bool = False):
        """Adopt a membership list. ``exact`` (a coordinator's status push)
        also drops topology entries the status no longer lists, as
        mergeClusterStatus removes them (cluster.go:1890-1930)."""
        with self.mu:
            by_id = {n.id: n for n in nodes}
            by_id[self.node.id] = by_id.get(self.node.id, self.node)
            self.nodes = sorted(by_id.values(), key=lambda n: n.id)
            if coordinator_id is not None:
                self.coordinator_id = coordinator_id
            for n in self.nodes:
                n.is_coordinator = n.id == self.coordinator_id
            ids = {n.id for n in self.nodes}
            self.topology.node_ids = sorted(ids if exact else set(self.topology.node_ids) | ids)
            self.save_topology()

    def add_node(self, n: Node):
        with self.mu:
            if any(x.id == n.id for x in self.nodes):
                return
            # a joining node describes itself as it sees itself (its own
            # coordinator until it joins); here only the cluster's counts
            n.is_coordinator = n.id == self.coordinator_id
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

    def partition_nodes(self, pid: int, nodes: Optional[List[Node]] = None,
                        replica_n: Optional[int] = None) -> List[Node]:
        nodes = self.nodes if nodes is None else nodes
        if not nodes:
            return []
        rn = self.replica_n if replica_n is None else replica_n
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

    # ------------------------------------------------------------ resize planning
    def frag_combos(self, index: str, shards: Sequence[int], field_views: Dict[str, List[str]],
                    replica_n: Optional[int] = None) -> Dict[str, List[Tuple[str, str, int]]]:
        """Per node id, every (field, view, shard) it holds for ``index``
        (cluster.go:702 fragCombos)."""
        out: Dict[str, List[Tuple[str, str, int]]] = {}
        for shard in sorted(shards):
            for n in self.partition_nodes(self.partition(index, shard), replica_n=replica_n):
                lst = out.setdefault(n.id, [])
                for field in sorted(field_views):
                    for view in field_views[field]:
                        lst.append((field, view, shard))
        return out

    def frags_by_host(self, schema: Dict[str, Dict[str, List[str]]], available: Dict[str, Sequence[int]],
                      replica_n: Optional[int] = None) -> Dict[str, List[Tuple[str, str, str, int]]]:
        """frag_combos over every index: node id -> [(index, field, view, shard)]."""
        out: Dict[str, List[Tuple[str, str, str, int]]] = {}
        for index in sorted(schema):
            for nid, frags in self.frag_combos(index, available.get(index, []), schema[index],
                                               replica_n).items():
                out.setdefault(nid, []).extend((index,) + f for f in frags)
        return out

    def diff(self, other: "Cluster") -> Tuple[str, str]:
        """(action, node id) for a one-node membership change (cluster.go:721)."""
        from pilosa_amd.errors import PilosaError
        nf, nt = len(self.nodes), len(other.nodes)
        if nf == nt:
            raise PilosaError("clusters are the same size")
        if nf < nt:
            if nt - nf > 1:
                raise PilosaError("adding more than one node at a time is not supported")
            mine = set(self.node_ids())
            return RESIZE_ACTION_ADD, next(n.id for n in other.nodes if n.id not in mine)
        if nf - nt > 1:
            raise PilosaError("removing more than one node at a time is not supported")
        theirs = set(other.node_ids())
        return RESIZE_ACTION_REMOVE, next(n.id for n in self.nodes if n.id not in theirs)

    def frag_sources(self, to: Union["Cluster", List[Node]], holder_schema: Dict[str, Dict[str, List[str]]],
                     available: Dict[str, Sequence[int]]) -> Dict[str, List[dict]]:
        """For a resize from this membership to ``to``: per destination node
        id, the fragments it lacks and which current node serves each
        (cluster.go:760-844 fragSources).

        Adding a node only ever reads primaries (a replica-1 view of the old
        cluster); removing one reads whichever surviving node holds the
        fragment, so ReplicaN must be high enough to cover the leaver."""
        from pilosa_amd.errors import PilosaError
        if not isinstance(to, Cluster):
            to = Cluster.from_nodes(to, replica_n=self.replica_n, partition_n=self.partition_n,
                                    hasher=self.hasher)
        action, diff_id = self.diff(to)
        src_rn = 1 if action == RESIZE_ACTION_ADD and self.replica_n > 1 else None
        have = self.frags_by_host(holder_schema, available)
        want = to.frags_by_host(holder_schema, available)
        src_by_frag: Dict[tuple, str] = {}
        for nid, frags in sorted(self.frags_by_host(holder_schema, available, src_rn).items()):
            if action == RESIZE_ACTION_REMOVE and nid == diff_id:
                continue
            for fr in frags:
                src_by_frag.setdefault(fr, nid)
        out: Dict[str, List[dict]] = {n.id: [] for n in to.nodes}
        for nid, frags in want.items():
            held = set(have.get(nid, ()))
            for fr in frags:
                if fr in held:
                    continue
                src = src_by_frag.get(fr)
                if src is None:
                    raise PilosaError("not enough data to perform resize (replica factor may need to be increased)")
                index, field, view, shard = fr
                out[nid].append({"node": self.node_by_id(src).to_json(), "index": index, "field": field,
                                 "view": view, "shard": shard})
        return out

    def status(self) -> dict:
        with self.mu:
            return {"clusterID": self.topology.cluster_id, "state": self.state,
                    "nodes": [n.to_json() for n in self.nodes]}
