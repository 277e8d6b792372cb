"""Node runtime (reference: server.go, server/server.go, cluster.go resize,
holder.go syncer/cleaner, gossip/).

Wires holder + cluster + executor (+ GPU executor) + API + HTTP handler and
runs the background loops:

* membership: every node runs SWIM-style failure detection
  (parallel/swim.py, the ``[gossip]`` probe-interval / probe-timeout /
  suspicion-mult / nodes keys that drive memberlist in the reference):
  direct ``/version`` probes, indirect probes through peers
  (``/internal/probe``), suspicion timeout -> DOWN; the coordinator applies
  the verdicts and pushes the cluster status; joining nodes announce
  themselves to the coordinator; NodeStatus push-pull gossip spreads schema
  and shards;
* resize: node join/leave with data -> coordinator computes per-node fragment
  sources (cluster.frag_sources), nodes stream fragments over HTTP, report
  completion, coordinator commits the topology, nodes drop fragments they no
  longer own (holderCleaner);
* anti-entropy (ReplicaN > 1): block checksum compare, majority-vote merge,
  attribute diffs (holder.go:683-839, fragment.go:2849-3014);
* cache flush (holder.go:506) and runtime/GPU gauges.
"""
from __future__ import annotations

import base64
import io
import os
import threading
import time
from typing import Dict, List, Optional

import numpy as np

from pilosa_amd.executor import Executor
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.holder import Holder
from pilosa_amd.errors import PilosaError
from pilosa_amd.parallel.cluster import (NODE_DOWN, NODE_READY, RESIZE_ACTION_ADD, RESIZE_ACTION_REMOVE,
                                         RESIZE_JOB_ABORTED, RESIZE_JOB_DONE, STATE_DEGRADED, STATE_NORMAL,
                                         STATE_RESIZING, STATE_STARTING, Cluster, JumpHasher, ModHasher, Node, ResizeJob, URI)
from pilosa_amd.server.api import API
from pilosa_amd.shardwidth import SHARD_WIDTH
from pilosa_amd.server.client import InternalClient
from pilosa_amd.server.http_handler import Handler, make_http_server
from pilosa_amd.utils.logger import NopLogger, StandardLogger
from pilosa_amd.utils.stats import NopStatsClient, new_stats_client


def _gpu_present() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def _ssl_ctx(skip_verify: bool):
    import ssl
    if not skip_verify:
        return None
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    return ctx


def _probe_version(uri, timeout: float, skip_verify: bool = False) -> bool:
    """One liveness probe: GET /version answered 200 within ``timeout``."""
    from urllib import request as _rq
    url = f"{uri.scheme}://{uri.host_port()}/version"
    try:
        with _rq.urlopen(url, timeout=timeout, context=_ssl_ctx(skip_verify) if uri.scheme == "https" else None) as r:
            return r.status == 200
    except Exception:  # noqa: BLE001 - any failure is a missed ack
        return False


class Server:
    def __init__(self, data_dir: str, bind: str = "127.0.0.1:10101", node_id: Optional[str] = None,
                 replica_n: int = 1, hosts: Optional[List[str]] = None, coordinator: bool = True,
                 coordinator_uri: Optional[str] = None, gpu: str = "auto", workers: int = 8,
                 max_writes: int = 5000, anti_entropy_interval: float = 600.0, probe_interval: float = 1.0,
                 long_query_time: float = 60.0, stats: str = "expvar", logger=None, hasher: str = "jump",
                 max_opn: int = 10000, cluster_disabled: bool = False, mesh_block: int = 1,
                 translation_primary_url: str = "", tls_certificate: str = "", tls_key: str = "",
                 tls_skip_verify: bool = False, diagnostics_host: str = "", diagnostics_interval: Optional[float] = None,
                 gpu_device: Optional[int] = None, hbm_budget: int = 0, mesh_timeout_s: float = 120.0,
                 lazy_fragments: Optional[bool] = None, native_http: Optional[bool] = None,
                 gossip_interval: float = 30.0, allowed_origins: Optional[List[str]] = None,
                 advertise: str = "", probe_timeout: float = 0.5, suspicion_mult: float = 4,
                 indirect_checks: int = 3, to_the_dead_time: float = 30.0, stream_timeout: float = 10.0,
                 gossip_nodes: int = 3, gossip_port: int = 0, gossip_key: Optional[bytes] = None,
                 gossip_peer_ports: Optional[Dict[str, int]] = None):
        self.data_dir = data_dir
        # CORS origins ([handler] allowed-origins); none = no CORS headers at all
        self.allowed_origins = list(allowed_origins or [])
        # address other nodes reach this one at ([advertise], server/config.go
        # validateAdvertiseAddr); empty = the listen address
        self.advertise = advertise
        # native epoll front end (native/httpd.cpp) unless TLS is configured
        if native_http is None:
            native_http = os.environ.get("PILOSA_NATIVE_HTTP", "1") != "0"
        self.native_http = bool(native_http) and not (tls_certificate and tls_key)
        self.mesh_timeout_s = mesh_timeout_s
        self.bind = bind
        self.logger = logger or StandardLogger()
        self.stats = new_stats_client(stats) if isinstance(stats, str) else (stats or NopStatsClient())
        # a GPU node reads cold fragments straight into HBM (ops/loader.py); the
        # host copy of a fragment is only materialised when a host path needs it
        if lazy_fragments is None or lazy_fragments:
            lazy_fragments = (gpu or "auto").lower() not in ("off", "none", "cpu") and _gpu_present()
        self.holder = Holder(data_dir, max_opn=max_opn, stats=self.stats, lazy_fragments=lazy_fragments)
        self.holder.logger = self.logger
        self.client = InternalClient()
        # liveness probes use a short timeout so a hung peer is noticed quickly
        # (reference confirmNodeDown: 2 s per /version attempt, cluster.go:1699-1726)
        self.probe_client = InternalClient(timeout=2.0)
        # NodeStatus push-pull ([gossip] stream-timeout, memberlist TCPTimeout)
        self.stream_client = InternalClient(timeout=stream_timeout)
        self.long_query_time = long_query_time
        self.anti_entropy_interval = anti_entropy_interval
        self.probe_interval = probe_interval
        # [gossip] failure detection (parallel/swim.py, memberlist's settings in
        # the reference, gossip/gossip.go:269-272)
        self.probe_timeout = probe_timeout
        self.suspicion_mult = suspicion_mult
        self.indirect_checks = indirect_checks
        # [gossip] nodes: peers each push-pull round sends this node's state to
        # (memberlist GossipNodes, gossip/gossip.go:273 -- the fan-out, not the
        # indirect-probe count, which stays memberlist's fixed 3)
        self.gossip_nodes = max(1, int(gossip_nodes))
        # [gossip] port / key: SWIM probes over UDP on that port, HMAC-tagged
        # with the key (parallel/gossip_udp.py); 0 = probes over the HTTP port.
        # A peer's gossip port is the same port unless listed (one host, tests)
        self.gossip_port = int(gossip_port or 0)
        self.gossip_key = gossip_key
        self.gossip_peer_ports: Dict[str, int] = dict(gossip_peer_ports or {})
        self.udp_prober = None
        self.to_the_dead_time = to_the_dead_time
        self.stream_timeout = stream_timeout
        self.failure_detector = None
        self._down_since: Dict[str, float] = {}
        self.gossip_interval = gossip_interval
        self._gossip_i = 0
        self._gossip_misses: Dict[str, int] = {}
        self.hosts = [URI.parse(h) for h in (hosts or [])]
        self.coordinator_uri = URI.parse(coordinator_uri) if coordinator_uri else None
        self.is_coordinator_cfg = coordinator
        self.cluster_disabled = cluster_disabled
        self._node_id = node_id
        self.replica_n = replica_n
        # "jump" (the reference's default), "mod", or a hasher object with hash(key, n)
        self.hasher = hasher if hasattr(hasher, "hash") else ModHasher() if hasher == "mod" else JumpHasher()
        self.gpu = None
        self.gpu_mode = gpu
        self.gpu_device = gpu_device
        self.hbm_budget = hbm_budget
        self.mesh = None          # multi-GPU node: parallel.mesh.ShardMesh (this process is rank 0)
        self.mesh_block = mesh_block
        self.translation_primary = URI.parse(translation_primary_url) if translation_primary_url else None
        self.tls_certificate, self.tls_key = tls_certificate, tls_key
        self.client.skip_verify = self.probe_client.skip_verify = self.stream_client.skip_verify = tls_skip_verify
        self.diagnostics = None
        from pilosa_amd import buildinfo
        # release builds report hourly, others not at all (server/release.go, default.go)
        self.diagnostics_host = diagnostics_host
        self.diagnostics_interval = buildinfo.DEFAULT_DIAGNOSTICS_INTERVAL if diagnostics_interval is None \
            else diagnostics_interval
        self.gc_notifier = None
        self.workers = workers
        self.max_writes = max_writes
        self.cluster: Optional[Cluster] = None
        self.executor: Optional[Executor] = None
        self.api = API(self)
        self.handler = None
        self.httpd = None
        self._closing = threading.Event()
        self._threads: List[threading.Thread] = []
        self._misses: Dict[str, int] = {}
        self._resize: Optional[ResizeJob] = None
        self.join_error: Optional[str] = None
        self.mu = threading.RLock()

    # ------------------------------------------------------------ lifecycle
    def open(self):
        self.holder.open(background=True)
        nid = self._node_id or self.holder.load_node_id()
        host, _, port = self.bind.rpartition(":")
        handler = Handler(self.api, self, self.logger, self.stats)
        handler.allowed_origins = self.allowed_origins
        self.handler = handler
        self.httpd = None
        if self.native_http:
            from pilosa_amd.server import native_http
            if native_http.available():
                self.httpd = native_http.make_native_http_server(handler, self.bind)
        if self.httpd is None:
            self.httpd = make_http_server(handler, self.bind)
        scheme = "http"
        if self.tls_certificate and self.tls_key:
            import ssl
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(self.tls_certificate, self.tls_key)
            self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True)
            scheme = "https"
        port = self.httpd.server_address[1]
        adv = host if host not in ("", "0.0.0.0") else "127.0.0.1"
        if self.advertise:
            a = URI.parse(self.advertise)
            adv, port = a.host or adv, a.port or port
        self.node = Node(nid, URI(scheme, adv, port), state=NODE_READY)
        self.client.local_node = self.node.to_json()
        self.cluster = Cluster(self.node, replica_n=self.replica_n, hasher=self.hasher, path=self.data_dir)
        self.cluster.on_state_change = lambda s: self.logger.debugf("cluster state -> %s", s)
        self._init_gpu()
        self.executor = Executor(self.holder, cluster=self.cluster, client=self.client, gpu=self.gpu,
                                 workers=self.workers, max_writes=self.max_writes, stats=self.stats)
        self.executor.logger = self.logger
        if self.gpu is not None:
            self.gpu.executor = self.executor
        self._init_mesh()
        self.holder.on_create_shard = self._on_create_shard
        self.holder.on_schema_change = lambda: self.gpu.invalidate() if self.gpu is not None else None
        t = threading.Thread(target=self.httpd.serve_forever, name="http", daemon=True)
        t.start()
        self._threads.append(t)
        if self.is_coordinator_cfg and not self.cluster_disabled:
            try:
                self.cluster.check_coordinator_topology()
            except PilosaError:
                self.close()
                raise
        if self.cluster_disabled or (not self.hosts and self.coordinator_uri is None):
            self.cluster.set_state(STATE_NORMAL if not self.cluster.need_topology_agreement() else STATE_STARTING)
        elif self.is_coordinator_cfg:
            self.cluster.set_coordinator(self.node.id)
            self.cluster.set_state(self.cluster.determine_state())
        else:
            self._join()
        if not self.cluster_disabled and self.gossip_port > 0:
            from pilosa_amd.parallel.gossip_udp import UdpProber
            try:
                self.udp_prober = UdpProber(self.node.id, host if host not in ("",) else "0.0.0.0", self.gossip_port,
                                            lambda: list(self.cluster.nodes), self._gossip_addr, self.gossip_key,
                                            self.logger)
            except OSError as e:   # the port is taken: probes stay on the HTTP port
                self.logger.printf("gossip: cannot listen on udp port %d (%s): probing over HTTP",
                                   self.gossip_port, e)
        if not self.cluster_disabled and self.probe_interval > 0:
            self._start_loop(self._swim_loop, "swim")
        if not self.cluster_disabled and self.gossip_interval > 0:
            self._start_loop(self._gossip_loop, "gossip")
        if self.replica_n > 1 and self.anti_entropy_interval > 0:
            self._start_loop(self._anti_entropy_loop, "anti-entropy")
        self._start_loop(self._runtime_loop, "runtime")
        if self.translation_primary is not None:
            self._start_translate_replica()
        elif not self.cluster_disabled:
            self._start_translate_follower()
        from pilosa_amd.utils import gctune
        from pilosa_amd.utils.gcnotify import GCNotifier
        self.gc_notifier = GCNotifier(self.stats).start()
        # long-lived objects out of the collector's walk (utils/gctune.py)
        self._refreezer = None
        if gctune.enabled():
            gctune.configure()
            gctune.freeze_long_lived()
            self._refreezer = gctune.Refreezer()
        from pilosa_amd.utils.diagnostics import DiagnosticsCollector
        self.diagnostics = DiagnosticsCollector(self.diagnostics_host, self.diagnostics_interval, self.logger)
        if self.diagnostics_host and self.diagnostics_interval > 0:
            self.diagnostics.start(self._refresh_diagnostics)
        return self

    # ------------------------------------------------------------ translate replica
    def _start_translate_replica(self):
        """Non-primary translate store: read-only, tails the primary's log from
        its byte offset over /internal/translate/data and forwards unknown keys
        to the primary (reference translate.go:423-474, http/translator.go)."""
        ts = self.holder.translate
        ts.read_only = True
        primary = self.translation_primary
        ts.forward = lambda index, field, keys: self.client.translate_keys(primary, index, field, keys)

        def loop():
            while not self._closing.is_set():
                try:
                    data = self.client.translate_data(primary, ts.size)
                    if data:
                        ts.apply_log(data)
                        continue
                except Exception as e:  # noqa: BLE001 - primary briefly unavailable
                    self.logger.debugf("translate replication: %s", e)
                self._closing.wait(0.5)
        self._start_loop(loop, "translate-replica")

    def _start_translate_follower(self):
        """Without a configured primary, the cluster's coordinator is the
        translate primary: every other node tails its key log and forwards
        keys it has not seen, so ids agree cluster-wide and any node answers
        with keys (the reference replicates the translate log between nodes
        on membership changes, cluster.go:1969-1971, translate.go:197-240).
        Re-evaluated as the coordinator changes."""
        ts = self.holder.translate
        state = {"primary": None}

        def primary_uri():
            c = self.cluster.coordinator() if self.cluster is not None else None
            return None if c is None or c.id == self.node.id else c.uri

        def forward(index, field, keys):
            uri = state["primary"]
            if uri is None:
                raise PilosaError("translate primary unavailable")
            return self.client.translate_keys(uri, index, field, keys)

        def loop():
            while not self._closing.is_set():
                uri = primary_uri()
                if uri != state["primary"]:
                    state["primary"] = uri
                    ts.read_only = uri is not None
                    ts.forward = forward if uri is not None else None
                if uri is not None:
                    try:
                        data = self.client.translate_data(uri, ts.size)
                        if data:
                            ts.apply_log(data)
                            continue
                    except Exception as e:  # noqa: BLE001 - coordinator briefly unavailable
                        self.logger.debugf("translate replication: %s", e)
                self._closing.wait(0.2)
        self._start_loop(loop, "translate-follower")

    def _refresh_diagnostics(self):
        d = self.diagnostics
        d.set("Version", d.version)
        d.set("Host", self.uri.host)
        d.set("Cluster", ",".join(n.id for n in self.cluster.nodes))
        d.set("NumNodes", len(self.cluster.nodes))
        d.set("NodeID", self.node.id)
        d.set("ClusterID", getattr(self.cluster, "id", ""))
        d.set("GPUs", len(self.diagnostics.sysinfo.gpus()) if self.gpu is not None else 0)
        d.enrich_with_cpu()
        d.enrich_with_os()
        d.enrich_with_memory()
        d.enrich_with_schema(self.holder)

    def _init_mesh(self):
        """Under torch.distributed.run with WORLD_SIZE > 1 this process is the
        front end (rank 0) of a one-process-per-GPU node; the other ranks run
        parallel.mesh.run_worker."""
        from pilosa_amd.parallel import mesh as M
        rank, world, local = M.dist_env()
        if world <= 1:
            return
        if rank != 0:
            raise RuntimeError("Server must run on rank 0; other ranks run parallel.mesh.run_worker")
        M.init_process_group(local, timeout_s=self.mesh_timeout_s)
        self.mesh = M.ShardMesh(self.executor, block=self.mesh_block,
                                peer_dirs={r: M.rank_data_dir(self.data_dir, r) for r in range(world)})
        self.executor.mesh = self.mesh
        self.mesh.apply_schema()

    def _init_gpu(self):
        mode = (self.gpu_mode or "auto").lower()
        if mode in ("off", "none", "cpu"):
            return
        from pilosa_amd import shardwidth
        if not shardwidth.device_supported():
            if mode == "on":
                raise RuntimeError(f"gpu=on needs shards of 2^{shardwidth.MIN_EXPONENT}..2^"
                                   f"{shardwidth.DEVICE_EXPONENT} columns (PILOSA_SHARD_WIDTH={shardwidth.EXPONENT})")
            self.logger.printf("shard width 2^%d: the device arenas hold shards of at most 2^%d columns, "
                               "queries run on the host", shardwidth.EXPONENT, shardwidth.DEVICE_EXPONENT)
            return
        try:
            import torch
            if not torch.cuda.is_available():
                if mode == "on":
                    raise RuntimeError("gpu=on but no GPU is visible")
                return
            from pilosa_amd.ops.gpu_executor import GpuExecutor
            from pilosa_amd.parallel.mesh import dist_env
            dev = self.gpu_device if self.gpu_device is not None else dist_env()[2]
            self.gpu = GpuExecutor(self.holder, f"cuda:{dev}", hbm_budget=self.hbm_budget)
        except ImportError:
            if mode == "on":
                raise

    def gpu_info(self) -> dict:
        if self.gpu is None:
            return {"enabled": False}
        import torch
        p = torch.cuda.get_device_properties(self.gpu.device)
        out = {"enabled": True, "name": p.name, "arch": getattr(p, "gcnArchName", ""), "hbmBytes": p.total_memory}
        out.update(self.gpu.stats())
        return out

    def close(self):
        self._closing.set()
        if self.diagnostics is not None:
            self.diagnostics.stop()
        if self.gc_notifier is not None:
            self.gc_notifier.stop()
        if self.mesh is not None:
            self.mesh.stop()
        if self.udp_prober is not None:
            self.udp_prober.close()
        if self.httpd is not None:
            self.httpd.shutdown()
            self.httpd.server_close()
        if self.executor is not None:
            self.executor.close()
        self.holder.close()

    @property
    def uri(self) -> URI:
        return self.node.uri

    def _start_loop(self, fn, name):
        t = threading.Thread(target=fn, name=name, daemon=True)
        t.start()
        self._threads.append(t)

    # ------------------------------------------------------------ broadcast
    def broadcast(self, msg: dict):
        """SendSync to every other node (server.go:646-667)."""
        if self.cluster is None:
            return
        errs = []
        for n in list(self.cluster.nodes):
            if n.id == self.node.id or n.state == NODE_DOWN:
                continue
            try:
                self.client.send_message(n, msg)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        if errs:
            self.logger.printf("broadcast %s: %d errors, first: %s", msg.get("type"), len(errs), errs[0])

    def _on_create_shard(self, index, field, shard):
        """Announce a new shard; like view.go:239-262 the write waits for the
        broadcast at most 50 ms and lets it finish in the background."""
        done = threading.Event()

        def send():
            try:
                self.broadcast({"type": "CreateShard", "index": index, "field": field, "shard": shard})
            finally:
                done.set()
        threading.Thread(target=send, name="create-shard", daemon=True).start()
        if not done.wait(0.05):
            self.logger.debugf("broadcasting create shard took >50ms")

    def receive_message(self, msg: dict):
        """Dispatch of internal cluster messages (server.go:549-643)."""
        t = msg.get("type")
        h = self.holder
        if t == "CreateIndex":
            o = msg.get("options", {})
            h.create_index_if_not_exists(msg["index"], keys=o.get("keys", False),
                                         track_existence=o.get("trackExistence", True))
        elif t == "DeleteIndex":
            if h.index(msg["index"]) is not None:
                h.delete_index(msg["index"])
        elif t == "CreateField":
            idx = h.index(msg["index"])
            if idx is not None and idx.field(msg["field"]) is None:
                o = msg.get("options", {})
                idx.create_field(msg["field"], _field_options(o))
        elif t == "DeleteField":
            idx = h.index(msg["index"])
            if idx is not None and idx.field(msg["field"]) is not None:
                idx.delete_field(msg["field"])
        elif t == "DeleteAvailableShard":
            f = h.field(msg["index"], msg["field"])
            if f is not None:
                f.remove_available_shard(msg["shard"])
        elif t == "DeleteView":
            f = h.field(msg["index"], msg["field"])
            if f is not None and f.view(msg["view"]) is not None:
                f.delete_view(msg["view"])
        elif t == "CreateView":
            f = h.field(msg["index"], msg["field"])
            if f is None:
                raise PilosaError(f"local field not found: {msg['field']}")
            f.create_view_if_not_exists(msg["view"])
        elif t == "NodeState":
            if self.cluster.set_node_state(msg["nodeID"], msg["state"]) and self.cluster.is_coordinator():
                self._publish_status()
        elif t == "NodeUpdate":
            pass    # intentionally not implemented, as in the reference (cluster.go:1762)
        elif t == "CreateShard":
            f = h.field(msg["index"], msg["field"])
            if f is not None:
                f.add_remote_available_shards([msg["shard"]])
        elif t == "ApplySchema":
            h.apply_schema(msg["schema"])
        elif t == "RecalculateCaches":
            h.recalculate_caches()
        elif t in ("SetCoordinator", "UpdateCoordinator"):
            self.cluster.set_coordinator(msg["node"]["id"])
        elif t == "ClusterStatus":
            self._merge_cluster_status(msg["status"])
        elif t == "NodeJoin":
            self._node_join(Node.from_json(msg["node"]))
        elif t == "NodeLeave":
            self._node_down(msg["node"]["id"])
        elif t == "NodeStatus":
            self._merge_node_status(msg)
        elif t == "ResizeInstruction":
            threading.Thread(target=self._follow_resize, args=(msg,), daemon=True).start()
        elif t == "ResizeInstructionComplete":
            self._resize_complete(msg)
        elif t == "ResizeAbort":
            self.cluster.set_state(self.cluster.determine_state() if self.cluster.state != STATE_RESIZING
                                   else STATE_NORMAL)
        else:
            raise ValueError(f"unknown message type: {t}")

    # ------------------------------------------------------------ membership
    def _join(self):
        """Announce this node to the cluster through the first seed that
        answers (the coordinator URI, then the configured hosts); a seed that
        is not the coordinator forwards the join (gossip seeds, server.go)."""
        seeds = ([self.coordinator_uri] if self.coordinator_uri else []) + \
            [h for h in self.hosts if h != self.node.uri and h != self.coordinator_uri]
        if not seeds:
            self.cluster.set_state(STATE_NORMAL)
            return
        deadline = time.time() + 30
        msg = {"type": "NodeJoin", "node": self.node.to_json(), "status": self._node_status()}
        while not self._closing.is_set():
            err = None
            for target in seeds:
                try:
                    self.client.send_message(Node("?", target), msg)
                    return
                except Exception as e:  # noqa: BLE001
                    if "not in topology" in str(e):    # refused by the coordinator: retrying cannot help
                        self.join_error = getattr(e, "body", str(e))
                        self.logger.printf("join %s refused: %s", target, e)
                        return
                    err = e
            if time.time() > deadline:
                self.logger.printf("join %s failed: %s", seeds, err)
                return
            time.sleep(0.2)

    def _node_status(self) -> dict:
        return {"node": self.node.to_json(), "schema": self.holder.schema(),
                "shards": {n: {f.name: f.available_shards() for f in idx.fields.values()}
                           for n, idx in self.holder.indexes.items()}}

    def _merge_node_status(self, msg: dict):
        st = msg.get("status") or msg
        if st.get("schema"):
            self.holder.apply_schema(st["schema"])
        for index, fields in (st.get("shards") or {}).items():
            for fname, shards in fields.items():
                f = self.holder.field(index, fname)
                if f is not None and shards:
                    f.add_remote_available_shards(shards)

    def _node_join(self, n: Node):
        if not self.cluster.is_coordinator():
            c = self.cluster.coordinator()
            if c is not None and c.id != self.node.id:
                self.client.send_message(c, {"type": "NodeJoin", "node": n.to_json()})
            return
        with self.mu:
            if self.cluster.need_topology_agreement() and not self.cluster.topology.contains_id(n.id):
                # a restarting cluster only admits the nodes of its persisted topology (cluster.go:1775)
                raise PilosaError(f"host is not in topology: {n.id}")
            known = self.cluster.node_by_id(n.id)
            if known is not None:
                known.uri = n.uri
                self.cluster.set_node_state(n.id, NODE_READY)
                self._publish_status()
                return
            has_data = any(idx.available_shards() for idx in self.holder.indexes.values())
            n.state = NODE_READY
            if has_data and n.id not in self.cluster.topology.node_ids:
                self._start_resize(self.cluster.nodes + [n], joining=n)
                return
            self.cluster.add_node(n)
            self._publish_status()

    def _node_down(self, nid: str):
        if self.cluster.set_node_state(nid, NODE_DOWN):
            self.cluster.set_state(self.cluster.determine_state())
            if self.cluster.is_coordinator():
                self._publish_status()

    def _publish_status(self):
        self.cluster.set_state(self.cluster.determine_state())
        st = self.cluster.status()
        st["coordinator"] = self.cluster.coordinator_id
        msg = {"type": "ClusterStatus", "status": st, "schema": self.holder.schema()}
        self.broadcast(msg)

    def _merge_cluster_status(self, st: dict):
        nodes = [Node.from_json(d) for d in st.get("nodes", [])]
        coord = st.get("coordinator") or next((d["id"] for d in st.get("nodes", []) if d.get("isCoordinator")),
                                               None)
        self.cluster.topology.cluster_id = st.get("clusterID", self.cluster.topology.cluster_id)
        self.cluster.set_nodes(nodes, coord, exact=True)
        me = self.cluster.node_by_id(self.node.id)
        if me is not None:
            me.state = NODE_READY
        self.cluster.set_state(st.get("state", STATE_NORMAL))

    def _swim_loop(self):
        """Failure detection on every node (parallel/swim.py: direct probe,
        indirect probes through ``indirect_checks`` peers, suspicion timeout
        from ``suspicion_mult``).  The coordinator applies the verdicts and
        publishes the cluster status; another node reports a DOWN verdict to
        the coordinator (NodeState), as memberlist's leave event reaches the
        reference's coordinator.  A DOWN node that answers again is READY."""
        from pilosa_amd.parallel.swim import DOWN, FailureDetector
        up = self.udp_prober
        det = FailureDetector(self.node.id, up.ping if up is not None else self._swim_probe,
                              up.ping_req if up is not None else self._swim_indirect,
                              probe_interval=self.probe_interval, probe_timeout=self.probe_timeout,
                              suspicion_mult=self.suspicion_mult, indirect_checks=self.indirect_checks)
        self.failure_detector = det
        try:
            while not self._closing.wait(self.probe_interval):
                det.probe_interval, det.probe_timeout = self.probe_interval, self.probe_timeout
                nodes = list(self.cluster.nodes)
                if len(nodes) < 2:
                    continue
                coord = self.cluster.is_coordinator()
                changed = False
                for nid, ev in det.tick(nodes):
                    if ev == DOWN:
                        self.logger.printf("swim: node %s unreachable past the suspicion timeout", nid)
                        self._down_since[nid] = time.monotonic()
                        if coord:
                            changed |= self.cluster.set_node_state(nid, NODE_DOWN)
                        else:
                            self._report_down(nid)
                    else:
                        self._down_since.pop(nid, None)
                        if coord:
                            changed |= self.cluster.set_node_state(nid, NODE_READY)
                if coord:
                    new_state = self.cluster.determine_state()
                    if changed or new_state != self.cluster.state:
                        self._publish_status()
        finally:
            det.close()

    def _gossip_addr(self, node):
        """(host, UDP gossip port) of a node."""
        return node.uri.host, self.gossip_peer_ports.get(node.id, self.gossip_port)

    def _swim_probe(self, node, timeout: float) -> bool:
        """Direct probe: the node's /version within ``timeout``."""
        return _probe_version(node.uri, timeout, self.probe_client.skip_verify)

    def _swim_indirect(self, helper, target, timeout: float) -> bool:
        """Indirect probe: ask ``helper`` to probe ``target`` (POST
        /internal/probe), memberlist's indirect ping."""
        import json as _json
        from urllib import request as _rq
        url = f"{helper.uri.scheme}://{helper.uri.host_port()}/internal/probe"
        body = _json.dumps({"uri": target.uri.normalize(), "timeout": timeout}).encode()
        req = _rq.Request(url, data=body, method="POST", headers={"Content-Type": "application/json"})
        with _rq.urlopen(req, timeout=timeout * 2 + 0.5, context=_ssl_ctx(self.probe_client.skip_verify)) as r:
            return bool(_json.loads(r.read() or b"{}").get("ok"))

    def probe_for_peer(self, uri: str, timeout: float) -> Optional[bool]:
        """A peer's indirect probe of ``uri`` through this node.  Only a
        member of this cluster is probed (memberlist's indirect ping targets
        known members only); None for any other address, so the route cannot
        be used to reach arbitrary hosts.  The timeout is capped
        at 2 s."""
        try:
            target = URI.parse(uri)
        except Exception:  # noqa: BLE001 - not an address
            return None
        if not any(n.uri == target for n in self.cluster.nodes if n.id != self.node.id):
            return None
        return _probe_version(target, max(0.0, min(float(timeout), 2.0)), self.probe_client.skip_verify)

    def _report_down(self, nid: str):
        coord = self.cluster.coordinator()
        if coord is not None and coord.id not in (nid, self.node.id):
            try:
                self.client.send_message(coord, {"type": "NodeState", "nodeID": nid, "state": NODE_DOWN})
            except Exception as e:  # noqa: BLE001
                self.logger.printf("swim: reporting %s down: %s", nid, e)
        else:
            self._node_down(nid)

    def _gossip_loop(self):
        """Push-pull of NodeStatus between every pair of nodes (the role of
        memberlist's LocalState/MergeRemoteState, gossip/gossip.go:295-443):
        each round this node pushes its schema + available shards to the next
        ``gossip_nodes`` peers in turn, and receives every peer's push in turn.  Failure detection is
        the SWIM loop's; a peer DOWN for longer than ``to_the_dead_time``
        stops receiving pushes (memberlist's GossipToTheDeadTime)."""
        while not self._closing.wait(self.gossip_interval):
            now = time.monotonic()
            peers = [n for n in self.cluster.nodes if n.id != self.node.id and
                     not (n.state == NODE_DOWN and now - self._down_since.get(n.id, now) > self.to_the_dead_time)]
            if not peers:
                continue
            status = None
            for _ in range(min(self.gossip_nodes, len(peers))):
                n = peers[self._gossip_i % len(peers)]
                self._gossip_i += 1
                try:
                    if status is None:
                        status = self._node_status()
                    self.stream_client.send_message(n, {"type": "NodeStatus", "status": status})
                except Exception as e:  # noqa: BLE001 - the SWIM loop judges liveness
                    self._gossip_misses[n.id] = self._gossip_misses.get(n.id, 0) + 1

    # ------------------------------------------------------------ resize
    def _holder_layout(self) -> Dict[str, Dict[str, List[str]]]:
        return {n: {f.name: sorted(f.views) for f in idx.fields.values()} for n, idx in self.holder.indexes.items()}

    def _start_resize(self, new_nodes: List[Node], joining: Optional[Node] = None, leaving: Optional[Node] = None):
        layout = self._holder_layout()
        avail = {n: idx.available_shards() for n, idx in self.holder.indexes.items()}
        sources = self.cluster.frag_sources(new_nodes, layout, avail)
        action = RESIZE_ACTION_ADD if joining is not None else RESIZE_ACTION_REMOVE
        job = ResizeJob(self.cluster.nodes, joining if joining is not None else leaving, action,
                        job_id=int(time.time() * 1000))
        job.nodes = list(new_nodes)
        self._resize = job
        self.cluster.set_state(STATE_RESIZING)
        status = self.cluster.status()
        for n in new_nodes:
            msg = {"type": "ResizeInstruction", "jobID": job.id, "node": n.to_json(),
                   "coordinator": self.node.to_json(), "sources": sources.get(n.id, []),
                   "schema": self.holder.schema(), "status": status, "nodeStatus": self._node_status()}
            try:
                if n.id == self.node.id:
                    threading.Thread(target=self._follow_resize, args=(msg,), daemon=True).start()
                else:
                    self.client.send_message(n, msg)
            except Exception as e:  # noqa: BLE001
                job.mark(n.id, str(e))

    def _follow_resize(self, msg: dict):
        err = ""
        try:
            self.cluster.set_state(STATE_RESIZING)
            self.holder.apply_schema(msg.get("schema", []))
            if msg.get("nodeStatus"):
                # the coordinator's view of which shards exist cluster-wide
                self._merge_node_status(msg["nodeStatus"])
            # pull sources a few at a time (resizeFollower fetches per source;
            # cluster.go:1378-1460) and stop as soon as the job is aborted: the
            # coordinator's abort leaves RESIZING through the status push
            from concurrent.futures import ThreadPoolExecutor

            def pull(src):
                if self._resize_aborted():
                    raise PilosaError("resize aborted")
                sn = Node.from_json(src["node"])
                data = self.client.fragment_data(sn.uri, src["index"], src["field"], src["view"], src["shard"])
                if self._resize_aborted():
                    raise PilosaError("resize aborted")
                f = self.holder.field(src["index"], src["field"])
                frag = f.create_view_if_not_exists(src["view"]).create_fragment_if_not_exists(src["shard"])
                frag.read_from(io.BytesIO(data))
            srcs = msg.get("sources", [])
            if srcs:
                with ThreadPoolExecutor(max_workers=min(4, len(srcs))) as pool:
                    for fut in [pool.submit(pull, s_) for s_ in srcs]:
                        fut.result()
        except Exception as e:  # noqa: BLE001
            err = str(e)
        done = {"type": "ResizeInstructionComplete", "jobID": msg["jobID"], "node": self.node.to_json(),
                "error": err}
        coord = Node.from_json(msg["coordinator"])
        if coord.id == self.node.id:
            self._resize_complete(done)
        else:
            self.client.send_message(coord, done)

    def _resize_complete(self, msg: dict):
        with self.mu:
            job = self._resize
            if job is None or msg.get("jobID") != job.id:
                return
            if not job.mark(msg["node"]["id"], msg.get("error") or ""):
                return
            self._resize = None
            if job.errors:
                self.logger.printf("resize job %s failed: %s", job.id, job.errors[0])
            else:
                self.cluster.set_nodes(job.nodes, self.cluster.coordinator_id)
                if job.leaving:
                    self.cluster.remove_node(job.leaving)
            self.cluster.state = STATE_NORMAL
            self._publish_status()
            self.clean_holder()
            self.broadcast({"type": "RecalculateCaches"})
            job.finish(RESIZE_JOB_ABORTED if job.errors else RESIZE_JOB_DONE)

    def node_leave(self, n: Node):
        """Coordinator-side checks before removing a node (cluster.go:1841-1880)."""
        c = self.cluster
        if not c.is_coordinator():
            co = c.coordinator()
            raise PilosaError("node removal requests are only valid on the coordinator node: "
                              f"{co.id if co else c.coordinator_id}")
        if c.state not in (STATE_NORMAL, STATE_DEGRADED):
            raise PilosaError(f"cluster must be '{STATE_NORMAL}' to remove a node but is '{c.state}'")
        if not c.topology.contains_id(n.id) and c.node_by_id(n.id) is None:
            raise PilosaError(f"Node is not a member of the cluster: {n.id}")
        if n.id == self.node.id:
            raise PilosaError("coordinator cannot be removed; first, make a different node the new coordinator")
        try:
            self.resize_remove_node(n)
        except PilosaError as e:
            raise PilosaError(f"generating job: {e}") from e

    def resize_remove_node(self, n: Node):
        remaining = [x for x in self.cluster.nodes if x.id != n.id]
        has_data = any(idx.available_shards() for idx in self.holder.indexes.values())
        if has_data:
            self._start_resize(remaining, leaving=n)
        else:
            self.cluster.remove_node(n.id)
            self._publish_status()

    def abort_resize(self) -> bool:
        with self.mu:
            if self._resize is None:
                return False
            self._resize.finish(RESIZE_JOB_ABORTED)
            self._resize = None
            self.cluster.state = STATE_NORMAL
            self._publish_status()     # followers leave RESIZING through the status push
            return True

    def clean_holder(self):
        """Delete local fragments this node no longer owns (holderCleaner)."""
        for idx in list(self.holder.indexes.values()):
            for f in list(idx.fields.values()):
                for v in list(f.views.values()):
                    for shard in list(v.fragments):
                        if not self.cluster.owns_shard(self.node.id, idx.name, shard):
                            v.delete_fragment(shard)
                            # still available in the cluster: its owner holds it now
                            f.add_remote_available_shards([shard])
        if self.gpu is not None:
            self.gpu.invalidate()

    # ------------------------------------------------------------ anti-entropy
    def _resize_aborted(self) -> bool:
        return self._closing.is_set() or self.cluster.state != STATE_RESIZING

    def _anti_entropy_loop(self):
        while not self._closing.wait(self.anti_entropy_interval):
            if self.cluster.state != STATE_NORMAL:
                continue
            try:
                if not self.sync_holder():
                    self.logger.printf("anti-entropy: pass aborted (cluster state %s)", self.cluster.state)
            except Exception as e:  # noqa: BLE001
                self.logger.printf("anti-entropy: %s", e)

    def _sync_should_abort(self) -> bool:
        """holderSyncer.IsClosing: a pass stops once the node closes or the
        cluster leaves NORMAL (a resize began), cluster.go:253-275,465."""
        return self._closing.is_set() or self.cluster.state != STATE_NORMAL

    def sync_holder(self) -> bool:
        """One anti-entropy pass over every local fragment and attr store.
        Returns False when the pass was aborted part-way."""
        for idx in list(self.holder.indexes.values()):
            if self._sync_should_abort():
                return False
            self._sync_attrs(idx.name, None, idx.column_attr_store)
            for f in list(idx.fields.values()):
                self._sync_attrs(idx.name, f.name, f.row_attr_store)
                for v in list(f.views.values()):
                    for shard, frag in list(v.fragments.items()):
                        if self._sync_should_abort():
                            return False
                        self._sync_fragment(idx.name, f.name, v.name, shard, frag)
        return True

    def _sync_attrs(self, index, field, store):
        blocks = [{"id": b, "checksum": base64.b64encode(c).decode()} for b, c in store.blocks()]
        for n in self.cluster.nodes:
            if n.id == self.node.id or n.state != NODE_READY:
                continue
            try:
                diff = self.client.attr_diff(n.uri, index, field, blocks)
            except Exception:  # noqa: BLE001
                continue
            if diff:
                store.set_bulk_attrs(diff)

    def _sync_fragment(self, index, field, view, shard, frag):
        owners = [n for n in self.cluster.shard_nodes(index, shard) if n.id != self.node.id]
        if not owners:
            return
        local = dict(frag.blocks())
        remote_blocks = {}
        for n in owners:
            try:
                remote_blocks[n.id] = {b["id"]: base64.b64decode(b["checksum"] or "")
                                       for b in self.client.fragment_blocks(n.uri, index, field, view, shard)}
            except Exception:  # noqa: BLE001
                remote_blocks[n.id] = None
        live = [n for n in owners if remote_blocks.get(n.id) is not None]
        ids = set(local)
        for n in live:
            ids |= set(remote_blocks[n.id])
        for bid in sorted(ids):
            if all(remote_blocks[n.id].get(bid) == local.get(bid) for n in live):
                continue
            data = [self.client.block_data(n.uri, index, field, view, shard, bid) for n in live]
            sets, clears = frag.merge_block(bid, data)
            base = shard * SHARD_WIDTH
            for n, (sr, sc), (cr, cc) in zip(live, sets, clears):
                if sr:
                    self.client.import_bits(n, index, field, shard, sr, [base + c for c in sc],
                                            ignore_key_check=True)
                if cr:
                    self.client.import_bits(n, index, field, shard, cr, [base + c for c in cc], clear=True,
                                            ignore_key_check=True)

    # ------------------------------------------------------------ runtime gauges
    def _runtime_loop(self):
        while not self._closing.wait(10.0):
            try:
                import resource
                ru = resource.getrusage(resource.RUSAGE_SELF)
                self.stats.gauge("maxrss_kb", ru.ru_maxrss)
                self.stats.gauge("open_files", len(os.listdir("/proc/self/fd")))
                self.stats.gauge("threads", threading.active_count())
                gcn = getattr(self, "gc_notifier", None)
                if gcn is not None:
                    gcn.flush()
                rf = getattr(self, "_refreezer", None)
                if rf is not None:
                    rf.tick()
                if self.gpu is not None:
                    st = self.gpu.stats()
                    self.stats.gauge("gpu.arena_bytes", st["arenaBytes"])
                    self.stats.gauge("gpu.launches", st["launches"])
                    self.stats.gauge("gpu.arena_rebuilds", st["rebuilds"])
                    self.stats.gauge("gpu.arena_row_updates", st["rowUpdates"])
                    for t, n in st["containers"].items():
                        self.stats.gauge(f"gpu.containers.{t}", n)
            except Exception:  # noqa: BLE001
                pass


def _field_options(o: dict) -> FieldOptions:
    return FieldOptions(type=o.get("type", "set"), cache_type=o.get("cacheType", ""), cache_size=o.get("cacheSize", 0),
                        time_quantum=o.get("timeQuantum", ""), min=o.get("min", 0), max=o.get("max", 0),
                        keys=o.get("keys", False), no_standard_view=o.get("noStandardView", False),
                        base=o.get("base", 0), bit_depth=o.get("bitDepth", 0))
