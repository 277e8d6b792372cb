"""Usage diagnostics (reference: diagnostics.go:32-347, server.go:740-790).

The reference periodically POSTs a JSON document (version, host facts,
schema size, cluster shape) to a collection endpoint and checks for a newer
release.  Here the collector builds the same document; sending happens only
when an endpoint is configured (``metric.diagnostics`` with a
``diagnostics.host`` URL) -- there is no default phone-home."""
from __future__ import annotations

import json
import threading
import time
import urllib.request
from typing import Callable, Dict, Optional

from pilosa_amd import __version__
from pilosa_amd.utils.sysinfo import SystemInfo


def compare_versions(a: str, b: str) -> int:
    """semver-ish compare of 'vX.Y.Z[-suffix]' strings (-1, 0, 1)."""
    def parts(v):
        v = v.lstrip("v").split("-", 1)[0]
        out = []
        for x in v.split("."):
            try:
                out.append(int(x))
            except ValueError:
                out.append(0)
        return (out + [0, 0, 0])[:3]
    pa, pb = parts(a), parts(b)
    return (pa > pb) - (pa < pb)


class DiagnosticsCollector:
    def __init__(self, host: str = "", interval: float = 3600.0, logger=None):
        self.host = host
        self.interval = interval
        self.logger = logger
        self.version = __version__
        self.start_time = time.time()
        self.metrics: Dict[str, object] = {}
        self.mu = threading.Lock()
        self.sysinfo = SystemInfo()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def set(self, name: str, value):
        with self.mu:
            self.metrics[name] = value

    def enrich_with_os(self):
        s = self.sysinfo
        self.set("HostUptime", s.uptime())
        self.set("OS", s.platform())
        self.set("OSFamily", s.family())
        self.set("OSVersion", s.os_version())
        self.set("KernelVersion", s.kernel_version())

    def enrich_with_cpu(self):
        s = self.sysinfo
        self.set("CPUArch", __import__("platform").machine())
        self.set("CPUModel", s.cpu_model())
        self.set("CPUMHz", s.cpu_mhz())
        self.set("CPUPhysicalCores", s.cpu_cores())
        self.set("CPULogicalCores", s.cpu_threads())

    def enrich_with_memory(self):
        self.set("MemTotal", self.sysinfo.mem_total())
        self.set("MemUsed", self.sysinfo.mem_used())

    def enrich_with_schema(self, holder):
        idx = holder.index_list()
        nfields = sum(len([f for f in i.fields if not f.startswith("_")]) for i in idx)
        nshards = 0
        int_fields = time_fields = 0
        for i in idx:
            shards = set()
            for f in i.fields.values():
                shards |= set(f.available_shards())
                t = f.type
                int_fields += t == "int"
                time_fields += t == "time"
            nshards = max(nshards, len(shards))
        self.set("NumIndexes", len(idx))
        self.set("NumFields", nfields)
        self.set("NumShards", nshards)
        self.set("BSIFieldCount", int_fields)
        self.set("TimeQuantumFieldCount", time_fields)

    def payload(self) -> bytes:
        with self.mu:
            m = dict(self.metrics)
        m["Version"] = self.version
        m["Uptime"] = int(time.time() - self.start_time)
        return json.dumps(m, sort_keys=True).encode()

    def flush(self) -> bool:
        """POST the document to the configured endpoint (no-op without one)."""
        if not self.host:
            return False
        req = urllib.request.Request(self.host, data=self.payload(), method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=10) as r:
                r.read()
            return True
        except Exception as e:  # noqa: BLE001 - diagnostics never fail the server
            if self.logger is not None:
                self.logger.debugf("diagnostics flush: %s", e)
            return False

    def check_version(self, latest: str) -> Optional[str]:
        """Message when ``latest`` is newer than this build (diagnostics.go:120-150)."""
        if latest and compare_versions(latest, self.version) > 0:
            return f"you are running Pilosa-AMD {self.version}, a newer version ({latest}) is available"
        return None

    def start(self, refresh: Callable[[], None]):
        def loop():
            while not self._stop.wait(self.interval):
                try:
                    refresh()
                    self.flush()
                except Exception:  # noqa: BLE001
                    pass
        self._thread = threading.Thread(target=loop, name="diagnostics", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
