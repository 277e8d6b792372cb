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


def version_segments(v: str):
    """'v1.2.3-rc1' -> [1, 2, 3] (diagnostics.go versionSegments)."""
    out = []
    for x in v.strip("v").split("-", 1)[0].split("."):
        try:
            out.append(int(x))
        except ValueError:
            out.append(0)
    return out


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
        if isinstance(value, str) and value == "":
            return   # empty strings are not recorded (diagnostics.go Set)
        with self.mu:
            self.metrics[name] = value

    def set_version(self, v: str):
        self.version = v

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

    def encode(self) -> bytes:
        """The recorded metrics as the JSON document (diagnostics.go encode)."""
        with self.mu:
            return json.dumps(self.metrics, sort_keys=True).encode()

    payload = encode

    def flush(self) -> bool:
        """Record Uptime, then POST the document to the configured endpoint
        (no-op without one; diagnostics.go Flush)."""
        self.set("Uptime", int(time.time() - self.start_time))
        if not self.host:
            return False
        req = urllib.request.Request(self.host, data=self.encode(), method="POST",
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=10) as r:
                r.read()
            return True
        except Exception as e:  # noqa: BLE001 - diagnostics never fail the server
            if self.logger is not None:
                self.logger.debugf("diagnostics flush: %s", e)
            return False

    def compare_version(self, value: str) -> Optional[str]:
        """The upgrade message when release ``value`` is newer than this
        build -- major, minor or patch -- else None (diagnostics.go:135-148)."""
        cur, loc = (version_segments(value) + [0, 0, 0])[:3], (version_segments(self.version) + [0, 0, 0])[:3]
        url = "https://github.com/pilosa/pilosa/releases"
        if loc[0] < cur[0]:
            return f"you are running Pilosa {self.version}, a newer version ({value}) is available: {url}"
        if loc[1] < cur[1] and loc[0] == cur[0]:
            return f"you are running Pilosa {self.version}, the latest minor release is {value}: {url}"
        if loc[2] < cur[2] and loc[0] == cur[0] and loc[1] == cur[1]:
            return f"there is a new patch release of Pilosa available: {value}: {url}"
        return None

    def check_version(self, latest: str) -> Optional[str]:
        """Message when ``latest`` is newer than this build."""
        return self.compare_version(latest) if latest else None

    version_url = ""
    _last_version = ""

    def check_version_url(self) -> None:
        """GET ``version_url`` ({"version": ...}) and log the upgrade message
        once per new release seen (diagnostics.go CheckVersion)."""
        with urllib.request.urlopen(self.version_url, timeout=10) as r:
            if r.status != 200:
                raise RuntimeError(f"http: status={r.status}")
            v = json.loads(r.read() or b"{}").get("version", "")
        if v == self._last_version:
            return
        self._last_version = v
        msg = self.compare_version(v)
        if msg and self.logger is not None:
            self.logger.printf("%s\n", msg)

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
