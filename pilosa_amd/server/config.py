"""Server configuration (reference: server/config.go, cmd/root.go).

Precedence: command-line flags > ``PILOSA_*`` environment variables
(``-``/``.`` -> ``_``, upper-cased) > TOML file > defaults.  Unknown TOML keys
are rejected (cmd/root.go:119-125).  Key names follow the reference
(``data-dir``, ``bind``, ``cluster.replicas`` ...) plus a ``gpu`` section
(``gpu.mode`` auto/on/off, ``gpu.devices``).
"""
from __future__ import annotations

import copy
import os
from typing import Any, Dict, List, Optional

DURATION_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(v) -> float:
    """Go ``time.ParseDuration`` ('1m30s', '500ms', '-1.5h') -> seconds
    (toml/toml.go Duration.UnmarshalText); the reference's error texts."""
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    orig = s
    if not s:
        return 0.0
    neg = s[0] == "-"
    if s[0] in "+-":
        s = s[1:]
    if s == "0":
        return 0.0
    if not s:
        raise ValueError(f"time: invalid duration {orig}")
    total, i = 0.0, 0
    while i < len(s):
        j = i
        while j < len(s) and (s[j].isdigit() or s[j] == "."):
            j += 1
        num = s[i:j]
        if not num or num == "." or num.count(".") > 1:
            raise ValueError(f"time: invalid duration {orig}")
        k = j
        while k < len(s) and not (s[k].isdigit() or s[k] == "."):
            k += 1
        unit = s[j:k]
        if not unit:
            raise ValueError(f"time: missing unit in duration {orig}")
        if unit not in DURATION_UNITS:
            raise ValueError(f"time: unknown unit {unit} in duration {orig}")
        total += float(num) * DURATION_UNITS[unit]
        i = k
    return -total if neg else total


def format_duration(sec: float) -> str:
    """Go ``time.Duration.String``: '3m2s', '1h0m0s', '1.5s', '500ms', '0s'."""
    ns = int(round(sec * 1e9))
    if ns == 0:
        return "0s"
    sign = "-" if ns < 0 else ""
    ns = abs(ns)

    def frac(v: int, unit: int) -> str:
        w, f = divmod(v, unit)
        if not f:
            return str(w)
        digits = len(str(unit)) - 1
        return f"{w}.{str(f).rjust(digits, '0').rstrip('0')}"
    if ns < 1000:
        return f"{sign}{ns}ns"
    if ns < 1_000_000:
        return f"{sign}{frac(ns, 1000)}\u00b5s"
    if ns < 1_000_000_000:
        return f"{sign}{frac(ns, 1_000_000)}ms"
    h, rem = divmod(ns, 3600 * 1_000_000_000)
    m, rem = divmod(rem, 60 * 1_000_000_000)
    out = f"{frac(rem, 1_000_000_000)}s"
    if h:
        return f"{sign}{h}h{m}m{out}"
    if m:
        return f"{sign}{m}m{out}"
    return sign + out


DEFAULTS: Dict[str, Any] = {
    "data-dir": "~/.pilosa",
    "bind": ":10101",
    "advertise": "",
    "max-writes-per-request": 5000,
    "log-path": "",
    "verbose": False,
    "max-map-count": 1000000,
    "max-file-count": 1000000,
    "worker-pool-size": os.cpu_count() or 8,
    "import-worker-pool-size": os.cpu_count() or 8,
    "handler": {"allowed-origins": []},
    "tls": {"certificate": "", "key": "", "skip-verify": False},
    "cluster": {"disabled": False, "coordinator": False, "replicas": 1, "hosts": [], "long-query-time": "1m0s",
                "coordinator-uri": ""},
    "gossip": {"port": "14000", "seeds": [], "key": "", "stream-timeout": "10s", "suspicion-mult": 4,
               "push-pull-interval": "30s", "probe-interval": "1s", "probe-timeout": "500ms",
               "interval": "200ms", "nodes": 3, "to-the-dead-time": "30s"},
    "translation": {"map-size": 10737418240, "primary-url": ""},
    "anti-entropy": {"interval": "10m0s"},
    "metric": {"service": "none", "host": "", "poll-interval": "0s", "diagnostics": True, "diagnostics-host": ""},
    "tracing": {"sampler-type": "remote", "sampler-param": 0.001, "agent-host-port": ""},
    "profile": {"block-rate": 10000000, "mutex-fraction": 100},
    "gpu": {"mode": "auto", "devices": [], "hbm-budget": 0, "shard-block": 1, "rccl-timeout": "2m",
            "lazy-fragments": True, "native-http": True},
}


class ConfigError(ValueError):
    pass


class Config:
    def __init__(self, values: Optional[dict] = None):
        self.v = copy.deepcopy(DEFAULTS)
        if values:
            self.merge(values, strict=True)

    # dotted access
    def get(self, key: str):
        cur = self.v
        for part in key.split("."):
            cur = cur[part]
        return cur

    def set(self, key: str, value):
        parts = key.split(".")
        cur = self.v
        for p in parts[:-1]:
            if p not in cur or not isinstance(cur[p], dict):
                raise ConfigError(f"unknown config key: {key}")
            cur = cur[p]
        if parts[-1] not in cur:
            raise ConfigError(f"unknown config key: {key}")
        old = cur[parts[-1]]
        cur[parts[-1]] = _coerce(value, old)

    def merge(self, d: dict, strict: bool = True, prefix: str = ""):
        for k, v in d.items():
            key = f"{prefix}{k}"
            if isinstance(v, dict):
                try:
                    if not isinstance(self.get(key), dict):
                        raise ConfigError(f"unknown config key: {key}")
                except KeyError:
                    raise ConfigError(f"unknown config key: {key}")
                self.merge(v, strict, key + ".")
            else:
                try:
                    self.set(key, v)
                except (ConfigError, KeyError):
                    if strict:
                        raise ConfigError(f"unknown config key: {key}")

    def load_toml(self, path: str):
        import tomli
        with open(os.path.expanduser(path), "rb") as fh:
            data = tomli.load(fh)
        bad = [k for k in _flat_keys(data) if not self._known(k)]
        if bad:   # cmd/root.go: every key of the file must be a known option
            raise ConfigError(f"invalid option in configuration file: {bad[0]}")
        self.merge(data, strict=True)

    def _known(self, key: str) -> bool:
        try:
            self.get(key)
            return True
        except (KeyError, TypeError):
            return False

    def load_env(self, env=None):
        env = os.environ if env is None else env
        for key in _flat_keys(self.v):
            name = "PILOSA_" + key.replace("-", "_").replace(".", "_").upper()
            if name in env:
                self.set(key, env[name])

    def to_toml(self) -> str:
        lines = []
        top = {k: v for k, v in self.v.items() if not isinstance(v, dict)}
        for k, v in top.items():
            lines.append(f"{k} = {_toml_value(v)}")
        for k, v in self.v.items():
            if isinstance(v, dict):
                lines.append("")
                lines.append(f"[{k}]")
                for kk, vv in v.items():
                    lines.append(f"  {kk} = {_toml_value(vv)}")
        return "\n".join(lines) + "\n"

    # ---- typed helpers
    def data_dir(self) -> str:
        return os.path.expanduser(self.get("data-dir"))

    def duration(self, key: str) -> float:
        return parse_duration(self.get(key))


# ------------------------------------------------------------ gossip
def validate_gossip(cfg: "Config") -> None:
    """The ``[gossip]`` keys this build acts on (parallel/swim.py failure
    detection, NodeStatus push-pull) must hold usable values: positive
    probe interval / timeout, suspicion multiplier >= 1, indirect probers
    >= 0, a port number, durations that parse, and a ``gossip.key`` file of
    16, 24 or 32 bytes (memberlist's key sizes): the UDP probes on
    ``gossip.port`` carry an HMAC of it (parallel/gossip_udp.py)."""
    try:
        pi = cfg.duration("gossip.probe-interval")
        pt = cfg.duration("gossip.probe-timeout")
        for k in ("gossip.push-pull-interval", "gossip.interval", "gossip.to-the-dead-time", "gossip.stream-timeout"):
            if cfg.duration(k) < 0:
                raise ConfigError(f"{k} must not be negative")
    except ValueError as e:
        raise ConfigError(f"gossip: {e}")
    if pi <= 0:
        raise ConfigError("gossip.probe-interval must be positive")
    if pt <= 0:
        raise ConfigError("gossip.probe-timeout must be positive")
    if float(cfg.get("gossip.suspicion-mult")) < 1:
        raise ConfigError("gossip.suspicion-mult must be at least 1")
    if int(cfg.get("gossip.nodes")) < 0:
        raise ConfigError("gossip.nodes must not be negative")
    port = str(cfg.get("gossip.port"))
    if not port.isdigit() or not 0 <= int(port) <= 65535:
        raise ConfigError(f"gossip.port: invalid port {port!r}")
    if cfg.get("gossip.key"):
        from pilosa_amd.parallel.gossip_udp import load_key
        try:
            load_key(str(cfg.get("gossip.key")))
        except (OSError, ValueError) as e:
            raise ConfigError(f"gossip.key: {e}")


# ------------------------------------------------------------ listen / advertise
# (server/config.go validateAddrs, validateAdvertiseAddr, validateListenAddr)
DEFAULT_PORT = "10101"


def split_scheme(addr: str):
    scheme, sep, rest = addr.partition("://")
    return (scheme, rest) if sep else ("", addr)


def split_host_port(hostport: str):
    """net.SplitHostPort: "host:port" / "[v6]:port" -> (host, port)."""
    if hostport.startswith("["):
        end = hostport.find("]")
        if end < 0:
            raise ConfigError(f"address {hostport}: missing ']' in address")
        host, rest = hostport[1:end], hostport[end + 1:]
        if not rest.startswith(":"):
            raise ConfigError(f"address {hostport}: missing port in address")
        return host, rest[1:]
    i = hostport.rfind(":")
    if i < 0:
        raise ConfigError(f"address {hostport}: missing port in address")
    host, port = hostport[:i], hostport[i + 1:]
    if ":" in host:
        raise ConfigError(f"address {hostport}: too many colons in address")
    return host, port


def join_host_port(host: str, port: str) -> str:
    return f"[{host}]:{port}" if ":" in host else f"{host}:{port}"


def lookup_port(port: str) -> str:
    """net.LookupPort("tcp", port): numeric (signed) or a service name."""
    import socket
    try:
        n = int(port, 10)
    except ValueError:
        try:
            n = socket.getservbyname(port, "tcp")
        except OSError:
            raise ConfigError(f"lookup tcp/{port}: unknown port")
    if not 0 <= n <= 65535:
        raise ConfigError(f"address {port}: invalid port")
    return str(n)


def lookup_addr(host: str) -> str:
    """First IPv4 address of ``host`` (else the first address)."""
    import socket
    try:
        infos = socket.getaddrinfo(host, None, proto=socket.IPPROTO_TCP)
    except (OSError, UnicodeError):
        raise ConfigError(f"looking up IP addresses: lookup {host}: no such host")
    if not infos:
        raise ConfigError(f"cannot resolve {host!r} to an address")
    for fam, *_, sa in infos:
        if fam == socket.AF_INET:
            return sa[0]
    return infos[0][4][0]


def outbound_ip() -> str:
    """The address this host would use towards the outside (no packet is sent)."""
    import socket
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as sk:
            sk.connect(("8.8.8.8", 80))
            return sk.getsockname()[0]
    except OSError:   # no route out (an isolated host): the loopback address
        return "127.0.0.1"


def _split_addr(addr: str):
    scheme, hostport = split_scheme(addr)
    host, port = "", ""
    if hostport:
        host, port = split_host_port(hostport)
    return scheme, host, port or DEFAULT_PORT


def _scheme_host_port(scheme: str, host: str, port: str) -> str:
    return (f"{scheme}://" if scheme else "") + join_host_port(host, port)


def validate_addrs(bind: str, advertise: str):
    """(bind, advertise) normalised as the reference's Config.validateAddrs:
    default port 10101, service names resolved, host names resolved to IPs
    for the listener, and an empty advertise host taken from the listener
    (or the outbound address when listening on 0.0.0.0)."""
    try:
        l_scheme, l_host, l_port = _split_addr(bind)
        a_scheme, a_hostport = split_scheme(advertise)
        a_host, a_port = split_host_port(a_hostport) if a_hostport else ("", "")
        a_scheme = a_scheme or l_scheme
        if a_port in ("", "0"):
            a_port = l_port
        a_port = lookup_port(a_port)
        if not a_host:
            a_host = outbound_ip() if l_host == "0.0.0.0" else l_host
    except ConfigError as e:
        raise ConfigError(f"validating advertise address: {e}")
    adv = _scheme_host_port(a_scheme, a_host, a_port)
    try:
        l_port = lookup_port(l_port)
        if l_host not in ("", "localhost"):
            l_host = lookup_addr(l_host)
    except ConfigError as e:
        raise ConfigError(f"validating listen address: resolving address: {e}")
    return _scheme_host_port(l_scheme, l_host, l_port), adv


def _flat_keys(d: dict, prefix=""):
    for k, v in d.items():
        if isinstance(v, dict):
            yield from _flat_keys(v, f"{prefix}{k}.")
        else:
            yield f"{prefix}{k}"


def _coerce(value, old):
    if isinstance(old, bool):
        if isinstance(value, str):
            if value.lower() in ("true", "1", "yes"):
                return True
            if value.lower() in ("false", "0", "no", ""):
                return False
            raise ConfigError(f"invalid bool: {value}")
        return bool(value)
    if isinstance(old, int) and not isinstance(old, bool):
        return int(value)
    if isinstance(old, float):
        return float(value)
    if isinstance(old, list):
        if isinstance(value, str):
            return [x.strip() for x in value.split(",") if x.strip()]
        return list(value)
    return value if not isinstance(value, (int, float)) or isinstance(old, (int, float)) else str(value)


def _toml_value(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return repr(v)
    if isinstance(v, list):
        return "[" + ", ".join(_toml_value(x) for x in v) + "]"
    return '"' + str(v).replace("\\", "\\\\").replace('"', '\\"') + '"'
