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
    """Go-style durations ('1m30s', '500ms', '10m') -> seconds."""
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    if not s:
        return 0.0
    total, num = 0.0, ""
    i = 0
    while i < len(s):
        ch = s[i]
        if ch.isdigit() or ch == ".":
            num += ch
            i += 1
            continue
        unit = ""
        while i < len(s) and not (s[i].isdigit() or s[i] == "."):
            unit += s[i]
            i += 1
        if unit not in DURATION_UNITS or not num:
            raise ValueError(f"invalid duration: {v!r}")
        total += float(num) * DURATION_UNITS[unit]
        num = ""
    if num:
        if total == 0 and float(num) == 0:
            return 0.0
        raise ValueError(f"missing unit in duration {v!r}")
    return total


def format_duration(sec: float) -> str:
    if sec == 0:
        return "0s"
    if sec % 3600 == 0:
        return f"{int(sec // 3600)}h0m0s"
    if sec % 60 == 0:
        return f"{int(sec // 60)}m0s"
    if sec >= 1 and float(sec).is_integer():
        return f"{int(sec)}s"
    return f"{int(round(sec * 1000))}ms"


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
            self.merge(tomli.load(fh), strict=True)

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
