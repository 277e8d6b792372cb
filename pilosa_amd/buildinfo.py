"""Build-time knobs (reference: Makefile:9-19 ``-ldflags`` Version /
BuildTime / Enterprise, ``server/release.go`` vs ``server/default.go``,
``version.go``).

The reference bakes them into the binary with ldflags and build tags; here
``native/build.py`` writes them next to the package as ``_buildinfo.json``
when the native modules are built, from ``PILOSA_VERSION``,
``PILOSA_RELEASE=1`` and ``PILOSA_ENTERPRISE=1``.  Without that file (a
source checkout), the values are the reference's defaults: the package
version, "not recorded", enterprise off, and a non-release build, whose
diagnostics interval is 0 (diagnostics off) instead of a release's hour.
"""
from __future__ import annotations

import datetime as _dt
import json
import os

from pilosa_amd import __version__

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_buildinfo.json")


def _load() -> dict:
    try:
        with open(PATH) as fh:
            d = json.load(fh)
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


INFO = _load()
VERSION = str(INFO.get("version") or __version__)
BUILD_TIME = str(INFO.get("build_time") or "not recorded")
ENTERPRISE_ENABLED = str(INFO.get("enterprise", "0")) == "1"
RELEASE = bool(INFO.get("release", False))
# server/release.go (1 h) vs server/default.go (0 = off)
DEFAULT_DIAGNOSTICS_INTERVAL = 3600.0 if RELEASE else 0.0


def write(env=None) -> dict:
    """Record the knobs of this build (called by native/build.py)."""
    env = os.environ if env is None else env
    info = {"version": env.get("PILOSA_VERSION") or __version__,
            "build_time": _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S+0000"),
            "enterprise": "1" if env.get("PILOSA_ENTERPRISE") == "1" else "0",
            "release": env.get("PILOSA_RELEASE") == "1"}
    tmp = PATH + ".tmp"
    with open(tmp, "w") as fh:
        json.dump(info, fh)
    os.replace(tmp, PATH)
    return info
