"""Debug tooling: the instrumented roaring build (reference roaringstats build
tag, roaring/roaring_stats.go) and the /debug/pprof/ profiles
(http/handler.go:280 mounts net/http/pprof)."""
import threading
import time

import numpy as np
import pytest


def test_roaring_stats_variant_counts_container_events():
    rs = pytest.importorskip("pilosa_amd._roaring_stats")
    from pilosa_amd import _roaring
    assert rs.ROARING_STATS and not _roaring.ROARING_STATS
    assert set(_roaring.roaring_stats()) == set(rs.roaring_stats())
    assert all(v == 0 for v in _roaring.roaring_stats().values())
    rs.roaring_stats(reset=True)
    b = rs.Bitmap()
    for v in range(5000):            # appends, then the 4097th value converts to a bitmap
        b.add(v)
    b.add(70000)                     # a second container
    for v in range(5000):
        b.remove(v)                  # bitmap -> array on the way down, then the container goes
    b.add(1)
    b.add(0)                         # insert before the end
    st = rs.roaring_stats()
    assert st["NewContainer"] == 3
    assert st["arrayAdd/append"] >= 4096 and st["arrayAdd/insert"] >= 1
    assert st["arrayAdd/arrayToBitmap"] == 1
    assert st["bitmapRemove/bitmapToArray"] == 1
    assert st["sliceContainers/Remove"] == 1
    c = rs.Bitmap(np.arange(0, 3000, dtype=np.uint64))
    c.optimize()                     # one long run
    assert rs.roaring_stats(reset=True)["optimize/toRun"] == 1
    assert all(v == 0 for v in rs.roaring_stats().values())


def test_pprof_profiles():
    from pilosa_amd.utils import pprof
    assert "profile" in pprof.render("", {})
    stop = threading.Event()

    def busy_loop_for_profile():
        while not stop.is_set():
            sum(range(1000))
    t = threading.Thread(target=busy_loop_for_profile, name="busy", daemon=True)
    t.start()
    try:
        out = pprof.render("profile", {"seconds": "0.3", "hz": "200"})
    finally:
        stop.set()
        t.join()
    lines = out.splitlines()
    assert lines[0].startswith("# pilosa_amd cpu profile")
    hot = [ln for ln in lines[1:] if "busy_loop_for_profile" in ln]
    assert hot and all(ln.startswith("busy;") for ln in hot)
    assert int(hot[0].rsplit(" ", 1)[1]) > 5
    assert "threads:" in pprof.render("goroutine", {"debug": "1"})
    assert "live objects by type" in pprof.render("heap", {})
    h = pprof.render("heap", {"start": "1", "stop": "1"})
    assert "tracemalloc: current" in h
    assert "MainThread" in pprof.render("threadcreate", {})
    with pytest.raises(KeyError):
        pprof.render("bogus", {})


def test_pprof_http_endpoint():
    import urllib.request
    import tempfile
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    s = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger(), native_http=False).open()
    try:
        base = s.uri.normalize()
        with urllib.request.urlopen(base + "/debug/pprof/profile?seconds=0.2&hz=50", timeout=30) as r:
            assert r.status == 200 and r.read().startswith(b"# pilosa_amd cpu profile")
        try:
            urllib.request.urlopen(base + "/debug/pprof/nope", timeout=30)
            assert False, "expected 404"
        except urllib.error.HTTPError as e:
            assert e.code == 404
    finally:
        s.close()
