"""Reference stats/stats_test.go (6 tests), statsd_test.go and
prometheus_test.go, ported: which events are counted, on which client,
with which tags (expvar / statsd / prometheus backends of utils/stats.py)."""
import json
import socket
import tempfile
import urllib.request

import pytest

from pilosa_amd.executor import Executor
from pilosa_amd.models.holder import Holder
from pilosa_amd.shardwidth import SHARD_WIDTH as SW
from pilosa_amd.utils import stats


class MockStats(stats.NopStatsClient):
    """stats_test.go MockStats: records Count / CountWithCustomTags calls."""

    def __init__(self):
        self.counts = []
        self.tagged = []

    def with_tags(self, *tags):
        return self

    def count(self, name, value=1, rate=1.0):
        self.counts.append(name)

    def count_with_tags(self, name, value, tags, rate=1.0):
        self.tagged.append((name, list(tags)))


def _holder(st):
    return Holder(tempfile.mkdtemp(), stats=st).open()


def test_multi_stat_client_expvar():
    """TestMultiStatClient_Expvar: fragment writes count under the index tag;
    gauges and sets overwrite; timings and histograms are recorded."""
    c = stats.ExpvarStatsClient()
    h = _holder(stats.MultiStatsClient(c))
    try:
        f = h.create_index("d").create_field("f")
        for col in (0, 1, SW, SW + 2):
            f.set_bit(0, col)
        f.clear_bit(0, 1)
        ev = c.expvar()
        assert ev["setBit{index:d}"] == 4 and ev["clearBit{index:d}"] == 1
        h.stats.count_with_tags("cc", 1, ["foo:bar"])
        assert c.expvar()["cc{foo:bar}"] == 1
        h.stats.gauge("g", 5)
        h.stats.gauge("g", 8)
        assert c.expvar()["g"] == 8
        h.stats.set("s", "4")
        h.stats.set("s", "7")
        h.stats.timing("tt", 123e-6)
        h.stats.histogram("hh", 3)
        ev = c.expvar()
        assert ev["tt"]["count"] == 1 and ev["hh"]["p50"] == 3
        assert h.stats.tags() == []     # the root client carries no tags
    finally:
        h.close()


def _run(h, q):
    ex = Executor(h)
    try:
        return ex.execute("d", q).results
    finally:
        ex.close()


def test_stats_count_topn():
    """TestStatsCount_TopN: the executor counts TopN with index:d."""
    m = MockStats()
    h = _holder(m)
    try:
        f = h.create_index("d").create_field("f")
        for col in (0, 1, SW, SW + 2):
            f.set_bit(0, col)
        m.tagged.clear()
        _run(h, "TopN(f, n=2)")
        assert ("TopN", ["index:d"]) in m.tagged
    finally:
        h.close()


def test_stats_count_bitmap():
    """TestStatsCount_Bitmap: Row(f=0) counts Row with index:d."""
    m = MockStats()
    h = _holder(m)
    try:
        f = h.create_index("d").create_field("f")
        f.set_bit(0, 0)
        f.set_bit(0, 1)
        m.tagged.clear()
        _run(h, "Row(f=0)")
        assert m.tagged == [("Row", ["index:d"])]
    finally:
        h.close()


def test_stats_count_set_row_attrs():
    """TestStatsCount_SetColumnAttrs (sic): SetRowAttrs counts on the field's client."""
    m = MockStats()
    h = _holder(m)
    try:
        f = h.create_index("d").create_field("f")
        f.set_bit(10, 0)
        m.counts.clear()
        _run(h, 'SetRowAttrs(f, 10, foo="bar")')
        assert "SetRowAttrs" in m.counts
    finally:
        h.close()


def test_stats_count_set_profile_attrs():
    """TestStatsCount_SetProfileAttrs: SetColumnAttrs counts SetProfileAttrs on the index's client."""
    m = MockStats()
    h = _holder(m)
    try:
        f = h.create_index("d").create_field("f")
        f.set_bit(10, 0)
        m.counts.clear()
        _run(h, 'SetColumnAttrs(10, foo="bar")')
        assert "SetProfileAttrs" in m.counts
    finally:
        h.close()


def test_stats_count_api_calls():
    """TestStatsCount_APICalls: createIndex / createField / deleteField /
    deleteIndex through the HTTP handler, on the holder's client."""
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    srv = Server(tempfile.mkdtemp(), bind="127.0.0.1:0", gpu="off", logger=CaptureLogger()).open()
    m = MockStats()
    srv.holder.stats = m
    base = f"http://127.0.0.1:{srv.uri.port}"

    def req(method, path):
        r = urllib.request.Request(base + path, data=b"" if method == "POST" else None, method=method)
        urllib.request.urlopen(r, timeout=10).read()
    try:
        req("POST", "/index/i")
        assert "createIndex" in m.counts
        req("POST", "/index/i/field/f")
        assert ("createField", ["index:i"]) in m.tagged
        req("DELETE", "/index/i/field/f")
        assert ("deleteField", ["index:i"]) in m.tagged
        req("DELETE", "/index/i")
        assert "deleteIndex" in m.counts
    finally:
        srv.close()


def test_statsd_client_sends_datagrams():
    """statsd_test.go: counters and gauges leave as DataDog statsd lines with tags."""
    sk = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sk.bind(("127.0.0.1", 0))
    sk.settimeout(5)
    try:
        c = stats.StatsDClient(f"127.0.0.1:{sk.getsockname()[1]}").with_tags("index:d")
        c.count("setBit", 2)
        got = sk.recv(4096).decode()
        assert got.startswith("pilosa.setBit:2|c") and "index:d" in got
        c.gauge("g", 7)
        got = sk.recv(4096).decode()
        assert got.startswith("pilosa.g:7") and "|g" in got
    finally:
        sk.close()


def test_prometheus_exposition():
    """prometheus_test.go: tagged counters become labelled series."""
    c = stats.ExpvarStatsClient().with_tags("index:d")
    c.count("setBit", 3)
    c.gauge("maxShard", 4)
    text = c.prometheus()
    assert 'pilosa_setBit_total{index="d"} 3' in text
    assert 'pilosa_maxShard{index="d"} 4' in text
