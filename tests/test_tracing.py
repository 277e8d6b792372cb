"""Tracing span trees (reference tracing/tracing.go + the StartSpanFromContext
sites of executor.go:117,235,278,2459,2521): a request's spans nest under
Executor.Execute across the map/reduce fan-out threads, the context crosses
process boundaries as a header / mesh command field, and on the GPU the
launch and copy spans carry HIP-event device time."""
import pytest

from pilosa_amd.utils import tracing
from tests.test_fanout import _executor, _SlowClient


@pytest.fixture
def tracer():
    t = tracing.RecordingTracer()
    prev = tracing.global_tracer()
    tracing.set_global_tracer(t)
    yield t
    tracing.set_global_tracer(prev)


def _names(node):
    out = [node["name"]]
    for c in node["children"]:
        out += _names(c)
    return out


def _find(node, name):
    if node["name"] == name:
        return node
    for c in node["children"]:
        got = _find(c, name)
        if got is not None:
            return got
    return None


def test_span_tree_spans_fanout_threads(tracer):
    client = _SlowClient(0.05)
    ex, holder = _executor(client)
    try:
        with tracing.span("test.request") as root:
            ex.execute("i", "Count(Row(f=1))", shards=list(range(6)))
    finally:
        ex.close()
        holder.close()
    tree = tracer.tree(root.trace_id)
    assert len(tree) == 1 and tree[0]["name"] == "test.request"
    exe = _find(tree[0], "Executor.Execute")
    mr = _find(exe, "Executor.mapReduce")
    assert mr is not None and mr["tags"]["shards"] == "6"
    remotes = [c for c in mr["children"] if c["name"] == "Executor.remoteExec"]
    # both remote nodes' requests ran in fan-out threads, yet hang under mapReduce
    assert sorted(c["tags"]["node"] for c in remotes) == ["n1", "n2"]
    assert any(c["name"] == "Executor.mapperLocal" for c in mr["children"])


def test_context_string_round_trip(tracer):
    with tracing.span("front") as s:
        ctx = tracing.context()
    assert ctx == f"{s.trace_id}:{s.span_id}"
    with tracing.remote_parent(ctx):
        with tracing.span("worker") as w:
            pass
    assert w.trace_id == s.trace_id and w.parent_id == s.span_id
    with tracing.remote_parent(""):
        assert tracing.current_span() is None


def test_gpu_flag_is_harmless_without_events(tracer):
    with tracing.span("GpuEngine.launchCount", gpu=True) as s:
        pass
    assert s.device_ms() is None and "device_ms" not in s.to_dict()


@pytest.mark.gpu
def test_gpu_count_request_span_tree_has_kernel_time():
    """One GPU Count request: its span tree holds the native plan, the kernel
    launch and the D2H copy, the latter two with HIP-event device time."""
    import tempfile

    import numpy as np

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor

    t = tracing.HipEventTracer()
    prev = tracing.global_tracer()
    tracing.set_global_tracer(t)
    holder = Holder(tempfile.mkdtemp()).open()
    try:
        f = holder.create_index("i").create_field("f")
        rng = np.random.default_rng(1)
        cols = rng.integers(0, 4 << 20, 200000).astype(np.uint64)
        f.import_bits(rng.integers(0, 4, len(cols)).astype(np.uint64), cols)
        gpu = GpuExecutor(holder, "cuda:0")
        ex = Executor(holder, gpu=gpu)
        gpu.executor = ex
        ex.strict_gpu = True
        text = "Count(Intersect(Row(f=1), Row(f=2))) Count(Row(f=3))"
        ex.execute("i", text)   # warm: arena load
        with tracing.span("test.request") as root:
            got = ex.execute("i", text).results
        tree = t.tree(root.trace_id, wait=True)
        host = Executor(holder)
        assert got == host.execute("i", text).results
        host.close()
        names = _names(tree[0])
        for n in ("Executor.Execute", "Executor.countTextNative", "GpuExecutor.planCountText",
                  "GpuEngine.launchCount", "GpuEngine.d2h"):
            assert n in names, (n, names)
        launch = _find(tree[0], "GpuEngine.launchCount")
        assert launch["device_ms"] > 0
        assert _find(tree[0], "GpuEngine.d2h")["device_ms"] >= 0
        ex.close()
    finally:
        holder.close()
        tracing.set_global_tracer(prev)
