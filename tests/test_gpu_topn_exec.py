"""TopN through Executor.execute on the device (ops/topn_exec.py): a lazily
opened holder answers cache-only and src-filtered TopN from the fragments'
``.cache`` files and the HBM arena, with every fragment still cold afterwards,
and the answers equal the host executor's (fragment.top two-phase TopN,
executor.go:863-1000) computed on the same data before the lazy reopen."""
import os
import threading

import numpy as np
import pytest

from pilosa_amd.executor import Executor
from pilosa_amd.models.holder import Holder
from pilosa_amd import shardwidth
from tests.helpers import SW, Env

pytestmark = pytest.mark.gpu

QUERIES = ["TopN(h, n=10)", "TopN(h, n=100)", "TopN(h)", "TopN(h, n=20, threshold=300)",
           "TopN(h, Row(f=1), n=5)", "TopN(h, Row(f=0), n=50)", "TopN(h, Row(h=3), n=20)",
           "TopN(h, Row(f=2), n=7, threshold=2)", "TopN(h, ids=[1, 5, 7, 2999])",
           "TopN(h, Row(f=1), ids=[0, 2, 4, 6, 8])", "TopN(h, Intersect(Row(f=0), Row(f=1)), n=10)",
           # n / threshold beyond int32: clamped, not a device fault
           "TopN(h, n=3000000000)", "TopN(h, n=3000000000, threshold=5000000000)"]


@pytest.fixture(scope="module")
def lazy_env():
    """(lazy holder, GPU executor, {query: host answer}, multi-call answer)."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    env = Env()
    rng = np.random.default_rng(7)
    env.create_index("i")
    env.field("i", "f")
    env.field("i", "h", cache_type="ranked", cache_size=2000)
    idx = env.holder.index("i")
    nshard = 3
    for r in range(4):
        k = int([0.3, 0.05, 0.01, 0.002][r] * nshard * SW)
        idx.field("f").import_bits(np.full(k, r, np.uint64),
                                   rng.choice(nshard * SW, size=k, replace=False).astype(np.uint64))
    hr = (rng.zipf(1.3, size=300000) % 3000).astype(np.uint64)
    hc = rng.integers(0, nshard * SW, size=len(hr)).astype(np.uint64)
    idx.field("h").import_bits(hr, hc)
    for frag in env.holder.all_fragments():
        frag.rebuild_cache()
        frag.flush_cache()
    want = {q: env.q1("i", q) for q in QUERIES}
    want_multi = env.q("i", " ".join(QUERIES[:8]))
    env.holder.close()
    holder = Holder(env.dir, lazy_fragments=True).open()
    gpu = GpuExecutor(holder, "cuda:0")
    ex = Executor(holder, gpu=gpu)
    gpu.executor = ex
    ex.strict_gpu = True
    yield holder, ex, gpu, want, want_multi
    ex.close()
    holder.close()
    env.executor.close()
    import shutil
    shutil.rmtree(env.dir, ignore_errors=True)


def _pairs(r):
    return [(p.id, p.count) for p in r]


@pytest.mark.parametrize("q", QUERIES)
def test_topn_executor_matches_host_and_stays_cold(lazy_env, q):
    holder, ex, gpu, want, _ = lazy_env
    n0 = gpu.launches
    got = ex.execute("i", q).results[0]
    assert gpu.launches > n0, "device path not taken"
    assert _pairs(got) == _pairs(want[q])
    assert ex.gpu_faults == 0
    frags = holder.view("i", "h", "standard").all_fragments()
    assert frags and all(f.is_cold() for f in frags), "TopN read a fragment on the host"


def test_multi_call_topn_request_one_batch(lazy_env):
    holder, ex, gpu, want, want_multi = lazy_env
    got = ex.execute("i", " ".join(QUERIES[:8])).results
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want_multi]
    assert all(f.is_cold() for f in holder.view("i", "h", "standard").all_fragments())


def test_concurrent_topn_requests_coalesce(lazy_env):
    holder, ex, gpu, want, _ = lazy_env
    qs = [QUERIES[k % 8] for k in range(48)]
    out = [None] * len(qs)
    f0 = ex.topn_coalescer.fallbacks

    def run(k):
        out[k] = ex.execute("i", qs[k]).results[0]
    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(qs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k, q in enumerate(qs):
        assert _pairs(out[k]) == _pairs(want[q]), q
    # every width: src calls batch on the slot index (per arena sub-shard at
    # wider shards), no per-call fallback
    assert ex.topn_coalescer.fallbacks == f0, (repr(ex.topn_coalescer.last_error), ex.topn_batch_declined,
                                               gpu.topn_decline)


def test_rank_caches_from_cache_files_equal_host_caches(lazy_env):
    """The device rank lists of cold fragments (.cache ids + arena counts)
    are the host rank caches the reference's openCache builds."""
    holder, ex, gpu, _, _ = lazy_env
    shards = holder.index("i").available_shards()
    rv = gpu.view_arena("i", "h", "standard", shards)
    frags = [holder.fragment("i", "h", "standard", s) for s in shards]
    rc = gpu._rank_caches("i", "h", shards, frags, rv)
    assert rc.cold_shards == len(shards)
    rows, counts = rc.host_lists()
    from pilosa_amd import _roaring
    for si, s in enumerate(shards):
        with open(frags[si].path, "rb") as fh:
            bm = _roaring.Bitmap.from_bytes(fh.read())
        offs, ids, _ = _roaring.read_cache_files([frags[si].cache_path()])
        host = sorted(((int(i), int(bm.count_range(int(i) * SW, (int(i) + 1) * SW))) for i in ids),
                      key=lambda p: (-p[1], p[0]))
        host = [p for p in host if p[1] > 0][:frags[si].cache_size]   # rankCache keeps cache_size entries
        live = counts[si] > 0
        assert list(zip(rows[si][live].tolist(), counts[si][live].tolist())) == host
    assert all(f.is_cold() for f in frags)


def test_topn_after_writes_uses_warm_caches(lazy_env):
    """A fragment written to after open is warm: its live host cache feeds the
    device ranks, and the answers still equal the host path."""
    holder, ex, gpu, _, _ = lazy_env
    ex.execute("i", "Set(5, h=2999) Set(6, h=2999) Set(7, h=2999)")
    got = ex.execute("i", "TopN(h, n=15) TopN(h, Row(f=1), n=6)").results
    ex.gpu = None
    try:
        want = ex.execute("i", "TopN(h, n=15) TopN(h, Row(f=1), n=6)").results
    finally:
        ex.gpu = gpu
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want]


def test_single_bit_writes_to_cold_fragment_reach_device_ranks(lazy_env):
    """Set on a mapped (cold) fragment goes to the mapped overlay and opens
    the fragment's in-memory rank cache while the fragment stays cold: from
    then on the live cache, not the stale ``.cache`` file, ranks that shard,
    so a new row written there shows up in the device TopN."""
    holder, ex, gpu, _, _ = lazy_env
    frag = holder.fragment("i", "h", "standard", 1)
    ex.execute("i", "TopN(h)")     # device ranks built while the shard is file-backed
    ex.execute("i", " ".join(f"Set({SW + 10 + k}, h=5000)" for k in range(60)))
    assert frag.is_cold() and frag.cache_is_live()
    frag.cache.recalculate()       # past the rank cache's 10 s recalculation throttle
    qs = "TopN(h) TopN(h, n=2500) TopN(h, Row(f=0), n=3000)"
    got = ex.execute("i", qs).results
    ex.gpu = None
    try:
        want = ex.execute("i", qs).results
    finally:
        ex.gpu = gpu
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want]
    assert 5000 in [p.id for p in got[0]]


def test_nosrc_dense_batch_equals_two_phase(lazy_env):
    """The sync-free cache-only batch (one [Q, candidates] accumulator, one
    re-count per threshold, one top-k) answers exactly as phase 1 + ids=
    re-count + finish_batch_dev, for mixed n (0 = all) and thresholds."""
    from pilosa_amd.ops.topn_index import finish_batch_dev
    holder, ex, gpu, want, _ = lazy_env
    ex.execute("i", "TopN(h, n=10)")
    rc = next(iter(gpu._rank_cache_map.values()))[1]
    ns = [10, 100, 0, 20, 1, 7, 100, 3, rc.K + 500]   # the last asks for more rows than a cache holds
    ths = [1, 1, 1, 300, 1, 2, 50, 1, 1]
    got = rc._topn_nosrc_dense(ns, ths)
    pq, pd, _ = rc.nosrc_phase1(ns, ths)
    ref = finish_batch_dev(rc.view.rows, len(ns), pq, pd, rc.recount(pq, pd, ths), ns)
    assert [_pairs(r) for r in got] == [_pairs(r) for r in ref]
    assert _pairs(got[0]) == _pairs(want["TopN(h, n=10)"])


def test_nosrc_fused_kernels_equal_torch_batch(lazy_env, monkeypatch):
    """The hand-written cache-only batch (topn_cache_member / totals / select
    kernels) answers exactly as the torch batch and the two-phase reference,
    for mixed n (0 = all, n beyond the cache width) and thresholds; the
    executor's TopN runs through it; an oversized candidate set declines to
    the torch batch."""
    from pilosa_amd.ops import topn_exec
    from pilosa_amd.ops.topn_index import finish_batch_dev
    holder, ex, gpu, want, _ = lazy_env
    ex.execute("i", "TopN(h, n=10)")
    rc = next(iter(gpu._rank_cache_map.values()))[1]
    ns = [10, 100, 0, 20, 1, 7, 100, 3, rc.K + 500, 50, 50]
    ths = [1, 1, 1, 300, 1, 2, 50, 1, 1, 5000, 20]
    got = rc._topn_nosrc_fused(ns, ths)
    assert got is not None
    dense = rc._topn_nosrc_dense(ns, ths)
    pq, pd, _ = rc.nosrc_phase1(ns, ths)
    ref = finish_batch_dev(rc.view.rows, len(ns), pq, pd, rc.recount(pq, pd, ths), ns)
    assert [_pairs(r) for r in got] == [_pairs(r) for r in dense] == [_pairs(r) for r in ref]
    assert _pairs(got[0]) == _pairs(want["TopN(h, n=10)"])
    assert rc.__dict__.get("_fused"), "fused memo never built"
    rc.__dict__.pop("_fused", None)
    monkeypatch.setattr(topn_exec, "FUSED_MAX_CELLS", 0)
    assert rc._topn_nosrc_fused(ns, ths) is None
    assert [_pairs(r) for r in rc.topn_nosrc(ns, ths)] == [_pairs(r) for r in ref]


@pytest.mark.parametrize("native", [False, True])
def test_nosrc_fused_concurrent_batches_on_lanes(lazy_env, monkeypatch, native):
    """Concurrent cache-only batches each check out a (side stream, pinned
    parameter buffer) lane -- a Python lane, or a slot of the native request
    object (binding.cpp CacheTopN) -- : 8 threads x 12 batches of different
    n / threshold mixes answer exactly as the same batches run one at a time,
    and the lanes are reused (the pool never holds more than the concurrency)."""
    from pilosa_amd.ops import topn_exec
    monkeypatch.setattr(topn_exec, "NATIVE_FUSED", native)
    holder, ex, gpu, _, _ = lazy_env
    ex.execute("i", "TopN(h, n=10)")
    rc = next(iter(gpu._rank_cache_map.values()))[1]
    rc.__dict__.pop("_fused", None)   # an earlier test memoised declines under FUSED_MAX_CELLS = 0
    rng = np.random.default_rng(5)
    batches = []
    for _ in range(96):
        q = int(rng.integers(1, 17))
        batches.append(([int(x) for x in rng.choice([0, 1, 5, 10, 50, 100, 400], q)],
                        [int(x) for x in rng.choice([1, 2, 20, 300], q)]))
    want = [[_pairs(r) for r in rc._topn_nosrc_fused(ns, ths)] for ns, ths in batches]
    assert want == [[_pairs(r) for r in rc._topn_nosrc_dense(ns, ths)] for ns, ths in batches]
    n0 = len(topn_exec._LANES.get(rc.view.device, []))
    got = [None] * len(batches)
    err = []

    def worker(w):
        try:
            for k in range(w, len(batches), 8):
                got[k] = [_pairs(r) for r in rc._topn_nosrc_fused(*batches[k])]
        except BaseException as e:  # noqa: BLE001
            err.append(e)
    ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not err, err[0]
    assert got == want
    lanes = topn_exec._LANES.get(rc.view.device, [])
    if native:
        assert rc.__dict__.get("_nat"), "the native request object never ran"
        assert len(lanes) == n0
    else:
        assert 1 <= len(lanes) <= n0 + 8


def test_nosrc_native_request_equals_python_lane(lazy_env, monkeypatch):
    """The native cache-only request (CacheTopN.run: parameters, kernels, D2H
    and decode in C++) answers every batch exactly as the Python lane path
    over the same memo, including n = 0, n beyond the candidates, int32-edge
    n / thresholds and duplicate thresholds; results are columnar PairArrays."""
    from pilosa_amd.models.cache import PairArray
    from pilosa_amd.ops import topn_exec
    holder, ex, gpu, _, _ = lazy_env
    ex.execute("i", "TopN(h, n=10)")
    rc = next(iter(gpu._rank_cache_map.values()))[1]
    rc.__dict__.pop("_fused", None)
    rng = np.random.default_rng(11)
    batches = [([0, 10, (1 << 31) - 1], [1, 1, (1 << 31) - 1]), ([rc.K + 7], [2]), ([5] * 16, [3] * 16)]
    for _ in range(40):
        q = int(rng.integers(1, 33))
        batches.append(([int(x) for x in rng.choice([0, 1, 3, 10, 64, 200, 999], q)],
                        [int(x) for x in rng.choice([1, 2, 7, 40, 1000], q)]))
    for ns, ths in batches:
        monkeypatch.setattr(topn_exec, "NATIVE_FUSED", False)
        want = rc._topn_nosrc_fused(ns, ths)
        monkeypatch.setattr(topn_exec, "NATIVE_FUSED", True)
        got = rc._topn_nosrc_fused(ns, ths)
        assert want is not None and got is not None
        assert all(isinstance(r, PairArray) for r in got)
        assert [_pairs(r) for r in got] == [_pairs(r) for r in want], (ns, ths)
    assert rc.__dict__.get("_nat")
    # the member buffer is reused with a cycling epoch mark and cleared only
    # when it wraps (every ~253 batches per slot): answers stay exact across
    # several wraps, alternating batch shapes so stale marks would show
    monkeypatch.setattr(topn_exec, "NATIVE_FUSED", True)
    ref = {i: [_pairs(r) for r in rc._topn_nosrc_fused(*batches[i])] for i in (3, 4)}
    for k in range(600):
        i = 3 + (k & 1)
        assert [_pairs(r) for r in rc._topn_nosrc_fused(*batches[i])] == ref[i], k


def test_src_topn_after_write_burst_refreshes_index_in_place(lazy_env):
    """A write burst into one shard (new bits, and a tail row pushed up the
    rank order) re-indexes only that shard's slot region in place: the next
    src TopN is answered by the slot index (no throttled rebuild, no
    pair-count fallback) and equals the host path."""
    holder, ex, gpu, _, _ = lazy_env
    q = "TopN(h, Row(f=1), n=8) TopN(h, Row(f=0), n=5)"
    gpu._topn_indexes.clear()               # earlier tests may have left a throttled entry
    ex.execute("i", q)                      # index built over the current caches
    r0 = gpu.topn_index_refreshes
    d0 = ex.topn_batch_declined
    cols = np.arange(2 * SW + 1000, 2 * SW + 61000, 7, dtype=np.uint64)
    holder.index("i").field("h").import_bits(np.full(len(cols), 2998, np.uint64), cols)
    ex.execute("i", "Set(%d, h=7) Clear(%d, h=7)" % (2 * SW + 3, 2 * SW + 3))
    got = ex.execute("i", q).results
    assert gpu.topn_index_refreshes > r0, gpu._topn_index_why if hasattr(gpu, "_topn_index_why") else ""
    assert ex.topn_batch_declined == d0
    ex.gpu = None
    try:
        want = ex.execute("i", q).results
    finally:
        ex.gpu = gpu
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want]


def test_src_topn_concurrent_with_write_bursts(lazy_env):
    """Request threads keep running src TopN while another thread writes
    bursts into one shard: the in-place index refreshes wait for the batches
    in flight (reader/writer lock), nothing fails, and afterwards the answers
    equal the host path."""
    holder, ex, gpu, _, _ = lazy_env
    q = "TopN(h, Row(f=1), n=8) TopN(h, Row(f=2), n=4)"
    errs = []
    stop = threading.Event()

    def reader():
        try:
            while not stop.is_set():
                ex.execute("i", q)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    def writer():
        try:
            rng = np.random.default_rng(11)
            for k in range(6):
                cols = (np.uint64(SW) + rng.choice(SW, 3000, replace=False).astype(np.uint64))
                holder.index("i").field("h").import_bits(np.full(len(cols), 2990 + k, np.uint64), cols)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
    rs = [threading.Thread(target=reader) for _ in range(3)]
    w = threading.Thread(target=writer)
    for t in rs:
        t.start()
    w.start()
    w.join(timeout=120)
    stop.set()
    for t in rs:
        t.join(timeout=120)
    assert not errs, errs[:2]
    assert not w.is_alive() and not any(t.is_alive() for t in rs)
    got = ex.execute("i", q).results
    ex.gpu = None
    try:
        want = ex.execute("i", q).results
    finally:
        ex.gpu = gpu
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want]


@pytest.mark.parametrize("hot", [0, 64, 700])
def test_slot_index_on_fragment_caches_matches_host(lazy_env, hot):
    """The slot index over the executor's per-fragment rank caches, with the
    cache ranks split between the hot-rank matrix and the tail histogram
    (hot=0: histogram only).  At a wide shard width (PILOSA_SHARD_WIDTH=22,
    test_gpu_shardwidth.py) each fragment is M arena sub-shards: the index
    is per sub-shard and the hot counts and histograms are summed per
    fragment before the heap walk (topn_kernels.hip topn_src_kernel)."""
    from pilosa_amd.ops.topn_index import DeviceTopNIndex
    from pilosa_amd.pql import parse_string
    holder, ex, gpu, _, _ = lazy_env
    # earlier tests of the module write to h: settle every rank cache now.
    # The host path re-ranks a dirty cache once its 10 s throttle expires
    # (fragment._top_bitmap_pairs -> invalidate); without this, a re-rank
    # landing between the device snapshot below and the host answers moved
    # the cache boundary (n=0 walks the whole cache) -- a timing flake
    if not os.environ.get("PILOSA_TEST_NO_SETTLE"):
        holder.recalculate_caches()
    shards = holder.index("i").available_shards()
    rv = gpu.view_arena("i", "h", "standard", shards)
    frags = [holder.fragment("i", "h", "standard", s) for s in shards]
    rc = gpu._rank_caches("i", "h", shards, frags, rv)
    idx = DeviceTopNIndex(rv, rc, hot=hot)
    assert idx.ok and idx.M == rc.M and idx.Sd == rv.S and idx.R == min(hot, rc.K)
    if shardwidth.WIDE:
        assert idx.M > 1
    cases = ["Row(f=0)", "Row(f=1)", "Row(f=3)", "Row(h=3)", "Intersect(Row(f=0), Row(f=1))"]
    srcs = [gpu.plan("i", parse_string(q).calls[0], shards) for q in cases]
    for n, th in ((5, 1), (50, 1), (0, 1), (20, 40)):
        got = idx.topn(gpu.engine, srcs, [n] * len(srcs), [th] * len(srcs))
        ex.gpu = None
        try:
            want = [ex.execute("i", f"TopN(h, {q}, n={n}, threshold={th})").results[0] for q in cases]
        finally:
            ex.gpu = gpu
        for q, g, w in zip(cases, got, want):
            if _pairs(g) != _pairs(w):
                gd, wd = dict(_pairs(g)), dict(_pairs(w))
                diff = sorted(set(gd.items()) ^ set(wd.items()))[:8]
                print("SLOTDIFF", q, n, th, hot, "device-only", sorted(set(gd.items()) - set(wd.items()))[:8],
                      "host-only", sorted(set(wd.items()) - set(gd.items()))[:8], "len", len(gd), len(wd))
                for rid, _ in diff[:4]:
                    per = []
                    for si, f in enumerate(frags):
                        c = f.cache
                        per.append((si, c.get(rid), len(c), getattr(c, "threshold_value", None),
                                    f.row_count(rid), f.is_cold()))
                    print("SLOTROW", rid, [x for x in per if x[1] or x[4]][:12])
            assert _pairs(g) == _pairs(w), (q, n, th, hot)


def test_src_topn_uses_the_slot_index_at_every_width(lazy_env):
    """Src TopN calls through the executor are answered by the device slot
    index (not the pair-count path) whatever the shard width."""
    holder, ex, gpu, _, _ = lazy_env
    holder.recalculate_caches()   # no re-rank between the device and host answers
    gpu._topn_indexes.clear()
    b0 = gpu.topn_index_batches
    q = "TopN(h, Row(f=1), n=5) TopN(h, Row(f=0), n=9)"
    got = ex.execute("i", q).results
    assert gpu.topn_index_batches > b0, getattr(gpu, "_topn_index_why", "")
    ex.gpu = None
    try:
        want = ex.execute("i", q).results
    finally:
        ex.gpu = gpu
    assert [_pairs(r) for r in got] == [_pairs(r) for r in want]


def test_cache_only_batch_with_varied_n_matches_host(lazy_env):
    """Cache-only calls whose n spans several prefix buckets (the count
    matrix / candidate memo is per power-of-two prefix) in one request, and
    again in another order: == the host answers."""
    holder, ex, gpu, _, _ = lazy_env
    holder.recalculate_caches()   # no re-rank between the device and host answers
    calls = ["TopN(h, n=3)", "TopN(h, n=17, threshold=5)", "TopN(h, n=700)", "TopN(h, n=129, threshold=40)",
             "TopN(h, n=1)", "TopN(h, n=33)"]
    for order in (calls, calls[::-1], calls[2:] + calls[:2]):
        q = " ".join(order)
        got = ex.execute("i", q).results
        assert gpu.__dict__.get("_plain_memo"), "the plain cache-only TopN path was not taken"
        ex.gpu = None
        try:
            want = ex.execute("i", q).results
        finally:
            ex.gpu = gpu
        assert [_pairs(r) for r in got] == [_pairs(r) for r in want], q
