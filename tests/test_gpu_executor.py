"""GPU executor vs host executor on the same holder (differential test)."""
import numpy as np
import pytest

from tests.helpers import SW, Env, cols

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def envs():
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    cpu = Env()
    rng = np.random.default_rng(3)
    for e in (cpu,):
        e.create_index("i")
        e.field("i", "f")
        e.field("i", "g")
        e.field("i", "t", type="time", time_quantum="YMD")
        e.field("i", "n", type="int", min=-1000, max=100000)
        e.field("i", "m", type="int", min=-5000, max=-10)
        e.field("i", "h", cache_type="ranked", cache_size=5000)
    idx = cpu.holder.index("i")
    f, g, t, n = (idx.field(x) for x in "fgtn")
    nshard = 4
    for r in range(12):
        density = [0.5, 0.05, 0.002, 0.0001][r % 4]
        k = int(density * nshard * SW)
        c = rng.choice(nshard * SW, size=k, replace=False).astype(np.uint64)
        f.import_bits(np.full(k, r, np.uint64), c)
        c2 = rng.choice(nshard * SW, size=k // 2 + 1, replace=False).astype(np.uint64)
        g.import_bits(np.full(len(c2), r % 5, np.uint64), c2)
    # runs
    f.import_bits(np.full(200000, 20, np.uint64), np.arange(100000, 300000, dtype=np.uint64))
    import datetime as dt
    cc = rng.choice(nshard * SW, size=5000, replace=False)
    ts = [dt.datetime(2020, 1 + int(x % 12), 1 + int(x % 27)) for x in cc]
    t.import_bits(np.full(len(cc), 1, np.uint64), cc.astype(np.uint64), timestamps=ts)
    vc = rng.choice(nshard * SW, size=20000, replace=False).astype(np.uint64)
    n.import_values(vc, rng.integers(-1000, 100000, size=len(vc)))
    # many rows with Zipf-like sizes: TopN replays need several counted prefixes
    hr = (rng.zipf(1.3, size=400000) % 3000).astype(np.uint64)
    hc = rng.integers(0, nshard * SW, size=len(hr)).astype(np.uint64)
    idx.field("h").import_bits(hr, hc)
    mc = rng.choice(nshard * SW, size=3000, replace=False).astype(np.uint64)
    idx.field("m").import_values(mc, rng.integers(-5000, -10, size=len(mc)))
    idx.existence_field().import_bits(np.zeros(nshard * SW // 2, np.uint64),
                                      np.arange(nshard * SW // 2, dtype=np.uint64))
    for frag in cpu.holder.all_fragments():
        frag.rebuild_cache()
    gpu = GpuExecutor(cpu.holder, "cuda:0", executor=cpu.executor)
    yield cpu, gpu
    cpu.close()


def _dev(cpu, gpu, fn):
    """Run ``fn`` with the GPU attached; the device must really answer (a
    launch happened; faults raise in strict mode, tests/conftest.py)."""
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = fn()
        assert gpu.launches > n0, "device path not taken"
    finally:
        cpu.executor.gpu = None
    return got


QUERIES = [
    "Count(Row(f=0))", "Count(Row(f=3))", "Count(Intersect(Row(f=0), Row(f=1)))",
    "Count(Intersect(Row(f=1), Row(f=2)))", "Count(Intersect(Row(f=2), Row(f=3)))",
    "Count(Intersect(Row(f=0), Row(f=20)))", "Count(Union(Row(f=1), Row(f=2), Row(f=20)))",
    "Count(Difference(Row(f=0), Row(g=1)))", "Count(Xor(Row(f=4), Row(g=0)))",
    "Count(Not(Row(f=1)))", "Count(Intersect(Union(Row(f=0), Row(g=2)), Not(Row(f=5))))",
    "Count(Row(t=1, from=2020-03-01T00:00, to=2020-07-15T00:00))", "Count(Row(f=999))",
    "Count(Intersect(Row(f=0), Row(f=999)))",
]


@pytest.mark.parametrize("q", QUERIES)
def test_counts_match_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    got = _dev(cpu, gpu, lambda: cpu.q1("i", q))
    assert got == want


def test_count_batch(envs):
    cpu, gpu = envs
    want = cpu.q("i", " ".join(QUERIES))
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q("i", " ".join(QUERIES))
        assert gpu.launches == n0 + 1
    finally:
        cpu.executor.gpu = None
    assert got == want


@pytest.mark.parametrize("q", ["Row(f=2)", "Intersect(Row(f=0), Row(f=1))", "Union(Row(f=3), Row(f=20))",
                               "Difference(Row(f=20), Row(f=0))", "Not(Row(f=0))"])
def test_rows_match_host(envs, q):
    cpu, gpu = envs
    want = cols(cpu.q1("i", q))
    got = cols(_dev(cpu, gpu, lambda: cpu.q1("i", q)))
    assert got == want


@pytest.mark.parametrize("q", ["Sum(field=n)", "Sum(Row(f=0), field=n)", "TopN(f, Row(g=1), n=5)",
                               "TopN(f, Row(g=0))", "GroupBy(Rows(g), Rows(f), limit=20)",
                               "GroupBy(Rows(g), Rows(f), filter=Row(f=1), limit=7)"])
def test_aggregates_match_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    got = _dev(cpu, gpu, lambda: cpu.q1("i", q))
    assert got == want


def test_arena_invalidation_on_write(envs):
    cpu, gpu = envs
    cpu.executor.gpu = gpu
    try:
        before = cpu.q1("i", "Count(Row(f=7))")
        cpu.q("i", f"Set({3 * SW + 12345}, f=7)")
        after = cpu.q1("i", "Count(Row(f=7))")
    finally:
        cpu.executor.gpu = None
    assert after == cpu.q1("i", "Count(Row(f=7))")
    assert after in (before, before + 1)


BSI_QUERIES = [
    "Count(Row(n < 0))", "Count(Row(n <= -1))", "Count(Row(n > 500))", "Count(Row(n >= 0))",
    "Count(Row(n < -1))", "Count(Row(n > -1))", "Count(Row(n >= -7))", "Count(Row(n < 77777))",
    "Count(Row(n == 1234))", "Count(Row(n != 5))", "Count(Row(n >< [-100, 100]))",
    "Count(Row(n >< [10, 5000]))", "Count(Row(n >< [-900, -10]))", "Count(Row(n != null))",
    "Count(Intersect(Row(f=0), Row(n > 50000)))", "Count(Union(Row(n < -500), Row(m > -100)))",
    "Count(Row(m == -20))", "Count(Row(m < -4000))", "Count(Row(n > 200000))",
    "Min(field=n)", "Max(field=n)", "Min(Row(f=1), field=n)", "Max(Row(f=2), field=n)",
    "Min(field=m)", "Max(field=m)", "Max(Row(f=0), field=m)", "Min(Row(n > 90000), field=n)",
    "Sum(Row(n < 0), field=n)", "Sum(field=n)", "Sum(field=m)",
]


@pytest.mark.parametrize("q", BSI_QUERIES)
def test_bsi_on_device_matches_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q1("i", q)
        if "200000" not in q:  # out-of-range predicate: answered without a launch
            assert gpu.launches > n0, "device path not taken"
    finally:
        cpu.executor.gpu = None
    assert got == want


def test_bsi_counts_in_one_request_match_host(envs):
    """A request of many Count() calls mixing BSI conditions (fused
    predicate+count launches, one D2H) with plain trees: == host."""
    cpu, gpu = envs
    text = " ".join(q for q in BSI_QUERIES if q.startswith("Count("))
    want = cpu.q("i", text)
    got = _dev(cpu, gpu, lambda: cpu.q("i", text))
    assert got == want


def test_bsi_rows_match_host(envs):
    cpu, gpu = envs
    for q in ("Row(n > 99000)", "Row(n >< [-3, 3])", "Row(m < -4990)"):
        want = cols(cpu.q1("i", q))
        got = cols(_dev(cpu, gpu, lambda: cpu.q1("i", q)))
        assert got == want, q


@pytest.mark.parametrize("q", ["TopN(h, Row(f=2), n=5)", "TopN(h, Row(f=3), n=300)", "TopN(h, Row(f=0), n=50)",
                               "TopN(h, Row(g=1), n=1000)", "TopN(h, Row(f=1), ids=[1, 5, 7, 2999])",
                               "TopN(h, Row(f=0), n=20, threshold=50)"])
def test_topn_prefix_rounds_match_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    got = _dev(cpu, gpu, lambda: cpu.q1("i", q))
    assert got == want


@pytest.mark.skipif(__import__("pilosa_amd.shardwidth").shardwidth.WIDE,
                    reason="ops/topn.py ranks per 2^20-column arena shard (engine-level API); the executor's "
                           "per-fragment ranking at wider shards is tests/test_gpu_topn_exec.py")
def test_device_rank_cache_topn_batch_matches_host(envs):
    """HBM rank caches + batched two-phase TopN (ops/topn.py) == host TopN."""
    from pilosa_amd.ops.topn import DeviceRankCache, topn_batch
    from pilosa_amd.pql import parse_string
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    hv = gpu.view_arena("i", "h", "standard", shards)
    cache = DeviceRankCache.from_view(hv, k=5000)
    # the device cache order equals the fragments' rank caches (all rows fit)
    for si, s in enumerate(shards):
        frag = cpu.holder.fragment("i", "h", "standard", s)
        # (at narrow shard widths the run of f=20 reaches a shard h never has)
        host = [(p[0], p[1]) for p in frag._top_bitmap_pairs([])] if frag is not None else []
        dev = [(int(r), int(c)) for r, c in zip(cache.rows[si], cache.counts[si]) if c > 0]
        assert dev == host
    cases = [("Row(f=2)", 5), ("Row(f=3)", 300), ("Row(g=1)", 1000), ("Row(f=0)", 50)]
    srcs = [gpu.plan("i", parse_string(q).calls[0], shards) for q, _ in cases]
    for n in sorted({n for _, n in cases}):
        got = topn_batch(gpu.engine, hv, cache, srcs, n=n)
        for (q, _), g in zip(cases, got):
            want = cpu.q1("i", f"TopN(h, {q}, n={n})")
            assert [(p.id, p.count) for p in g] == [(p.id, p.count) for p in want], (q, n)


@pytest.mark.skipif(__import__("pilosa_amd.shardwidth").shardwidth.WIDE,
                    reason="ops/topn.py ranks per 2^20-column arena shard (engine-level API); the executor's "
                           "per-fragment ranking at wider shards is tests/test_gpu_topn_exec.py")
def test_cache_only_topn_matches_host(envs):
    from pilosa_amd.ops.topn import DeviceRankCache, finish_topn, topn_cache_phase1, topn_cache_phase2_counts
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    hv = gpu.view_arena("i", "h", "standard", shards)
    cache = DeviceRankCache.from_view(hv, k=5000, keep_row_counts=True)
    for n in (1, 10, 100):
        t = topn_cache_phase1(cache, n)
        ids = sorted(t)
        got = finish_topn(ids, topn_cache_phase2_counts(cache, hv, ids), n)
        want = cpu.q1("i", f"TopN(h, n={n})")
        assert [(p.id, p.count) for p in got] == [(p.id, p.count) for p in want], n


def test_generated_queries_gpu_vs_host(envs):
    """Random PQL (pilosa_amd/testing/querygen.py) through the executor with
    and without the GPU: identical results."""
    from pilosa_amd.testing.querygen import QueryGenerator
    cpu, gpu = envs
    g = QueryGenerator(seed=21, set_fields=["f", "g"], int_fields=["n"], time_fields=["t"], max_row=14,
                       int_range=(-1000, 100000))
    qs = g.queries(120, depth=3)
    want = [cpu.q("i", q) for q in qs]
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = [cpu.q("i", q) for q in qs]
        assert gpu.launches > n0 + 50
    finally:
        cpu.executor.gpu = None
    for q, w, r in zip(qs, want, got):
        if hasattr(w[0], "columns"):
            assert cols(r[0]) == cols(w[0]), q
        else:
            assert r == w, q


def test_incremental_shard_updates(envs):
    """Writes to a few shards patch the device arena in place (no full
    re-upload), including writes that create new row ids."""
    cpu, gpu = envs
    cpu.executor.gpu = gpu
    try:
        q = "Count(Intersect(Row(g=1), Row(f=0)))"
        cpu.q1("i", q)
        r0, u0 = gpu.rebuilds, gpu.shard_updates
        for k in range(20):
            cpu.q("i", f"Set({(k % 4) * SW + 777 + k}, g=1) Set({(k % 4) * SW + 777 + k}, f=0)")
            got = cpu.q1("i", q)
            cpu.executor.gpu = None
            want = cpu.q1("i", q)
            cpu.executor.gpu = gpu
            assert got == want
        assert gpu.rebuilds == r0, "writes to existing rows must not re-upload the view"
        assert gpu.shard_updates > u0
        # new row ids are inserted into the dense directory in place (no rebuild),
        # in the middle (g=3 < 4321 < ...) and past the end of the directory
        for rid, col in ((4321, 2 * SW + 5), (3, 3 * SW + 99), (2, 17), (99999, SW + 1)):
            cpu.q("i", f"Set({col}, g={rid})")
            for qq in (f"Count(Row(g={rid}))", "Count(Intersect(Row(g=1), Row(f=0)))", "Count(Row(g=2))",
                       "Count(Union(Row(g=3), Row(g=4321)))"):
                got = cpu.q1("i", qq)
                cpu.executor.gpu = None
                want = cpu.q1("i", qq)
                cpu.executor.gpu = gpu
                assert got == want, qq
        got = cpu.q1("i", "Rows(g)")
        cpu.executor.gpu = None
        want = cpu.q1("i", "Rows(g)")
        cpu.executor.gpu = gpu
        assert got == want
        assert gpu.rebuilds == r0, "a new row id must patch the directory, not re-upload the view"
    finally:
        cpu.executor.gpu = None


def test_hbm_budget_lru_eviction(envs):
    """gpu.hbm-budget: least recently used view arenas are dropped and
    rebuilt on demand; results stay exact."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    cpu, gpu = envs
    small = GpuExecutor(cpu.holder, "cuda:0", executor=cpu.executor, hbm_budget=1)
    qs = ["Count(Row(f=1))", "Count(Row(g=1))", "Count(Row(h=3))", "Count(Row(f=2))", "Count(Row(g=2))"]
    want = [cpu.q1("i", q) for q in qs]
    cpu.executor.gpu = small
    try:
        got = [cpu.q1("i", q) for q in qs]
    finally:
        cpu.executor.gpu = None
    assert got == want
    st = small.stats()
    assert st["evictions"] >= 3 and st["arenas"] == 1
    assert sum(st["containers"].values()) > 0


@pytest.mark.parametrize("k,hot", [(5000, 0), (5000, 37), (5000, None), (100, 0), (100, 64), (100, 100), (7, 3)])
def test_slot_index_topn_matches_replay(envs, k, hot):
    """Hot-rank count matrix + column-major slot index + LDS-histogram heap
    walk (ops/topn_index.py) == the exact host replay over the same device
    rank cache, for every split of the cache ranks between the two (hot=0:
    histogram only, hot=k: row-major only); small caches exercise the ids
    outside a shard's cache (in-kernel exact probe)."""
    from pilosa_amd.ops.topn import DeviceRankCache, topn_batch
    from pilosa_amd.ops.topn_index import DeviceTopNIndex
    from pilosa_amd.pql import parse_string
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    hv = gpu.view_arena("i", "h", "standard", shards)
    cache = DeviceRankCache.from_view(hv, k=k)
    idx = DeviceTopNIndex(hv, cache, hot=hot)
    assert idx.ok and (idx.entries > 0 or idx.R >= min(k, cache.rows.shape[1]))
    cases = ["Row(f=2)", "Row(f=3)", "Row(g=1)", "Row(f=0)", "Row(h=0)", "Intersect(Row(f=0), Row(g=2))",
             "Union(Row(f=20), Row(f=1))"]
    srcs = [gpu.plan("i", parse_string(q).calls[0], shards) for q in cases]
    for n, th in ((5, 1), (50, 1), (1000, 1), (20, 40), (0, 1)):
        got = idx.topn(gpu.engine, srcs, [n] * len(srcs), [th] * len(srcs))
        want = topn_batch(gpu.engine, hv, cache, srcs, n=n, threshold=th)
        for q, g, w in zip(cases, got, want):
            assert [(p.id, p.count) for p in g] == [(p.id, p.count) for p in w], (q, n, th, k)
        if k == 5000 and th == 1 and n:
            for q, g in zip(cases, got):
                want = cpu.q1("i", f"TopN(h, {q}, n={n})")
                assert [(p.id, p.count) for p in g] == [(p.id, p.count) for p in want], (q, n)


@pytest.mark.parametrize("hot", [None, 64])
def test_slot_index_topn_32_query_launch(envs, hot, monkeypatch):
    """17..32 srcs per launch take topn_hot_kernel<32> (u32 masks of half a
    key per workgroup): its hot counts equal two 16-query launches', and the
    TopN answers equal the exact replay."""
    import torch

    from pilosa_amd.ops import topn_index
    from pilosa_amd.ops.topn import DeviceRankCache, topn_batch
    monkeypatch.setattr(topn_index, "HOT_Q", 32)
    from pilosa_amd.ops.topn_index import DeviceTopNIndex
    from pilosa_amd.pql import parse_string
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    hv = gpu.view_arena("i", "h", "standard", shards)
    cache = DeviceRankCache.from_view(hv, k=5000)
    idx = DeviceTopNIndex(hv, cache, hot=hot)
    cases = ["Row(f=2)", "Row(f=3)", "Row(g=1)", "Row(f=0)", "Row(h=0)", "Intersect(Row(f=0), Row(g=2))",
             "Union(Row(f=20), Row(f=1))", "Row(h=1)", "Row(h=2)", "Row(g=0)"] * 3
    srcs = [gpu.plan("i", parse_string(q).calls[0], shards) for q in cases]
    assert 16 < len(srcs) <= 32
    src = idx.materialize(gpu.engine, srcs)
    h32 = idx.hot_counts(src, len(srcs)).view(idx.S, len(srcs), idx.R)
    for lo, hi in ((0, 16), (16, len(srcs))):
        sub = idx.materialize(gpu.engine, srcs[lo:hi])
        h16 = idx.hot_counts(sub, hi - lo).view(idx.S, hi - lo, idx.R)
        assert torch.equal(h32[:, lo:hi], h16), (lo, hi)
    for n, th in ((5, 1), (100, 1), (20, 40)):
        got = idx.topn(gpu.engine, srcs, [n] * len(srcs), [th] * len(srcs))
        want = topn_batch(gpu.engine, hv, cache, srcs, n=n, threshold=th)
        for q, g, w in zip(cases, got, want):
            assert [(p.id, p.count) for p in g] == [(p.id, p.count) for p in w], (q, n, th)


def test_topn_nosrc_matches_cache_replay(envs):
    """Ranked-cache TopN(field, n) batches on the device (sorted unique
    candidate keys, device ids= re-count, device finish) == the per-query
    host replay of the same device rank caches, mixed n and thresholds."""
    from pilosa_amd.ops.topn import DeviceRankCache, finish_topn, topn_cache_phase1, topn_cache_phase2_counts
    from pilosa_amd.ops.topn_index import DeviceTopNIndex
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    hv = gpu.view_arena("i", "h", "standard", shards)
    for k in (5000, 7):
        cache = DeviceRankCache.from_view(hv, k=k, keep_row_counts=True)
        idx = DeviceTopNIndex(hv, cache)
        ns = [5, 100, 0, 1, 20, 3000]
        ths = [1, 1, 1, 1, 40, 2]
        got = idx.topn_nosrc(cache.row_counts, ns, ths)
        for n, th, g in zip(ns, ths, got):
            ids = sorted(topn_cache_phase1(cache, n, th))
            want = finish_topn(ids, topn_cache_phase2_counts(cache, hv, ids, th), n)
            assert [(p.id, p.count) for p in g] == [(p.id, p.count) for p in want], (k, n, th)


def test_concurrent_counts_coalesce_on_gpu(envs):
    """Independent concurrent Count() requests share GPU launches
    (ops/coalescer.py) and each gets exactly its host result."""
    import threading
    cpu, gpu = envs
    qs = [QUERIES[i % len(QUERIES)] for i in range(96)]
    want = [cpu.q1("i", q) for q in qs]
    got = [None] * len(qs)
    cpu.executor.gpu = gpu
    try:
        co = cpu.executor.coalescer
        b0, n0 = co.batches, co.batched + co.fallbacks

        def work(i):
            got[i] = cpu.q1("i", qs[i])

        ts = [threading.Thread(target=work, args=(i,)) for i in range(len(qs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=60)
        assert co.batched + co.fallbacks - n0 == len(qs)
        assert co.batches - b0 <= len(qs)
    finally:
        cpu.executor.gpu = None
    assert got == want


def test_native_count_batch_path(envs):
    """Batches of plain Row/set-op counts take the native-compiler fast path
    (GpuExecutor._count_batch_native) and match the host."""
    cpu, gpu = envs
    qs = ["Count(Row(f=0))", "Count(Intersect(Row(f=0), Row(f=1)))", "Count(Union(Row(f=1), Row(g=2), Row(f=20)))",
          "Count(Difference(Row(f=20), Row(f=0)))", "Count(Xor(Row(f=4), Row(g=0)))", "Count(Row(f=999))",
          "Count(Intersect(Row(f=0), Row(f=999)))", "Count(Row(h=3))"]
    want = cpu.q("i", " ".join(qs))
    from pilosa_amd.pql import parse_string
    calls = [parse_string(q).calls[0] for q in qs]
    shards = cpu.holder.index("i").available_shards()
    got = gpu._count_batch_native("i", calls, shards)
    assert got == want


@pytest.mark.parametrize("q", ["GroupBy(Rows(g), Rows(f))", "GroupBy(Rows(f), Rows(g), limit=7)",
                               "GroupBy(Rows(f), Rows(h), limit=50)",
                               "GroupBy(Rows(f, previous=3), Rows(g, previous=1), limit=10)",
                               "GroupBy(Rows(g), Rows(f), filter=Row(f=0))",
                               "GroupBy(Rows(f), Rows(g), previous=[2, 2], limit=5)"])
def test_groupby_count_matrix_matches_host(envs, monkeypatch, q):
    """Two-field GroupBy through the bit-GEMM count matrix (ops/groupby.py)."""
    import pilosa_amd.ops.gpu_executor as ge
    cpu, gpu = envs
    monkeypatch.setattr(ge, "GROUPBY_MATRIX_MIN", 1)
    want = cpu.q1("i", q)
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q1("i", q)
        assert gpu.launches > n0
    finally:
        cpu.executor.gpu = None
    assert got == want


def test_paranoia_cross_check_on_device(envs):
    """PILOSA_PARANOIA: every device result is re-derived on the host; the
    whole query mix must pass the cross-check."""
    cpu, gpu = envs
    cpu.executor.gpu = gpu
    cpu.executor.paranoia = True
    cpu.executor.coalesce = False
    try:
        for q in QUERIES + ["Row(f=2)", "Not(Row(f=0))", "TopN(h, Row(f=2), n=5)", "Sum(Row(f=0), field=n)"]:
            cpu.q1("i", q)
    finally:
        cpu.executor.paranoia = False
        cpu.executor.coalesce = True
        cpu.executor.gpu = None


SHIFT_QUERIES = [
    "Count(Shift(Row(f=0), n=1))", "Shift(Row(f=20), n=5)", "Count(Intersect(Shift(Row(f=0), n=3), Row(f=1)))",
    "Count(Not(Shift(Row(f=2), n=100)))", "Difference(Shift(Row(f=1), n=129), Row(f=0))",
    "Union(Shift(Row(f=0), n=64), Shift(Row(f=1), n=7))", "Shift(Row(f=3), n=0)",
    # shifts relative to the shard width (every width runs them on the device,
    # narrow 2^16 / 2^18 shards included: their spill starts at 2^e columns)
    f"Count(Union(Shift(Row(f=1), n={SW // 2 + 4464}), Row(g=1)))", f"Shift(Row(f=0), n={SW // 16})",
    f"Xor(Shift(Row(f=2), n={SW - 48576}), Row(f=3))", f"Count(Shift(Intersect(Row(f=0), Row(f=1)), n={SW - 1}))",
    # nested shifts (one spill level while the total stays below the width)
    "Shift(Shift(Row(f=0), n=5), n=7)", f"Count(Shift(Shift(Row(f=1), n={SW - 300}), n=200))",
    "Union(Shift(Shift(Row(f=2), n=100), n=65000), Row(g=1))",
    f"Count(Intersect(Shift(Shift(Row(f=0), n=3), n={SW // 4}), Row(f=1)))",
    "Shift(Union(Shift(Row(f=1), n=9), Row(f=3)), n=11)",
]
if SW > (1 << 21):
    # wide shards (PILOSA_SHARD_WIDTH=22): carries across 1..3 device sub-shards
    SHIFT_QUERIES += ["Shift(Row(f=20), n=1048576)", "Count(Shift(Row(f=0), n=3000000))",
                      "Xor(Shift(Row(f=1), n=2097153), Row(f=0))", "Shift(Row(f=3), n=4194303)"]


@pytest.mark.parametrize("q", SHIFT_QUERIES)
def test_shift_on_device_matches_host(envs, q):
    """Shift(row, n) through expr_dense + shift_dense (row_kernels.hip),
    including the bits each shard carries into the next shard's segment, at
    every shard width, nested shifts included."""
    cpu, gpu = envs
    want = cpu.q1("i", q)
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q1("i", q)
        assert gpu.launches > n0  # no silent host fallback
    finally:
        cpu.executor.gpu = None
    if hasattr(want, "columns"):
        assert cols(got) == cols(want)
    else:
        assert got == want


@pytest.mark.parametrize("q", ["Rows(f)", "Rows(g)", "Rows(f, previous=3)", "Rows(f, limit=4)",
                               "Rows(f, column=1234567)", "Rows(f, column=100000)", "Rows(h, limit=50)",
                               "Rows(t, from=2020-03-01T00:00, to=2020-06-01T00:00)", "Rows(f, column=4194303)",
                               "Rows(g, previous=1, limit=2)"])
def test_rows_listing_on_device_matches_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q1("i", q)
        assert gpu.launches > n0
    finally:
        cpu.executor.gpu = None
    assert got == want


@pytest.mark.parametrize("q", ["MinRow(field=f)", "MaxRow(field=f)", "MinRow(Row(g=1), field=f)",
                               "MaxRow(Row(g=2), field=f)", "MinRow(Intersect(Row(f=20), Row(g=1)), field=h)",
                               "MaxRow(Row(f=999), field=f)", "MaxRow(field=h)", "MinRow(Row(f=11), field=h)",
                               "MaxRow(Union(Row(f=3), Row(g=4)), field=h)", "MinRow(Shift(Row(f=2), n=9), field=f)"])
def test_minmax_row_on_device_matches_host(envs, q):
    cpu, gpu = envs
    want = cpu.q1("i", q)
    cpu.executor.gpu = gpu
    try:
        n0 = gpu.launches
        got = cpu.q1("i", q)
        assert "999" in q or gpu.launches > n0  # no silent host fallback
    finally:
        cpu.executor.gpu = None
    assert got == want


def test_count_text_fast_path_matches_host(envs):
    """A request of many Count() calls is compiled from its PQL text natively
    (Executor._count_text_fast -> GpuExecutor.try_count_text) in one launch."""
    cpu, gpu = envs
    qs = ["Count(Row(f=0))", "Count(Intersect(Row(f=0), Row(f=1)))", "Count(Union(Row(f=1), Row(g=2), Row(f=20)))",
          "Count(Difference(Row(f=20), Row(f=0)))", "Count(Xor(Row(f=4), Row(g=0)))", "Count(Row(f=999))",
          "Count(Intersect(Row(f=0), Row(f=999)))", "Count( Intersect( Row(f=2) ,Row(g=1) ) )"]
    text = "\n".join(qs)
    want = cpu.q("i", text)
    got = _dev(cpu, gpu, lambda: cpu.q("i", text))
    assert got == want
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    shards = cpu.holder.index("i").available_shards()
    assert gpu.try_count_text("i", text, shards) == want
    # outside the native subset: None (the general path answers)
    assert gpu.try_count_text("i", "Count(Row(f=1)) Count(Row(n > 5))", shards) is None
    assert gpu.try_count_text("i", "Count(Row(f=1)) TopN(f)", shards) is None


@pytest.mark.parametrize("q", ["GroupBy(Rows(g), Rows(f), Rows(h), limit=60)",
                               "GroupBy(Rows(f), Rows(g), Rows(h), filter=Row(f=1), limit=25)",
                               "GroupBy(Rows(g), Rows(f), Rows(g), previous=[1, 3, 2], limit=10)",
                               "GroupBy(Rows(f), Rows(g), Rows(f), Rows(h), limit=40)"])
def test_groupby_pruned_k3_matches_host(envs, q):
    """k >= 3 GroupBy: cumulative-intersection pruning on the device
    (GpuExecutor._pruned_groups) == host groupByIterator semantics."""
    cpu, gpu = envs
    want = cpu.q1("i", q)
    got = _dev(cpu, gpu, lambda: cpu.q1("i", q))
    assert got == want


def test_groupby_two_million_row_fields_limit():
    """GroupBy over two 1M-row fields with limit=100 answers without
    densifying 2M rows or allocating a 10^12-cell matrix (HBM guard ->
    pruned walk), and matches the diagonal it was built from."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    from tests.helpers import Env
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "a")
        env.field("i", "b")
        n = 1_000_000
        rows = np.arange(n, dtype=np.uint64)
        cols = (rows * np.uint64(3)) % np.uint64(4 << 20)   # no two rows share a column (any shard width)
        idx = env.holder.index("i")
        idx.field("a").import_bits(rows, cols)
        idx.field("b").import_bits(rows, cols)
        gpu = GpuExecutor(env.holder, "cuda:0", executor=env.executor)
        env.executor.gpu = gpu
        got = env.q1("i", "GroupBy(Rows(a), Rows(b), limit=100)")
        assert [(g.group[0].row_id, g.group[1].row_id, g.count) for g in got] == [(r, r, 1) for r in range(100)]
        assert not gpu._matrix_fits(n, n)
    finally:
        env.executor.gpu = None
        env.close()


@pytest.mark.parametrize("mode", [0, 2, 3, 4])
def test_bsi_sum_matrix_matches_per_filter_kernel(envs, mode):
    """Batched Sum as the bit-plane count matrix (ops/bsi.py, bitgemm VALU
    and MFMA modes) == the per-filter bsi_sum kernel == the host executor."""
    from pilosa_amd.ops.bsi import bsi_sum_matrix
    from pilosa_amd.pql import parse_string
    cpu, gpu = envs
    shards = cpu.holder.index("i").available_shards()
    bv = gpu.view_arena("i", "n", "bsig_n", shards)
    depth = cpu.holder.index("i").field("n").bsi_group("n").bit_depth
    qs = ["Row(f=0)", "Row(f=1)", "Row(g=2)", "Intersect(Row(f=0), Row(g=1))", None, "Row(f=999)",
          "Union(Row(f=2), Row(f=20))", "Not(Row(f=3))"] * 3
    filters = [None if q is None else gpu.plan("i", parse_string(q).calls[0], shards) for q in qs]
    s0, n0 = gpu.engine.bsi_sum_async(filters, bv, depth, matrix=False)
    s1, n1 = bsi_sum_matrix(gpu.engine, filters, bv, depth, mode=mode)
    assert s0.cpu().tolist() == s1.cpu().tolist() and n0.cpu().tolist() == n1.cpu().tolist()
    base = cpu.holder.index("i").field("n").bsi_group("n").base
    for q, s, n in list(zip(qs, s1.cpu().tolist(), n1.cpu().tolist()))[:8]:
        want = cpu.q1("i", f"Sum({q}, field=n)" if q else "Sum(field=n)")
        assert (want.val, want.count) == (s + n * base, n), q


def test_time_range_count_batches_match_host():
    """Count(Row(t=r, from=, to=)) calls sharing a range go through the
    vectorised union programs (GpuExecutor._count_time_rows, one launch per
    range group) and equal the host executor; mixed with other calls and
    ranges covering no view."""
    import datetime as dt

    from pilosa_amd.ops.gpu_executor import GpuExecutor
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "t", type="time", time_quantum="YMDH")
        env.field("i", "f")
        rng = np.random.default_rng(5)
        t = env.holder.index("i").field("t")
        rows, cs, ts = [], [], []
        for r in range(40):
            k = int(rng.integers(1, 3000))
            cc = rng.choice(3 * SW, size=k, replace=False)
            rows += [r] * k
            cs += cc.tolist()
            ts += [dt.datetime(2021, 1 + int(x % 3), 1 + int(x % 28), int(x % 24)) for x in cc]
        t.import_bits(np.array(rows, np.uint64), np.array(cs, np.uint64), timestamps=ts)
        env.holder.index("i").field("f").import_bits(np.zeros(100, np.uint64), np.arange(100, dtype=np.uint64))
        ranges = [("2021-01-03T05:00", "2021-02-11T13:00"), ("2021-01-01T00:00", "2021-04-01T00:00"),
                  ("2021-02-27T22:00", "2021-03-02T02:00"), ("2019-01-01T00:00", "2019-02-01T00:00")]
        q = " ".join(f"Count(Row(t={r}, from={a}, to={b}))" for a, b in ranges for r in list(range(0, 44, 3)))
        q += " Count(Row(f=0)) Count(Row(t=7, from=2021-01-05T00:00, to=2021-01-06T00:00))"
        want = env.q("i", q)
        gpu = GpuExecutor(env.holder, "cuda:0", executor=env.executor)
        env.executor.gpu = gpu
        try:
            n0 = gpu.launches
            got = env.q("i", q)
            assert gpu.launches > n0
        finally:
            env.executor.gpu = None
        assert got == want
        assert sum(want) > 0
    finally:
        env.close()


@pytest.mark.parametrize("q", ["TopN(h, Row(h=3), tanimotoThreshold=10)", "TopN(h, Row(f=1), n=5, tanimotoThreshold=1)",
                               "TopN(h, Row(h=7), n=20, tanimotoThreshold=60)",
                               'TopN(h, Row(f=0), n=8, attrName="cat", attrValues=[1, 3])',
                               'TopN(h, n=6, attrName="cat", attrValues=[2])',
                               'TopN(h, Row(f=2), ids=[1, 2, 3, 4, 5, 6], attrName="cat", attrValues=[1])'])
def test_topn_tanimoto_and_attr_filters_on_device(envs, q):
    """fragment.top's Tanimoto window and attribute filter (fragment.go:
    1586-1650) on the device path: counts on the GPU, the heap walk with both
    filters replayed exactly."""
    cpu, gpu = envs
    if not getattr(test_topn_tanimoto_and_attr_filters_on_device, "_attrs", False):
        for rid in range(40):
            cpu.q("i", f"SetRowAttrs(h, {rid}, cat={1 + rid % 3})")
        test_topn_tanimoto_and_attr_filters_on_device._attrs = True
    want = cpu.q1("i", q)
    got = _dev(cpu, gpu, lambda: cpu.q1("i", q))
    assert [(p.id, p.count) for p in got] == [(p.id, p.count) for p in want]

