"""Device write path (K11 AddN/RemoveN, K12 ImportRoaringBits on the GPU,
kernels/write_kernels.hip): after set / clear / roaring-import batches are
merged into the HBM arena by container_merge + container_emit, the arena
decodes to exactly the host roaring result (C++ CPU oracle)."""
import numpy as np
import pytest

from pilosa_amd import _roaring as R
from tests.helpers import SW, Env
from tests.test_arena_patch import _decode
from tests.test_gpu_kernels import _random_fragment

pytestmark = pytest.mark.gpu


@pytest.fixture
def view():
    import torch
    from pilosa_amd.ops.device import DeviceView
    rng = np.random.default_rng(11)
    # shard 1 holds every container flavour, shards 0 and 2 must stay untouched
    frags = [_random_fragment(rng, nrows=6, shard=0) for _ in range(3)]
    dv = DeviceView.from_bitmaps(frags, torch.device("cuda:0"), shards=[0, 1, 2], patchable=True)
    return dv, frags, rng


def _check(dv, host):
    for si, h in enumerate(host):
        assert _decode(dv, si) == h.slice().astype(np.int64).tolist(), f"shard {si}"


def test_set_positions_every_container_kind(view):
    dv, host, rng = view
    pos = np.concatenate([
        rng.integers(0, 6 * SW, 20000),                       # into existing rows
        np.uint64(3) * np.uint64(SW) + np.arange(5000, dtype=np.uint64),   # array -> bitmap conversions
        np.uint64(9) * np.uint64(SW) + rng.integers(0, SW, 300),            # a brand-new row
        np.uint64(7) * np.uint64(SW) + np.arange(65536, dtype=np.uint64),   # a full container
    ]).astype(np.uint64)
    assert dv.apply_positions(1, pos, clear=False)
    host[1].add_many(np.unique(pos), True)
    assert 9 in dv.rows.tolist()
    _check(dv, host)


def test_clear_positions_removes_emptied_containers(view):
    dv, host, rng = view
    everything = host[1].slice()
    key0 = everything[(everything >> np.uint64(16)) == (everything[0] >> np.uint64(16))]
    pos = np.concatenate([key0, rng.choice(everything, 5000, replace=False),
                          np.uint64(11) * np.uint64(SW) + np.arange(10, dtype=np.uint64)])  # absent row: no-op
    n_before = int(dv._rowptr_host[1][-1])
    assert dv.apply_positions(1, pos, clear=True)
    host[1].remove_many(np.unique(pos))
    assert int(dv._rowptr_host[1][-1]) < n_before
    _check(dv, host)


def test_point_writes_and_mixed_batches(view):
    dv, host, rng = view
    for k in range(40):
        p = np.array([int(rng.integers(0, 8 * SW))], np.uint64)
        clear = bool(k % 3 == 0)
        assert dv.apply_deltas(1, [("pos", p, clear)])
        (host[1].remove_many if clear else host[1].add_many)(*((p,) if clear else (p, True)))
    deltas = [("pos", rng.integers(0, 6 * SW, 500).astype(np.uint64), False),
              ("pos", rng.integers(0, 6 * SW, 500).astype(np.uint64), False),
              ("pos", rng.integers(0, 6 * SW, 800).astype(np.uint64), True)]
    assert dv.apply_deltas(1, deltas)
    for kind, p, clear in deltas:
        if clear:
            host[1].remove_many(np.unique(p))
        else:
            host[1].add_many(np.unique(p), True)
    _check(dv, host)


def test_import_roaring_containers(view):
    dv, host, rng = view
    src = _random_fragment(rng, nrows=8, shard=0)      # arrays, bitmaps and runs
    assert dv.apply_bitmap(1, src, clear=False)
    host[1] = R.Bitmap(np.union1d(host[1].slice(), src.slice()))
    _check(dv, host)
    cut = _random_fragment(rng, nrows=5, shard=0)
    assert dv.apply_bitmap(1, cut, clear=True)
    host[1] = R.Bitmap(np.setdiff1d(host[1].slice(), cut.slice()))
    _check(dv, host)


def test_executor_writes_merge_on_device():
    """Set/Clear queries, bulk imports and roaring imports against a GPU-
    resident view are replayed by the write kernels (no rebuild, no host
    container rebuild) and every shard still decodes to its fragment."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    shards = [0, 1, 2, 3]
    env = Env(gpu=lambda h: GpuExecutor(h, "cuda:0"))
    try:
        env.create_index("i")
        env.field("i", "g")
        f = env.holder.index("i").field("g")
        rng = np.random.default_rng(3)
        for r in range(6):
            c = rng.choice(4 * SW, 40000, replace=False).astype(np.uint64)
            f.import_bits(np.full(len(c), r, np.uint64), c)
        g = env.executor.gpu
        g.executor = env.executor
        g.view_arena("i", "g", "standard", shards)
        for k in range(60):
            c, r = int(rng.integers(0, 4 * SW)), int(rng.integers(0, 8))
            env.q("i", f"Set({c}, g={r})" if k % 3 else f"Clear({c}, g={r})")
            if k % 9 == 0:
                f.import_bits(np.full(3000, r, np.uint64), rng.integers(0, 4 * SW, 3000).astype(np.uint64))
            if k % 20 == 19:
                frag = env.holder.fragment("i", "g", "standard", 2)
                rb = R.Bitmap(np.uint64(r) * np.uint64(SW) + rng.integers(0, SW, 5000).astype(np.uint64))
                frag.import_roaring(rb.to_bytes(), clear=bool(k % 40 == 39))
            dv = g.view_arena("i", "g", "standard", shards)
        assert g.rebuilds == 1 and g.device_writes > 50
        for si, s in enumerate(shards):
            frag = env.holder.fragment("i", "g", "standard", s)
            assert _decode(dv, si) == frag.storage.slice().astype(np.int64).tolist()
        # and queries through the device agree with the host
        before = g.launches

        def cols(s, r):
            v = env.holder.fragment("i", "g", "standard", s).storage.slice()
            return v[(v >> np.uint64(20)) == np.uint64(r)] & np.uint64(SW - 1)
        for r in range(7):
            got = env.q("i", f"Count(Intersect(Row(g={r}), Row(g={r + 1})))")[0]
            want = sum(len(np.intersect1d(cols(s, r), cols(s, r + 1))) for s in shards)
            assert got == want
        assert g.launches > before and g.rebuilds == 1
    finally:
        env.close()


def test_row_rebuilds_after_recorded_batches():
    """Set -> ClearRow and Set -> Store between two device reads: the recorded
    position batches are replayed BEFORE the storage-described row rebuilds,
    so the device never re-applies a set on top of the cleared/stored row
    (gpu_executor refresh order)."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    shards = [0, 1]
    env = Env(gpu=lambda h: GpuExecutor(h, "cuda:0"))
    try:
        env.create_index("i")
        env.field("i", "g")
        f = env.holder.index("i").field("g")
        rng = np.random.default_rng(5)
        for r in range(4):
            c = rng.choice(2 * SW, 5000, replace=False).astype(np.uint64)
            f.import_bits(np.full(len(c), r, np.uint64), c)
        g = env.executor.gpu
        g.executor = env.executor
        env.executor.strict_gpu = True
        assert env.q("i", "Count(Row(g=1))")[0] > 0

        def host_count(r):
            return sum(int(env.holder.fragment("i", "g", "standard", s).storage.count_range(r * SW, (r + 1) * SW))
                       for s in shards)
        env.q("i", f"Set({SW + 17}, g=1)")
        env.q("i", "ClearRow(g=1)")
        assert env.q("i", "Count(Row(g=1))")[0] == host_count(1) == 0
        env.q("i", f"Set({SW + 99}, g=2)")
        env.q("i", f"Set(5, g=3)")
        env.q("i", "Store(Row(g=0), g=2)")
        assert env.q("i", "Count(Row(g=2))")[0] == host_count(2) == host_count(0)
        assert env.q("i", "Count(Row(g=3))")[0] == host_count(3)
        env.q("i", f"Set(7, g=1)")
        assert env.q("i", "Count(Row(g=1))")[0] == host_count(1) == 1
        assert g.rebuilds == 1
    finally:
        env.close()


def test_compaction_on_device(view):
    dv, host, rng = view
    for k in range(6):
        p = rng.integers(0, 6 * SW, 30000).astype(np.uint64)
        assert dv.apply_positions(k % 3, p, clear=bool(k % 2))
        if k % 2:
            host[k % 3].remove_many(np.unique(p))
        else:
            host[k % 3].add_many(np.unique(p), True)
    before = dv.payload_used
    assert dv.garbage_u16 > 0
    assert dv.compact()
    assert dv.payload_used < before and dv.garbage_u16 == 0
    _check(dv, host)
    # and writes keep working on the compacted buffer
    p = rng.integers(0, 6 * SW, 5000).astype(np.uint64)
    assert dv.apply_positions(2, p)
    host[2].add_many(np.unique(p), True)
    _check(dv, host)


def _types(dv, si):
    """{container key: encoding} of shard si as the arena holds it."""
    rp = dv._rowptr_host[si]
    base = int(dv._sb_host[si])
    out = {}
    for d in range(dv.D):
        row = int(dv.rows[d])
        for ci in range(base + rp[d], base + rp[d + 1]):
            m = int(dv._meta_host[ci])
            out[row * 16 + (m & 15)] = {1: "array", 2: "bitmap", 3: "run"}[(m >> 4) & 3]
    return out


def test_device_writes_emit_optimized_container_types(view):
    """K9: containers the device writes are encoded by the reference's
    Optimize rule (run / array / bitmap, roaring.go:2289-2338), exactly as the
    host roaring core optimises the same container (runs from a long range,
    arrays below 4096 bits, bitmaps at 4096 and above)."""
    dv, host, rng = view
    pos = np.concatenate([
        np.uint64(20) * np.uint64(SW) + np.arange(30000, dtype=np.uint64),                    # one long run
        np.uint64(21) * np.uint64(SW) + np.arange(0, 60000, 3, dtype=np.uint64),              # bitmap, many runs
        np.uint64(22) * np.uint64(SW) + np.sort(rng.choice(65536, 300, replace=False)).astype(np.uint64),  # array
        np.uint64(23) * np.uint64(SW) + np.arange(0, 8192, 2, dtype=np.uint64),               # exactly 4096 bits
        np.uint64(24) * np.uint64(SW) + (np.arange(2000, dtype=np.uint64) * np.uint64(32))[:, None].repeat(4, 1).ravel()
        + np.tile(np.arange(4, dtype=np.uint64), 2000),                                        # 2000 runs of 4
    ]).astype(np.uint64)
    assert dv.apply_positions(1, pos, clear=False)
    host[1].add_many(np.unique(pos), True)
    _check(dv, host)
    opt = host[1].clone()
    opt.optimize()
    want = {k: t for k, t, _ in opt.container_info()}
    got = _types(dv, 1)
    for k in (20 * 16, 21 * 16, 22 * 16, 23 * 16, 24 * 16):
        assert got[k] == want[k], (k, got[k], want[k])
    assert got[20 * 16] == "run" and got[22 * 16] == "array" and got[23 * 16] == "bitmap"


def test_device_write_replay_shares_launches_across_shards():
    """A bulk import request per shard (16 shards, as POST /import sends them)
    is replayed on the device at the next read in shared launches: one
    container_merge + container_emit pair for the whole refresh, not one per
    shard (reference fragment.go:1995-2156 imports shard by shard)."""
    from pilosa_amd.ops.gpu_executor import GpuExecutor

    shards = list(range(16))
    env = Env(gpu=lambda h: GpuExecutor(h, "cuda:0"))
    try:
        env.create_index("i")
        env.field("i", "g")
        f = env.holder.index("i").field("g")
        rng = np.random.default_rng(7)
        c = rng.choice(16 * SW, 200000, replace=False).astype(np.uint64)
        f.import_bits(rng.integers(0, 5, len(c)).astype(np.uint64), c)
        g = env.executor.gpu
        g.executor = env.executor
        g.view_arena("i", "g", "standard", shards)
        w0, l0 = g.device_writes, g.device_write_launches
        for s in shards:
            cols = np.uint64(s) * np.uint64(SW) + rng.integers(0, SW, 5000).astype(np.uint64)
            f.import_bits(rng.integers(0, 8, len(cols)).astype(np.uint64), cols)
        dv = g.view_arena("i", "g", "standard", shards)
        assert g.device_writes - w0 == 16
        assert g.device_write_launches - l0 <= 4, g.device_write_launches - l0
        for si, s in enumerate(shards):
            frag = env.holder.fragment("i", "g", "standard", s)
            assert _decode(dv, si) == frag.storage.slice().astype(np.int64).tolist()
    finally:
        env.close()
