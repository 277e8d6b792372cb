"""Fragment files -> device arena without host Bitmaps (native/arena_io.cpp,
ops/loader.py), checked on the CPU against the Bitmap-based arena builder:
plain snapshots, run containers, op logs after the snapshot (replayed), lazy
holders whose cold views load from the files, and writes after such a load
patching the arena (reference open path: fragment.go:311-456,
roaring/roaring.go:1562-1653)."""
import os

import numpy as np
import pytest

from pilosa_amd import _roaring
from tests.helpers import SW, Env
from tests.test_arena_patch import _decode

SHARDS = [0, 1, 2, 5]


def _populate(env):
    env.create_index("i")
    env.field("i", "g")
    f = env.holder.index("i").field("g")
    rng = np.random.default_rng(7)
    for r in range(8):
        k = [30000, 200, 5, 120000][r % 4]
        c = rng.choice(6 * SW, k, replace=False).astype(np.uint64)
        c = c[np.isin(c >> np.uint64(20), SHARDS)]
        f.import_bits(np.full(len(c), r * 3 + 1, np.uint64), c)
    f.import_bits(np.full(90000, 40, np.uint64), np.arange(100, 90100, dtype=np.uint64))  # runs
    f.import_bits(np.full(70000, 41, np.uint64), 5 * SW + np.arange(0, 140000, 2, dtype=np.uint64))
    return f


def _frags(env, shards=SHARDS):
    v = env.holder.view("i", "g", "standard")
    return [v.fragment(s) for s in shards]


def test_loader_matches_bitmap_arena_builder():
    from pilosa_amd.ops.loader import load_view
    env = Env()
    try:
        _populate(env)
        frags = _frags(env)
        for fr in frags:
            fr.snapshot()
        # an op log after the snapshot on one shard (replayed by the loader)
        env.q("i", f"Set({SW + 77}, g=999) Set({SW + 78}, g=4) Clear({SW + 78}, g=4) Set(5, g=1)")
        paths = [fr.path for fr in frags]
        with open(paths[1], "rb") as fh:
            data = fh.read()
        bms = [_roaring.Bitmap.from_bytes(open(p, "rb").read()) for p in paths]
        assert len(data) > len(bms[1].to_bytes())  # really has an op log
        want = _roaring.build_arena(bms, 16, 4)
        info = {}
        dv = load_view(paths, SHARDS, "cpu", patchable=False, stats=info)
        assert info["replayed_shards"] >= 1
        rows, rowptr, sb, meta, payload = want
        assert dv.rows.tolist() == rows.tolist()
        assert (dv.t_rowptr.numpy().view(np.uint32).reshape(len(SHARDS), -1) == rowptr).all()
        assert dv.t_shard_base.numpy().tolist() == sb.tolist()
        assert (dv.t_meta.numpy()[:int(sb[-1])] == meta[:int(sb[-1])]).all()
        P = int(payload.shape[0])
        assert (dv.t_payload.numpy().view(np.uint16)[:P] == payload).all()
        # patchable layout: every shard decodes to its file's bitmap
        dv2 = load_view(paths, SHARDS, "cpu", patchable=True)
        assert dv2._cap is not None and (dv2._cap >= np.diff(sb)).all()
        for si in range(len(SHARDS)):
            assert _decode(dv2, si) == bms[si].slice().astype(np.int64).tolist()
    finally:
        env.close()


def test_zipf_fragment_writer_matches_generator(tmp_path):
    cols, rows = 3 * SW + 12345, 3000
    d = str(tmp_path)
    out = _roaring.write_zipf_fragments(d, 0, 4, cols, rows, 8.0, 1.6, 50.0, 3, 4)
    assert out["shards"] == 4 and out["containers"] > 0
    arena = _roaring.gen_zipf_arena(0, 4, cols, rows, 8.0, 1.6, 50.0, 3, 4)
    total = 0
    for s in range(4):
        p = os.path.join(d, str(s))
        total += os.path.getsize(p)
        got = _roaring.Bitmap.from_bytes(open(p, "rb").read())
        assert got.equals(_roaring.arena_shard_bitmap(*arena, s)), s
    assert total == out["bytes"]


def test_lazy_holder_cold_view_loads_from_files():
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    env = Env()
    try:
        _populate(env)
        want = {s: fr.storage.slice().astype(np.int64).tolist() for s, fr in zip(SHARDS, _frags(env))}
        q = "Count(Intersect(Row(g=1), Row(g=4))) Count(Row(g=40)) TopN(g, n=3)"
        want_q = env.q("i", q)
        env.holder.close()
        env.holder = Holder(env.dir, lazy_fragments=True).open()
        env.executor.holder = env.holder
        frags = _frags(env)
        assert all(fr.is_cold() for fr in frags)
        g = GpuExecutor(env.holder, "cpu")
        dv = g.view_arena("i", "g", "standard", SHARDS)
        assert g.cold_loads == 1 and g.last_load["files"] == len(SHARDS)
        assert all(fr.is_cold() for fr in frags), "loading the arena must not read host storage"
        for si, s in enumerate(SHARDS):
            assert _decode(dv, si) == want[s]
        # host queries load the storage (and the rank cache) on first use
        assert env.q("i", q) == want_q
        assert not any(fr.is_cold() for fr in frags)
        # writes after the file load patch the arena in place
        env.q("i", f"Set({2 * SW + 9}, g=1) Set({5 * SW + 3}, g=12345)")
        dv = g.view_arena("i", "g", "standard", SHARDS)
        assert g.rebuilds == 1 and g.cold_loads == 1 and g.shard_updates >= 2
        for si, fr in enumerate(frags):
            assert _decode(dv, si) == fr.storage.slice().astype(np.int64).tolist()
    finally:
        env.close()


def test_lazy_fragment_close_keeps_files_and_cache():
    from pilosa_amd.models.holder import Holder
    env = Env()
    try:
        _populate(env)
        frags = _frags(env)
        env.holder.close()  # drains the snapshot queue, flushes caches
        sizes = [os.path.getsize(fr.path) for fr in frags]
        caches = [open(fr.cache_path(), "rb").read() for fr in frags]
        env.holder = Holder(env.dir, lazy_fragments=True).open()
        env.holder.flush_caches()
        env.holder.close()
        assert [os.path.getsize(fr.path) for fr in frags] == sizes
        assert [open(fr.cache_path(), "rb").read() for fr in frags] == caches
        env.holder = Holder(env.dir, lazy_fragments=True).open()
        env.executor.holder = env.holder
        fr = _frags(env)[0]
        assert fr.is_cold()
        # the cache opens from the mmapped file (fragment.go openCache): still cold
        assert fr.cache.ids() and fr.is_cold() and fr.mapped_stats() is not None
    finally:
        env.close()


def test_loader_rejects_corrupt_file(tmp_path):
    from pilosa_amd.ops.loader import load_view
    p = tmp_path / "0"
    bm = _roaring.Bitmap(np.arange(0, 5000, 3, dtype=np.uint64))
    data = bytearray(bm.to_bytes())
    data[4:8] = (10 ** 6).to_bytes(4, "little")  # key count past the end of the file
    p.write_bytes(bytes(data))
    with pytest.raises(RuntimeError, match="key-cardinality"):
        load_view([str(p)], [0], "cpu", patchable=False)
