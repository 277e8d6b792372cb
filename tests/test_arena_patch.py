"""In-place device-arena maintenance (ops/device.py DeviceView.update_rows /
update_shard, gpu_executor.view_arena) checked on the CPU: after random point
writes, clears and bulk imports the patched arena decodes to exactly the
fragment contents, without full re-uploads."""
import numpy as np

from tests.helpers import SW, Env

SHARDS = [0, 1, 2, 3]


def _decode(dv, si):
    rp = dv._rowptr_host[si]
    base = int(dv._sb_host[si])
    meta = dv._meta_host
    pay = dv.t_payload.cpu().numpy().view(np.uint16)
    out = []
    for d in range(dv.D):
        row = int(dv.rows[d])
        js = []
        for ci in range(base + rp[d], base + rp[d + 1]):
            m = int(meta[ci])
            j, t, n, off = m & 15, (m >> 4) & 3, (m >> 6) & 0x1FFFF, (m >> 23) * 8
            js.append(j)
            if t == 1:
                vs = pay[off:off + n].astype(np.int64)
            elif t == 2:
                vs = np.nonzero(np.unpackbits(pay[off:off + 4096].view(np.uint8), bitorder="little"))[0]
            else:
                nr = int(pay[off])
                vs = np.concatenate([np.arange(int(pay[off + 8 + 2 * k]), int(pay[off + 9 + 2 * k]) + 1)
                                     for k in range(nr)]) if nr else np.zeros(0, np.int64)
            assert len(vs) == n
            out.extend((row * SW + j * 65536 + vs.astype(np.int64)).tolist())
        assert js == sorted(set(js))
    return sorted(out)


def test_patched_arena_matches_fragments():
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "g")
        f = env.holder.index("i").field("g")
        rng = np.random.default_rng(1)
        for r in range(6):
            c = rng.choice(4 * SW, 40000, replace=False).astype(np.uint64)
            f.import_bits(np.full(len(c), r, np.uint64), c)
        f.import_bits(np.full(70000, 2, np.uint64), np.arange(10, 70010, dtype=np.uint64))  # runs/bitmaps
        g = GpuExecutor(env.holder, "cpu")
        g.view_arena("i", "g", "standard", SHARDS)
        for k in range(150):
            c, r = int(rng.integers(0, 4 * SW)), int(rng.integers(0, 6))
            env.q("i", f"Set({c}, g={r})" if k % 3 else f"Clear({c}, g={r})")
            if k % 9 == 0:
                f.import_bits(np.full(7, r, np.uint64), rng.integers(0, 4 * SW, 7).astype(np.uint64))
            if k % 50 == 49:
                env.q("i", f"ClearRow(g={r})")
            dv = g.view_arena("i", "g", "standard", SHARDS)
        assert g.rebuilds == 1 and g.row_updates > 100
        for si, s in enumerate(SHARDS):
            frag = env.holder.fragment("i", "g", "standard", s)
            assert _decode(dv, si) == frag.storage.slice().astype(np.int64).tolist()
        # brand-new row ids go into the directory in place (past the end and
        # in the middle); every shard still decodes to its fragment
        for col, rid in ((SW + 3, 999), (3 * SW + 70000, 7), (5, 999), (2 * SW + 1, 6)):
            env.q("i", f"Set({col}, g={rid})")
            dv = g.view_arena("i", "g", "standard", SHARDS)
        assert g.rebuilds == 1 and {6, 7, 999} <= set(dv.rows.tolist())
        assert dv.rows.tolist() == sorted(dv.rows.tolist())
        for si, s in enumerate(SHARDS):
            frag = env.holder.fragment("i", "g", "standard", s)
            assert _decode(dv, si) == frag.storage.slice().astype(np.int64).tolist()
            assert (dv.t_rowptr.view(dv.S, dv.D + 1)[si].numpy() == dv._rowptr_host[si]).all()
    finally:
        env.close()


def test_arena_rebuild_races_snapshots():
    """Stress of the scenario behind a CPU-suite crash: the native arena
    builder reads the fragments' bitmaps with no lock held while writes and
    the snapshot's to_bytes() (which optimises containers in place) change
    them.  The rebuild now takes a copy under each fragment lock; rebuilds
    racing writes + snapshots must not crash, and the quiescent arena
    decodes to the fragments.  (The window is narrow: this does not
    reproduce the crash reliably without the fix.)"""
    import threading

    from pilosa_amd.ops.gpu_executor import GpuExecutor
    env = Env()
    try:
        env.create_index("i")
        env.field("i", "g")
        f = env.holder.index("i").field("g")
        rng = np.random.default_rng(7)
        for r in range(4):
            f.import_bits(np.full(30000, r, np.uint64), rng.choice(4 * SW, 30000, replace=False).astype(np.uint64))
        frags = [env.holder.fragment("i", "g", "standard", s) for s in SHARDS]
        stop = threading.Event()

        wr = np.random.default_rng(8)

        def snapshots():
            # writes leave containers un-optimised; the snapshot's to_bytes()
            # then converts them in place
            while not stop.is_set():
                f.import_bits(np.full(64, int(wr.integers(0, 4)), np.uint64),
                              wr.integers(0, 4 * SW, 64).astype(np.uint64))
                for fr in frags:
                    fr.snapshot()
        t = threading.Thread(target=snapshots, daemon=True)
        t.start()
        try:
            for _ in range(12):
                GpuExecutor(env.holder, "cpu").view_arena("i", "g", "standard", SHARDS)
        finally:
            stop.set()
            t.join(timeout=30)
        # quiescent: a fresh arena decodes to exactly the fragments
        dv = GpuExecutor(env.holder, "cpu").view_arena("i", "g", "standard", SHARDS)
        for si, s in enumerate(SHARDS):
            assert _decode(dv, si) == frags[si].storage.slice().astype(np.int64).tolist()
    finally:
        env.close()
