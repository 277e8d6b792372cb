"""Zero-copy host reads for lazily opened fragments (VERDICT r02 item 5;
reference roaring/container_stash.go:262-346, roaring.go:1616-1622,
fragment.go:311-456,459): on a holder opened with lazy fragments, scattered
Set()/Clear() calls, row reads, Count(Row), TopN from the rank cache and the
``.cache`` open run against the mmapped files.  Every fragment stays cold (no
heap copy of its containers), host RSS grows by a small fraction of the data
size, and the answers equal those of the same data loaded whole."""
import os
import shutil
import tempfile

import numpy as np
import psutil

from pilosa_amd import _roaring
from pilosa_amd.executor import Executor
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.holder import Holder
from tests.helpers import SW

NSHARD = 12


def _rss_anon() -> int:
    """Anonymous (heap) resident bytes.  Pages of the mapped fragment files
    are file-backed (RssFile): the kernel reclaims them under pressure."""
    with open("/proc/self/status") as fh:
        for line in fh:
            if line.startswith("RssAnon:"):
                return int(line.split()[1]) * 1024
    return psutil.Process().memory_info().rss


def _make(base):
    h = Holder(base).open()
    h.create_index("i", track_existence=False)
    h.index("i").create_field("f", FieldOptions(cache_type="ranked", cache_size=2000))
    h.close()
    fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
    os.makedirs(fdir, exist_ok=True)
    _roaring.write_zipf_fragments(fdir, 0, NSHARD, NSHARD * SW, 200_000, 3.0, 1.6, 50.0, 3, 4, cache_size=2000)
    return sum(os.path.getsize(os.path.join(fdir, f)) for f in os.listdir(fdir))


def test_lazy_holder_serves_writes_and_reads_from_mapped_files():
    base = tempfile.mkdtemp(prefix="cold_reads_")
    try:
        nbytes = _make(base)
        rng = np.random.default_rng(5)
        cols = rng.integers(0, NSHARD * SW, size=300)
        rows = rng.integers(0, 50, size=300)
        sets = " ".join(f"Set({c}, f={r})" for c, r in zip(cols.tolist(), rows.tolist()))
        clears = " ".join(f"Clear({c}, f={r})" for c, r in zip(cols[:40].tolist(), rows[:40].tolist()))
        reads = "Count(Row(f=0)) Count(Row(f=3)) TopN(f, n=10) TopN(f, ids=[0, 1, 2, 49])"

        holder = Holder(base, lazy_fragments=True).open()
        ex = Executor(holder)
        rss0 = _rss_anon()
        got_sets = ex.execute("i", sets).results
        got_clears = ex.execute("i", clears).results
        got = ex.execute("i", reads).results
        row7 = ex.execute("i", "Row(f=7)").results[0].columns()
        grew = _rss_anon() - rss0
        frags = holder.view("i", "f", "standard").all_fragments()
        assert len(frags) == NSHARD and all(f.is_cold() for f in frags), "a fragment was read into heap"
        assert all(f.mapped_stats() is not None for f in frags)
        # the overlays hold only the containers the writes touched
        assert sum(f.mapped_stats()["overlay_containers"] for f in frags) <= 300
        # loading the fragments whole would take more than nbytes of heap; the
        # growth here is the rank caches, the copied containers and the query objects
        assert grew < 0.2 * nbytes, (grew, nbytes)
        ex.close()
        holder.close()

        # the same data loaded whole (file snapshot + the op log the writes appended)
        full = Holder(base).open()
        exf = Executor(full)
        want = exf.execute("i", reads).results
        assert [r if isinstance(r, int) else [(p.id, p.count) for p in r] for r in got] == \
            [r if isinstance(r, int) else [(p.id, p.count) for p in r] for r in want]
        assert np.array_equal(exf.execute("i", "Row(f=7)").results[0].columns(), row7)
        cleared = set(zip(cols[:40].tolist(), rows[:40].tolist()))
        for c, r in zip(cols.tolist(), rows.tolist()):
            frag = full.fragment("i", "f", "standard", c // SW)
            assert frag.bit(r, c) == ((c, r) not in cleared)
        assert any(got_sets) and all(got_clears)
        exf.close()
        full.close()
    finally:
        shutil.rmtree(base, ignore_errors=True)


def test_cold_bulk_import_and_snapshot_stay_off_heap():
    """Bulk imports (bits, roaring) into cold fragments go through the
    mapped overlay, and the snapshot they trigger streams the mapped file plus
    overlay to the new file (MappedBitmap.write_snapshot): the fragments stay
    cold, and a whole load of the new files equals a whole-load replay."""
    base = tempfile.mkdtemp(prefix="cold_import_")
    try:
        _make(base)
        rng = np.random.default_rng(9)
        holder = Holder(base, lazy_fragments=True).open()
        f = holder.index("i").field("f")
        n = 60_000   # > max_opn for every shard it lands in: snapshots run
        rows = rng.integers(0, 300, size=n).astype(np.uint64)
        cols = rng.integers(0, 4 * SW, size=n).astype(np.uint64)
        f.import_bits(rows, cols)
        f.import_bits(rows[:5000], cols[:5000], clear=True)
        frag0 = holder.fragment("i", "f", "standard", 0)
        blob = _roaring.Bitmap(np.unique(rng.integers(0, 64 * SW, size=20000)).astype(np.uint64)).to_bytes()
        frag0.import_roaring(blob)
        holder.snapshot_queue.drain() if getattr(holder, "snapshot_queue", None) is not None and \
            hasattr(holder.snapshot_queue, "drain") else None
        for s in range(4):
            holder.fragment("i", "f", "standard", s).snapshot()
        frags = holder.view("i", "f", "standard").all_fragments()
        assert all(fr.is_cold() for fr in frags)
        counts = {r: holder.fragment("i", "f", "standard", 1).row_count(r) for r in range(0, 300, 37)}
        holder.close()
        full = Holder(base).open()
        for r, c in counts.items():
            assert full.fragment("i", "f", "standard", 1).row_count(r) == c
        fr0 = full.fragment("i", "f", "standard", 0)
        assert fr0.storage.check() == ""
        clear_set = set(zip(rows[:5000].tolist(), cols[:5000].tolist()))
        blob_bm = _roaring.Bitmap.from_bytes(blob)
        for r, c in list(zip(rows.tolist(), cols.tolist()))[::97]:
            sh = int(c) // SW
            exp = (r, c) not in clear_set or (sh == 0 and blob_bm.contains(r * SW + c % SW))
            assert full.fragment("i", "f", "standard", sh).bit(r, c) == exp
        full.close()
    finally:
        shutil.rmtree(base, ignore_errors=True)


def test_map_count_cap_falls_back_to_heap():
    """syswrap: past max-map-count a cold fragment is read into heap instead
    of mapped (reference syswrap/mmap.go ErrMaxMapCountReached), and closing
    fragments gives their map slots back."""
    from pilosa_amd.utils import syswrap
    base = tempfile.mkdtemp(prefix="cold_cap_")
    old_max = syswrap.max_map_count()
    try:
        _make(base)
        holder = Holder(base, lazy_fragments=True).open()
        frags = holder.view("i", "f", "standard").all_fragments()
        c0 = syswrap.map_count()
        syswrap.set_max_map_count(c0 + 2)
        for fr in frags[:3]:
            fr.row_count(1)
        assert [fr.mapped_stats() is not None for fr in frags[:3]] == [True, True, False]
        assert frags[0].is_cold() and frags[1].is_cold() and not frags[2].is_cold()
        assert syswrap.map_count() == c0 + 2
        holder.close()
        assert syswrap.map_count() == c0
    finally:
        syswrap.set_max_map_count(old_max)
        shutil.rmtree(base, ignore_errors=True)
