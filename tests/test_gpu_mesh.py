"""Two-rank shard mesh with a GPU executor per rank on the one GPU of the
box (gloo collectives through host copies: the rehearsal of the node's RCCL
mesh).  Pipelined Count texts and the tensor TopN batch (candidate union +
re-count all-reduce across ranks) must equal a single-process host
executor holding every shard."""
import json
import os
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.test_mesh import _canon, _data, _free_port, _load, _setup_schema

pytestmark = pytest.mark.gpu

QUERIES = ["Count(Row(f=1)) Count(Intersect(Row(f=1), Row(g=2))) Count(Union(Row(f=3), Row(g=1)))",
           "TopN(f, n=3)", "TopN(f, Row(g=3), n=2)", "TopN(f, n=4) TopN(f, Row(g=1), n=3) TopN(f)"]


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"gmesh{rank}_")).open()
    gpu = GpuExecutor(holder, "cuda:0")
    ex = Executor(holder, gpu=gpu)
    gpu.executor = ex
    ex.strict_gpu = True
    mesh = ShardMesh(ex, block=1, device="cuda:0")
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _data()
        _load(ex, bits, vals, mesh)
        for s in holder.all_fragments():
            s.recalculate_cache()
        got = [_canon(ex.execute("i", q).results) for q in QUERIES]
        with open(os.path.join(outdir, "gmesh.json"), "w") as fh:
            json.dump({"got": got, "topn_tensor": mesh.topn_tensor_batches, "seq": mesh.seq}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_gpu_mesh_counts_and_tensor_topn(tmp_path):
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder

    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    res = json.load(open(tmp_path / "gmesh.json"))
    holder = Holder(tempfile.mkdtemp(prefix="gmesh_ref_")).open()
    ex = Executor(holder)
    _setup_schema(holder)
    bits, vals = _data()
    _load(ex, bits, vals)
    want = [_canon(ex.execute("i", q).results) for q in QUERIES]
    ex.close()
    holder.close()
    for q, g, w in zip(QUERIES, res["got"], want):
        assert g == w, q
    assert res["seq"] >= 1, "Count text did not take the pipelined mesh path"
    assert res["topn_tensor"] >= 3, "TopN did not take the tensor mesh path"


# 300 bits of a new row 30 in shard 1 (rank 1's): enough to enter the top 5
WRITE = " ".join(f"Set({(1 << 20) + 7 * k}, f=30)" for k in range(300))
TOPN_QUERIES = ["TopN(f, n=5)", "TopN(f, Row(g=1), n=4)", "TopN(f, n=3) TopN(f, Row(g=2), n=6) TopN(f)"]


def _distinct_rows_data():
    """Even shards hold rows 0-4 and 10-14, odd shards rows 0-4 and 20-24, so
    the two ranks' row directories differ (the node row space is their union)."""
    rng = np.random.default_rng(11)
    bits = []
    for shard in range(6):
        extra = 10 if shard % 2 == 0 else 20
        for _ in range(400):
            col = shard * (1 << 20) + int(rng.integers(0, 1 << 20))
            r = int(rng.integers(0, 5))
            bits.append(("f", r if rng.random() < 0.5 else r + extra, col))
            if rng.random() < 0.5:
                bits.append(("g", int(rng.integers(0, 4)), col))
    return bits, []


def _topn_worker(rank, world, port, outdir):
    import threading

    # rebuild the slot index as soon as the node row space moves (the 10 s
    # re-rank throttle would send the src batches to the general path)
    os.environ["PILOSA_TOPN_INDEX_REBUILD_S"] = "0"

    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"gmesht{rank}_")).open()
    gpu = GpuExecutor(holder, "cuda:0")
    ex = Executor(holder, gpu=gpu)
    gpu.executor = ex
    ex.strict_gpu = True
    mesh = ShardMesh(ex, block=1, device="cuda:0")
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _distinct_rows_data()
        _load(ex, bits, vals, mesh)
        mesh.recalculate_caches()
        shards = list(range(6))
        before = [_canon(ex.execute("i", q, shards=shards).results) for q in TOPN_QUERIES]
        # a write that adds a row on rank 1 only (shard 1): only that rank's
        # row space moves; the next batch must refresh it on every rank
        ex.execute("i", WRITE)
        mesh.recalculate_caches()
        after = [_canon(ex.execute("i", q, shards=shards).results) for q in TOPN_QUERIES]
        b0 = mesh.topn_tensor_batches
        mesh.max_in_flight = 0
        got = [None] * 24

        def run(k):
            got[k] = _canon(ex.execute("i", TOPN_QUERIES[k % len(TOPN_QUERIES)], shards=shards).results)
        ts = [threading.Thread(target=run, args=(k,)) for k in range(len(got))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        with open(os.path.join(outdir, "gmesht.json"), "w") as fh:
            json.dump({"before": before, "after": after, "concurrent": got,
                       "concurrent_batches": mesh.topn_tensor_batches - b0, "max_in_flight": mesh.max_in_flight}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()


def test_gpu_mesh_topn_distinct_row_spaces_and_writes(tmp_path):
    """the slot index must be built over the node row space, and
    a write that moves one rank's row directory must make every rank
    re-gather the space (a collective decision), before and during
    concurrent TopN requests."""
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder

    mp.start_processes(_topn_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "gmesht.json"))
    holder = Holder(tempfile.mkdtemp(prefix="gmesht_ref_")).open()
    ex = Executor(holder)
    _setup_schema(holder)
    bits, vals = _distinct_rows_data()
    _load(ex, bits, vals)
    holder.recalculate_caches()
    want_before = [_canon(ex.execute("i", q).results) for q in TOPN_QUERIES]
    ex.execute("i", WRITE)
    holder.recalculate_caches()
    want_after = [_canon(ex.execute("i", q).results) for q in TOPN_QUERIES]
    ex.close()
    holder.close()
    assert res["before"] == want_before
    assert res["after"] == want_after
    assert want_after != want_before
    for k, g in enumerate(res["concurrent"]):
        assert g == want_after[k % len(TOPN_QUERIES)], k
    assert res["concurrent_batches"] >= 20, res
    assert res["max_in_flight"] >= 2, res


def test_gpu_mesh_cache_only_fused_one_collective(tmp_path):
    """The cache-only groups of the TopN batches above ran the node-wide
    fused path (one all-reduce of membership + partial totals per batch) on
    both ranks; answers are checked by the two tests above."""
    mp.start_processes(_fused_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = json.load(open(tmp_path / "gfused.json"))
    assert res["fused"] >= 4, res
    assert res["per_batch"] and max(res["per_batch"]) <= 2, res


def _fused_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor
    from pilosa_amd.parallel.mesh import ShardMesh

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = Holder(tempfile.mkdtemp(prefix=f"gfused{rank}_")).open()
    gpu = GpuExecutor(holder, "cuda:0")
    ex = Executor(holder, gpu=gpu)
    gpu.executor = ex
    ex.strict_gpu = True
    mesh = ShardMesh(ex, block=1, device="cuda:0")
    ex.mesh = mesh
    try:
        if rank != 0:
            mesh.serve()
            return
        _setup_schema(holder)
        mesh.apply_schema()
        bits, vals = _distinct_rows_data()
        _load(ex, bits, vals, mesh)
        mesh.recalculate_caches()
        shards = list(range(6))
        ex.execute("i", "TopN(f, n=5) TopN(f, n=2, threshold=3)", shards=shards)
        per_batch = []
        for q in ("TopN(f, n=5) TopN(f, n=2, threshold=3)", "TopN(f, n=3)", "TopN(f)", "TopN(f, n=1) TopN(f)"):
            ex.execute("i", q, shards=shards)   # first of each prefix length refreshes its space
            c0 = mesh.comm.data_calls
            ex.execute("i", q, shards=shards)
            per_batch.append(mesh.comm.data_calls - c0)
        with open(os.path.join(outdir, "gfused.json"), "w") as fh:
            json.dump({"fused": gpu.topn_mesh_fused, "per_batch": per_batch}, fh)
        mesh.stop()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()
