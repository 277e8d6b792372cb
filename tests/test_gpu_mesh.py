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
