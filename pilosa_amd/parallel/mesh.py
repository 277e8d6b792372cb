"""Intra-node multi-GPU execution: one process per GPU over torch.distributed.

Reference analog: the coordinator map/reduce of executor.go:2458-2555, where
every node executes a call over its shards and the coordinator folds the
per-node results (HTTP + protobuf).  Inside one MI355X node we replace that
hop with a process group (backend ``nccl`` = RCCL over xGMI on the GPU box,
``gloo`` for CPU tests):

* rank 0 is the front end (HTTP API, key translation, attribute stores,
  schema of record); ranks 1..N-1 run :meth:`ShardMesh.serve`.
* each rank owns shards ``s`` with ``(s // block) % world == rank`` and keeps
  their fragments (and device arenas) in its own holder; block-cyclic rather
  than one contiguous range so ownership is stable while an index grows.
* every read call is broadcast once (the canonical PQL string, like the
  reference's remote QueryRequest), each rank runs it over the shards it owns
  with ``remote`` semantics (TopN phase-1 pairs, unmerged row segments), and
  the partial results are reduced with collectives: ``all_reduce(SUM)`` of
  int64 tensors for Count / batched Counts / Sum, an object gather folded
  with the executor's own reduce function for everything else (TopN pairs,
  Rows, GroupBy, MinRow/MaxRow, Min/Max, Row segments).
* writes and imports are routed to the owning rank only.

Collectives are issued strictly in the same order on every rank, so the front
end serialises mesh operations with a lock.
"""
from __future__ import annotations

import threading
import traceback
from typing import Any, Callable, Dict, List, Optional, Sequence

SHARD_WIDTH = 1 << 20


class MeshError(RuntimeError):
    pass


# ---------------------------------------------------------------- transport
def encode_result(r):
    """Make a partial result picklable (Row segments hold native bitmaps)."""
    from pilosa_amd.models.row import Row

    if isinstance(r, Row):
        return ("__row__", {int(s): bm.to_bytes() for s, bm in r.segments.items()})
    if isinstance(r, BaseException):
        return ("__err__", f"{type(r).__name__}: {r}", traceback.format_exception(type(r), r, r.__traceback__))
    return r


def decode_result(r):
    from pilosa_amd import _roaring
    from pilosa_amd.models.row import Row

    if isinstance(r, tuple) and r and r[0] == "__row__":
        return Row(segments={s: _roaring.Bitmap.from_bytes(b) for s, b in r[1].items()})
    if isinstance(r, tuple) and r and r[0] == "__err__":
        raise MeshError(r[1])
    return r


class ShardMesh:
    """Shard-owner routing and collective reductions for one node's GPUs."""

    def __init__(self, executor, group=None, block: int = 1, device=None):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.block = max(1, int(block))
        self.executor = executor
        backend = dist.get_backend(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        self.lock = threading.RLock()
        self.ops = 0

    # ------------------------------------------------------------ ownership
    def owner(self, shard: int) -> int:
        return (int(shard) // self.block) % self.world

    def owned(self, shards: Sequence[int], rank: Optional[int] = None) -> List[int]:
        r = self.rank if rank is None else rank
        return [int(s) for s in shards if self.owner(s) == r]

    @property
    def is_frontend(self) -> bool:
        return self.rank == 0

    # ------------------------------------------------------------ plumbing
    def _bcast(self, cmd):
        box = [cmd]
        self.dist.broadcast_object_list(box, src=0, group=self.group, device=self._obj_device())
        return box[0]

    def _obj_device(self):
        return self.device if self.device.type == "cuda" else None

    def _gather(self, obj) -> Optional[list]:
        out = [None] * self.world if self.rank == 0 else None
        self.dist.gather_object(encode_result(obj), out, dst=0, group=self.group)
        return out

    def _sum_i64(self, values: Sequence[int]) -> List[int]:
        t = self.torch.tensor(list(values), dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return [int(x) for x in t.cpu().tolist()]

    def _run(self, cmd):
        """Front end: broadcast ``cmd`` and take part in it like any rank."""
        if not self.is_frontend:
            raise MeshError("only rank 0 issues mesh commands")
        with self.lock:
            self.ops += 1
            self._bcast(cmd)
            return self._dispatch(cmd)

    # ------------------------------------------------------------ front-end API
    def map_local(self, index: str, c, shards: Sequence[int], opt, reduce_fn: Callable[[Any, Any], Any]):
        """Execute call ``c`` over ``shards`` on their owner ranks and fold the
        partial results with ``reduce_fn`` (the executor's reduce step)."""
        if c.name == "Count":
            return self._run(("count", index, [str(c)], list(shards)))[0]
        parts = self._run(("call", index, str(c), list(shards), _opt_dict(opt)))
        result = None
        for p in parts:
            result = reduce_fn(result, decode_result(p))
        return result

    def count_batch(self, index: str, calls, shards: Sequence[int]) -> List[int]:
        return self._run(("count", index, [str(c) for c in calls], list(shards)))

    def forward_write(self, index: str, c, shard: int, opt) -> Any:
        parts = self._run(("write", index, str(c), int(shard), _opt_dict(opt)))
        out = decode_result(parts[self.owner(shard)])
        self._note_shard(index, shard)
        return out

    def forward_import(self, kind: str, index: str, field: str, shard: int, payload: dict):
        parts = self._run(("import", kind, index, field, int(shard), payload))
        decode_result(parts[self.owner(shard)])
        self._note_shard(index, shard)

    def apply_schema(self):
        """Push the front end's schema to every rank (after schema changes)."""
        schema = self.executor.holder.schema()
        self._run(("schema", schema))

    def delete_index(self, name: str):
        self._run(("delete_index", name))

    def delete_field(self, index: str, name: str):
        self._run(("delete_field", index, name))

    def shard_counts(self) -> Dict[int, Dict[str, List[int]]]:
        """Available shards per rank (status/debug)."""
        parts = self._run(("shards",))
        return {r: decode_result(p) for r, p in enumerate(parts)}

    def stop(self):
        if self.is_frontend:
            with self.lock:
                self._bcast(("stop",))

    def _note_shard(self, index: str, shard: int):
        idx = self.executor.holder.index(index)
        if idx is None:
            return
        for f in list(idx.fields.values()):
            if int(shard) not in f.remote_available_shards:
                f.add_remote_available_shards([int(shard)])

    # ------------------------------------------------------------ worker loop
    def serve(self):
        """Ranks > 0: execute broadcast commands until ``stop``."""
        while True:
            cmd = self._bcast(None)
            if cmd[0] == "stop":
                return
            self._dispatch(cmd)

    # ------------------------------------------------------------ all ranks
    def _dispatch(self, cmd):
        kind = cmd[0]
        ex = self.executor
        if kind == "count":
            _, index, pqls, shards = cmd
            local = [0] * len(pqls)
            err = None
            try:
                local = self._local_counts(index, pqls, self.owned(shards))
            except Exception as e:  # noqa: BLE001 - reported through the gather below
                err = e
            out = self._sum_i64(local)
            errs = self._gather(err)
            if self.is_frontend:
                for e in errs:
                    decode_result(e)
            return out
        if kind == "call":
            _, index, pql, shards, optd = cmd
            try:
                mine = self._local_call(index, pql, self.owned(shards), optd)
            except Exception as e:  # noqa: BLE001
                mine = e
            return self._gather(mine)
        if kind == "write":
            _, index, pql, shard, optd = cmd
            mine = None
            if self.owner(shard) == self.rank:
                try:
                    mine = self._local_call(index, pql, [shard], optd)
                except Exception as e:  # noqa: BLE001
                    mine = e
            return self._gather(mine)
        if kind == "import":
            _, what, index, field, shard, payload = cmd
            mine = None
            if self.owner(shard) == self.rank:
                try:
                    self._local_import(what, index, field, shard, payload)
                except Exception as e:  # noqa: BLE001
                    mine = e
            return self._gather(mine)
        if kind == "schema":
            if not self.is_frontend:
                ex.holder.apply_schema(cmd[1])
            return self._gather(None)
        if kind == "delete_index":
            if not self.is_frontend and ex.holder.index(cmd[1]) is not None:
                ex.holder.delete_index(cmd[1])
            return self._gather(None)
        if kind == "delete_field":
            if not self.is_frontend:
                idx = ex.holder.index(cmd[1])
                if idx is not None and idx.field(cmd[2]) is not None:
                    idx.delete_field(cmd[2])
            return self._gather(None)
        if kind == "shards":
            mine = {name: idx.available_shards() for name, idx in ex.holder.indexes.items()}
            if self.is_frontend:
                mine = {name: sorted({s for f in idx.fields.values() for s in f.local_shards})
                        for name, idx in ex.holder.indexes.items()}
            return self._gather(mine)
        raise MeshError(f"unknown mesh command {kind!r}")

    def _local_opt(self, optd: dict):
        from pilosa_amd.executor import ExecOptions

        o = ExecOptions(remote=True, exclude_row_attrs=optd.get("exclude_row_attrs", False),
                        exclude_columns=optd.get("exclude_columns", False))
        o.mesh_local = True
        return o

    def _local_call(self, index: str, pql: str, shards: List[int], optd: dict):
        from pilosa_amd.pql import parse_string

        ex = self.executor
        if ex.holder.index(index) is None:
            raise MeshError(f"index not found on rank {self.rank}: {index}")
        c = parse_string(pql).calls[0]
        if not shards and c.name not in ("Set", "Clear", "SetRowAttrs", "SetColumnAttrs"):
            return None
        return ex.execute_call(index, c, shards, self._local_opt(optd))

    def _local_counts(self, index: str, pqls: List[str], shards: List[int]) -> List[int]:
        from pilosa_amd.pql import parse_string

        ex = self.executor
        if not shards:
            return [0] * len(pqls)
        calls = [parse_string(p).calls[0] for p in pqls]
        if ex.gpu is not None and len(calls) > 1:
            res = ex.gpu.try_count_batch(index, calls, shards)
            if res is not None:
                return [int(x) for x in res]
        opt = self._local_opt({})
        return [int(ex.execute_call(index, c, shards, opt) or 0) for c in calls]

    def _local_import(self, what: str, index: str, field: str, shard: int, p: dict):
        import numpy as np

        holder = self.executor.holder
        idx = holder.index(index)
        if idx is None:
            raise MeshError(f"index not found on rank {self.rank}: {index}")
        f = idx.field(field)
        if f is None:
            raise MeshError(f"field not found on rank {self.rank}: {field}")
        ef = idx.existence_field()
        if what == "bits":
            cols = np.asarray(p["cols"], np.uint64)
            if not p.get("clear") and ef is not None and len(cols):
                ef.import_bits(np.zeros(len(cols), np.uint64), cols)
            f.import_bits(p["rows"], p["cols"], p.get("timestamps"), clear=p.get("clear", False))
        elif what == "values":
            cols = np.asarray(p["cols"], np.uint64)
            if not p.get("clear") and ef is not None and len(cols):
                ef.import_bits(np.zeros(len(cols), np.uint64), cols)
            f.import_values(p["cols"], p["values"], clear=p.get("clear", False))
        elif what == "roaring":
            f.import_roaring(shard, p["views"], p.get("clear", False))
        else:
            raise MeshError(f"unknown import kind {what!r}")


def _opt_dict(opt) -> dict:
    if opt is None:
        return {}
    return {"exclude_row_attrs": bool(getattr(opt, "exclude_row_attrs", False)),
            "exclude_columns": bool(getattr(opt, "exclude_columns", False))}


# ---------------------------------------------------------------- process setup
def dist_env():
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    import os

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_process_group(local_rank: int, backend: Optional[str] = None):
    """One process per GPU: RCCL ("nccl") when GPUs are visible, else gloo."""
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_backend()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    return backend


def rank_data_dir(data_dir: str, rank: int) -> str:
    """Rank 0 uses the node's data dir; rank r keeps its shards in ``.rank<r>``
    inside it (dot-dirs are skipped by the holder scan)."""
    import os

    return data_dir if rank == 0 else os.path.join(data_dir, f".rank{rank}")


def run_worker(data_dir: str, gpu_mode: str = "auto", block: int = 1, logger=None) -> int:
    """Entry point of ranks > 0 of a multi-GPU server (``pilosa_amd server``
    under ``torch.distributed.run``): own holder + GPU engine, serve the mesh."""
    import torch
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder

    rank, world, local = dist_env()
    init_process_group(local)
    holder = Holder(rank_data_dir(data_dir, rank)).open()
    gpu = None
    if (gpu_mode or "auto").lower() not in ("off", "none", "cpu") and torch.cuda.is_available():
        from pilosa_amd.ops.gpu_executor import GpuExecutor
        gpu = GpuExecutor(holder, f"cuda:{local}")
    ex = Executor(holder, gpu=gpu)
    if gpu is not None:
        gpu.executor = ex
    holder.on_schema_change = lambda: gpu.invalidate() if gpu is not None else None
    mesh = ShardMesh(ex, block=block)
    if logger is not None:
        logger.printf("mesh worker rank %d/%d on %s", rank, world, f"cuda:{local}" if gpu else "cpu")
    try:
        mesh.serve()
    finally:
        ex.close()
        holder.close()
        dist.destroy_process_group()
    return 0
