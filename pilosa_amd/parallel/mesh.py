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
  int64 tensors for Count / batched Counts (an error flag rides in the same
  tensor), whole TopN batches on the device with a candidate union and an
  all-reduced re-count (OP_TOPN), and for every other call one
  variable-length all-gather of each rank's partial as a typed int64 tensor
  (collectives.encode_partial: ValCount, Pair, TopN pairs, Rows ids, GroupBy
  matrices; a GPU rank's Row as its device result containers,
  collectives.encode_row_block, decoded with one D2H on the front end)
  folded with the executor's own
  reduce function; results carrying strings (keys, attributes) ride as
  msgpack bytes inside the same tensor.
* writes and imports are routed to the owning rank only.

Transport is tensors only (parallel/collectives.py): a command is an int64
header plus a uint8 payload tensor, no pickled objects.  Collectives are
issued strictly in the same order on every rank, so the front end serialises
the ISSUE of mesh operations with a lock: the command broadcast, this rank's
share of the work and the start of the operation's last collective.  Count
batches, general calls (OP_CALL) and TopN batches (OP_TOPN) leave that last
collective in flight (a ``collectives.Pending``) and complete it -- wait,
decode, reduce, trim -- outside the lock, so up to MAX_IN_FLIGHT requests per
rank overlap (the reference runs every query's mapReduce independently,
executor.go:2458-2518).  Every collective has the process group's
timeout; when one fails (a rank died or hung) the front end fails over: it
adopts the other ranks' fragment files from their data dirs into its own
holder (lazily opened, loaded into its HBM on first use) and keeps serving
single-GPU (a dead GPU's shard range is reloaded onto the
survivors).
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Dict, List, Optional, Sequence

from pilosa_amd.utils import tracing


class MeshError(RuntimeError):
    pass


# ---------------------------------------------------------------- transport
(OP_STOP, OP_COUNT, OP_CALL, OP_WRITE, OP_IMPORT, OP_SCHEMA, OP_DEL_INDEX, OP_DEL_FIELD, OP_SHARDS, OP_COUNT_TEXT,
 OP_ERRORS, OP_TOPN, OP_SYNC, OP_RECALC, OP_TOPN_PLAIN, OP_TOPN_CAND, OP_SHARDSET, OP_TOPN_SPACES) = range(18)
MAX_IN_FLIGHT = 4     # count batches a worker keeps in flight before it waits for the oldest
MAX_SHARD_SETS = 4096  # shard lists registered with the ranks (OP_SHARDSET); more go the general way
CALL_MIN_CAP = 1024    # int64 words per rank of a general call's partial gather (grows per call name)
# bitmap calls whose rank partial can travel as device container blocks
_ROW_CALLS = ("Row", "Range", "Bitmap", "Intersect", "Union", "Difference", "Xor", "Not", "Shift")
_OP_NAMES = {OP_STOP: "stop", OP_COUNT: "count", OP_CALL: "call", OP_WRITE: "write", OP_IMPORT: "import",
             OP_SCHEMA: "schema", OP_DEL_INDEX: "deleteIndex", OP_DEL_FIELD: "deleteField", OP_SHARDS: "shards",
             OP_COUNT_TEXT: "countText", OP_ERRORS: "errors", OP_TOPN: "topn", OP_SYNC: "sync",
             OP_RECALC: "recalculateCaches", OP_TOPN_PLAIN: "topnPlain", OP_TOPN_CAND: "topnCand",
             OP_SHARDSET: "shardSet", OP_TOPN_SPACES: "topnSpaces"}
_VOTES = {1: "declined", 2: "stale"}
_PIPELINED = (OP_COUNT_TEXT, OP_CALL, OP_TOPN, OP_TOPN_PLAIN)


def _raise_remote(parts):
    from .collectives import RemoteError

    for p in parts:
        if isinstance(p, RemoteError):
            raise MeshError(str(p))


class ShardMesh:
    """Shard-owner routing and collective reductions for one node's GPUs."""

    def __init__(self, executor, group=None, block: int = 1, device=None, peer_dirs: Optional[Dict[int, str]] = None,
                 ctrl_group="auto", force: bool = False):
        import collections

        import torch.distributed as dist

        from .collectives import Comm

        if ctrl_group == "auto":
            # every rank builds its mesh in the same order, so this collective
            # group creation lines up; commands then travel on gloo (host).  An
            # RCCL mesh always gets one (a world-size-1 RCCL mesh too: the
            # 1-GPU rehearsal of the node's transport, ``force``)
            multi = dist.get_world_size() > 1 or dist.get_backend() == "nccl"
            ctrl_group = dist.new_group(backend="gloo") if group is None and multi else None
        self.comm = Comm(group, device=device, ctrl_group=ctrl_group)
        # commands travel through a shared-memory ring (native/shmring.cpp)
        # when every rank can attach to it: set up collectively, here, where
        # every rank builds its mesh in the same order
        self.ring = self.comm.attach_ring()
        self.torch = self.comm.torch
        self.dist = self.comm.dist
        self.group = group
        self.rank = self.comm.rank
        self.world = self.comm.world
        self.block = max(1, int(block))
        self.executor = executor
        self.device = self.comm.device
        self.lock = threading.RLock()
        self.ops = 0
        # rank -> data dir of that rank's holder (failover adopts its fragments)
        self.peer_dirs: Dict[int, str] = dict(peer_dirs or {})
        self.failed_over = False
        self.failover_error: Optional[str] = None
        self.seq = 0                      # count-text batches issued (front end)
        self.in_flight = 0                # front end: batches issued, result not yet read
        self.max_in_flight = 0
        self.row_blocks = 0      # Row partials sent as device container blocks
        self._pending = collections.deque()   # worker: (tensor, work) of batches in flight
        self._errors: Dict[int, BaseException] = {}
        self.last_count_text_errors: List[str] = []
        self.topn_tensor_batches = 0
        # route calls through the mesh even at world size 1 (the executor
        # otherwise answers a 1-rank node directly): runs the RCCL transport
        # on a 1-GPU box, bench.py --mesh
        self.always = bool(force)
        # shard lists named by a small id, registered once with every rank
        # (OP_SHARDSET): a request names its ~1k shards with one int, and each
        # rank's owned subset is computed once
        self._shardsets: Dict[tuple, tuple] = {}     # front end: shards -> (id, owned)
        self._sets_by_id: Dict[int, tuple] = {}      # every rank: id -> (shards, owned)
        self._cand_gen = 0                           # node candidate space generations issued
        self.topn_plain_batches = 0
        self.topn_plain_refreshes = 0
        self.topn_plain_retries = 0
        self._call_cap: Dict[str, int] = {}          # OP_CALL gather capacity per call name (front end)
        self.call_retries = 0

    # ------------------------------------------------------------ ownership
    def owner(self, shard: int) -> int:
        return (int(shard) // self.block) % self.world

    def owned(self, shards: Sequence[int], rank: Optional[int] = None) -> List[int]:
        r = self.rank if rank is None else rank
        # memoised per shard list: a request over ~1k shards re-derived the
        # owner of every shard (~0.17 ms of the front end's time under the
        # mesh lock per TopN request)
        key = (r, self.world, self.block, tuple(shards))
        memo = self.__dict__.setdefault("_owned_memo", {})
        got = memo.get(key)
        if got is None:
            got = [int(s) for s in shards if self.owner(s) == r]
            if len(memo) >= 64:
                memo.clear()
            memo[key] = got
        return list(got)

    @property
    def is_frontend(self) -> bool:
        return self.rank == 0

    # ------------------------------------------------------------ plumbing
    def _gather(self, obj) -> list:
        """Every rank's partial result (typed int64 tensors, one all-gather)."""
        return self.comm.gather_partials(obj)

    def _run(self, op: int, *args):
        """Front end: broadcast the command and take part in it like any rank.
        A failed collective turns into failover (MeshError for this call)."""
        from .collectives import CommError, encode

        if not self.is_frontend:
            raise MeshError("only rank 0 issues mesh commands")
        with self.lock, tracing.span(f"Mesh.{_OP_NAMES.get(op, op)}"):
            if self.failed_over:
                raise MeshError(f"mesh failed over: {self.failover_error}")
            self.ops += 1
            try:
                self.comm.bcast_bytes(op, encode([tracing.context()] + list(args)))
                return self._dispatch(op, list(args))
            except CommError as e:
                self.failover(e)
                raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e

    # ------------------------------------------------------------ front-end API
    def map_local(self, index: str, c, shards: Sequence[int], opt, reduce_fn: Callable[[Any, Any], Any]):
        """Execute call ``c`` over ``shards`` on their owner ranks and fold the
        partial results with ``reduce_fn`` (the executor's reduce step)."""
        from .collectives import Overflow
        if c.name == "Count":
            return self._run(OP_COUNT, index, [str(c)], list(shards))[0]
        pql, optd = str(c), _opt_dict(opt)
        while True:
            # the partials travel in ONE fixed-capacity all-gather (no size
            # exchange, no host read before the data moves); the capacity is
            # learnt per call name and carried in the command
            cap, quiet = self._call_cap.get(c.name, (CALL_MIN_CAP, 0))
            # a partial that fits the results board is gathered there (cap 0:
            # no collective at all); larger ones in the RCCL all-gather
            board = self.comm.board and cap * 8 <= self.comm.ring.board_bytes
            parts = self._run_pipelined(OP_CALL, index, pql, list(shards), optd, 0 if board else cap)
            if not isinstance(parts, Overflow):
                break
            self.call_retries += 1
            self._call_cap[c.name] = (max(cap * 2 if board else 0, 1 << int(parts.need + parts.need // 4).bit_length()),
                                      0)
        # a capacity far above what the call sends is halved after a quiet
        # spell (a one-off large Row result does not pad every later one)
        longest = getattr(self, "_call_longest", 0)
        if cap > CALL_MIN_CAP and longest * 8 < cap:
            self._call_cap[c.name] = (cap // 2, 0) if quiet >= 15 else (cap, quiet + 1)
        _raise_remote(parts)
        result = None
        for p in parts:
            result = reduce_fn(result, p)
        return result

    def count_batch(self, index: str, calls, shards: Sequence[int]) -> List[int]:
        return self._run(OP_COUNT, index, [str(c) for c in calls], list(shards))

    def count_text(self, index: str, text: str, shards: Sequence[int]) -> Optional[List[int]]:
        """A request of Count() calls as PQL text, pipelined: the lock covers
        only the command broadcast and the launch of this rank's share plus
        its all-reduce (every rank issues collectives in command order); the
        wait for the reduced counts happens outside it, so the next request's
        broadcast, planning and kernels overlap this one's (executor.go
        mapReduce)."""
        from .collectives import CommError, encode

        if not self.is_frontend:
            raise MeshError("only rank 0 issues mesh commands")
        q = text.count("Count(")
        with self.lock, tracing.span("Mesh.countTextIssue", calls=q):
            if self.failed_over:
                raise MeshError(f"mesh failed over: {self.failover_error}")
            self.ops += 1
            self.seq += 1
            seq = self.seq
            try:
                self.comm.bcast_bytes(OP_COUNT_TEXT, encode([tracing.context(), index, text, list(shards), q, seq]))
                t, work = self._count_text_issue(index, text, list(shards), q, seq)
            except CommError as e:
                self.failover(e)
                raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e
            self.in_flight += 1
            self.max_in_flight = max(self.max_in_flight, self.in_flight)
        try:
            with tracing.span("Mesh.countTextWait", gpu=True):
                self.comm.wait(work)
                out = self._host_list(t)
        except CommError as e:
            with self.lock:
                self.failover(e)
            raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e
        finally:
            with self.lock:
                self.in_flight -= 1
        if out[-1]:
            # a rank could not count it: collect the errors (logged), and let
            # the caller run the request on the general path, which raises
            # the reference's error for it (parse errors, unknown fields, ...)
            from .collectives import RemoteError
            errs = [p for p in self._run_collect(OP_ERRORS, seq) if isinstance(p, RemoteError)]
            self.last_count_text_errors = [str(e) for e in errs]
            return None
        return out[:-1]

    def _run_collect(self, op: int, *args) -> list:
        """Like :meth:`_run` but returns the per-rank parts without raising
        the remote errors among them."""
        from .collectives import CommError, encode

        with self.lock:
            if self.failed_over:
                raise MeshError(f"mesh failed over: {self.failover_error}")
            try:
                self.comm.bcast_bytes(op, encode([tracing.context()] + list(args)))
                mine = self._errors.pop(int(args[0]), None) if op == OP_ERRORS else None
                return self._gather(mine)
            except CommError as e:
                self.failover(e)
                raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e

    def topn_batch(self, index: str, calls, shards: Sequence[int], text: Optional[str] = None):
        """Whole TopN calls on every rank's GPU with the node-wide merge on
        tensors (ops/topn_exec.py / topn_index.py with ``comm``): the ranks
        all-gather and union their phase-1 candidate keys and all-reduce the
        ids= re-counts, so the answers come back complete on every rank
        (executor.go:863-903 over RCCL instead of per-shard pair lists).  The
        ranks first agree (one all-reduce of a flag) that each can run the
        batch on its device; None = use the general path."""
        from pilosa_amd.executor import DEFAULT_FIELD
        payload = text if text is not None else [str(c) for c in calls]
        for attempt in range(2):
            res = self._run_pipelined(OP_TOPN, index, payload, list(shards))
            if isinstance(res, str):
                # a batch whose vote rode in its first collective: some rank
                # declined (the general path answers) or found its node row
                # space stale (rebuilt collectively, then the batch re-runs)
                if res == "stale" and attempt == 0:
                    fnames = sorted({str(c.args.get("_field") or DEFAULT_FIELD) for c in calls})
                    self._run(OP_TOPN_SPACES, index, fnames, list(shards))
                    continue
                return None
            if res is not None:
                self.topn_tensor_batches += 1
            return res
        return None

    def shard_set(self, shards: Sequence[int]):
        """(id, owned shards) of a shard list, registered with every rank on
        first use (one OP_SHARDSET command); None once MAX_SHARD_SETS lists
        are registered (the caller then takes the general path)."""
        key = tuple(shards)
        got = self._shardsets.get(key)
        if got is not None:
            return got
        with self.lock:
            got = self._shardsets.get(key)
            if got is None:
                if len(self._shardsets) >= MAX_SHARD_SETS:
                    return None
                sid = len(self._shardsets) + 1
                self._run(OP_SHARDSET, sid, list(key))
                got = self._shardsets[key] = (sid, self._sets_by_id[sid][1])
        return got

    def topn_plain(self, index: str, fname: str, ns: Sequence[int], ths: Sequence[int], shards: Sequence[int]):
        """A request of plain cache-only TopN calls of one field -- TopN(f[,
        n=][, threshold=]), recognised natively on the front end
        (Executor._topn_plain_fast) -- on every rank's GPU as ONE all-reduce
        (OP_TOPN_PLAIN): the command carries the parsed (n, threshold)
        arrays, the shard-set id and the node candidate space's generation
        and size; each rank adds its partial over that space, with its vote
        (stale / declined) folded into the same buffer, and the front end
        selects each call's top n from the sum.  No rank parses PQL and no
        host reads a tensor before the data collective (executor.go:863-930
        over mapReduce :2458-2555, on RCCL).  A space that some rank finds
        stale is rebuilt collectively (OP_TOPN_CAND) and the batch re-run
        once.  None = the general path."""
        from pilosa_amd.ops.gpu_executor import _nreq

        gpu = getattr(self.executor, "gpu", None)
        if gpu is None or not hasattr(gpu, "topn_plain_mesh"):
            return None
        ss = self.shard_set(shards)
        if ss is None:
            return None
        sid, own = ss
        nreq = _nreq(ns)
        ns = [int(n) for n in ns]
        ths = [int(t) for t in ths]
        force = False
        for attempt in range(2):
            st = None if force else gpu.plain_cand_state(index, fname, own, sid, nreq)
            if st is None:
                with self.lock:
                    self._cand_gen += 1
                    gen = self._cand_gen
                self.topn_plain_refreshes += 1
                self._run(OP_TOPN_CAND, index, fname, sid, nreq, gen)
                st = gpu.plain_cand_state(index, fname, own, sid, nreq)
                if st is None:
                    return None
            gen, U, fits, bucket = st
            if not fits:
                return None
            res = self._run_pipelined(OP_TOPN_PLAIN, index, fname, ns, ths, sid, bucket, gen, U)
            if isinstance(res, str):
                if res == "stale" and attempt == 0:
                    self.topn_plain_retries += 1
                    force = True   # another rank's copy was stale: rebuild the space node-wide
                    continue
                return None
            self.topn_plain_batches += 1
            return res
        return None

    def _run_pipelined(self, op: int, *args):
        """Front end: broadcast + issue under the lock (this rank's share
        and the start of the last collective), completion outside it, so
        the next request's issue overlaps this one's transfer and decode."""
        from .collectives import CommError, encode, resolve

        if not self.is_frontend:
            raise MeshError("only rank 0 issues mesh commands")
        name = _OP_NAMES.get(op, op)
        with self.lock, tracing.span(f"Mesh.{name}Issue"):
            if self.failed_over:
                raise MeshError(f"mesh failed over: {self.failover_error}")
            self.ops += 1
            try:
                self.comm.bcast_bytes(op, encode([tracing.context()] + list(args)))
                h = self._issue(op, list(args))
            except CommError as e:
                self.failover(e)
                raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e
            self.in_flight += 1
            self.max_in_flight = max(self.max_in_flight, self.in_flight)
        try:
            with tracing.span(f"Mesh.{name}Complete", gpu=True):
                return resolve(h)
        except CommError as e:
            with self.lock:
                self.failover(e)
            raise MeshError(f"mesh collective failed, failed over to rank 0: {e}") from e
        finally:
            with self.lock:
                self.in_flight -= 1

    def _host_list(self, t) -> List[int]:
        gpu = getattr(self.executor, "gpu", None)
        if t.device.type == "cuda" and gpu is not None and hasattr(gpu, "engine"):
            return gpu.engine.to_host(t).tolist()
        return t.cpu().tolist()

    def forward_write(self, index: str, c, shard: int, opt) -> Any:
        parts = self._run(OP_WRITE, index, str(c), int(shard), _opt_dict(opt))
        self._note_shard(index, shard)
        return parts[self.owner(shard)]

    def forward_import(self, kind: str, index: str, field: str, shard: int, payload: dict):
        self._run(OP_IMPORT, kind, index, field, int(shard), _plain(payload))
        self._note_shard(index, shard)

    def apply_schema(self):
        """Push the front end's schema to every rank (after schema changes)."""
        schema = self.executor.holder.schema()
        self._run(OP_SCHEMA, schema)

    def delete_index(self, name: str):
        self._run(OP_DEL_INDEX, name)

    def delete_field(self, index: str, name: str):
        self._run(OP_DEL_FIELD, index, name)

    def shard_counts(self) -> Dict[int, Dict[str, List[int]]]:
        """Available shards per rank (status/debug)."""
        parts = self._run(OP_SHARDS)
        return {r: p for r, p in enumerate(parts)}

    def recalculate_caches(self):
        """Every rank re-ranks its fragments' caches now (the reference's
        /recalculate-caches, holder.go:544, on each GPU's holder)."""
        self._run(OP_RECALC)

    def sync(self) -> List[int]:
        """Quiesce the node: every rank completes its requests in flight and
        synchronises its device, then the ranks meet (one gather).  Returns
        each rank's monotonic clock (ns) at that point, so the time between
        two syncs can be taken as the max over ranks (bench.py)."""
        return [int(x) for x in self._run(OP_SYNC)]

    def stop(self):
        if self.is_frontend and not self.failed_over:
            with self.lock:
                try:
                    self.comm.bcast_bytes(OP_STOP, b"")
                except Exception:  # noqa: BLE001 - peers already gone
                    pass

    def _note_shard(self, index: str, shard: int):
        idx = self.executor.holder.index(index)
        if idx is None:
            return
        for f in list(idx.fields.values()):
            if int(shard) not in f.remote_available_shards:
                f.add_remote_available_shards([int(shard)])

    # ------------------------------------------------------------ failover
    def failover(self, err: BaseException):
        """A collective failed: stop using the mesh and adopt every other
        rank's fragment files (their data dirs) into the front end's holder,
        so all shards are served by this process's GPU (or host)."""
        if self.failed_over:
            return
        self.failed_over = True
        self.failover_error = f"{type(err).__name__}: {err}"
        self.comm.close_ring()   # ranks still waiting for a command stop
        ex = self.executor
        if getattr(ex, "mesh", None) is self:
            ex.mesh = None
        adopted = 0
        for r, d in sorted(self.peer_dirs.items()):
            if r == self.rank:
                continue
            try:
                adopted += adopt_holder_dir(ex.holder, d)
            except Exception as e:  # noqa: BLE001 - keep serving what we have
                if getattr(ex, "logger", None) is not None:
                    ex.logger.printf("mesh failover: cannot adopt rank %d (%s): %s", r, d, e)
        if ex.gpu is not None:
            ex.gpu.invalidate()
        if getattr(ex, "logger", None) is not None:
            ex.logger.printf("mesh failover after %s: adopted %d fragments", self.failover_error, adopted)
        return adopted

    # ------------------------------------------------------------ worker loop
    def serve(self):
        """Ranks > 0: execute broadcast commands until ``stop``."""
        from pilosa_amd.utils import gctune

        from .collectives import decode

        refreeze = None
        if gctune.enabled():
            # this rank's holder and arena are built: keep them out of the
            # cyclic collector's walk (utils/gctune.py), as the front end does
            gctune.configure()
            gctune.freeze_long_lived()
            refreeze = gctune.Refreezer()
        while True:
            if refreeze is not None:
                refreeze.tick()
            op, payload = self.comm.bcast_bytes()
            if op == OP_STOP:
                while self._pending:
                    self._pending.popleft().wait()
                return
            args = decode(payload) or [""]
            ctx, args = args[0], args[1:]
            with tracing.remote_parent(ctx), tracing.span(f"Mesh.serve.{_OP_NAMES.get(op, op)}", rank=self.rank):
                self._serve_one(op, args)

    def _serve_one(self, op: int, args: list):
        if op not in _PIPELINED:
            self._dispatch(op, args)
            return
        if op == OP_COUNT_TEXT:
            from .collectives import Pending
            index, text, shards, q, seq = args
            t, work = self._count_text_issue(index, text, shards, q, seq)
            h = Pending(self.comm, work, lambda: None, keep=t)
        else:
            h = self._issue(op, args)
        if hasattr(h, "wait"):
            # keep tensors alive until their collective is done; bound the queue
            self._pending.append(h)
        while self._pending and (len(self._pending) > MAX_IN_FLIGHT or self._pending[0].done()):
            self._pending.popleft().wait()

    # ------------------------------------------------------------ all ranks
    def _dispatch(self, op: int, args: list):
        ex = self.executor
        if op == OP_COUNT:
            index, pqls, shards = args
            torch = self.torch
            err = None
            local = [0] * len(pqls)
            try:
                local = self._local_counts(index, pqls, self.owned(shards))
            except Exception as e:  # noqa: BLE001 - flagged in the reduced tensor below
                err = e
            if self.comm.board and len(pqls) <= 1024:
                # host-side counts: the shared-memory results board, no
                # collective (the size test is the command's, so every rank
                # takes the same path; 1024 counts fit an entry)
                from .collectives import RemoteError, decode, encode
                got = self.comm.board_gather(encode([[int(x) for x in local],
                                                     f"{type(err).__name__}: {err}" if err is not None else ""]))
                if not self.is_frontend:
                    return None
                parts = [decode(b) for b in got.result()]
                errs = [RemoteError(e) for _, e in parts if e]
                if errs:
                    raise MeshError(str(errs[0]))
                return [sum(int(p[0][i]) for p in parts) for i in range(len(pqls))]
            t = torch.tensor(list(local) + [1 if err is not None else 0], dtype=torch.int64, device=self.device)
            self.comm.all_reduce(t)
            out = [int(x) for x in t.cpu().tolist()]
            if out[-1]:
                parts = self._gather(err)
                if self.is_frontend:
                    _raise_remote(parts)
            return out[:-1]
        mine = None
        try:
            if op == OP_WRITE:
                index, pql, shard, optd = args
                if self.owner(shard) == self.rank:
                    mine = self._local_call(index, pql, [shard], optd)
            elif op == OP_IMPORT:
                what, index, field, shard, payload = args
                if self.owner(shard) == self.rank:
                    self._local_import(what, index, field, shard, payload)
            elif op == OP_SCHEMA:
                if not self.is_frontend:
                    ex.holder.apply_schema(args[0])
            elif op == OP_DEL_INDEX:
                if not self.is_frontend and ex.holder.index(args[0]) is not None:
                    ex.holder.delete_index(args[0])
            elif op == OP_DEL_FIELD:
                if not self.is_frontend:
                    idx = ex.holder.index(args[0])
                    if idx is not None and idx.field(args[1]) is not None:
                        idx.delete_field(args[1])
            elif op == OP_ERRORS:
                mine = self._errors.pop(int(args[0]), None)
            elif op == OP_SHARDSET:
                sid, shards = int(args[0]), [int(x) for x in args[1]]
                self._sets_by_id[sid] = (shards, self.owned(shards))
            elif op == OP_TOPN_CAND:
                self._topn_cand_refresh(*args)
            elif op == OP_TOPN_SPACES:
                index, fnames, shards = args
                self._topn_spaces_refresh(index, fnames, self.owned(shards))
            elif op == OP_RECALC:
                ex.holder.recalculate_caches()
            elif op == OP_SYNC:
                while self._pending:
                    self._pending.popleft().wait()
                if self.device.type == "cuda":
                    self.torch.cuda.synchronize(self.device)
                import time
                mine = time.perf_counter_ns()
            elif op == OP_SHARDS:
                mine = {name: idx.available_shards() for name, idx in ex.holder.indexes.items()}
                if self.is_frontend:
                    mine = {name: sorted({s for f in idx.fields.values() for s in f.local_shards})
                            for name, idx in ex.holder.indexes.items()}
            else:
                raise MeshError(f"unknown mesh command {op!r}")
        except Exception as e:  # noqa: BLE001 - reported through the gather below
            if isinstance(e, MeshError) and "unknown mesh command" in str(e):
                raise
            mine = e
        parts = self._gather(mine)
        if self.is_frontend:
            _raise_remote(parts)
        return parts

    def _issue(self, op: int, args: list):
        """This rank's share of a pipelined operation, up to the start of its
        last collective: a Pending (or a plain value when nothing is left in
        flight).  Any failure of the local work travels as the rank's partial
        (OP_CALL) or as a declined readiness vote (OP_TOPN), never as a
        missing collective."""
        from .collectives import decode_partial, encode_partial, encode_row_block

        if op == OP_TOPN:
            return self._topn_batch_local(*args)
        if op == OP_TOPN_PLAIN:
            return self._topn_plain_local(*args)
        if op != OP_CALL:
            raise MeshError(f"mesh command {op!r} is not pipelined")
        index, pql, shards, optd, cap = args
        try:
            mine = self._local_call(index, pql, self.owned(shards), optd)
        except Exception as e:  # noqa: BLE001 - reported through the gather below
            mine = e
        from pilosa_amd.ops.device import DeviceRowBlock

        from .collectives import Overflow
        if int(cap) == 0:
            # results board: the partial as host bytes into this rank's slot
            import numpy as np
            w = encode_row_block(mine, self.device).cpu().numpy() if isinstance(mine, DeviceRowBlock) else \
                encode_partial(mine)

            def decode_board(ps):
                if isinstance(ps, Overflow) or ps is None:
                    return ps
                self._call_longest = max(len(b) for b in ps) // 8 if ps else 0
                return [decode_partial(np.frombuffer(b, dtype=np.int64)) for b in ps]
            return _Chain(self.comm.board_gather(np.ascontiguousarray(w, dtype=np.int64).tobytes()), decode_board)
        if isinstance(mine, DeviceRowBlock):
            t = encode_row_block(mine, self.device)
        else:
            t = self.torch.from_numpy(encode_partial(mine)).to(self.device)

        def decode(ps):
            if isinstance(ps, Overflow):
                return ps
            out = [decode_partial(p.cpu().numpy()) for p in ps]
            self._call_longest = getattr(ps, "longest", 0)
            return out
        return _Chain(self.comm.all_gather_cap_async(t, int(cap)), decode)

    def _refresh_spaces(self, index: str, fnames: List[str], own: List[int], vote: bool = True):
        """Collective refresh of the node row spaces of a TopN batch: every
        rank reports whether its copy is stale (a write moved its own view),
        and if ANY rank says so every rank re-gathers, field by field in the
        same order -- the decision is never rank-local.  ``vote=False``: the
        ranks already agreed to refresh (the folded OP_TOPN vote)."""
        torch = self.torch
        gpu = self.executor.gpu
        if vote:
            stale = 0
            try:
                if gpu is not None and hasattr(gpu, "node_space_stale"):
                    stale = int(any(gpu.node_space_stale(index, f, own) for f in fnames))
            except Exception:  # noqa: BLE001 - a rank that cannot tell asks for a refresh
                stale = 1
            flag = torch.tensor([stale], dtype=torch.int64, device=self.device)
            self.comm.all_reduce(flag)
            if not int(flag.item()):
                return
        if gpu is not None and hasattr(gpu, "refresh_node_spaces"):
            gpu.refresh_node_spaces(index, fnames, own, self.comm)
        else:
            for _ in fnames:   # take part with no rows
                self.comm.all_gather_var(torch.zeros(0, dtype=torch.int64, device=self.device))

    def _topn_cand_refresh(self, index: str, fname: str, sid: int, nreq: int, gen: int):
        """OP_TOPN_CAND on every rank: exactly one candidate-row all-gather
        whatever this rank holds (GpuExecutor.refresh_plain_cand)."""
        gpu = self.executor.gpu
        own = (self._sets_by_id.get(int(sid)) or ((), []))[1]
        if gpu is not None and hasattr(gpu, "refresh_plain_cand"):
            gpu.refresh_plain_cand(index, fname, own, int(sid), int(nreq), int(gen), self.comm)
        else:   # take part with a failed head: the node declines the fused path
            self.comm.all_gather_var(self.torch.tensor([-1, 0], dtype=self.torch.int64, device=self.device))

    def _topn_plain_local(self, index: str, fname: str, ns: List[int], ths: List[int], sid: int, nreq: int,
                          gen: int, U: int):
        """This rank's share of an OP_TOPN_PLAIN batch: its partial and vote
        in the one all-reduce (a rank without the GPU path declines, with a
        buffer of the commanded size)."""
        gpu = self.executor.gpu
        ss = self._sets_by_id.get(int(sid))
        if gpu is None or not hasattr(gpu, "topn_plain_mesh") or ss is None:
            from pilosa_amd.ops.topn_exec import mesh_cache_batch
            return mesh_cache_batch(None, ns, ths, self.comm, None, int(U), declined=1, defer=True,
                                    device=self.device)
        return gpu.topn_plain_mesh(index, fname, ns, ths, ss[1], int(sid), int(nreq), int(gen), int(U), self.comm)

    def _topn_spaces_refresh(self, index: str, fnames: List[str], own: List[int]):
        """OP_TOPN_SPACES on every rank: the node row spaces of ``fnames``
        re-gathered (one all-gather per field, whatever this rank holds)."""
        gpu = self.executor.gpu
        prev = gpu.comm if gpu is not None else None
        try:
            if gpu is not None:
                gpu.comm = self.comm
            self._refresh_spaces(index, fnames, own, vote=False)
        finally:
            if gpu is not None:
                gpu.comm = prev

    @staticmethod
    def _single_src_group(calls) -> bool:
        """Every call a TopN over one src of one field, with no ids= /
        Tanimoto / attribute filter: the batch is one slot-index group, whose
        first collective (the candidate union) can carry the readiness vote.
        Decided from the command text alone, so every rank decides alike."""
        if not calls:
            return False
        fields = set()
        for c in calls:
            if c.name != "TopN" or len(c.children) != 1 or any(
                    k in c.args for k in ("ids", "tanimotoThreshold", "attrName", "attrValues")):
                return False
            fields.add(str(c.args.get("_field") or ""))
        return len(fields) == 1

    def _topn_batch_local(self, index: str, pqls: List[str], shards: List[int]):
        from pilosa_amd.pql import parse_string

        from .collectives import MeshVote

        torch = self.torch
        ex = self.executor
        gpu = ex.gpu
        from pilosa_amd.executor import DEFAULT_FIELD

        own = self.owned(shards)
        calls = []
        try:
            # one request text (parsed once) or the calls printed one by one
            calls = parse_string(pqls).calls if isinstance(pqls, str) else [parse_string(p).calls[0] for p in pqls]
            if not all(c.name == "TopN" for c in calls):
                calls = []
        except Exception:  # noqa: BLE001 - the same text fails on every rank
            calls = []
        # the batch's fields come from the command text: every rank lists the
        # same ones in the same order for the collective space refresh
        fnames = sorted({str(c.args.get("_field") or DEFAULT_FIELD) for c in calls})
        prev = gpu.comm if gpu is not None else None
        if gpu is not None:
            gpu.comm = self.comm

        def ready() -> bool:
            try:
                return bool(calls) and gpu is not None and ex.holder.index(index) is not None and \
                    gpu.topn_batch_ready(index, calls, own)
            except Exception:  # noqa: BLE001 - a rank that cannot take part declines
                return False

        def space_stale() -> int:
            try:
                if gpu is not None and hasattr(gpu, "node_space_stale") and fnames:
                    return int(any(gpu.node_space_stale(index, f, own) for f in fnames))
            except Exception:  # noqa: BLE001 - a rank that cannot tell asks for a refresh
                return 1
            return 0
        try:
            if self._single_src_group(calls):
                # src batch: the vote rides in the candidate union (Comm.union
                # vote=): union + re-count = 2 data collectives in the steady
                # state.  A rank that cannot take part sends its vote in the
                # union and every rank abandons the batch after it.
                vote = 2 if space_stale() else (0 if ready() else 1)
                res = None
                try:
                    if not vote:
                        res = gpu.topn_batch(index, calls, own, defer=True)
                    if res is None:   # declined before its first collective: vote in it
                        self.comm.union(torch.zeros(0, dtype=torch.int64, device=self.device), tag="topn_src",
                                        vote=vote or 1)
                except MeshVote as v:
                    return _VOTES.get(v.kind, "declined")
                return res
            # other shapes: ONE all-reduce (MAX) of [space stale, decline,
            # cand]: the refresh vote and the readiness vote folded together.
            # A rank whose own copy of a node row space is stale cannot judge
            # readiness yet (the slot index depends on the space): it votes
            # stale only, and then every rank refreshes and votes readiness
            # again (a second all-reduce, only after writes moved a row
            # directory).
            stale = space_stale()
            decline = 0 if stale else (0 if ready() else 1)
            # cache-only groups also need this rank's node candidate space
            # (built from its current rank caches): stale = refresh them too
            cand = 1 if stale else 0
            if not stale and not decline and hasattr(gpu, "topn_cand_stale"):
                try:
                    cand = int(gpu.topn_cand_stale(index, calls, own))
                except Exception:  # noqa: BLE001 - a rank that cannot tell asks for a refresh
                    cand = 1
            flag = torch.tensor([stale, decline, cand], dtype=torch.int64, device=self.device)
            self.comm.all_reduce(flag, op=self.dist.ReduceOp.MAX)
            voted_stale, voted_decline, voted_cand = (int(x) for x in flag.cpu().tolist())
            if voted_stale:
                self._refresh_spaces(index, fnames, own, vote=False)
                flag = torch.tensor([0 if ready() else 1], dtype=torch.int64, device=self.device)
                self.comm.all_reduce(flag, op=self.dist.ReduceOp.MAX)
                voted_decline = int(flag.item())
            if voted_decline:
                return None
            if (voted_stale or voted_cand) and hasattr(gpu, "refresh_cand_spaces"):
                gpu.refresh_cand_spaces(index, calls, own, self.comm)
            # the fused-or-not choice of every cache-only group is taken NOW,
            # from the entries every rank holds after the vote (a write on
            # another thread may replace this rank's caches before the batch
            # runs; the captured entries keep the node's collectives paired)
            cands = gpu.capture_cands(index, calls, own) if hasattr(gpu, "capture_cands") else None
            res = gpu.topn_batch(index, calls, own, defer=True, cands=cands) if cands is not None else \
                gpu.topn_batch(index, calls, own, defer=True)
        finally:
            if gpu is not None:
                gpu.comm = prev
        if res is None:   # every rank checked readiness: a decline now would desynchronise
            raise MeshError(f"rank {self.rank}: TopN batch declined after the readiness check")
        return res

    def _count_text_issue(self, index: str, text: str, shards: List[int], q: int, seq: int):
        """This rank's counts for its own shards as a device tensor (plus an
        error flag) and the started all-reduce of it."""
        torch = self.torch
        err = None
        t = None
        try:
            t = self._local_count_text(index, text, self.owned(shards), q)
            if t is None or t.numel() != q:
                raise MeshError(f"rank {self.rank}: {0 if t is None else t.numel()} counts for {q} calls")
        except Exception as e:  # noqa: BLE001 - flagged in the reduced tensor, text via OP_ERRORS
            err = e
            t = torch.zeros(q, dtype=torch.int64, device=self.device)
        if err is not None:
            self._errors[seq] = err
            while len(self._errors) > 64:
                self._errors.pop(next(iter(self._errors)))
        flag = torch.full((1,), 1 if err is not None else 0, dtype=torch.int64, device=self.device)
        tt = torch.cat([t.to(self.device, torch.int64), flag])
        return tt, self.comm.all_reduce_async(tt)

    def _local_count_text(self, index: str, text: str, shards: List[int], q: int):
        torch = self.torch
        ex = self.executor
        if not shards:
            return torch.zeros(q, dtype=torch.int64, device=self.device)
        if ex.holder.index(index) is None:
            raise MeshError(f"index not found on rank {self.rank}: {index}")
        gpu = ex.gpu
        if gpu is not None and hasattr(gpu, "try_count_text"):
            res = gpu.try_count_text(index, text, shards, device_out=True)
            if res is not None:
                return res
        from pilosa_amd.pql import parse_string
        pqls = [str(c) for c in parse_string(text).calls]
        return torch.tensor(self._local_counts(index, pqls, shards), dtype=torch.int64, device=self.device)

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
        if c.name in _ROW_CALLS and ex.gpu is not None and hasattr(ex.gpu, "bitmap_block"):
            # a Row partial stays on the device: its containers go straight
            # into the all-gather (collectives.encode_row_block); the front end
            # attaches row attributes after the reduce, as for any partial.
            # Anything the device declines (or any error) takes the regular
            # path below, which reports exactly what the executor would.
            try:
                blk = ex.gpu.bitmap_block(index, c, list(shards))
                self.row_blocks += 1
                if blk is not None:
                    return blk
                from pilosa_amd.models.row import Row
                return Row()
            except Exception:  # noqa: BLE001 - the regular path answers (or raises the real error)
                pass
        return ex.execute_call(index, c, shards, self._local_opt(optd))

    def _local_counts(self, index: str, pqls: List[str], shards: List[int]) -> List[int]:
        from pilosa_amd.pql import parse_string

        ex = self.executor
        if not shards:
            return [0] * len(pqls)
        if ex.gpu is not None and len(pqls) > 1 and hasattr(ex.gpu, "try_count_text"):
            res = ex.gpu.try_count_text(index, " ".join(pqls), shards)
            if res is not None:
                return [int(x) for x in res]
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


class _Chain:
    """A pending result post-processed by ``fn`` on completion."""

    __slots__ = ("p", "fn")

    def __init__(self, p, fn):
        self.p, self.fn = p, fn

    def wait(self):
        self.p.wait()

    def done(self) -> bool:
        return self.p.done()

    def result(self):
        return self.fn(self.p.result())


def _plain(v):
    """numpy arrays -> lists for the msgpack codec."""
    import numpy as np

    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.integer):
        return int(v)
    return v


def adopt_holder_dir(holder, data_dir: str) -> int:
    """Move every fragment of the holder at ``data_dir`` (another rank's, whose
    process is gone) into ``holder``'s views, lazily opened from their files.
    Returns the number of fragments adopted."""
    from pilosa_amd.models.holder import Holder

    peer = Holder(data_dir, lazy_fragments=True).open()
    n = 0
    for iname, pidx in peer.indexes.items():
        idx = holder.index(iname)
        if idx is None:
            continue
        for fname, pf in pidx.fields.items():
            f = idx.field(fname)
            if f is None:
                continue
            for vname, pv in pf.views.items():
                v = f.create_view_if_not_exists(vname)
                for shard, frag in list(pv.fragments.items()):
                    if shard in v.fragments:
                        continue
                    v.fragments[shard] = frag
                    pv.fragments.pop(shard)
                    f.local_shards.add(int(shard))
                    n += 1
    if n:
        # the peer Holder.open bumped the epoch before the move: bump it again
        # so no available_shards() memo taken meanwhile hides the adopted shards
        from pilosa_amd.models.fragment import bump_shard_epoch
        bump_shard_epoch()
    return n


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


def init_process_group(local_rank: int, backend: Optional[str] = None, timeout_s: float = 120.0):
    """One process per GPU: RCCL ("nccl") when GPUs are visible, else gloo,
    with a collective timeout (parallel/collectives.py init)."""
    from .collectives import init

    return init(backend, local_rank, timeout_s)


def rank_data_dir(data_dir: str, rank: int) -> str:
    """Rank 0 uses the node's data dir; rank r keeps its shards in ``.rank<r>``
    inside it (dot-dirs are skipped by the holder scan)."""
    import os

    return data_dir if rank == 0 else os.path.join(data_dir, f".rank{rank}")


def run_worker(data_dir: str, gpu_mode: str = "auto", block: int = 1, logger=None, timeout_s: float = 120.0) -> int:
    """Entry point of ranks > 0 of a multi-GPU server (``pilosa_amd server``
    under ``torch.distributed.run``): own holder + GPU engine, serve the mesh."""
    import torch
    import torch.distributed as dist

    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder

    rank, world, local = dist_env()
    init_process_group(local, timeout_s=timeout_s)
    use_gpu = (gpu_mode or "auto").lower() not in ("off", "none", "cpu") and torch.cuda.is_available()
    holder = Holder(rank_data_dir(data_dir, rank), lazy_fragments=use_gpu).open()
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
