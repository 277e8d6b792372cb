"""Tensor-only collectives for the intra-node mesh (RCCL over xGMI on the GPU
box, gloo for CPU tests) and a compact binary codec for partial results.

Reference analog: the coordinator fan-out/reduce of executor.go:2458-2555 and
the QueryResponse protobuf a remote node returns (internal/public.proto).  Here
the ranks of one node exchange only tensors:

* ``bcast_bytes``  command broadcast: an int64 header (op, length) then the
  payload as a uint8 tensor (2 collectives, no pickling);
* ``all_reduce``   counts / sums (int64) with an error flag folded into the
  same tensor, so a healthy Count batch costs one collective;
* ``all_gather_var`` variable-length 1-D tensors (sizes first, then one padded
  all_gather): TopN candidate ids, encoded partial results;
* ``union``        sorted distinct values over ranks (TopN phase-1 candidate
  sets: only membership matters because phase 2 re-counts exactly, so fixed-k
  candidate lists are gathered instead of a dense [Q x rows] all-reduce).

Every collective runs under the process group's timeout (``init(timeout=)``;
RCCL aborts the communicator when it expires), and a failure marks the Comm
broken so callers can fail over instead of hanging.

Partial call results travel as typed int64 tensors (``encode_partial``:
ValCount, Pair, TopN pairs, row ids, GroupBy matrices, Row segments as
roaring bytes); results with strings and errors fall back to msgpack (a
schema-less binary format; no code is executed on decode) with extension
types for the executor's result objects, packed into the same tensor.
"""
from __future__ import annotations

import datetime as _dt
import os
from typing import List, Optional, Sequence

import numpy as np

from pilosa_amd.utils import tracing


BCAST_INLINE = 4080          # command payload bytes carried in the header broadcast
RING_SLOTS = 64              # commands a reader may lag behind the front end
RING_SLOT_BYTES = 1 << 18    # a Count text of ~5k calls fits one slot; longer ones follow on gloo
RING_BIG = 1 << 40           # op flag: the payload follows on the command group
RING_SPIN_US = 300.0         # a waiting rank spins this long before it sleeps on the futex
RING_PUBLISH_TIMEOUT_S = 120.0
RING_BOARD_BYTES = 1 << 14   # per-rank result bytes of the results board (one-shot gather of small partials)
BOARD_TIMEOUT_S = 120.0
UNION_MIN_CAP = 1024         # initial per-rank pad of a speculative union gather


class CommError(RuntimeError):
    """A collective failed or timed out; the mesh must fail over."""


class GatherParts(list):
    """The per-rank tensors of a fixed-capacity gather, with the largest
    rank's length (the caller's capacity policy reads it)."""

    def __init__(self, parts, longest: int):
        super().__init__(parts)
        self.longest = int(longest)


class Overflow:
    """A speculative fixed-capacity gather some rank did not fit into:
    ``need`` words would have (Comm.all_gather_cap_async)."""

    __slots__ = ("need",)

    def __init__(self, need: int):
        self.need = int(need)


class MeshVote(Exception):
    """Some rank voted against a batch inside one of its data collectives
    (``Comm.union(vote=)``): every rank raises it after the same collective,
    so all abandon the batch at the same point.  ``kind`` is the largest
    vote: 1 = declined (the general path answers), 2 = a stale node row space
    (refresh, then re-run)."""

    def __init__(self, kind: int):
        super().__init__(f"mesh batch vote {kind}")
        self.kind = int(kind)


class Comm:
    def __init__(self, group=None, device=None, host_copies: bool = False, ctrl_group=None):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.device = torch.device(device)
        # gloo rehearsal of a GPU run: collectives on host copies
        self.host_copies = host_copies or (backend == "gloo" and self.device.type == "cuda")
        self.backend = backend
        self.broken: Optional[BaseException] = None
        self.calls = 0
        self.data_calls = 0       # collectives on the data group (device tensors on RCCL)
        self.union_retries = 0    # speculative union gathers that overflowed their pad
        self._union_cap: dict = {}
        # command channel: a gloo group of its own, so a command broadcast is
        # never queued behind the data collectives of batches still in flight
        self.ctrl = ctrl_group
        self.ctrl_device = torch.device("cpu") if ctrl_group is not None else self.device
        # commands through a shared-memory ring (native/shmring.cpp) once
        # attach_ring() set it up: no TCP round trip per request, and an idle
        # node's ranks wait without a collective timeout
        self.ring = None
        self.ring_reader = -1
        self.ring_msgs = 0
        self.cmd_seq = -1          # sequence number of the last command sent / received on the ring
        self.board_gathers = 0
        self.use_board = True      # small OP_CALL partials through the results board (when the ring has one)
        self._ar_opts: dict = {}
        # RCCL all-reduces of all_reduce_async on the caller's stream
        # (asyncOp = False: no event hop to the process group's stream and
        # back) instead of the process group's own stream
        self.ar_current_stream = backend == "nccl" and os.environ.get("PILOSA_MESH_AR_STREAM", "pg") == "current"

    # ------------------------------------------------------------ guard
    def _guard(self, fn, *a, **kw):
        if self.broken is not None:
            raise CommError(f"communicator broken: {self.broken}")
        self.calls += 1
        if "group" in kw and (self.ctrl is None or kw["group"] is not self.ctrl):
            self.data_calls += 1
        try:
            if tracing.enabled():
                # one span per collective; RCCL ones are HIP-event timed (the
                # collective kernel on the device), async ones time the issue
                dev = self.device.type == "cuda" and not self.host_copies and kw.get("group") is not self.ctrl
                with tracing.span(f"Comm.{getattr(fn, '__name__', 'op')}", gpu=dev and not kw.get("async_op"),
                                  ranks=self.world, control=kw.get("group") is self.ctrl):
                    return fn(*a, **kw)
            return fn(*a, **kw)
        except Exception as e:  # noqa: BLE001 - timeouts / peer loss surface here
            self.broken = e
            raise CommError(f"collective failed: {type(e).__name__}: {e}") from e

    def _on(self, t):
        return t.cpu() if self.host_copies and t.device.type != "cpu" else t

    # ------------------------------------------------------------ primitives
    def all_reduce(self, t, op=None):
        """In-place sum (or ``op``) of ``t`` over the ranks."""
        op = self.dist.ReduceOp.SUM if op is None else op
        h = self._on(t)
        self._guard(self.dist.all_reduce, h, op=op, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def broadcast(self, t, src: int = 0):
        h = self._on(t)
        self._guard(self.dist.broadcast, h, src=src, group=self.group)
        if h is not t:
            t.copy_(h)
        return t

    def attach_ring(self, nslots: int = RING_SLOTS, slot_bytes: int = RING_SLOT_BYTES) -> bool:
        """Collective on every rank (in the same order as the other setup
        collectives): rank 0 creates the command ring in /dev/shm, names it
        over the command group, the other ranks attach as readers, and all
        agree (one all-reduce) that every rank could -- else every rank keeps
        the gloo broadcast.  Returns whether the ring is in use."""
        import os
        import uuid
        ring = None
        name = ""
        if self.rank == 0 and os.environ.get("PILOSA_MESH_RING", "1") != "0":
            try:
                from pilosa_amd import _shmring
                name = f"/pilosa_mesh_{os.getpid()}_{uuid.uuid4().hex[:10]}"
                ring = _shmring.Ring(name, True, nslots=nslots, slot_bytes=slot_bytes,
                                     nreaders=max(0, self.world - 1), board_bytes=RING_BOARD_BYTES)
            except Exception:  # noqa: BLE001 - no ring: the gloo broadcast stays
                ring, name = None, ""
        _, got = self._bcast_bytes_group(0, name.encode())
        name = got.decode()
        ok = 1
        if name and self.rank != 0:
            try:
                from pilosa_amd import _shmring
                ring = _shmring.Ring(name, False)
                ring.attach(self.rank - 1)
            except Exception:  # noqa: BLE001 - e.g. another host: everyone falls back
                ring, ok = None, 0
        if not name:
            ok = 0
        flag = self.torch.tensor([ok], dtype=self.torch.int64)
        if self.ctrl is not None:
            self._guard(self.dist.all_reduce, flag, op=self.dist.ReduceOp.MIN, group=self.ctrl)
        elif self.world > 1:
            self.all_reduce(flag.to(self.device), op=self.dist.ReduceOp.MIN)
            flag = flag.cpu()
        if int(flag.item()) and ring is not None:
            self.ring = ring
            self.ring_reader = self.rank - 1
            return True
        return False

    def close_ring(self):
        """Front end: wake every reader with an error (shutdown / failover)."""
        if self.ring is not None and self.rank == 0:
            try:
                self.ring.close()
            except Exception:  # noqa: BLE001
                pass

    def bcast_bytes(self, op: int = 0, payload: bytes = b"", src: int = 0):
        """Rank ``src`` sends (op, payload); every rank returns them: through
        the shared-memory command ring when the node has one (a payload
        larger than a slot follows on the command group), else on the
        command group (gloo) or the data group."""
        if self.ring is None or src != 0:
            return self._bcast_bytes_group(op, payload, src)
        if self.broken is not None:
            raise CommError(f"communicator broken: {self.broken}")
        try:
            if self.rank == src:
                big = len(payload) > self.ring.slot_bytes
                if tracing.enabled():
                    with tracing.span("Comm.command", ranks=self.world, bytes=len(payload)):
                        self.cmd_seq = self.ring.publish(int(op) | RING_BIG if big else int(op),
                                                         b"" if big else bytes(payload), RING_PUBLISH_TIMEOUT_S)
                else:
                    self.cmd_seq = self.ring.publish(int(op) | RING_BIG if big else int(op),
                                                     b"" if big else bytes(payload), RING_PUBLISH_TIMEOUT_S)
                self.ring_msgs += 1
                if big:
                    self._bcast_bytes_group(op, payload, src)
                return int(op), payload
            o, data, self.cmd_seq = self.ring.read(self.ring_reader, RING_SPIN_US)
        except (RuntimeError, ValueError) as e:
            self.broken = e
            raise CommError(f"command ring failed: {e}") from e
        self.ring_msgs += 1
        if o & RING_BIG:
            return self._bcast_bytes_group(o & ~RING_BIG, b"", src)
        return int(o), data

    def _bcast_bytes_group(self, op: int = 0, payload: bytes = b"", src: int = 0):
        torch = self.torch
        dev = self.ctrl_device

        def bc(t):
            if self.ctrl is None:
                return self.broadcast(t, src)
            self._guard(self.dist.broadcast, t, src=src, group=self.ctrl)
            return t
        # one fixed-size broadcast carries (op, length) and a payload of up to
        # BCAST_INLINE bytes (every TopN batch, most calls); longer payloads
        # (Count texts of thousands of calls) follow in a second broadcast
        words = 2 + BCAST_INLINE // 8
        if self.rank == src:
            h = np.zeros(words, np.int64)
            h[0], h[1] = int(op), len(payload)
            if len(payload) <= BCAST_INLINE:
                h[2:].view(np.uint8)[:len(payload)] = np.frombuffer(payload, np.uint8)
            hdr = torch.from_numpy(h).to(dev)
        else:
            hdr = torch.empty(words, dtype=torch.int64, device=dev)
        bc(hdr)
        hh = hdr.cpu().numpy()
        op_, n = int(hh[0]), int(hh[1])
        if n == 0:
            return op_, b""
        if n <= BCAST_INLINE:
            return op_, hh[2:].view(np.uint8)[:n].tobytes()
        buf = torch.empty(n, dtype=torch.uint8, device=dev)
        if self.rank == src:
            buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
        bc(buf)
        return op_, buf.cpu().numpy().tobytes()

    def all_reduce_async(self, t, op=None):
        """Start an in-place sum of ``t``; returns a handle for :meth:`wait`.
        RCCL enqueues it behind the work already on the caller's stream and
        the host goes on (the next batch can be planned and launched)."""
        op = self.dist.ReduceOp.SUM if op is None else op
        if self.host_copies:   # gloo rehearsal of a GPU run: host copies, synchronous
            self.all_reduce(t, op)
            return None
        pg = self._pg()
        if pg is not None and not tracing.enabled():
            # the process group's own entry point: what dist.all_reduce does
            # after its Python-side checks and logging (~15 us a call, which a
            # sub-millisecond TopN request pays once)
            opts = self._ar_opts.get(op)
            if opts is None:
                opts = self.dist.AllreduceOptions()
                opts.reduceOp = op
                opts.asyncOp = not self.ar_current_stream
                self._ar_opts[op] = opts
            if self.broken is not None:
                raise CommError(f"communicator broken: {self.broken}")
            self.calls += 1
            self.data_calls += 1
            try:
                return pg.allreduce([t], opts)
            except Exception as e:  # noqa: BLE001 - timeouts / peer loss surface here
                self.broken = e
                raise CommError(f"collective failed: {type(e).__name__}: {e}") from e
        return self._guard(self.dist.all_reduce, t, op=op, group=self.group, async_op=True)

    def _pg(self):
        """The data group's ProcessGroup object (None: use the dist API)."""
        pg = getattr(self, "_pg_obj", False)
        if pg is False:
            try:
                pg = self.group if self.group is not None else self.dist.group.WORLD
                if not hasattr(pg, "allreduce"):
                    pg = None
            except Exception:  # noqa: BLE001
                pg = None
            self._pg_obj = pg
        return pg

    def wait(self, work):
        """Complete a collective started by :meth:`all_reduce_async`."""
        if work is not None:
            self._guard(work.wait)

    @staticmethod
    def done(work) -> bool:
        return work is None or work.is_completed()

    def all_gather_var(self, t) -> List:
        """1-D tensors of any length per rank -> list of per-rank tensors."""
        torch = self.torch
        t = t.reshape(-1)
        n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        hs = [self._on(x) for x in sizes]
        self._guard(self.dist.all_gather, hs, self._on(n), group=self.group)
        lens = [int(x.item()) for x in hs]
        m = max(lens) if lens else 0
        if m == 0:
            return [t[:0] for _ in range(self.world)]
        pad = torch.zeros(m, dtype=t.dtype, device=t.device)
        pad[:t.numel()] = t
        outs = [torch.empty(m, dtype=t.dtype, device=t.device) for _ in range(self.world)]
        ho = [self._on(x) for x in outs]
        self._guard(self.dist.all_gather, ho, self._on(pad), group=self.group)
        return [x[:k].to(t.device) for x, k in zip(ho, lens)]

    def all_gather_var_async(self, t) -> "Pending":
        """Like :meth:`all_gather_var`, with the data all-gather left in
        flight: the sizes travel first (one tiny synchronous all-gather, so
        every rank pads alike), then the padded all-gather is started and
        the returned :class:`Pending` yields the per-rank tensors."""
        torch = self.torch
        t = t.reshape(-1)
        n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        hs = [self._on(x) for x in sizes]
        self._guard(self.dist.all_gather, hs, self._on(n), group=self.group)
        lens = [int(x.item()) for x in hs]
        m = max(lens) if lens else 0
        if m == 0:
            return Pending(self, None, lambda: [t[:0] for _ in range(self.world)])
        pad = torch.zeros(m, dtype=t.dtype, device=t.device)
        pad[:t.numel()] = t
        outs = [torch.empty(m, dtype=t.dtype, device=t.device) for _ in range(self.world)]
        if self.host_copies:   # gloo rehearsal of a GPU run: host copies, synchronous
            ho = [self._on(x) for x in outs]
            self._guard(self.dist.all_gather, ho, self._on(pad), group=self.group)
            return Pending(self, None, lambda: [x[:k].to(t.device) for x, k in zip(ho, lens)])
        work = self._guard(self.dist.all_gather, outs, pad, group=self.group, async_op=True)
        return Pending(self, work, lambda: [x[:k] for x, k in zip(outs, lens)], keep=(pad, outs))

    @property
    def board(self) -> bool:
        """The node has a shared-memory results board (Comm.board_gather)."""
        return self.use_board and self.ring is not None and bool(getattr(self.ring, "board_bytes", 0))

    def board_gather(self, payload: bytes) -> "BoardPending":
        """One-shot gather of a small host-side partial of the current
        command (the one bcast_bytes last delivered) through the results
        board in shared memory: every rank writes its bytes into its own
        slot, the front end reads them all -- no collective, no device copy,
        no ring of hops (tiny partials off the ring; the
        reference's per-node reduce, executor.go:2487-2516).  Workers return
        at once; the front end's pending result is every rank's bytes, or an
        :class:`Overflow` when some rank's did not fit an entry."""
        if self.broken is not None:
            raise CommError(f"communicator broken: {self.broken}")
        seq = self.cmd_seq
        try:
            self.ring.post(self.rank, seq, payload)
        except (RuntimeError, ValueError) as e:
            self.broken = e
            raise CommError(f"results board failed: {e}") from e
        self.board_gathers += 1
        return BoardPending(self, seq if self.rank == 0 else None)

    def all_gather_cap_async(self, t, cap: int) -> "Pending":
        """Variable-length 1-D int64 tensors of every rank in ONE all-gather
        with no size exchange first: each rank sends ``[len, values...,
        padding]`` padded to ``cap`` words (the capacity comes from the
        command, so every rank pads alike), or ``[-len]`` when its tensor does
        not fit.  The pending result is the list of per-rank tensors, or an
        :class:`Overflow` naming the capacity that would fit -- the caller
        re-issues the whole operation with it (one more command, never a
        collective inside a completion)."""
        torch = self.torch
        t = t.reshape(-1).to(torch.int64)
        n = int(t.numel())
        cap = max(1, int(cap))
        buf = torch.zeros(cap + 1, dtype=torch.int64, device=t.device)
        if n <= cap:
            buf[0] = n
            if n:
                buf[1:1 + n] = t
        else:
            buf[0] = -n
        out = torch.empty(self.world * (cap + 1), dtype=torch.int64, device=t.device)

        def finish(ho):
            ho = ho.view(self.world, cap + 1)
            lens = ho[:, 0].cpu().numpy()
            if len(lens) and int(lens.min()) < 0:
                return Overflow(int(np.abs(lens).max()))
            return GatherParts([ho[r, 1:1 + int(k)] for r, k in enumerate(lens)], int(lens.max()) if len(lens) else 0)
        if self.host_copies:   # gloo rehearsal of a GPU run: host copies, synchronous
            ho = self._on(out)
            self._guard(self.dist.all_gather_into_tensor, ho, self._on(buf), group=self.group)
            return Pending(self, None, lambda: finish(ho))
        work = self._guard(self.dist.all_gather_into_tensor, out, buf, group=self.group, async_op=True)
        return Pending(self, work, lambda: finish(out), keep=(buf, out))

    def union(self, t, tag: str = "union", vote: int = 0):
        """Sorted distinct values of int64 ``t`` over all ranks (the same on
        every rank).  One all-gather in the steady state: every rank sends
        ``[count, values..., padding]`` padded to a capacity all ranks share
        (per ``tag``), so no size exchange has to finish -- with its host
        sync -- before the data moves.  Every rank reads every count from the
        gather, so the ranks agree when one overflowed the pad: they then
        re-gather at the exact size (one more collective) and raise the
        capacity alike for the next call.

        ``vote`` > 0: this rank cannot take part in the batch (1 declined, 2
        its node row space is stale); it sends ``-vote`` in place of its
        count, and every rank -- reading the counts it already reads --
        raises :class:`MeshVote` after this one collective.  A batch's
        readiness vote thus needs no collective of its own."""
        torch = self.torch
        t = t.reshape(-1).to(torch.int64)
        n = int(t.numel()) if not vote else 0
        cap = self._union_cap.get(tag, (UNION_MIN_CAP, 0))
        cap, quiet = cap
        buf = torch.empty(cap + 1, dtype=torch.int64, device=t.device)
        buf[0] = n if not vote else -int(vote)
        k = min(n, cap)
        if k:
            buf[1:1 + k] = t[:k]
        out = torch.empty(self.world * (cap + 1), dtype=torch.int64, device=t.device)
        ho = self._on(out)
        self._guard(self.dist.all_gather_into_tensor, ho, self._on(buf), group=self.group)
        ho = ho.view(self.world, cap + 1)
        counts = ho[:, 0].cpu().numpy()
        if len(counts) and int(counts.min()) < 0:
            raise MeshVote(-int(counts.min()))
        mx = int(counts.max()) if len(counts) else 0
        # capacity for the next call: grow past the largest count (with room),
        # halve after a long quiet spell well below it; same on every rank
        if mx > cap:
            ncap = 1 << max(UNION_MIN_CAP.bit_length() - 1, int(mx + mx // 4).bit_length())
            self._union_cap[tag] = (ncap, 0)
        elif mx * 8 < cap and cap > UNION_MIN_CAP:
            quiet += 1
            self._union_cap[tag] = (cap // 2, 0) if quiet >= 32 else (cap, quiet)
        else:
            self._union_cap[tag] = (cap, 0)
        if mx > cap:
            self.union_retries += 1
            parts = self.all_gather_var(t)
            return torch.unique(torch.cat(parts)) if parts else t
        ho = ho.to(t.device)
        keep = torch.arange(cap, device=t.device)[None, :] < ho[:, :1]
        return torch.unique(ho[:, 1:][keep])

    def gather_bytes(self, payload: bytes) -> List[bytes]:
        """Every rank's bytes, on every rank (small control-plane payloads)."""
        torch = self.torch
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if payload else torch.zeros(0, dtype=torch.uint8)
        parts = self.all_gather_var(t.to(self.device))
        return [p.cpu().numpy().tobytes() for p in parts]

    def gather_partials(self, obj) -> list:
        """Every rank's partial call result, on every rank: the typed int64
        encoding (encode_partial) of each rank travels in ONE variable-length
        all-gather of device tensors (RCCL over xGMI on a GPU node)."""
        torch = self.torch
        t = torch.from_numpy(encode_partial(obj)).to(self.device)
        return [decode_partial(p.cpu().numpy()) for p in self.all_gather_var(t)]

    def barrier(self):
        self.all_reduce(self.torch.zeros(1, dtype=self.torch.int64, device=self.device))


class Pending:
    """A result whose last collective is still in flight (the mesh keeps
    several requests in flight: parallel/mesh.py).  ``wait()`` completes the
    collective only (what a worker rank needs before it drops the tensors);
    ``result()`` also runs ``finish`` (decode / trim on the front end).
    Nothing after the collective's start may issue another collective, so
    completions can run in any order, outside the mesh lock."""

    __slots__ = ("_comm", "_work", "_finish", "_keep")

    def __init__(self, comm, work, finish, keep=None):
        self._comm, self._work, self._finish, self._keep = comm, work, finish, keep

    def wait(self):
        if self._work is not None:
            w, self._work = self._work, None
            self._comm.wait(w)
        self._keep = None

    def done(self) -> bool:
        return self._work is None or Comm.done(self._work)

    def result(self):
        self.wait()
        return self._finish()


class BoardPending:
    """A results-board gather (Comm.board_gather): nothing to wait for on a
    worker; on the front end ``result()`` collects every rank's bytes."""

    __slots__ = ("_comm", "_seq", "_got")

    def __init__(self, comm, seq):
        self._comm, self._seq, self._got = comm, seq, None

    def wait(self):
        pass

    def done(self) -> bool:
        return True

    def result(self):
        if self._seq is None:
            return None
        if self._got is None:
            try:
                got = self._comm.ring.collect(self._seq, BOARD_TIMEOUT_S, RING_SPIN_US)
            except (RuntimeError, ValueError) as e:
                self._comm.broken = e
                raise CommError(f"results board failed: {e}") from e
            over = [-x for x in got if isinstance(x, int)]
            self._got = Overflow(max(over) // 8 + 1) if over else got
        return self._got


class PendingAll:
    """Several :class:`Pending` parts finished together by ``combine``."""

    __slots__ = ("parts", "combine")

    def __init__(self, parts, combine):
        self.parts, self.combine = list(parts), combine

    def wait(self):
        for p in self.parts:
            if hasattr(p, "wait"):
                p.wait()

    def done(self) -> bool:
        return all(p.done() for p in self.parts if hasattr(p, "done"))

    def result(self):
        return self.combine([p.result() if hasattr(p, "result") else p for p in self.parts])


def resolve(x):
    """The value of a possibly pending result."""
    return x.result() if callable(getattr(x, "result", None)) and callable(getattr(x, "wait", None)) else x


def init(backend: Optional[str] = None, local_rank: int = 0, timeout_s: float = 120.0):
    """One process per GPU: RCCL ("nccl") when GPUs are visible, else gloo;
    collectives time out after ``timeout_s`` (RCCL: the communicator aborts
    and the waiting call raises)."""
    import os

    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_backend()
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    to = _dt.timedelta(seconds=float(timeout_s))
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=to)
    else:
        dist.init_process_group(backend, timeout=to)
    return backend


# ---------------------------------------------------------------- result codec
_EXT_ROW, _EXT_PAIR, _EXT_VALCOUNT, _EXT_GROUPCOUNT, _EXT_ROWIDS, _EXT_FIELDROW, _EXT_ERR, _EXT_U64 = range(1, 9)


def _default(o):
    import msgpack

    from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
    from pilosa_amd.models.cache import Pair
    from pilosa_amd.models.row import Row

    if isinstance(o, Row):
        segs = {int(s): bm.to_bytes() for s, bm in o.segments.items()}
        return msgpack.ExtType(_EXT_ROW, msgpack.packb([segs, o.attrs, o.keys], default=_default))
    if isinstance(o, Pair):
        return msgpack.ExtType(_EXT_PAIR, msgpack.packb([int(o.id), int(o.count), getattr(o, "key", "") or ""]))
    if isinstance(o, ValCount):
        return msgpack.ExtType(_EXT_VALCOUNT, msgpack.packb([int(o.val), int(o.count)]))
    if isinstance(o, GroupCount):
        return msgpack.ExtType(_EXT_GROUPCOUNT, msgpack.packb([[_default(g) for g in o.group], int(o.count)],
                                                              default=_default))
    if isinstance(o, RowIdentifiers):
        return msgpack.ExtType(_EXT_ROWIDS, msgpack.packb([list(o.rows), o.keys]))
    if isinstance(o, FieldRow):
        return msgpack.ExtType(_EXT_FIELDROW, msgpack.packb([o.field, int(o.row_id), o.row_key]))
    if isinstance(o, BaseException):
        return msgpack.ExtType(_EXT_ERR, msgpack.packb(f"{type(o).__name__}: {o}"))
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    raise TypeError(f"cannot encode {type(o).__name__}")


def _ext_hook(code, data):
    import msgpack

    from pilosa_amd import _roaring
    from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
    from pilosa_amd.models.cache import Pair
    from pilosa_amd.models.row import Row

    v = msgpack.unpackb(data, ext_hook=_ext_hook, strict_map_key=False)
    if code == _EXT_ROW:
        segs, attrs, keys = v
        r = Row(segments={int(s): _roaring.Bitmap.from_bytes(b) for s, b in segs.items()})
        r.attrs, r.keys = attrs, keys
        return r
    if code == _EXT_PAIR:
        p = Pair(v[0], v[1])
        if v[2]:
            p.key = v[2]
        return p
    if code == _EXT_VALCOUNT:
        return ValCount(v[0], v[1])
    if code == _EXT_GROUPCOUNT:
        return GroupCount(list(v[0]), v[1])
    if code == _EXT_ROWIDS:
        return RowIdentifiers(v[0], v[1])
    if code == _EXT_FIELDROW:
        return FieldRow(v[0], v[1], v[2])
    if code == _EXT_ERR:
        return RemoteError(v)
    return msgpack.ExtType(code, data)


class RemoteError(Exception):
    """An error raised on another rank, carried back in a partial result."""


def encode(obj) -> bytes:
    import msgpack
    return msgpack.packb(obj, default=_default, strict_types=False, use_bin_type=True)


def decode(data: bytes):
    import msgpack
    if not data:
        return None
    return msgpack.unpackb(data, ext_hook=_ext_hook, strict_map_key=False, raw=False)


# ---------------------------------------------------------------- typed partials
# A rank's partial result of one call as a flat int64 tensor, so the mesh
# moves call results as tensors (one all_gather_var, i.e. RCCL on the GPU
# box) and the front end decodes them with numpy views instead of walking a
# msgpack object tree.  Layout: [tag, ...payload].  Shapes with strings (keys,
# attributes), errors and anything else ride as TAG_MSGPACK (the bytes
# packed into int64 words), so every rank always takes part in the same one
# collective whatever it produced (the reference's QueryResponse per node,
# internal/public.proto, reduced by executor.go mapReduce).
(TAG_NONE, TAG_MSGPACK, TAG_VALCOUNT, TAG_PAIR, TAG_PAIRS, TAG_ROWIDS, TAG_GROUPS, TAG_ROW,
 TAG_INT, TAG_BOOL, TAG_DEVROW) = range(11)


def encode_row_block(blk, device):
    """A rank's Row partial left on its GPU (ops/device.DeviceRowBlock) ->
    one device int64 tensor, built with device copies only: [TAG_DEVROW,
    nblocks] then per block (the row, then its Shift spill) [S, payload
    words, shards[S], counts (int32 pairs), u16 offsets[S*16], payload].
    The rank never copies its row to the host or serialises it; the front
    end decodes every rank's containers with one D2H (decode_partial)."""
    import torch

    parts = []
    blocks = [b for b in (blk, blk.spill) if b is not None]
    parts.append(torch.tensor([TAG_DEVROW, len(blocks)], dtype=torch.int64))
    dev_parts = []
    for b in blocks:
        S = len(b.shards)
        pay = b.payload.reshape(-1)
        if pay.numel() % 4:
            pay = torch.cat([pay, pay.new_zeros(4 - pay.numel() % 4)])
        hdr = torch.tensor([S, pay.numel() // 4] + list(b.shards), dtype=torch.int64)
        dev_parts += [hdr.to(device, non_blocking=True), b.counts.reshape(-1).contiguous().view(torch.int64),
                      b.offs.reshape(-1).to(torch.int64), pay.contiguous().view(torch.int64)]
    return torch.cat([parts[0].to(device, non_blocking=True)] + dev_parts)


def _bytes_to_words(b: bytes) -> np.ndarray:
    pad = (-len(b)) % 8
    return np.frombuffer(b + b"\0" * pad, dtype=np.int64)


def _words_to_bytes(w: np.ndarray, n: int) -> bytes:
    return np.ascontiguousarray(w, dtype=np.int64).tobytes()[:n]


def encode_partial(obj) -> np.ndarray:
    """One rank's partial result -> int64[...] (see the TAG_ layout)."""
    from pilosa_amd.executor import GroupCount, RowIdentifiers, ValCount
    from pilosa_amd.models.cache import Pair, PairArray
    from pilosa_amd.models.row import Row

    def msg():
        b = encode(obj)
        return np.concatenate([np.array([TAG_MSGPACK, len(b)], np.int64), _bytes_to_words(b)])

    if obj is None:
        return np.array([TAG_NONE], np.int64)
    if isinstance(obj, bool):
        return np.array([TAG_BOOL, int(obj)], np.int64)
    if isinstance(obj, (int, np.integer)) and -(1 << 63) <= int(obj) < (1 << 63):
        return np.array([TAG_INT, int(obj)], np.int64)
    if isinstance(obj, ValCount):
        return np.array([TAG_VALCOUNT, obj.val, obj.count], np.int64)
    if isinstance(obj, Pair) and not getattr(obj, "key", ""):
        return np.array([TAG_PAIR, obj.id, obj.count], np.uint64).view(np.int64)
    if isinstance(obj, PairArray):
        flat = np.stack([obj.ids, obj.counts.view(np.uint64)], axis=1).reshape(-1).view(np.int64)
        return np.concatenate([np.array([TAG_PAIRS, len(obj)], np.int64), flat])
    if isinstance(obj, list) and all(isinstance(p, Pair) and not getattr(p, "key", "") for p in obj):
        flat = np.array([(p.id, p.count) for p in obj], np.uint64).reshape(-1).view(np.int64) if obj else \
            np.zeros(0, np.int64)
        return np.concatenate([np.array([TAG_PAIRS, len(obj)], np.int64), flat])
    if isinstance(obj, list) and all(isinstance(x, (int, np.integer)) for x in obj):
        a = np.asarray(obj, dtype=np.uint64).view(np.int64) if obj else np.zeros(0, np.int64)
        return np.concatenate([np.array([TAG_ROWIDS, len(obj)], np.int64), a])
    if isinstance(obj, list) and obj and all(isinstance(g, GroupCount) for g in obj):
        fields = [fr.field for fr in obj[0].group]
        k = len(fields)
        if all(len(g.group) == k and all(fr.field == f and not fr.row_key for fr, f in zip(g.group, fields))
               for g in obj):
            names = encode(fields)
            mat = np.array([[fr.row_id for fr in g.group] + [g.count] for g in obj], np.uint64).view(np.int64)
            return np.concatenate([np.array([TAG_GROUPS, len(obj), k, len(names)], np.int64), _bytes_to_words(names),
                                   mat.reshape(-1)])
        return msg()
    if isinstance(obj, Row) and not obj.keys and not obj.attrs:
        segs = [(int(s), bm.to_bytes()) for s, bm in sorted(obj.segments.items())]
        head = [TAG_ROW, len(segs)]
        for s, b in segs:
            head += [s, len(b)]
        return np.concatenate([np.array(head, np.int64)] + [_bytes_to_words(b) for _, b in segs])
    if isinstance(obj, RowIdentifiers) and not obj.keys:
        a = np.asarray(obj.rows, dtype=np.uint64).view(np.int64) if obj.rows else np.zeros(0, np.int64)
        return np.concatenate([np.array([TAG_ROWIDS, -1 - len(obj.rows)], np.int64), a])
    return msg()


def decode_partial(w: np.ndarray):
    """Inverse of :func:`encode_partial`."""
    from pilosa_amd import _roaring
    from pilosa_amd.executor import FieldRow, GroupCount, RowIdentifiers, ValCount
    from pilosa_amd.models.cache import Pair
    from pilosa_amd.models.row import Row

    w = np.asarray(w, dtype=np.int64)
    if len(w) == 0:
        return None
    tag = int(w[0])
    if tag == TAG_NONE:
        return None
    if tag == TAG_BOOL:
        return bool(w[1])
    if tag == TAG_INT:
        return int(w[1])
    if tag == TAG_MSGPACK:
        return decode(_words_to_bytes(w[2:], int(w[1])))
    if tag == TAG_VALCOUNT:
        return ValCount(int(w[1]), int(w[2]))
    if tag == TAG_PAIR:
        return Pair(int(w[1:2].view(np.uint64)[0]), int(w[2]))
    if tag == TAG_PAIRS:
        n = int(w[1])
        a = w[2:2 + 2 * n].view(np.uint64).reshape(n, 2)
        return [Pair(int(i), int(c)) for i, c in a.tolist()]
    if tag == TAG_ROWIDS:
        n = int(w[1])
        if n < 0:   # RowIdentifiers
            m = -1 - n
            return RowIdentifiers(w[2:2 + m].view(np.uint64).tolist())
        return w[2:2 + n].view(np.uint64).tolist()
    if tag == TAG_GROUPS:
        n, k, nb = int(w[1]), int(w[2]), int(w[3])
        nw = (nb + 7) // 8
        fields = decode(_words_to_bytes(w[4:4 + nw], nb))
        mat = w[4 + nw:4 + nw + n * (k + 1)].view(np.uint64).reshape(n, k + 1).tolist()
        return [GroupCount([FieldRow(f, r) for f, r in zip(fields, row[:k])], row[k]) for row in mat]
    if tag == TAG_DEVROW:
        from pilosa_amd.ops.device import GpuEngine
        from pilosa_amd.ops.gpu_executor import row_from_bitmaps
        o = 2
        out = []
        for _ in range(int(w[1])):
            S, npw = int(w[o]), int(w[o + 1])
            shards = w[o + 2:o + 2 + S].tolist()
            o += 2 + S
            c = w[o:o + S * 8].view(np.int32)
            o += S * 8
            offs = w[o:o + S * 16]
            o += S * 16
            pay = w[o:o + npw].view(np.uint16)
            o += npw
            out.append((GpuEngine.block_bitmaps(shards, c, offs, pay), shards))
        spill = out[1] if len(out) > 1 else ((), ())
        return row_from_bitmaps(out[0][0], out[0][1], *spill)
    if tag == TAG_ROW:
        ns = int(w[1])
        hdr = w[2:2 + 2 * ns].reshape(ns, 2)
        o = 2 + 2 * ns
        segs = {}
        for s, nb in hdr.tolist():
            nw = (nb + 7) // 8
            segs[int(s)] = _roaring.Bitmap.from_bytes(_words_to_bytes(w[o:o + nw], nb))
            o += nw
        return Row(segments=segs)
    raise ValueError(f"unknown partial tag {tag}")


def pairs_to_arrays(totals: Sequence[dict]):
    """[{id: count}] per query -> (q, id, count) int64 arrays."""
    q, ids, cnt = [], [], []
    for k, t in enumerate(totals):
        for i, c in t.items():
            q.append(k)
            ids.append(int(i))
            cnt.append(int(c))
    return np.array(q, np.int64), np.array(ids, np.int64), np.array(cnt, np.int64)
