"""Test harness: an in-process holder + executor on a temp dir
(reference test/holder.go, test/pilosa.go MustRunCluster(t, 1))."""
from __future__ import annotations

import os
import shutil
import tempfile

from pilosa_amd.executor import Executor
from pilosa_amd.models.field import FieldOptions
from pilosa_amd.models.holder import Holder

from pilosa_amd.shardwidth import SHARD_WIDTH as SW  # noqa: E402


class Env:
    def __init__(self, gpu=None, max_opn=10000):
        self.dir = tempfile.mkdtemp(prefix="pilosa_amd_test_")
        self.holder = Holder(self.dir, max_opn=max_opn).open()
        self.gpu = gpu
        self.executor = Executor(self.holder, gpu=gpu(self.holder) if callable(gpu) else gpu)

    def create_index(self, name="i", keys=False, track_existence=True):
        return self.holder.create_index(name, keys=keys, track_existence=track_existence)

    def field(self, index, name, **opts):
        idx = self.holder.index(index)
        return idx.create_field(name, FieldOptions(**opts) if opts else None)

    def q(self, index, pql, **kw):
        return self.executor.execute(index, pql, **kw).results

    def q1(self, index, pql, **kw):
        return self.q(index, pql, **kw)[0]

    def reopen(self):
        self.holder.close()
        self.holder = Holder(self.dir).open()
        self.executor.holder = self.holder
        if self.executor.gpu is not None:
            self.executor.gpu.holder = self.holder

    def close(self):
        self.executor.close()
        self.holder.close()
        shutil.rmtree(self.dir, ignore_errors=True)


def cols(row):
    return [int(c) for c in row.columns()]


def free_port() -> int:
    """A currently free TCP port below the kernel's ephemeral range.

    A port taken from ``bind(0)`` and released is soon handed out again to
    some other test's ``bind(0)`` server (xdist workers run side by side), so
    a test that picks a port for a server started later could end up talking
    to another test's server.  Ports below 32768 are never assigned by
    ``bind(0)``."""
    import random
    import socket
    rng = random.Random()
    for _ in range(1000):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port below 32000")
