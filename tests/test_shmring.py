"""The mesh command ring (native/shmring.cpp): one producer, several reader
processes, messages in order with no loss when the ring wraps, readers that
wait through an idle spell, and readers that raise once the producer is gone
or the ring is closed (parallel/mesh.py uses it in place of a gloo broadcast
per command)."""
import multiprocessing as mp
import os
import time
import uuid

import pytest

from pilosa_amd import _shmring


def _reader(name, r, n, q):
    ring = _shmring.Ring(name, False)
    ring.attach(r)
    q.put(("ready", r))
    got = []
    try:
        for _ in range(n):
            got.append(ring.read(r, 50.0))
        q.put(("done", r, [(op, len(b), b[:8]) for op, b, _ in got]))
        ring.read(r, 50.0)           # blocks until the producer closes the ring
    except RuntimeError as e:
        q.put(("closed", r, str(e)))


def test_ring_fanout_order_wrap_idle_close():
    name = f"/pilosa_test_{uuid.uuid4().hex[:12]}"
    ring = _shmring.Ring(name, True, nslots=8, slot_bytes=4096, nreaders=3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n = 200
    ps = [ctx.Process(target=_reader, args=(name, r, n, q)) for r in range(3)]
    for p in ps:
        p.start()
    ready = {q.get(timeout=60)[1] for _ in range(3)}
    assert ready == {0, 1, 2}
    time.sleep(0.5)              # idle: readers sleep on the futex, no timeout
    msgs = []
    for i in range(n):
        payload = bytes([i % 251]) * (i * 17 % 4096)
        ring.publish(i, payload)  # 8 slots, 200 messages: the ring wraps many times
        msgs.append((i, len(payload), payload[:8]))
    done = [q.get(timeout=60) for _ in range(3)]
    for d in done:
        assert d[0] == "done" and d[2] == msgs
    with pytest.raises(Exception):
        ring.publish(0, b"x" * 5000)        # larger than a slot
    ring.close()
    closed = [q.get(timeout=60) for _ in range(3)]
    assert all(c[0] == "closed" and "closed" in c[2] for c in closed)
    for p in ps:
        p.join(30)
    del ring
    assert not os.path.exists("/dev/shm" + name)


def _producer_dies(name):
    ring = _shmring.Ring(name, True, nslots=4, slot_bytes=256, nreaders=1)
    ring.publish(1, b"hello")
    time.sleep(0.3)
    os._exit(0)                  # no close: the reader must notice the death


def test_reader_raises_when_producer_dies():
    name = f"/pilosa_test_{uuid.uuid4().hex[:12]}"
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_producer_dies, args=(name,))
    p.start()
    for _ in range(200):
        try:
            ring = _shmring.Ring(name, False)
            break
        except RuntimeError:
            time.sleep(0.02)
    ring.attach(0)
    p.join(30)
    t0 = time.time()
    with pytest.raises(RuntimeError, match="gone"):
        ring.read(0, 10.0)
    assert time.time() - t0 < 5
    if os.path.exists("/dev/shm" + name):
        os.unlink("/dev/shm" + name)


def _poster(name, r, q):
    ring = _shmring.Ring(name, False)
    ring.attach(r)
    q.put("ready")
    for _ in range(3):
        op, data, seq = ring.read(r, 50.0)
        payload = b"x" * (20000 if op == 2 else 10 * (r + 1))
        ring.post(r + 1, seq, payload)


def test_results_board_one_shot_gather():
    """The results board: every rank posts its result of command `seq`; the
    producer collects all of them with no collective; a result larger than
    the board's entry posts its size only (the caller falls back)."""
    name = f"/pilosa_test_{uuid.uuid4().hex[:12]}"
    ring = _shmring.Ring(name, True, nslots=4, slot_bytes=256, nreaders=2, board_bytes=8192)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_poster, args=(name, r, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in range(2):
        q.get(timeout=60)
    for op in (1, 1, 2):
        seq = ring.publish(op, b"cmd")
        ring.post(0, seq, b"front")
        got = ring.collect(seq, 30.0, 50.0)
        if op == 1:
            assert got == [b"front", b"x" * 10, b"x" * 20]
        else:
            assert got == [b"front", -20000, -20000]
    for p in ps:
        p.join(30)
    with pytest.raises(RuntimeError, match="timed out"):
        ring.collect(ring.publish(1, b""), 0.2, 10.0)
