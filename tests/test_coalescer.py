"""Cross-request Count batching (pilosa_amd/ops/coalescer.py): results,
batching under concurrency, leadership hand-off and per-call fallback."""
import threading
import time

from pilosa_amd.ops.coalescer import CountCoalescer


def _run_threads(n, fn):
    out = [None] * n
    errs = []

    def work(i):
        try:
            out[i] = fn(i)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    assert not errs, errs
    return out


def test_concurrent_requests_share_batches():
    sizes = []

    def run(key, calls):
        sizes.append(len(calls))
        time.sleep(0.01)
        return [c * 10 for c in calls]

    co = CountCoalescer(run)
    out = _run_threads(64, lambda i: co.submit("k", i, lambda: -1))
    assert out == [i * 10 for i in range(64)]
    assert sum(sizes) == 64 and co.batched == 64
    assert len(sizes) < 64  # requests arriving during a launch were batched


def test_lone_request_runs_immediately():
    co = CountCoalescer(lambda key, calls: [7] * len(calls))
    t0 = time.perf_counter()
    assert co.submit("k", 1, lambda: -1) == 7
    assert time.perf_counter() - t0 < 0.5
    assert co.batches == 1


def test_unsupported_or_failing_batches_fall_back_per_call():
    def run(key, calls):
        if any(c == 3 for c in calls):
            raise ValueError("boom")
        return None if any(c == 5 for c in calls) else [c for c in calls]

    co = CountCoalescer(run)
    out = _run_threads(16, lambda i: co.submit(i % 2, i, lambda i=i: ("host", i)))
    for i, r in enumerate(out):
        assert r == i or r == ("host", i)
    assert out[3] == ("host", 3) and out[5] == ("host", 5)
    assert co.batched + co.fallbacks == 16


def test_keys_are_batched_separately():
    seen = []

    def run(key, calls):
        seen.append((key, tuple(calls)))
        time.sleep(0.005)
        return [(key, c) for c in calls]

    co = CountCoalescer(run, max_batch=4)
    out = _run_threads(24, lambda i: co.submit(i % 3, i, lambda: None))
    assert out == [(i % 3, i) for i in range(24)]
    assert all(len(c) <= 4 and all(x % 3 == k for x in c) for k, c in seen)

