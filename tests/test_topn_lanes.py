"""Lane pool of the cache-only fused TopN batch (ops/topn_exec.py): a lane
(side stream + pinned / device buffers) is owned by one batch at a time and
reused after; concurrent takers get distinct lanes."""
import threading

import torch

from pilosa_amd.ops import topn_exec


def test_lanes_are_exclusive_and_reused(monkeypatch):
    dev = torch.device("cpu")
    monkeypatch.setattr(topn_exec, "_LANES", {})
    a = topn_exec._lane_take(dev)
    b = topn_exec._lane_take(dev)
    assert a is not b and a.stream is None
    topn_exec._lane_give(dev, a)
    assert topn_exec._lane_take(dev) is a          # reused, not rebuilt
    topn_exec._lane_give(dev, a)
    topn_exec._lane_give(dev, b)
    held, mu, seen = set(), threading.Lock(), []

    def worker():
        for _ in range(200):
            lane = topn_exec._lane_take(dev)
            with mu:
                assert id(lane) not in held
                held.add(id(lane))
                seen.append(id(lane))
            with mu:
                held.discard(id(lane))
            topn_exec._lane_give(dev, lane)
    ts = [threading.Thread(target=worker) for _ in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(set(seen)) <= 8 and len(topn_exec._LANES[dev]) == len(set(seen) | {id(a), id(b)})


def test_lane_buffers_grow_and_are_reused():
    lane = topn_exec._Lane(torch.device("cpu"))
    x = lane.buf("out", 100, torch.int64)
    assert x.numel() == 100 and x.dtype == torch.int64
    base = lane._bufs["out"].data_ptr()
    y = lane.buf("out", 900, torch.int64)        # within the first allocation (1024 * 1.5)
    assert y.numel() == 900 and lane._bufs["out"].data_ptr() == base
    z = lane.buf("out", 5000, torch.int64)
    assert z.numel() == 5000 and lane._bufs["out"].numel() >= 5000   # (pinned buffers need a GPU)
