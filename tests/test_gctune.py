"""GC policy (utils/gctune.py): freezing, thresholds, periodic refreeze."""
import gc

from pilosa_amd.utils import gctune


def test_freeze_and_refreeze():
    old = gc.get_threshold()
    try:
        gctune.configure(12345)
        assert gc.get_threshold()[0] >= 12345
        keep = [[i] for i in range(1000)]
        assert gctune.freeze_long_lived() >= 1000
        r = gctune.Refreezer(every=1.0, full_every=10.0)
        t0 = r._last
        assert r.tick(t0 + 0.5) == ""
        assert r.tick(t0 + 1.5) == "freeze"
        assert r.tick(t0 + 11.0) == "full" and gc.get_freeze_count() > 0
        del keep
    finally:
        gc.unfreeze()
        gc.set_threshold(*old)
