#!/usr/bin/env python3
"""Per-batch host cost of the Count group commit (Executor._count_text_fast
on a 40-request group) on a served data dir, with a cProfile breakdown."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from bench import zipf_rows
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils.logger import CaptureLogger
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    srv = Server(d, bind="127.0.0.1:0", gpu="on", logger=CaptureLogger()).open()
    try:
        ex = srv.executor
        rng = np.random.default_rng(3)
        texts = []
        for _ in range(50):
            a, b = zipf_rows(rng, n, 1_000_000), zipf_rows(rng, n, 1_000_000)
            texts.append("\n".join(f"Count(Intersect(Row(f={x}), Row(f={y})))" for x, y in zip(a, b)))
        ex._count_text_fast("i", texts[0], None, None, min_calls=1)
        t0 = time.perf_counter()
        for t in texts:
            ex._count_text_fast("i", t, None, None, min_calls=1)
        el = (time.perf_counter() - t0) / len(texts)
        pr = cProfile.Profile()
        pr.enable()
        for t in texts:
            ex._count_text_fast("i", t, None, None, min_calls=1)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue())
        print(json.dumps({"batch": n, "ms_per_batch": round(el * 1000, 3)}))
    finally:
        srv.close()


if __name__ == "__main__":
    main()
