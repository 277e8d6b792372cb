"""cProfile of executor-path TopN requests on a small disk index (diagnostics)."""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilosa_amd import _roaring  # noqa: E402
from pilosa_amd.executor import Executor  # noqa: E402
from pilosa_amd.models.field import FieldOptions  # noqa: E402
from pilosa_amd.models.holder import Holder  # noqa: E402
from pilosa_amd.ops.gpu_executor import GpuExecutor  # noqa: E402

S = int(os.environ.get("SHARDS", "24"))
base = tempfile.mkdtemp(prefix="prof_topn_")
h = Holder(base).open()
h.create_index("i", track_existence=False)
h.index("i").create_field("f", FieldOptions())
h.close()
fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
os.makedirs(fdir, exist_ok=True)
_roaring.write_zipf_fragments(fdir, 0, S, S << 20, 1_000_000, 8.0, 1.6, 50.0, 1, 16, cache_size=50000)
holder = Holder(base, lazy_fragments=True).open()
gpu = GpuExecutor(holder, torch.device("cuda:0"))
ex = Executor(holder, gpu=gpu)
gpu.executor = ex
ex.strict_gpu = True
shards = list(range(S))
gpu.view_arena("i", "f", "standard", shards)
torch.cuda.synchronize()
for name, text in (("cache", " ".join(["TopN(f, n=100)"] * 16)),
                   ("src", " ".join(f"TopN(f, Row(f={r}), n=100)" for r in range(16)))):
    for k in range(3):
        t0 = time.perf_counter()
        pr = cProfile.Profile()
        pr.enable()
        ex.execute("i", text, shards=shards)
        torch.cuda.synchronize()
        pr.disable()
        print(f"{name} request {k}: {time.perf_counter() - t0:.3f} s", flush=True)
        if k in (0, 2):
            pstats.Stats(pr).sort_stats("tottime").print_stats(12)
import threading  # noqa: E402
for name, text in (("cache", " ".join(["TopN(f, n=100)"] * 16)),
                   ("src", " ".join(f"TopN(f, Row(f={r}), n=100)" for r in range(16)))):
    for nthreads in (1, 3):
        t0 = time.perf_counter()

        def work():
            for _ in range(8):
                ex.execute("i", text, shards=shards)
        ts = [threading.Thread(target=work) for _ in range(nthreads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"{name} threads={nthreads}: {8 * nthreads} requests in {el:.3f} s -> {16 * 8 * nthreads / el:.0f} q/s",
              flush=True)
