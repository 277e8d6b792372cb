"""Host-side cost of one Count batch through Executor.execute on a 120-shard
disk index (one rank's share at 8 GPUs): stage timings and a cProfile of
single-threaded requests (diagnostics for VERDICT r02 item 2)."""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pilosa_amd import _pql, _roaring  # noqa: E402
from pilosa_amd.executor import Executor  # noqa: E402
from pilosa_amd.models.field import FieldOptions  # noqa: E402
from pilosa_amd.models.holder import Holder  # noqa: E402
from pilosa_amd.ops.gpu_executor import GpuExecutor  # noqa: E402

S = int(os.environ.get("SHARDS", "120"))
B = int(os.environ.get("BATCH", "4096"))
base = tempfile.mkdtemp(prefix="prof_count_")
h = Holder(base).open()
h.create_index("i", track_existence=True)
h.index("i").create_field("f", FieldOptions())
h.close()
fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
os.makedirs(fdir, exist_ok=True)
_roaring.write_zipf_fragments(fdir, 0, S, S << 20, 1_000_000, 8.0, 1.6, 50.0, 1, 16, cache_size=0)
holder = Holder(base, lazy_fragments=True).open()
gpu = GpuExecutor(holder, torch.device("cuda:0"))
ex = Executor(holder, gpu=gpu)
ex.strict_gpu = True
shards = list(range(S))
dv = gpu.view_arena("i", "f", "standard", shards)
torch.cuda.synchronize()
rng = np.random.default_rng(3)
ra = (rng.zipf(1.6, size=B * 40) - 1) % 1_000_000
rb = (rng.zipf(1.6, size=B * 40) - 1) % 1_000_000
texts = [" ".join(f"Count(Intersect(Row(f={a}), Row(f={b})))" for a, b in zip(ra[i * B:(i + 1) * B], rb[i * B:(i + 1) * B]))
         for i in range(40)]


def tm(fn, n=10):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e3


eng = gpu.engine
for pt in (1, 4, 8, 16):
    print(f"plan_count_text nthreads={pt}: {tm(lambda: _pql.plan_count_text(texts[0], {'f': 0}, [dv.rows], True, True, pt)):.3f} ms")
print(f"count_text_fields: {tm(lambda: _pql.count_text_fields(texts[0])):.3f} ms")
Q, segs, buf = _pql.plan_count_text(texts[0], {'f': 0}, [dv.rows], True, True, 8)
print(f"prepare_planned: {tm(lambda: eng.prepare_planned(Q, segs, buf, [dv], dv.S)):.3f} ms")
hd = eng.prepare_planned(Q, segs, buf, [dv], dv.S)
torch.cuda.synchronize()
print(f"launch_count (enqueue only): {tm(lambda: eng.launch_count(hd), 3):.3f} ms")
torch.cuda.synchronize()
print(f"launch_count + sync: {tm(lambda: eng.launch_count(hd).cpu(), 5):.3f} ms")
print(f"try_count_text: {tm(lambda: gpu.try_count_text('i', texts[1], shards), 5):.3f} ms")
print(f"Executor.execute: {tm(lambda: ex.execute('i', texts[2], shards=shards), 5):.3f} ms")
pr = cProfile.Profile()
pr.enable()
for k in range(5):
    ex.execute("i", texts[3 + k], shards=shards)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
