"""cProfile of config-5 requests (1024 Count(Row(t=r, from, to)) calls each)
through Executor.execute on a disk-loaded YMDH time field (diagnostics)."""
import cProfile
import os
import pstats
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import TIME_RANGE, TIME_VIEWS, zipf_rows  # noqa: E402
from pilosa_amd import _roaring  # noqa: E402
from pilosa_amd.executor import Executor  # noqa: E402
from pilosa_amd.models.field import FieldOptions  # noqa: E402
from pilosa_amd.models.holder import Holder  # noqa: E402
from pilosa_amd.ops.gpu_executor import GpuExecutor  # noqa: E402

S = int(os.environ.get("SHARDS", "954"))
base = tempfile.mkdtemp(prefix="prof_cfg5_")
h = Holder(base).open()
idx = h.create_index("c", track_existence=False)
idx.create_field("t", FieldOptions(type="time", time_quantum="YMDH"))
h.close()
cols = min(S << 20, 1_000_000_000)
for k, (vname, bpc) in enumerate(TIME_VIEWS):
    d = os.path.join(base, "c", "t", "views", vname, "fragments")
    os.makedirs(d, exist_ok=True)
    _roaring.write_zipf_fragments(d, 0, S, cols, 1_000_000, bpc, 1.6, 50.0, 100 + k, 16, cache_size=0)
holder = Holder(base, lazy_fragments=True).open()
gpu = GpuExecutor(holder, torch.device("cuda:0"))
ex = Executor(holder, gpu=gpu)
gpu.executor = ex
ex.strict_gpu = True
shards = list(range(S))
rng = np.random.default_rng(5)
texts = [" ".join(f"Count(Row(t={int(r)}, {TIME_RANGE}))" for r in zipf_rows(rng, 1024, 1_000_000)) for _ in range(7)]
ex.execute("c", texts[0], shards=shards)
torch.cuda.synchronize()
t0 = time.perf_counter()
for t in texts[1:4]:
    ex.execute("c", t, shards=shards)
torch.cuda.synchronize()
print(f"sequential: {(time.perf_counter() - t0) / 3 * 1000:.2f} ms per request", flush=True)
pr = cProfile.Profile()
pr.enable()
for t in texts[4:7]:
    ex.execute("c", t, shards=shards)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
import shutil  # noqa: E402
shutil.rmtree(base, ignore_errors=True)
