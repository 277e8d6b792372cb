"""Kernel-trace target: executor-path src TopN requests (16 calls each) on a
disk-loaded index of SHARDS shards (default the headline 954), for
rocprofv3 --kernel-trace --stats (scripts/gpu_r03_topnprof.sh)."""
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import zipf_rows  # noqa: E402
from pilosa_amd import _roaring  # noqa: E402
from pilosa_amd.executor import Executor  # noqa: E402
from pilosa_amd.models.field import FieldOptions  # noqa: E402
from pilosa_amd.models.holder import Holder  # noqa: E402
from pilosa_amd.ops.gpu_executor import GpuExecutor  # noqa: E402

S = int(os.environ.get("SHARDS", "954"))
N = int(os.environ.get("REQUESTS", "12"))
base = tempfile.mkdtemp(prefix="prof_topn_")
h = Holder(base).open()
h.create_index("i", track_existence=False)
h.index("i").create_field("f", FieldOptions())
h.close()
fdir = os.path.join(base, "i", "f", "views", "standard", "fragments")
os.makedirs(fdir, exist_ok=True)
cols = min(S << 20, 1_000_000_000)
_roaring.write_zipf_fragments(fdir, 0, S, cols, 1_000_000, 8.0, 1.6, 50.0, 1, 16, cache_size=50000)
print("written", flush=True)
holder = Holder(base, lazy_fragments=True).open()
gpu = GpuExecutor(holder, torch.device("cuda:0"))
ex = Executor(holder, gpu=gpu)
gpu.executor = ex
ex.strict_gpu = True
shards = list(range(S))
gpu.view_arena("i", "f", "standard", shards)
torch.cuda.synchronize()
rng = np.random.default_rng(99)
hot = zipf_rows(rng, 16 * (N + 1), 1000)
texts = [" ".join(f"TopN(f, Row(f={a}), n=100)" for a in hot[i * 16:(i + 1) * 16]) for i in range(N + 1)]
ex.execute("i", texts[0], shards=shards)     # builds rank caches + slot index
torch.cuda.synchronize()
print("warm", flush=True)
t0 = time.perf_counter()
for t in texts[1:]:
    ex.execute("i", t, shards=shards)
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"src: {N} requests x 16 calls in {el:.3f} s -> {16 * N / el:.0f} q/s, {el / N * 1000:.2f} ms per request",
      flush=True)
import shutil  # noqa: E402
shutil.rmtree(base, ignore_errors=True)
