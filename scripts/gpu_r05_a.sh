#!/bin/bash
# Round 5, first GPU call: RCCL executed.  The world-size-1 nccl mesh GPU
# test + the gloo 2-rank mesh tests, then bench.py --gpus 1 --mesh (the N>1
# product path under torch.distributed.run over RCCL) against the plain
# 1-GPU run, then the 4-rank gloo rehearsal vs 1 rank on a reduced index.
set -o pipefail
O=gpurun_out/r05_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_mesh.py tests/test_gpu_mesh.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -c 6000 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
ARGS="--steps 20 --warmup 5 --configs= --serve-seconds 0 --topn-batches 20 --topn-pairs-batches 0"
timeout -k 10 900 python -u bench.py --gpus 1 --mesh $ARGS > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 5000 $O/bench_mesh.err; exit 1; }
timeout -k 10 900 python -u bench.py --gpus 1 $ARGS > $O/bench_plain.log 2> $O/bench_plain.err || { tail -c 5000 $O/bench_plain.err; exit 1; }
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python -u bench.py --gpus 4 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 $RARGS > $O/bench1.log 2> $O/bench1.err || { tail -c 5000 $O/bench1.err; exit 1; }
python - <<'PY'
import json
for n in ("mesh", "plain", "4", "1"):
    d = json.loads([l for l in open(f"gpurun_out/r05_a/bench{'_' if not n.isdigit() else ''}{n}.log") if l.startswith("{")][-1])
    e = d["extra"]
    t = e.get("topn", {})
    print(n, "n_gpus", d["n_gpus"], "value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"],
          "backend", e.get("backend"), "world", e.get("world_size"), "inflight", e.get("mesh_max_in_flight"))
    print("  topn cache", {k: t.get("cache", {}).get(k) for k in ("qps", "ms_per_request", "max_in_flight")},
          "src", {k: t.get("src", {}).get(k) for k in ("qps", "ms_per_request")}, "verify", t.get("verify"))
PY
