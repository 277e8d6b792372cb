#!/bin/bash
# Round 4, first GPU call: the mesh GPU tests (distinct row spaces, writes,
# concurrent TopN), then bench.py --gpus 4 with no launcher as a gloo
# rehearsal on the one GPU vs the 1-rank run on the same reduced index.
set -o pipefail
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_topn_exec.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -c 5000 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
ARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 3 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python -u bench.py --gpus 4 $ARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 $ARGS > $O/bench1.log 2> $O/bench1.err || { tail -c 5000 $O/bench1.err; exit 1; }
python - <<'PY'
import json
for n in (1, 4):
    d = json.loads([l for l in open(f"gpurun_out/r04_a/bench{n}.log") if l.startswith("{")][-1])
    e = d["extra"]
    t = e.get("topn", {})
    print(n, "n_gpus", d["n_gpus"], "value", d["value"], "verified", d["verified"], "mean", e.get("mean_count"),
          "backend", e.get("backend"), "per_rank", e.get("shards_per_rank"), "inflight", e.get("mesh_max_in_flight"))
    print("  topn cache", {k: t.get("cache", {}).get(k) for k in ("qps", "sample_top3", "max_in_flight")},
          "src", {k: t.get("src", {}).get(k) for k in ("qps", "sample_top3", "max_in_flight")}, "verify", t.get("verify"))
PY
# pair kernel: v10 (flat stream per staged run) vs v6, correctness + timing
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "and2 or array_size" --timeout 300 --timeout-method thread > $O/pytest_pairs.log 2>&1 || { tail -c 4000 $O/pytest_pairs.log; exit 1; }
tail -2 $O/pytest_pairs.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 10 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
tail -3 $O/kbench.log
