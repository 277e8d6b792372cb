#!/bin/bash
# Executor-path TopN: GPU tests, then the bench at one rank's share and full size.
set -o pipefail
mkdir -p gpurun_out/r03_topn
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_topn_exec.py \
  tests/test_gpu_write.py tests/test_gpu_executor.py -k "topn or TopN or write or rebuild or aggregates" \
  > gpurun_out/r03_topn/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_topn/pytest.log; exit 1; }
tail -3 gpurun_out/r03_topn/pytest.log
timeout -k 10 300 python -u bench.py --cols 125000000 --steps 10 --warmup 3 --configs none \
  > gpurun_out/r03_topn/bench_small.log 2>&1 || { tail -c 4000 gpurun_out/r03_topn/bench_small.log; exit 1; }
tail -c 2500 gpurun_out/r03_topn/bench_small.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --configs none \
  > gpurun_out/r03_topn/bench_full.log 2>&1 || { tail -c 4000 gpurun_out/r03_topn/bench_full.log; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r03_topn/bench_small.log", "gpurun_out/r03_topn/bench_full.log"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, d["value"], d["verified"], json.dumps(d["extra"].get("topn"))[:1500])
PY
