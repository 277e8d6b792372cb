#!/bin/bash
# Hot ranks 4096 (pipelined small-row loads) and the single-sort TopN finish:
# TopN / executor / write GPU suites, then the driver bench command.
set -o pipefail
mkdir -p gpurun_out/r03_hot4k
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_write.py tests/test_gpu_executor.py > gpurun_out/r03_hot4k/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r03_hot4k/pytest.log | tail -12
[ $rc -eq 0 ] || { grep -B30 "Error\b" gpurun_out/r03_hot4k/pytest.log | tail -60; exit 1; }
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_hot4k/bench.log 2> gpurun_out/r03_hot4k/bench.err || { tail -c 3000 gpurun_out/r03_hot4k/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r03_hot4k/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"], "load_s", e.get("load_s"), "page_cache", e.get("page_cache"))
print("load", json.dumps(e.get("load")))
print("topn", json.dumps({k: e["topn"].get(k) for k in ("cache", "src", "after_write", "fragments_cold_after_topn", "verify")}))
PY
