#!/bin/bash
# Round-3 final pass (after the TopN hot-split change): the whole GPU test suite, smoke, then the driver's bench
# command (defaults: disk mode, TopN through the executor, configs 4/5, serving).
set -o pipefail
mkdir -p gpurun_out/r03_final2
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r03_final2/pytest_gpu.log 2>&1 \
  || { tail -c 4000 gpurun_out/r03_final2/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03_final2/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final2/smoke.log 2>&1 || { cat gpurun_out/r03_final2/smoke.log; exit 1; }
tail -1 gpurun_out/r03_final2/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_final2/bench.log 2> gpurun_out/r03_final2/bench.err || { tail -c 3000 gpurun_out/r03_final2/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r03_final2/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
print("topn", json.dumps({k: e["topn"][k] for k in ("cache", "src", "fragments_cold_after_topn", "verify")}))
print("serving", json.dumps({k: e["serving"][k] for k in ("count", "count_topn_mix")})[:1500]); print("after_write", e["topn"].get("after_write")); print("load", e.get("load_s"), e.get("page_cache"))
PY
