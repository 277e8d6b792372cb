#!/bin/bash
# Round-4 checkpoint: the whole GPU test suite, smoke, then the driver's bench
# command (disk mode, distinct-call TopN, configs 4/5 through the native
# time-range path, serving + native import decode).  Test failures (rc 1) do
# not stop the bench; a timeout, crash or GPU fault does.
set -o pipefail
O=gpurun_out/r04_full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -c 3000 $O/pytest_gpu.log | grep -E "FAILED|ERROR|passed|failed" 
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04_full/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
t = e["topn"]
print("topn", json.dumps({k: t.get(k) for k in ("cache", "cache_repeated", "src", "verify")})[:1500])
print("cfg5", json.dumps(e.get("config5_time_union"))[:800])
print("cfg4", json.dumps(e.get("config4_bsi", {}).get("queries"))[:800])
print("serving", json.dumps({k: e["serving"][k] for k in ("count", "count_topn_mix", "import")})[:1800])
PY
exit $rc
