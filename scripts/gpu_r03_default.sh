#!/bin/bash
# The driver's bench command (defaults: disk mode, TopN, configs 4 and 5).
set -o pipefail
mkdir -p gpurun_out/r03_default
df -h /tmp | tail -1
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_default/bench.log 2> gpurun_out/r03_default/bench.err || { tail -c 3000 gpurun_out/r03_default/bench.err; exit 1; }
tail -c 600 gpurun_out/r03_default/bench.err
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r03_default/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "verified", d["verified"])
print("topn", json.dumps({k: e["topn"][k] for k in ("cache", "src", "fragments_cold_after_topn", "verify")}))
print("cfg4", json.dumps(e.get("config4_bsi"))[:2500])
print("cfg5", json.dumps(e.get("config5_time_union"))[:1500])
print("data", e.get("data"))
print("serving", json.dumps(e.get("serving"))[:3000])
PY
