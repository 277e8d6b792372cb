#!/bin/bash
# Round 5, call F: checkpoint of the driver's bench command (all extras:
# TopN, configs 4/5, serving) after the columnar TopN results, BSI host
# trims and mesh changes; then the Count group-commit micro profile
# (per-batch host cost at 40 and 128 requests) on the same data dir.
set -o pipefail
O=gpurun_out/r05_f
mkdir -p $O
D=${TMPDIR:-/tmp}/pilosa_r05f
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 --data-dir $D --keep-data > $O/bench.log 2> $O/bench.err || { tail -c 5000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_f/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
t = e["topn"]
print("topn", json.dumps({k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_repeated", "src")}))
print("cfg5", json.dumps(e.get("config5_time_union", {}).get("qps")))
print("cfg4", json.dumps({k: v["ms_per_request"] for k, v in e.get("config4_bsi", {}).get("queries", {}).items()}))
s = e["serving"]
print("serving", json.dumps({k: s[k] for k in ("count", "count_topn_mix", "import") if k in s})[:1500])
PY
timeout -k 10 300 python -u scripts/serve_micro.py $D 40 > $O/micro40.log 2>&1 || { tail -c 3000 $O/micro40.log; exit 1; }
tail -1 $O/micro40.log
timeout -k 10 300 python -u scripts/serve_micro.py $D 128 > $O/micro128.log 2>&1 || { tail -c 3000 $O/micro128.log; exit 1; }
tail -1 $O/micro128.log
