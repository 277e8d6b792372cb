#!/bin/bash
# Round 6, call E: the whole GPU suite on the stripped kernel build (shipped
# variants only, planner dedupe, mesh TopN paths), smoke, then the driver's
# bench command.
set -o pipefail
O=gpurun_out/r06_e
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_e/bench.log") if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print("value", d["value"], "ms", d["ms_per_step"], "verified", d.get("verified"))
print("topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
print("serving", {k: v for k, v in (e.get("serving") or {}).items() if k in ("count", "count_topn_mix")})
print("bsi", {k: v for k, v in (e.get("config4_bsi") or {}).items() if "ms" in k})
PY
echo done
