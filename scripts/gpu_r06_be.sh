#!/bin/bash
# Round 6, call BE: the driver's bench command (N=1, defaults) on the final code.
set -o pipefail
O=gpurun_out/r06_be
mkdir -p $O
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - $O/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print("value", d["value"], "ms", d["ms_per_step"], "verified", d.get("verified"))
print("topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
print("serving", {k: (v.get("req_per_s") if isinstance(v, dict) else v) for k, v in (e.get("serving") or {}).items()})
PY
echo done
