#!/bin/bash
# Round 6, call AT: run-to-run spread of the headline -- the driver's bench
# command three times on one box (fresh process each).
set -o pipefail
O=gpurun_out/r06_at
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 600 python3 -u bench.py --serve-seconds 0 --configs= > $O/bench_$r.log 2> $O/bench_$r.err || { tail -c 3000 $O/bench_$r.err; exit 1; }
  python3 - $O/bench_$r.log $r <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"]["topn"]
print("run", sys.argv[2], d["value"], d["ms_per_step"], d.get("verified"), {k: t[k]["qps"] for k in ("cache", "cache_cycling", "src")})
PY
done
echo done
