#!/bin/bash
# Round 6, call A: round-start baseline. Driver bench command, then the same
# bench through the world-size-1 RCCL mesh (--mesh).
set -o pipefail
O=gpurun_out/r06_a
mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --mesh --serve-seconds 0 --configs "" > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench", "bench_mesh"):
    d = json.loads([l for l in open(f"gpurun_out/r06_a/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "value", d["value"], "verified", d.get("verified"), "backend", e.get("backend"))
    print("  topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
    print("  serving", {k: (v.get("req_per_s") if isinstance(v, dict) else v) for k, v in (e.get("serving") or {}).items()})
PY
echo done
