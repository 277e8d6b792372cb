#!/bin/bash
# Round 6, call C: mesh vs plain TopN with equal warm-up, sampled host profiles of the cache-only phase.
set -o pipefail
O=gpurun_out/r06_c
mkdir -p $O
ARGS="--serve-seconds 0 --configs= --steps 3 --warmup 1"
timeout -k 10 400 env PILOSA_BENCH_TOPN_PROFILE=$O/prof_plain.folded python3 -u bench.py $ARGS > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
timeout -k 10 400 env PILOSA_BENCH_TOPN_PROFILE=$O/prof_mesh.folded python3 -u bench.py --mesh $ARGS > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench", "bench_mesh"):
    d = json.loads([l for l in open(f"gpurun_out/r06_c/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "value", d["value"], "verified", d.get("verified"), "backend", e.get("backend"))
    for k in ("cache", "cache_cycling", "cache_repeated", "src"):
        r = t.get(k) or {}
        print("  ", k, r.get("qps"), r.get("ms_per_request"), r.get("space_refreshes"), r.get("device_batches"))
    print("  verify", t.get("verify"))
PY
echo done
