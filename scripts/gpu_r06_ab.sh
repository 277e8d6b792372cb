#!/bin/bash
# Round 6, call AB: world-size-1 RCCL mesh breakdown of src TopN requests
# (sequential, HIP-event tracer) next to Count and cache-only TopN.
set -o pipefail
O=gpurun_out/r06_ab
mkdir -p $O
timeout -k 10 600 python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 --mesh-breakdown 20 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_ab/bench_mesh.log") if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print({k: ((t.get(k) or {}).get("qps"), (t.get(k) or {}).get("ms_per_request")) for k in ("cache", "src")})
b = e.get("mesh_breakdown") or {}
for kind in ("topn_src", "topn_cache"):
    if kind in b:
        print(kind, "wall ms/request", b[kind]["wall_ms_per_request"])
        for name, v in list(b[kind]["spans"].items())[:25]:
            print("   ", name, v)
PY
echo done
