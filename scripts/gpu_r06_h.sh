#!/bin/bash
# Round 6, call H: device Shift at every width + nested shifts, the RCCL
# mesh test, then the mesh bench (cache-only TopN after space reuse, native
# upload, vectorised decode) with the per-span breakdown.
set -o pipefail
O=gpurun_out/r06_h
mkdir -p $O
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $T -k "shift or Shift" tests/test_gpu_executor.py > $O/shift20.log 2>&1 || { tail -c 4000 $O/shift20.log; exit 1; }
tail -1 $O/shift20.log
for e in 16 18 22; do
  timeout -k 10 400 env PILOSA_SHARD_WIDTH=$e $T -k "shift or Shift" tests/test_gpu_executor.py > $O/shift$e.log 2>&1 || { tail -c 4000 $O/shift$e.log; exit 1; }
  tail -1 $O/shift$e.log
done
timeout -k 10 400 $T tests/test_gpu_rccl_mesh.py > $O/rccl.log 2>&1 || { tail -c 4000 $O/rccl.log; exit 1; }
tail -1 $O/rccl.log
timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= --mesh-breakdown 20 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_h/bench_mesh.log") if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print("mesh value", d["value"], {k: ((t.get(k) or {}).get("qps"), (t.get(k) or {}).get("space_refreshes")) for k in ("cache", "cache_cycling", "src")})
for kind, b in (e.get("mesh_breakdown") or {}).items():
    print("  ", kind, "wall ms/request", b["wall_ms_per_request"])
    for name, v in list(b["spans"].items())[:12]:
        print("     ", name, v)
PY
echo done
