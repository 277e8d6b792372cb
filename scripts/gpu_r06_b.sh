#!/bin/bash
# Round 6, call B: mesh TopN fast path (OP_TOPN_PLAIN, src vote in the union).
# GPU tests of the RCCL mesh and TopN, then plain vs --mesh bench (TopN phases).
set -o pipefail
O=gpurun_out/r06_b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl_mesh.py tests/test_gpu_topn_exec.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
ARGS="--serve-seconds 0 --configs= --steps 5 --warmup 2"
timeout -k 10 400 python3 -u bench.py $ARGS > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --mesh $ARGS > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench", "bench_mesh"):
    d = json.loads([l for l in open(f"gpurun_out/r06_b/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "value", d["value"], "verified", d.get("verified"), "backend", e.get("backend"))
    print("  topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")}, t.get("verify"))
PY
echo done
