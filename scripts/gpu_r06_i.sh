#!/bin/bash
# Round 6, call I: mesh with the results board (small partials off the
# collectives) and the direct ProcessGroup all-reduce: RCCL mesh test, the
# world-size-1 RCCL mesh bench with its breakdown, the 4-rank rehearsal.
set -o pipefail
O=gpurun_out/r06_i
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_mesh.py > $O/rccl.log 2>&1 || { tail -c 4000 $O/rccl.log; exit 1; }
tail -1 $O/rccl.log
timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= --mesh-breakdown 20 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-src-batches 40 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python3 -u bench.py --gpus 4 --mesh-breakdown 20 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench_mesh", "bench4"):
    d = json.loads([l for l in open(f"gpurun_out/r06_i/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "value", d["value"], {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "src")}, t.get("verify"))
    for kind, b in (e.get("mesh_breakdown") or {}).items():
        print("  ", kind, "wall ms/request", b["wall_ms_per_request"])
        for name, v in list(b["spans"].items())[:10]:
            print("     ", name, v)
PY
echo done
