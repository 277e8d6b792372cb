#!/bin/bash
# Round 6, call P: native mesh cache-only TopN issue/finish
# (binding.cpp mesh_cache_issue / mesh_cache_finish) next to the native
# 1-GPU request object: GPU tests, then the world-size-1 RCCL mesh bench and
# the plain 1-GPU bench, both with the native paths.
set -o pipefail
O=gpurun_out/r06_p
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_mesh.py tests/test_gpu_topn_exec.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 --mesh-breakdown 20 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
timeout -k 10 500 env PILOSA_TOPN_NATIVE=0 python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 > $O/bench_mesh_py.log 2> $O/bench_mesh_py.err || { tail -c 3000 $O/bench_mesh_py.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench_mesh", "bench_mesh_py"):
    d = json.loads([l for l in open(f"gpurun_out/r06_p/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "value", d["value"], {k: ((t.get(k) or {}).get("qps"), (t.get(k) or {}).get("ms_per_request")) for k in ("cache", "cache_cycling", "cache_repeated", "src")}, t.get("verify"))
    for kind, b in (e.get("mesh_breakdown") or {}).items():
        print("  ", kind, "wall ms/request", b["wall_ms_per_request"])
        for name, v in list(b["spans"].items())[:12]:
            print("     ", name, v)
PY
echo done
