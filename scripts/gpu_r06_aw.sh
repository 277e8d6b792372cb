#!/bin/bash
# Round 6, call AW: mesh cache-only partial with membership + totals in one launch (world-size-1
# RCCL): mesh GPU tests, then the mesh bench.
set -o pipefail
O=gpurun_out/r06_aw
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_mesh.py tests/test_gpu_mesh.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_aw/bench_mesh.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v}, t.get("verify"))
PY
echo done
