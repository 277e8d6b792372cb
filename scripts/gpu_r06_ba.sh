#!/bin/bash
# Round 6, call BA: RCCL all-reduce of the mesh on the caller's stream (asyncOp = False) vs the
# process group's stream: world-size-1 mesh tests under "current", then bench --mesh both ways.
set -o pipefail
O=gpurun_out/r06_ba
mkdir -p $O
export PILOSA_MESH_AR_STREAM=current
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl_mesh.py > $O/pytest_rccl_current.log 2>&1 || { tail -c 4000 $O/pytest_rccl_current.log; exit 1; }
tail -2 $O/pytest_rccl_current.log
D=/tmp/pilosa_ba_data
for m in pg current current pg; do
  export PILOSA_MESH_AR_STREAM=$m
  timeout -k 10 400 python3 -u bench.py --mesh --serve-seconds 0 --configs "" --topn-pairs-batches 0 --data-dir $D --keep-data > $O/bench_mesh_$m.log 2> $O/bench_mesh_$m.err || { tail -c 3000 $O/bench_mesh_$m.err; exit 1; }
  python3 - $O/bench_mesh_$m.log $m <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print(sys.argv[2], "value", d["value"], "verified", d.get("verified"), "topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
PY
  cat $O/bench_mesh_$m.log | python3 -c "import sys" ; mv $O/bench_mesh_$m.log $O/bench_mesh_${m}_$RANDOM.log
done
echo done
