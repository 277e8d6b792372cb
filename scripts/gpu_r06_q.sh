#!/bin/bash
# Round 6, call Q: world-size-1 RCCL mesh cache-only TopN with 2 / 3 / 4
# pipelined request threads (issue under the mesh lock, completion outside).
set -o pipefail
O=gpurun_out/r06_q
mkdir -p $O
for c in 2 3 4; do
  timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 --topn-cache-clients $c > $O/bench_mesh_c$c.log 2> $O/bench_mesh_c$c.err || { tail -c 3000 $O/bench_mesh_c$c.err; exit 1; }
  python3 - $O/bench_mesh_c$c.log $c <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"].get("topn", {})
print("clients", sys.argv[2], d["value"], {k: ((t.get(k) or {}).get("qps"), (t.get(k) or {}).get("ms_per_request")) for k in ("cache", "cache_cycling", "src")}, t.get("verify"))
PY
done
echo done
