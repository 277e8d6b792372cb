#!/bin/bash
# Round 6, call F: the mesh after OP_TOPN_PLAIN + the shared-memory command
# ring. (1) bench --mesh on the full index (world-size-1 RCCL) vs call E's
# plain run; (2) 4-rank gloo rehearsal on one GPU vs 1 rank, reduced index.
set -o pipefail
O=gpurun_out/r06_f
mkdir -p $O
timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-src-batches 40 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 python3 -u bench.py --gpus 1 $RARGS > $O/bench1.log 2> $O/bench1.err || { tail -c 5000 $O/bench1.err; exit 1; }
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python3 -u bench.py --gpus 4 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench_mesh", "bench1", "bench4"):
    d = json.loads([l for l in open(f"gpurun_out/r06_f/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, "n_gpus", d["n_gpus"], "value", d["value"], "verified", d.get("verified"), "backend", e.get("backend"))
    for k in ("cache", "cache_cycling", "cache_repeated", "src"):
        r = t.get(k) or {}
        print("   ", k, r.get("qps"), r.get("ms_per_request"), "refreshes", r.get("space_refreshes"), "p50", r.get("p50_ms"))
    print("    verify", t.get("verify"))
PY
echo done
