#!/bin/bash
# Round 5, call AJ (final code): the 4-rank gloo rehearsal of the mesh TopN path (4 ranks
# sharing the one GPU) against 1 rank on the same reduced index (125M
# columns), cache-only (wide and cycling sets) and src.
set -o pipefail
O=gpurun_out/r05_aj
mkdir -p $O
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 python -u bench.py --gpus 1 $RARGS > $O/bench1.log 2> $O/bench1.err || { tail -c 5000 $O/bench1.err; exit 1; }
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python -u bench.py --gpus 4 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
python - <<'PY'
import json
for n in ("1", "4"):
    d = json.loads([l for l in open(f"gpurun_out/r05_aj/bench{n}.log") if l.startswith("{")][-1])
    e = d["extra"]
    t = e.get("topn", {})
    print(n, "n_gpus", d["n_gpus"], "value", d["value"], "verified", d["verified"], "backend", e.get("backend"))
    print("  topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")}, "verify", t.get("verify"))
PY
echo done
