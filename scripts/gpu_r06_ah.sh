#!/bin/bash
# Round 6, call AH: the 4-rank rehearsal, again after the src TopN fixed-cost changes (4 ranks time-sharing the GPU, gloo
# collectives on host copies) with the native mesh TopN issue/finish and the
# flat phase-1 histogram, against 1 rank on the same reduced index.
set -o pipefail
O=gpurun_out/r06_ah
mkdir -p $O
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-src-batches 40 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python3 -u bench.py --gpus 4 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --gpus 1 --mesh $RARGS > $O/bench1_mesh.log 2> $O/bench1_mesh.err || { tail -c 3000 $O/bench1_mesh.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --gpus 1 $RARGS > $O/bench1.log 2> $O/bench1.err || { tail -c 3000 $O/bench1.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench4", "bench1_mesh", "bench1"):
    d = json.loads([l for l in open(f"gpurun_out/r06_ah/{n}.log") if l.startswith("{")][-1])
    t = d["extra"].get("topn", {})
    print(n, "value", d["value"], {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "src")}, t.get("verify"), d["extra"].get("verified"))
PY
echo done
