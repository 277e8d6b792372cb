#!/bin/bash
# Cache-only TopN: sampled host stacks of the request threads during the timed run.
set -o pipefail
O=gpurun_out/r04_i
mkdir -p $O
timeout -k 10 600 env PILOSA_BENCH_TOPN_PROFILE=$O/cache_stacks.txt python -u bench.py --steps 2 --warmup 1 \
    --configs none --serve-seconds 0 --topn-batches 40 > $O/bench.log 2> $O/bench.err || { tail -c 2000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04_i/bench.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print("cache", t["cache"].get("qps"), "gc", t["cache"].get("gc_pause_s"), t["cache"].get("gc_collections"),
      "repeated", t["cache_repeated"].get("qps"), "src", t["src"].get("qps"))
PY
