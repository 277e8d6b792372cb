#!/bin/bash
# Serving-mix repeat (Count + cache-only TopN over native HTTP) to size its
# run-to-run spread: two bench runs without configs 4/5.
set -o pipefail
mkdir -p gpurun_out/r03_mix
for i in 1 2; do
  timeout -k 10 500 python -u bench.py --gpus 1 --steps 5 --warmup 2 --configs "" > gpurun_out/r03_mix/bench$i.log 2> gpurun_out/r03_mix/bench$i.err || { tail -c 3000 gpurun_out/r03_mix/bench$i.err; exit 1; }
  python - $i <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/r03_mix/bench{sys.argv[1]}.log") if l.startswith("{")][-1])
s = d["extra"]["serving"]
print("run", sys.argv[1], "count", s["count"]["req_per_s"], s["count"]["p99_ms"], "mix", s["count_topn_mix"]["req_per_s"], s["count_topn_mix"]["p99_ms"])
PY
done
