#!/bin/bash
# Round 5, call AM: the driver bench command after the Min/Max fold change.
set -o pipefail
O=gpurun_out/r05_am
mkdir -p $O
timeout -k 10 1000 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_am/bench.log").read().strip().splitlines()[-1])
ex = d["extra"]
print("headline", d["value"], d["ms_per_step"])
print("topn", {k: v.get("qps") for k, v in ex["topn"].items() if isinstance(v, dict)})
print("serving", ex["serving"]["count"]["req_per_s"], ex["serving"]["count"]["p99_ms"], ex["serving"]["count_topn_mix"]["req_per_s"], ex["serving"]["count_topn_mix"]["p99_ms"])
print("bsi", {k: v["ms_per_request"] for k, v in ex["config4_bsi"]["queries"].items()})
print("config5", ex["config5_time_union"]["qps"])
PY
echo done
