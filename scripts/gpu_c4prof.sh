#!/bin/bash
# Kernel trace of BASELINE config 4 (BSI) incl. the batched-Sum paths.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/c4prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c4prof -o c4 -- python3 $R/bench.py --mode synthetic --steps 2 --warmup 1 --topn-batches 0 --configs 4 --batch 256 > $R/gpurun_out/c4prof/bench.log 2>&1 || { tail -30 $R/gpurun_out/c4prof/bench.log; exit 1; }
cd $R; python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/c4prof/*kernel_stats.csv")[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
d = json.loads(open("gpurun_out/c4prof/bench.log").read().strip().splitlines()[-1])
e = d["extra"]["config4_bsi"]
print({k: v.get("ms", v.get("ms_per_batch")) for k, v in e["queries"].items()}, e["batched_sum_paths_agree"])
PY
