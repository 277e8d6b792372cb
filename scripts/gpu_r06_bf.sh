#!/bin/bash
# Round 6, call BF: headline request threads 2 vs 3, alternating on one box and one data dir
# (headline phase only).
set -o pipefail
O=gpurun_out/r06_bf
mkdir -p $O
D=/tmp/pilosa_bf_data
i=0
for c in 2 3 2 3; do
  i=$((i+1))
  timeout -k 10 240 python3 -u bench.py --clients $c --serve-seconds 0 --configs "" --topn-batches 0 --data-dir $D --keep-data > $O/bench_c${c}_$i.log 2> $O/bench_c${c}_$i.err || { tail -c 2000 $O/bench_c${c}_$i.err; exit 1; }
  python3 - $O/bench_c${c}_$i.log $c <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("clients", sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "verified", d.get("verified"))
PY
done
echo done
