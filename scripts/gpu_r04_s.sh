#!/bin/bash
# One rank's share at 8 GPUs (120 shards): request threads 2 vs 3.
set -o pipefail
O=gpurun_out/r04_s
mkdir -p $O
D=/tmp/pilosa_r04s
for C in 2 3; do
  timeout -k 10 600 python -u bench.py --cols 125000000 --steps 40 --warmup 5 --clients $C --configs none --serve-seconds 0 \
      --topn-batches 0 --data-dir $D --keep-data > $O/bench_c$C.log 2> $O/bench_c$C.err || { tail -c 2000 $O/bench_c$C.err; exit 1; }
  python - "$O/bench_c$C.log" "$C" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("clients", sys.argv[2], "value", d["value"], "ms_per_step", d["ms_per_step"], "verified", d.get("verified"))
PY
done
