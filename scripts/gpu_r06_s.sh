#!/bin/bash
# Round 6, call S: headline Count(Intersect) with each request thread on a
# HIP stream of its own (the next batch's pair build and small kernels can
# fill the pair kernel's tail) vs the shared default stream.
set -o pipefail
O=gpurun_out/r06_s
D=/tmp/r06s_data
mkdir -p $O
run() {  # name, thread streams, clients
  timeout -k 10 420 env PILOSA_BENCH_THREAD_STREAMS=$2 python3 -u bench.py --serve-seconds 0 --configs= --topn-batches 0 --steps 40 --warmup 3 --clients $3 --data-dir $D --keep-data > $O/$1.log 2> $O/$1.err || { tail -c 3000 $O/$1.err; exit 1; }
  python3 - $O/$1.log $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["extra"].get("verified"))
PY
}
run base_c2 0 2
run ts_c2 1 2
run ts_c3 1 3
run base_c2b 0 2
run ts_c2b 1 2
rm -rf $D
echo done
