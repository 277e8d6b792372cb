#!/bin/bash
# Round 6, call O: native cache-only TopN request object (binding.cpp
# CacheTopN) -- GPU tests against the Python lane path, then the bench's
# cache-only phases native vs Python and with 1 / 2 / 3 request threads.
set -o pipefail
O=gpurun_out/r06_o
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_topn_exec.py > $O/pytest_topn.log 2>&1 || { tail -40 $O/pytest_topn.log; exit 1; }
tail -3 $O/pytest_topn.log
run() {  # name, native (1/0), cache-phase request threads
  local name=$1
  timeout -k 10 420 env PILOSA_TOPN_NATIVE=$2 python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 --topn-cache-clients $3 > $O/bench_$name.log 2> $O/bench_$name.err || { tail -c 3000 $O/bench_$name.err; exit 1; }
  python3 - $O/bench_$name.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d.get("extra", {}).get("topn", {})
print(sys.argv[2], d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v})
PY
}
run native1 1 1
run python1 0 1
run native2 1 2
run native3 1 3
echo done
