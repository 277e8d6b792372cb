#!/bin/bash
# Round 6, call K: serving batches on variant 39 (batched staging, 4 / 16
# queries per wave): pair-kernel GPU tests, then the driver bench command.
set -o pipefail
O=gpurun_out/r06_k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $O/pytest_kernels.log 2>&1 || { tail -c 4000 $O/pytest_kernels.log; exit 1; }
tail -1 $O/pytest_kernels.log
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_k/bench.log") if l.startswith("{")][-1])
e = d["extra"]; t = e.get("topn", {})
print("value", d["value"], "ms", d["ms_per_step"], "verified", d.get("verified"))
print("topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
s = e.get("serving") or {}
print("serving count", s.get("count"))
print("serving mix", s.get("count_topn_mix"))
print("httpd", s.get("httpd"))
PY
echo done
