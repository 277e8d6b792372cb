#!/bin/bash
# Round 5, call R: cache-only TopN (wide call set) at 1 / 2 / 3 request
# threads with memo reuse across prefix buckets; the unrolled Min/Max fold
# and BSI tests; then the driver's bench command.
set -o pipefail
O=gpurun_out/r05_r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "not boundaries" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 300 --paths local --wide --clients 1 --top 25 > $O/prof_topn_wide.log 2>&1 || { tail -c 3000 $O/prof_topn_wide.log; exit 1; }
grep -E "request thread" $O/prof_topn_wide.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 5000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_r/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
t = e["topn"]
print("topn", json.dumps({k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")}), json.dumps(t.get("verify")))
print("cfg4", json.dumps({k: v["ms_per_request"] for k, v in e.get("config4_bsi", {}).get("queries", {}).items()}))
s = e["serving"]
print("serving", json.dumps({k: s[k] for k in ("count", "count_topn_mix") if k in s})[:1200])
PY
echo done
