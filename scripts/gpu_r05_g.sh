#!/bin/bash
# Round 5, call G: GPU tests touched by the TopN group commit / BSI host
# trims, the cache-only TopN request profile at full scale (954 shards, local
# and world-1 mesh), then the driver's bench command (serving mix now with the
# TopN group commit).
set -o pipefail
O=gpurun_out/r05_g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py tests/test_native_http.py tests/test_gpu_kernels.py tests/test_gpu_rccl_mesh.py "tests/test_gpu_shardwidth.py::test_gpu_executor_suite_at_wide_width" -x -q --timeout 900 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 6000 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 5000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_g/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
t = e["topn"]
print("topn", json.dumps({k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_repeated", "src")}))
print("cfg5", json.dumps(e.get("config5_time_union", {}).get("qps")))
print("cfg4", json.dumps({k: v["ms_per_request"] for k, v in e.get("config4_bsi", {}).get("queries", {}).items()}))
s = e["serving"]
print("serving", json.dumps({k: s[k] for k in ("count", "count_topn_mix") if k in s})[:1200])
print("httpd", json.dumps(s.get("httpd"))[:600])
PY
# serving Count: group-commit thread sweep with the prep / wait split per batch
timeout -k 10 400 python -u scripts/bench_server.py --seconds 4 --batchers 1,2,3,4,6 > $O/serve_sweep.log 2>&1 || { tail -c 3000 $O/serve_sweep.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05_g/serve_sweep.log"):
    if l.startswith("{"):
        d = json.loads(l); s = d["server_stats"]
        print("batchers", s.get("count_batchers"), "rps", d["value"], "p50", d["p50_ms"], "p99", d["p99_ms"],
              "batch", round(s["batched_requests"] / max(s["batches"], 1), 1), "ms/batch", s["count_ms_per_batch"],
              "prep", s.get("text_prep_ms_per_batch"), "wait", s.get("text_wait_ms_per_batch"))
PY
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_serve -o serve -- python3 -u scripts/bench_server.py --seconds 4 > $O/serve_prof.log 2>&1 || { tail -c 3000 $O/serve_prof.log; exit 1; }
echo done
