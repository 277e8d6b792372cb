#!/bin/bash
# Round 5, call K: dense bitmap shadows of the hottest rows for the pair
# kernels (variants 41 / 42): correctness, headline and serving batch
# timings against the shadow-less kernels, serving with and without, then
# the driver's bench command.
set -o pipefail
O=gpurun_out/r05_k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_executor.py tests/test_gpu_topn_exec.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/kbench.py --batch 4096 --reps 5 --no-tile --cq 64 --variants 41 > $O/kbench_b4096.log 2>&1 || { tail -c 3000 $O/kbench_b4096.log; exit 1; }
grep -v "^{" $O/kbench_b4096.log
timeout -k 10 400 python -u scripts/kbench.py --batch 32 --reps 20 --no-tile --cq 8 --variants 40@8,42@8,41@32 > $O/kbench_b32.log 2>&1 || { tail -c 3000 $O/kbench_b32.log; exit 1; }
grep -v "^{" $O/kbench_b32.log
timeout -k 10 400 python -u scripts/kbench.py --batch 64 --reps 20 --no-tile --cq 8 --variants 40@8,42@8 > $O/kbench_b64.log 2>&1 || { tail -c 3000 $O/kbench_b64.log; exit 1; }
grep -v "^{" $O/kbench_b64.log
for SH in 1 0; do
  PILOSA_SHADOW=$SH timeout -k 10 300 python -u scripts/bench_server.py --seconds 5 --batchers 2,3 > $O/serve_sh$SH.log 2>&1 || { tail -c 3000 $O/serve_sh$SH.log; exit 1; }
  python - $O/serve_sh$SH.log "shadow $SH" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); s = d["server_stats"]
        print(sys.argv[2], "batchers", s.get("count_batchers"), "rps", d["value"], "p50", d["p50_ms"], "p99", d["p99_ms"],
              "batch", round(s["batched_requests"] / max(s["batches"], 1), 1), "prep", s.get("text_prep_ms_per_batch"),
              "wait", s.get("text_wait_ms_per_batch"), "mism", d["mismatches"])
PY
done
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 5000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_k/bench.log") if l.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"])
t = e["topn"]
print("topn", json.dumps({k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")}))
print("cfg5", json.dumps(e.get("config5_time_union", {}).get("qps")))
print("cfg4", json.dumps({k: v["ms_per_request"] for k, v in e.get("config4_bsi", {}).get("queries", {}).items()}))
s = e["serving"]
print("serving", json.dumps({k: s[k] for k in ("count", "count_topn_mix") if k in s})[:1200])
PY
echo done
