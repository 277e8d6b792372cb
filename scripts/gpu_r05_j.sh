#!/bin/bash
# Round 5, call J: batched array staging (variant 39) and one-off direct
# probes + batched staging (40) against the shipped v6, at the headline
# batch and at serving batch sizes, then the serving sweep with them.
set -o pipefail
O=gpurun_out/r05_j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "boundaries or scatter" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/kbench.py --batch 4096 --reps 5 --no-tile --cq 64 --variants 39,40 > $O/kbench_b4096.log 2>&1 || { tail -c 3000 $O/kbench_b4096.log; exit 1; }
grep -v "^{" $O/kbench_b4096.log
timeout -k 10 400 python -u scripts/kbench.py --batch 32 --reps 20 --no-tile --cq 32,8 --variants 38,39,40,40@8,40@16 > $O/kbench_b32.log 2>&1 || { tail -c 3000 $O/kbench_b32.log; exit 1; }
grep -v "^{" $O/kbench_b32.log
timeout -k 10 400 python -u scripts/kbench.py --batch 64 --reps 20 --no-tile --cq 32,8 --variants 39,40,40@8,40@16 > $O/kbench_b64.log 2>&1 || { tail -c 3000 $O/kbench_b64.log; exit 1; }
grep -v "^{" $O/kbench_b64.log
for V in "32 6" "32 40" "8 40"; do
  set -- $V
  PILOSA_AND2_CQ=$1 PILOSA_AND2_VARIANT=$2 timeout -k 10 300 python -u scripts/bench_server.py --seconds 4 --batchers 2,3 > $O/serve_cq$1_v$2.log 2>&1 || { tail -c 3000 $O/serve_cq$1_v$2.log; exit 1; }
  python - $O/serve_cq$1_v$2.log "cq $1 v $2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); s = d["server_stats"]
        print(sys.argv[2], "batchers", s.get("count_batchers"), "rps", d["value"], "p50", d["p50_ms"], "p99", d["p99_ms"],
              "batch", round(s["batched_requests"] / max(s["batches"], 1), 1), "prep", s.get("text_prep_ms_per_batch"),
              "wait", s.get("text_wait_ms_per_batch"), "mism", d["mismatches"])
PY
done
echo done
