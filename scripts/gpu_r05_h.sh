#!/bin/bash
# Round 5, call H: the small-batch (serving) pair-kernel study -- where a
# 32..96-query batch's GPU time goes (cost-isolation variants, queries per
# wave 32/16/8/4, the tile kernel), the serving sweep per chunk size, and
# BSI config 4 under a kernel trace + FETCH_SIZE (HBM roofline).
set -o pipefail
O=gpurun_out/r05_h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/kbench.py --batch 32 --reps 20 --cq 32,16,8,4 --variants 38,38@16,38@8,31,33,34,35 > $O/kbench_b32.log 2>&1 || { tail -c 3000 $O/kbench_b32.log; exit 1; }
grep -v "^{" $O/kbench_b32.log
timeout -k 10 400 python -u scripts/kbench.py --batch 96 --reps 20 --cq 32,16,8,4 --variants 38,38@16,38@8 > $O/kbench_b96.log 2>&1 || { tail -c 3000 $O/kbench_b96.log; exit 1; }
grep -v "^{" $O/kbench_b96.log
for CQ in 16 8 4; do
  PILOSA_AND2_CQ=$CQ timeout -k 10 300 python -u scripts/bench_server.py --seconds 4 --batchers 1,2,3 > $O/serve_cq$CQ.log 2>&1 || { tail -c 3000 $O/serve_cq$CQ.log; exit 1; }
  python - $O/serve_cq$CQ.log $CQ <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); s = d["server_stats"]
        print("cq", sys.argv[2], "batchers", s.get("count_batchers"), "rps", d["value"], "p50", d["p50_ms"], "p99", d["p99_ms"],
              "batch", round(s["batched_requests"] / max(s["batches"], 1), 1), "prep", s.get("text_prep_ms_per_batch"),
              "wait", s.get("text_wait_ms_per_batch"), "mism", d["mismatches"])
PY
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 3 --no-profile > $O/pmc_c4.log 2>&1 || { tail -c 3000 $O/pmc_c4.log; exit 1; }
echo done
