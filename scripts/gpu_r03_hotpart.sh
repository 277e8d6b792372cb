#!/bin/bash
# Small hot rows with pipelined rank -> meta -> payload loads (groups claimed
# two ahead), at hot-rank splits 2048 / 4096 / 3072; then the TopN GPU tests.
set -o pipefail
mkdir -p gpurun_out/r03_hotpart
for cfg in "1 2048" "1 4096" "1 3072"; do
  set -- $cfg
  PILOSA_TOPN_HOT_PARTIALS=$1 PILOSA_TOPN_HOT=$2 timeout -k 10 300 python -u scripts/topn_kbench.py --reps 5 > gpurun_out/r03_hotpart/p$1_h$2.log 2>&1 || { tail -c 2000 gpurun_out/r03_hotpart/p$1_h$2.log; exit 1; }
  echo "partials=$1 hot=$2 $(grep '^{' gpurun_out/r03_hotpart/p$1_h$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["hot_ms"] for k, v in d["classes"].items()}, d["mix"])')"
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -k "topn or TopN or rank" > gpurun_out/r03_hotpart/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_hotpart/pytest.log; exit 1; }
tail -1 gpurun_out/r03_hotpart/pytest.log
