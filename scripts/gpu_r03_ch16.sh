#!/bin/bash
# Big-row walk with 16 array values per lane per step (two 16-byte loads):
# kernel timing on the headline arena, then the TopN GPU tests.
set -o pipefail
mkdir -p gpurun_out/r03_ch16
timeout -k 10 300 python -u scripts/topn_kbench.py --reps 5 > gpurun_out/r03_ch16/kbench.log 2>&1 || { tail -c 2000 gpurun_out/r03_ch16/kbench.log; exit 1; }
grep '^{' gpurun_out/r03_ch16/kbench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["hot_ms"] for k, v in d["classes"].items()}, d["mix"])'
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -k "topn or TopN or rank" > gpurun_out/r03_ch16/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_ch16/pytest.log; exit 1; }
tail -1 gpurun_out/r03_ch16/pytest.log
