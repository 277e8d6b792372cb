#!/bin/bash
# Written cold fragments rank through their live host cache; dense cache-only
# TopN keeps n rows past the cache width (TopN + executor suites).
set -o pipefail
mkdir -p gpurun_out/r03_coldrank
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py > gpurun_out/r03_coldrank/pytest.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r03_coldrank/pytest.log | tail -12
[ $rc -eq 0 ] || { grep -B40 "Error\b" gpurun_out/r03_coldrank/pytest.log | tail -80; exit 1; }
