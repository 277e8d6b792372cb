#!/bin/bash
# TopN suites after the reader/writer lock around in-place index refreshes.
set -o pipefail
mkdir -p gpurun_out/r03_rw
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_mesh.py > gpurun_out/r03_rw/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03_rw/pytest.log | tail -8
[ $rc -eq 0 ] || { grep -B40 "Error\b" gpurun_out/r03_rw/pytest.log | tail -60; exit 1; }
