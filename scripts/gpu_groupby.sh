#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_kernels.py -x -q -k "groupby or bitgemm or GroupBy" \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_groupby.log 2>&1 || { tail -40 gpurun_out/pytest_groupby.log; exit 1; }
tail -1 gpurun_out/pytest_groupby.log
