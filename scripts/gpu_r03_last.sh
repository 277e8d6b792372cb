#!/bin/bash
# Last check of the shipped build: TopN / executor GPU tests and smoke.
set -o pipefail
mkdir -p gpurun_out/r03_last
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py tests/test_gpu_kernels.py > gpurun_out/r03_last/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_last/pytest.log; exit 1; }
tail -1 gpurun_out/r03_last/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_last/smoke.log 2>&1 || { cat gpurun_out/r03_last/smoke.log; exit 1; }
tail -1 gpurun_out/r03_last/smoke.log
