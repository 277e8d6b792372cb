#!/bin/bash
# Hot-rank TopN kernel with rotating prefetch buffers and batched table
# reads: TopN GPU tests, then the kernel trace of executor-path src TopN.
set -o pipefail
mkdir -p gpurun_out/r03_hot
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -k "topn or TopN or rank" > gpurun_out/r03_hot/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_hot/pytest.log; exit 1; }
tail -1 gpurun_out/r03_hot/pytest.log
bash scripts/gpu_r03_topnprof.sh
