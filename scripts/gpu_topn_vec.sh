#!/bin/bash
# TopN GPU tests + src-TopN kbench (hot-rank vector loads).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py -x -q -k "topn or TopN" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_topn.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_topn.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_topn.log
PILOSA_TOPN_DBG=0 timeout -k 10 300 python -u scripts/topn_kbench.py --cols 1000000000 > gpurun_out/topn_kbench_vec.log 2>&1 || { tail -20 gpurun_out/topn_kbench_vec.log; exit 1; }
tail -1 gpurun_out/topn_kbench_vec.log
