#!/bin/bash
# TopN GPU tests (incl. the 32-query hot launch) + src-TopN kbench (BATCHES, default 16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py -x -q -k "topn or TopN" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_topn.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_topn.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_topn.log
for B in ${BATCHES:-16}; do  # 32 needs PILOSA_TOPN_HOT_Q=32
  timeout -k 10 300 python -u scripts/topn_kbench.py --cols 1000000000 --batch $B > gpurun_out/topn_kbench_b$B.log 2>&1 || { tail -20 gpurun_out/topn_kbench_b$B.log; exit 1; }
  tail -1 gpurun_out/topn_kbench_b$B.log
done
