#!/bin/bash
# Union-kernel GPU test + A/B first (short), then the round-end style pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_kernels.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_kernels.log
timeout -k 10 300 python -u scripts/union_ab.py > gpurun_out/union_ab.log 2>&1 || { tail -20 gpurun_out/union_ab.log; exit 1; }
tail -1 gpurun_out/union_ab.log
bash scripts/gpu_full.sh
