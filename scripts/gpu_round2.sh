#!/bin/bash
# GPU tests of the expression kernels after the meta-table change, the
# tile-kernel A/B point, then the pair-kernel PMC passes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_executor.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_expr.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_expr.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_expr.log
timeout -k 10 300 python -u scripts/kbench.py --reps 3 --cq 64 --batch 4096 > gpurun_out/kbench_tile.log 2>&1 || { tail -20 gpurun_out/kbench_tile.log; exit 1; }
tail -1 gpurun_out/kbench_tile.log
bash scripts/gpu_pmc_v6.sh
