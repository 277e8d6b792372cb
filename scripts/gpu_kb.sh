#!/bin/bash
# Kernel iteration pass: GPU kernel tests, pair-kernel A/B on the headline data, short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_kernels.log 2>&1 || { tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
timeout -k 10 300 python -u scripts/kbench.py --batch 4096 --reps 5 --cq ${KB_CQ:-64} ${KB_ARGS} > gpurun_out/kbench.log 2>&1 || { tail -30 gpurun_out/kbench.log; exit 1; }
grep -v "^{" gpurun_out/kbench.log
if [ -n "$FULL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_all.log
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
  tail -1 gpurun_out/bench_full.log | cut -c1-600
fi
