#!/bin/bash
# all GPU tests, then BASELINE config 5 (time-view union counts).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 400 python -u scripts/bench_configs.py --only 5 > gpurun_out/cfg5.log 2>&1 || { tail -20 gpurun_out/cfg5.log; exit 1; }
tail -1 gpurun_out/cfg5.log
