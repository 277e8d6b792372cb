#!/bin/bash
# all GPU tests, then the row-op timings on the config-2 index and a kernel trace of them.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 500 python -u scripts/bench_configs.py --only r > gpurun_out/rowops.log 2>&1 || { tail -20 gpurun_out/rowops.log; exit 1; }
tail -1 gpurun_out/rowops.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rowops -o run -- \
  python3 -u scripts/bench_configs.py --only r --reps 3 > gpurun_out/rowops_prof.log 2>&1 || { tail -20 gpurun_out/rowops_prof.log; exit 1; }
find gpurun_out/prof_rowops -name "*kernel_stats.csv" | head -3
