#!/bin/bash
# Pair kernel v6 with one-ahead prefetch in the multi-chunk array walks
# (variant 10) vs v6: kernel tests with variant 10, then kbench A/B.
set -o pipefail
mkdir -p gpurun_out/r03_pf
PILOSA_AND2_VARIANT=10 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r03_pf/pytest.log 2>&1 || { tail -c 3000 gpurun_out/r03_pf/pytest.log; exit 1; }
tail -1 gpurun_out/r03_pf/pytest.log
timeout -k 10 400 python -u scripts/kbench.py --batch 4096 --reps 7 --no-tile --cq 64 --variants 10,6,10 \
  > gpurun_out/r03_pf/kbench.log 2>&1 || { tail -c 3000 gpurun_out/r03_pf/kbench.log; exit 1; }
grep -v "^{" gpurun_out/r03_pf/kbench.log | tail -5
