#!/bin/bash
# Pair-kernel timing (shipped v6) + its GPU tests.
set -o pipefail
mkdir -p gpurun_out/r03_kb
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r03_kb/pytest.log 2>&1 || { tail -c 3000 gpurun_out/r03_kb/pytest.log; exit 1; }
tail -2 gpurun_out/r03_kb/pytest.log
timeout -k 10 400 python -u scripts/kbench.py --batch ${BATCH:-4096} --reps 7 --no-tile --cq ${CQ:-64} ${KB_ARGS} \
  > gpurun_out/r03_kb/kbench.log 2>&1 || { tail -c 3000 gpurun_out/r03_kb/kbench.log; exit 1; }
grep -v "^{" gpurun_out/r03_kb/kbench.log | tail -5
