#!/bin/bash
# GPU test suite + 2/4-rank disk rehearsal of the N>1 bench path (device-tensor
# all-reduce) after the mesh / cold-read / D2H changes.
set -o pipefail
mkdir -p gpurun_out/r03_check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_check/pytest_gpu.log 2>&1 \
  || { tail -c 4000 gpurun_out/r03_check/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03_check/pytest_gpu.log
NP=4 COLS=50000000 BATCH=1024 timeout -k 10 800 bash scripts/gpu_rehearse_disk.sh > gpurun_out/r03_check/rehearse.log 2>&1 \
  || { tail -c 3000 gpurun_out/r03_check/rehearse.log; exit 1; }
cat gpurun_out/r03_check/rehearse.log
cp gpurun_out/rehearse_disk*.log gpurun_out/r03_check/
