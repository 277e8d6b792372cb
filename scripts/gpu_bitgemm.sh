#!/bin/bash
# bitgemm correctness (MFMA and VALU vs host) then MFMA vs VALU timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k bitgemm --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_bitgemm.log 2>&1 || { tail -40 gpurun_out/pytest_bitgemm.log; exit 1; }
tail -1 gpurun_out/pytest_bitgemm.log
timeout -k 10 300 python -u scripts/bitgemm_bench.py ${BG_ARGS} > gpurun_out/bitgemm_bench.log 2>&1 \
  || { tail -20 gpurun_out/bitgemm_bench.log; exit 1; }
tail -1 gpurun_out/bitgemm_bench.log
