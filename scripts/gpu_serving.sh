#!/bin/bash
# GPU executor tests, then end-to-end HTTP serving throughput with and
# without cross-request coalescing (scripts/bench_server.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_exec.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_exec.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_exec.log
for c in 1 0; do
  PILOSA_COALESCE=$c timeout -k 10 300 python -u scripts/bench_server.py --shards ${SHARDS:-64} --seconds 10 \
    > gpurun_out/serving_c$c.log 2>&1 || { tail -20 gpurun_out/serving_c$c.log; exit 1; }
  tail -1 gpurun_out/serving_c$c.log
done
