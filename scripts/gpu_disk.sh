#!/bin/bash
# Round-2 pass: GPU tests (strict), disk-mode bench small then full, synthetic harness.
set -o pipefail
mkdir -p gpurun_out
df -h /tmp "${TMPDIR:-/tmp}" > gpurun_out/df.txt 2>&1; free -g >> gpurun_out/df.txt; nproc >> gpurun_out/df.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 300 python -u bench.py --mode disk --cols 125000000 --steps 10 --warmup 2 --topn-batches 0 \
  > gpurun_out/bench_disk_small.log 2>&1 || { tail -30 gpurun_out/bench_disk_small.log; exit 1; }
tail -1 gpurun_out/bench_disk_small.log
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_disk_full.log 2>&1 || { tail -30 gpurun_out/bench_disk_full.log; exit 1; }
tail -1 gpurun_out/bench_disk_full.log
