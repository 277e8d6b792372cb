#!/bin/bash
# Round-end style pass: all GPU tests, smoke, full bench, kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o final -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_final.log 2>&1 || { tail -20 $R/gpurun_out/prof_final.log; exit 1; }
echo PROFILED
