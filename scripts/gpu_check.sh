#!/bin/bash
# One GPU-box pass: build, GPU tests, bench, kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  R=$PWD
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof.log 2>&1 || { tail -30 $R/gpurun_out/prof.log; exit 1; }
  cd $R
fi
echo DONE
