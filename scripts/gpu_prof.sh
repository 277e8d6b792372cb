#!/bin/bash
# Kernel-trace profile of a short bench run: gpurun_out/prof/<tag>_kernel_stats.csv
set -o pipefail
TAG=${TAG:-bench}
R=$PWD
mkdir -p gpurun_out/prof
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o $TAG -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_$TAG.log
ls $R/gpurun_out/prof
