#!/bin/bash
# One rank's share at 8 GPUs (119 shards): q/s of the product path plus a
# kernel-trace profile, to size the fixed per-batch cost.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03_small
A="--cols 125000000 --steps 20 --warmup 5 --topn-batches 0 --configs none ${BENCH_ARGS}"
timeout -k 10 300 python -u bench.py $A > gpurun_out/r03_small/bench.log 2>&1 || { tail -c 3000 gpurun_out/r03_small/bench.log; exit 1; }
tail -c 1500 gpurun_out/r03_small/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_small/prof -o small -- \
  python3 $R/bench.py $A > $R/gpurun_out/r03_small/prof.log 2>&1 || { tail -c 2000 $R/gpurun_out/r03_small/prof.log; exit 1; }
find $R/gpurun_out/r03_small/prof -name '*kernel_stats.csv' -exec head -20 {} \;
