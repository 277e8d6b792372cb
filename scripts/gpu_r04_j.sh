#!/bin/bash
# Kernel stats of the TopN phases (cache-only batches: topn_cache_* kernels).
set -o pipefail
O=gpurun_out/r04_j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 \
    --configs none --serve-seconds 0 --topn-batches 40 > $O/bench.log 2> $O/bench.err || { tail -c 2000 $O/bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-220
