#!/bin/bash
# Headline Count(Intersect) path only: per-kernel stats of the driver's bench step.
set -o pipefail
O=gpurun_out/r04_n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 \
    --configs none --serve-seconds 0 --topn-batches 0 > $O/bench.log 2> $O/bench.err || { tail -c 2000 $O/bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-200
grep '^{' $O/bench.log | cut -c1-400
