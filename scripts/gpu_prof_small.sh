#!/bin/bash
# Kernel-trace of the disk bench at 1/8 of the shards (the per-rank work of an 8-GPU run).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/prof_small
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_small -o small -- python3 $R/bench.py --cols 125000000 --steps 10 --warmup 2 --topn-batches 0 > $R/gpurun_out/prof_small/bench.log 2>&1 || { tail -30 $R/gpurun_out/prof_small/bench.log; exit 1; }
cd $R; tail -1 gpurun_out/prof_small/bench.log | cut -c1-300
f=$(find gpurun_out/prof_small -name "*kernel_stats.csv" | head -1); head -14 $f | cut -d, -f1-4 | cut -c1-200
f=$(find gpurun_out/prof_small -name "*memory_copy_stats.csv" | head -1); [ -n "$f" ] && head -5 $f | cut -c1-200
