#!/bin/bash
# Pair-kernel cost isolation + kernel-trace stats of the A/B harness.
set -o pipefail
mkdir -p gpurun_out/kprof
R=$PWD
timeout -k 10 300 python -u scripts/kbench.py --batch 4096 --reps 3 --cq 64 --dbg > gpurun_out/kbench_dbg.log 2>&1 || { tail -30 gpurun_out/kbench_dbg.log; exit 1; }
grep -v "^{" gpurun_out/kbench_dbg.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kprof -o kb -- python3 $R/scripts/kbench.py --batch 4096 --reps 3 --cq 64 > $R/gpurun_out/kprof/kb.log 2>&1 || { tail -30 $R/gpurun_out/kprof/kb.log; exit 1; }
cd $R; find gpurun_out/kprof -name "*kernel_stats.csv" | head -3
head -8 $(find gpurun_out/kprof -name "*kernel_stats.csv" | head -1) | cut -c1-220
