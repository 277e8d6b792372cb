#!/bin/bash
# Kernel trace of the native serving path (scripts/bench_server.py, 5 s).
set -o pipefail
mkdir -p gpurun_out/servprof
R=$PWD
D=${TMPDIR:-/tmp}/pilosa_serve_data
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/servprof -o sv -- \
  python3 $R/scripts/bench_server.py --data-dir $D --seconds 5 > $R/gpurun_out/servprof/sv.log 2>&1 \
  || { tail -20 $R/gpurun_out/servprof/sv.log; exit 1; }
cd $R; grep '^{' gpurun_out/servprof/sv.log | tail -1
f=$(find gpurun_out/servprof -name "*kernel_stats.csv" | head -1); head -12 $f | cut -d, -f1-4 | cut -c1-160
timeout -k 10 200 python -u scripts/serve_micro.py $D 40 > gpurun_out/servprof/micro.log 2>&1 || { tail -20 gpurun_out/servprof/micro.log; exit 1; }
tail -1 gpurun_out/servprof/micro.log
