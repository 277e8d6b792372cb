#!/bin/bash
# Round 6, call L: serving Count. Group-commit thread sweep on the shipped
# serving variant (39), the same with round 5's variant 40 (kbench module),
# and a kernel trace of the serving run.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_l
mkdir -p $O
timeout -k 10 400 python3 -u scripts/bench_server.py --seconds 4 --batchers 1,2,3 > $O/serve_v39.log 2>&1 || { tail -c 3000 $O/serve_v39.log; exit 1; }
grep "^{" $O/serve_v39.log | cut -c 1-600
timeout -k 10 400 env PILOSA_HIPKERNELS=_hipkernels_kbench PILOSA_AND2_VARIANT=40 python3 -u scripts/bench_server.py --seconds 4 --batchers 2 > $O/serve_v40.log 2>&1 || { tail -c 3000 $O/serve_v40.log; exit 1; }
grep "^{" $O/serve_v40.log | cut -c 1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o serve -- python3 $R/scripts/bench_server.py --seconds 3 --batchers 2 > $O/serve_prof.log 2>&1 || { tail -c 3000 $O/serve_prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_head -o head -- python3 $R/bench.py --serve-seconds 0 --configs= --topn-batches 0 --topn-cache-batches 0 --topn-src-batches 0 --steps 10 --warmup 2 > $O/head_prof.log 2>&1 || { tail -c 3000 $O/head_prof.log; exit 1; }
cd $R
find $O/prof $O/prof_head -name "*kernel_stats.csv" | head -3
for f in $(find $O/prof $O/prof_head -name "*kernel_stats.csv"); do echo $f; head -12 $f | cut -c 1-220; done
echo done
