#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03_topn
timeout -k 10 280 python -u bench.py --cols 125000000 --steps 10 --warmup 3 --configs none 2>&1 | tee gpurun_out/r03_topn/bench_small.log | grep -v "^{" 
tail -c 2000 gpurun_out/r03_topn/bench_small.log
