#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03_topn
SHARDS=${SHARDS:-120} timeout -k 10 300 python -u scripts/prof_topn_exec.py > gpurun_out/r03_topn/prof_topn.log 2>&1 || { tail -c 3000 gpurun_out/r03_topn/prof_topn.log; exit 1; }
grep -E "request|threads" gpurun_out/r03_topn/prof_topn.log
