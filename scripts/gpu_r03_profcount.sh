#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03_profcount
timeout -k 10 300 python -u scripts/prof_count_exec.py > gpurun_out/r03_profcount/prof.log 2>&1; rc=$?
tail -c 5000 gpurun_out/r03_profcount/prof.log
exit $rc
