#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03_cfg5
timeout -k 10 600 python -u scripts/prof_cfg5.py > gpurun_out/r03_cfg5/prof.log 2>&1 || { tail -c 3000 gpurun_out/r03_cfg5/prof.log; exit 1; }
head -60 gpurun_out/r03_cfg5/prof.log | grep -v "^$"
