#!/bin/bash
# 1- and 2-rank disk-mode bench rehearsal (gloo through host copies on one
# GPU) after the round-3 changes; the mean counts must agree.
set -o pipefail
NP=2 COLS=60000000 BATCH=1024 timeout -k 10 900 bash scripts/gpu_rehearse_disk.sh > gpurun_out/r03_rehearse.log 2>&1 || { tail -c 3000 gpurun_out/r03_rehearse.log; exit 1; }
cat gpurun_out/r03_rehearse.log
