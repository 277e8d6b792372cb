#!/bin/bash
# Slot-index TopN kernel timings with cost isolation (scripts/topn_kbench.py).
# DBGS: PILOSA_TOPN_DBG values to run (0 full, 1 no histogram, 2 no walk).
set -o pipefail
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 3}; do
  PILOSA_TOPN_DBG=$d timeout -k 10 240 python -u scripts/topn_kbench.py --cols ${COLS:-1000000000} \
    >> gpurun_out/topn_kbench.log 2>&1 || { tail -20 gpurun_out/topn_kbench.log; exit 1; }
  tail -1 gpurun_out/topn_kbench.log
done
