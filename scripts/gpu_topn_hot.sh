#!/bin/bash
# Hot-rank TopN A/B (scripts/topn_kbench.py): histogram only (hot 0) vs hot
# ranks counted row-major (2048, 4096), then the GPU TopN tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "topn or TopN" \
  > gpurun_out/pt_topn.log 2>&1 || { tail -30 gpurun_out/pt_topn.log; exit 1; }
tail -1 gpurun_out/pt_topn.log
for h in ${HOTS:-0 2048 4096}; do
  PILOSA_TOPN_HOT=$h timeout -k 10 240 python -u scripts/topn_kbench.py --cols ${COLS:-1000000000} \
    >> gpurun_out/topn_hot.log 2>&1 || { tail -20 gpurun_out/topn_hot.log; exit 1; }
  tail -1 gpurun_out/topn_hot.log
done
