#!/bin/bash
# src-TopN kbench over the hot-rank split (PILOSA_TOPN_HOT = ranks counted row-major).
set -o pipefail
mkdir -p gpurun_out
for H in ${HOTS:-512 1024 2048 4096}; do
  PILOSA_TOPN_HOT=$H timeout -k 10 300 python -u scripts/topn_kbench.py --cols 1000000000 > gpurun_out/topn_hot_$H.log 2>&1 || { tail -20 gpurun_out/topn_hot_$H.log; exit 1; }
  echo "HOT=$H $(tail -1 gpurun_out/topn_hot_$H.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["mix"]["e2e_ms_per_batch"], d["mix"]["qps"], d["mix"]["parts_ms"], d["lds_bytes"])')"
done
