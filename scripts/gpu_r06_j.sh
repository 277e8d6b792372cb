#!/bin/bash
# Round 6, call J: serving-size pair-kernel sweep (kbench module): variants
# 6 / 38 / 39 / 40 / 13 at 2-16 queries per wave, 32- and 64-query batches.
set -o pipefail
O=gpurun_out/r06_j
mkdir -p $O
for B in 32 64 128; do
  timeout -k 10 300 python3 -u scripts/kbench.py --batch $B --reps 30 --cq "" --no-tile \
    --variants 40@8,40@4,39@8,39@4,38@8,38@4,6@8,6@4,13@8,40@16,39@16 > $O/kbench_b$B.log 2>&1 || { tail -30 $O/kbench_b$B.log; exit 1; }
  echo "batch $B"; grep -v "^{" $O/kbench_b$B.log | grep and2
done
echo done
