#!/bin/bash
# Pair-kernel A/B (v6 vs v7) on the headline arena.
set -o pipefail
mkdir -p gpurun_out/r03_kb
timeout -k 10 400 python -u scripts/kbench.py --batch ${BATCH:-4096} --reps 7 --no-tile --cq "" --variants ${VARIANTS:-6,7} ${KB_ARGS} \
  > gpurun_out/r03_kb/kbench.log 2>&1 || { tail -c 3000 gpurun_out/r03_kb/kbench.log; exit 1; }
grep -v "^{" gpurun_out/r03_kb/kbench.log | tail -5
