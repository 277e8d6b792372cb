#!/bin/bash
# v10 cost isolation (debug variants: no probes / no staging / no chunk loads / no singletons)
set -o pipefail
O=gpurun_out/r04_c
mkdir -p $O
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 3 --cq 64 --no-tile --variants 11,21,22,23,24 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
tail -7 $O/kbench.log
