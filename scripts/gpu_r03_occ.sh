#!/bin/bash
# Occupancy sensitivity of the pair kernel: v6 at 20 waves/CU (8 KiB LDS)
# against the same code with LDS padded to 10 KiB (16 waves/CU, variant 7)
# and 13 KiB (12 waves/CU, variant 8).  The probe variants were removed after
# the measurement (profiles/r03_occ/); variants 7 and 8 now run the shipped v6.
set -o pipefail
mkdir -p gpurun_out/r03_occ
timeout -k 10 400 python -u scripts/kbench.py --batch 4096 --reps 7 --no-tile --cq 64 --variants 7,8,6 \
  > gpurun_out/r03_occ/kbench.log 2>&1 || { tail -c 3000 gpurun_out/r03_occ/kbench.log; exit 1; }
grep -v "^{" gpurun_out/r03_occ/kbench.log | tail -6
