#!/bin/bash
# pair kernel: v6 at 16 / 32 / 64 queries per wave (L2 footprint of the units
# in flight per XCD) and variant 15 (non-temporal loads for single-use B containers).
set -o pipefail
O=gpurun_out/r04_o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "and2 or array_size" --timeout 300 --timeout-method thread > $O/pytest_pairs.log 2>&1 || { tail -c 4000 $O/pytest_pairs.log; exit 1; }
tail -2 $O/pytest_pairs.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 15 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
tail -6 $O/kbench.log
