#!/bin/bash
# pair kernel A/B: v6 vs the flat-stream kernel at prefetch depths 1-3
set -o pipefail
O=gpurun_out/r04_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "and2 or array_size" --timeout 300 --timeout-method thread > $O/pytest_pairs.log 2>&1 || { tail -c 4000 $O/pytest_pairs.log; exit 1; }
tail -2 $O/pytest_pairs.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 10,11,12 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
tail -5 $O/kbench.log
timeout -k 10 300 python -u -m pytest tests/test_tracing.py -x -q --timeout 200 --timeout-method thread > $O/pytest_tracing.log 2>&1 || { tail -c 4000 $O/pytest_tracing.log; exit 1; }
tail -2 $O/pytest_tracing.log
