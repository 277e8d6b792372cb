#!/bin/bash
# Round 5, call C: v16 (lane-parallel small-B pass) correctness + timing,
# attribution variants re-measured with v6's LDS pinned (occupancy 5), and
# the device Shift across wide-shard sub-shards.
set -o pipefail
O=gpurun_out/r05_c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "and2 or array_size" --timeout 300 --timeout-method thread > $O/pytest_pairs.log 2>&1 || { tail -c 5000 $O/pytest_pairs.log; exit 1; }
tail -2 $O/pytest_pairs.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 16,17,18,31,32,33,34,35 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
grep -v "^{" $O/kbench.log | tail -10
timeout -k 10 600 python -u -m pytest tests/test_gpu_executor.py -x -q -k "shift" --timeout 300 --timeout-method thread > $O/pytest_shift.log 2>&1 || { tail -c 5000 $O/pytest_shift.log; exit 1; }
tail -2 $O/pytest_shift.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_shardwidth.py -x -v -k "wide_width" --timeout 880 --timeout-method thread > $O/pytest_wide.log 2>&1 || { tail -c 5000 $O/pytest_wide.log; exit 1; }
tail -3 $O/pytest_wide.log
