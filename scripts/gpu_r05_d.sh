#!/bin/bash
# Round 5, call D: B-head prefetch depth (v6 PD 2/3/4, skeletons at PD 2/3),
# small-B lane pass with loads up front (SB 16/32); host profiles of the
# cache-only TopN request (local vs world-1 RCCL mesh) and of config 4.
set -o pipefail
O=gpurun_out/r05_d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "and2 or array_size" --timeout 300 --timeout-method thread > $O/pytest_pairs.log 2>&1 || { tail -c 5000 $O/pytest_pairs.log; exit 1; }
tail -2 $O/pytest_pairs.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 16,17,18,19,20,31,36,37 > $O/kbench.log 2>&1 || { tail -c 3000 $O/kbench.log; exit 1; }
grep -v "^{" $O/kbench.log | tail -10
timeout -k 10 600 python -u scripts/prof_topn_paths.py --reqs 300 > $O/prof_topn.log 2>&1 || { tail -c 3000 $O/prof_topn.log; exit 1; }
grep -E "requests x|mesh data" $O/prof_topn.log
timeout -k 10 600 python -u scripts/prof_configs.py --which 4 --reps 20 > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
head -c 1500 $O/prof_c4.log
