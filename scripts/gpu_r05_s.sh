#!/bin/bash
# Round 5, call S: the hot-rank TopN kernel with the full-chunk fast path
# (kbench + slot-index tests), and config 4 under a kernel trace (Sum after
# the double-buffered planes).
set -o pipefail
O=gpurun_out/r05_s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "slot_index or topn or TopN or bsi" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u scripts/topn_kbench.py --reps 3 > $O/topn_kbench.log 2>&1 || { tail -c 2000 $O/topn_kbench.log; exit 1; }
tail -1 $O/topn_kbench.log | cut -c1-800
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
echo done
