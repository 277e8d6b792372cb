#!/bin/bash
# Round 5, call M: cache-only TopN over the wide call set (n 1..1000, 72
# thresholds) at full scale: request timing, host profile and kernel trace
# with the single-pass totals kernel; BSI GPU tests (unfiltered Sum path).
set -o pipefail
O=gpurun_out/r05_m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 200 --paths local --wide > $O/prof_topn_wide.log 2>&1 || { tail -c 3000 $O/prof_topn_wide.log; exit 1; }
grep -E "requests x" $O/prof_topn_wide.log
timeout -k 10 600 python -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 200 --paths local > $O/prof_topn_cyc.log 2>&1 || { tail -c 3000 $O/prof_topn_cyc.log; exit 1; }
grep -E "requests x" $O/prof_topn_cyc.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_wide -o wide -- python3 -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 200 --paths local --wide --top 5 > $O/prof_wide_trace.log 2>&1 || { tail -c 3000 $O/prof_wide_trace.log; exit 1; }
echo done
