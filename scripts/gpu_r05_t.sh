#!/bin/bash
# Round 5, call T: carry-save counting in the hot-rank TopN kernel.
# Exactness against a dense fp32 reference (every lane-owned bound, both
# counting modes), the TopN suites, kernel timing per setting and per path
# (PILOSA_TOPN_DBG isolation), and config 4 under a kernel trace.
set -o pipefail
O=gpurun_out/r05_t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py -x -v --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "slot_index or topn or TopN or bsi" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "base:" "bytecnt:PILOSA_TOPN_DBG=128" "small1023:PILOSA_TOPN_SMALL_N=1023" "small4096:PILOSA_TOPN_SMALL_N=4096" "nolane:PILOSA_TOPN_DBG=8" "nocoop:PILOSA_TOPN_DBG=16" "bytecnt_nolane:PILOSA_TOPN_DBG=136"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(tail -1 $O/kb_$name.log | cut -c1-600)"
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
echo done
