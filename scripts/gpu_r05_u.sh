#!/bin/bash
# Round 5, call U: hot-rank TopN table build as a transpose of bitmap srcs
# (no per-bit LDS atomics); exactness, then kernel timing with isolation.
set -o pipefail
O=gpurun_out/r05_u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py -x -v --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
for cfg in "base:" "atomicbuild:PILOSA_TOPN_DBG=1024" "nolaneatomics:PILOSA_TOPN_DBG=256" "nocoopbitmap:PILOSA_TOPN_DBG=32" "nocooparray:PILOSA_TOPN_DBG=64" "nolane:PILOSA_TOPN_DBG=8" "nocoop:PILOSA_TOPN_DBG=16" "tableonly:PILOSA_TOPN_DBG=24"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(tail -1 $O/kb_$name.log | cut -c1-400)"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "slot_index or topn or TopN" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo done
