#!/bin/bash
# Round 6, call BB: device rank caches tie-break by row id (the width-18 slot-index flake of call AZ),
# the TopN modules at width 18 first, then the whole GPU suite and smoke.
set -o pipefail
O=gpurun_out/r06_bb
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shardwidth.py > $O/pytest_width.log 2>&1 || { tail -c 4000 $O/pytest_width.log; exit 1; }
tail -2 $O/pytest_width.log
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -c 3000 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo done
