#!/bin/bash
# Round 6, call AY: the whole GPU suite again (rank caches settled before device-vs-host TopN comparisons).
set -o pipefail
O=gpurun_out/r06_ay
mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
echo done
