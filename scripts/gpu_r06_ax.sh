#!/bin/bash
# Round 6, call AX: the whole GPU suite after the fused cache-only launches (final code).
set -o pipefail
O=gpurun_out/r06_ax
mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
echo done
