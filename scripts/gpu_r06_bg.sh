#!/bin/bash
# Round 6, call BG: the whole GPU suite a second time on the final code (flake check).
set -o pipefail
O=gpurun_out/r06_bg
mkdir -p $O
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
echo done
