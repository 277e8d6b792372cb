#!/bin/bash
# Round 6, call AS: the whole GPU suite once more after the last mesh change,
# then the driver's bench command twice (run-to-run spread of the headline).
set -o pipefail
O=gpurun_out/r06_as
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
echo done
