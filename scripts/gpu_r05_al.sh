#!/bin/bash
# Round 5, call AL: final state (after the Min/Max fold change) -- smoke, the whole GPU suite, the driver's bench.
set -o pipefail
O=gpurun_out/r05_al
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -c 3000 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || { tail -c 6000 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
echo done
