#!/bin/bash
# Round 6, call AZ: re-entry validation of HEAD on a fresh box: whole GPU suite, smoke, driver bench command.
set -o pipefail
O=gpurun_out/r06_az
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -3 $O/pytest_all.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -c 3000 $O/smoke.log; exit 1; }
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.log
echo done
