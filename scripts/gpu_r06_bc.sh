#!/bin/bash
# Round 6, call BC: the width-18 slot-index mismatch: the TopN module alone with and without the
# rank-cache settle, with per-row diagnostics on a mismatch.
set -o pipefail
O=gpurun_out/r06_bc
mkdir -p $O
run() {  # name, extra env
  env PILOSA_SHARD_WIDTH=18 $2 timeout -k 10 300 python3 -u -m pytest -x -s -q -p no:cacheprovider -m gpu --timeout 200 --timeout-method thread tests/test_gpu_topn_exec.py > $O/$1.log 2>&1
  rc=$?
  echo "$1 rc=$rc"; grep -E "SLOTDIFF|SLOTROW|passed|failed" $O/$1.log | cut -c1-1500
  [ $rc -le 1 ] || exit 1
}
run settle "PILOSA_TEST_DUMMY=1"
run nosettle "PILOSA_TEST_NO_SETTLE=1"
echo done
