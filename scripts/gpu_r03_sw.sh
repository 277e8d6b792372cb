#!/bin/bash
# Narrow shard widths on the device (2^16, 2^18): the GPU executor and TopN
# suites at that width (all failures listed), then the mesh GPU tests.
set -o pipefail
mkdir -p gpurun_out/r03_sw
for E in 16 18; do
  PILOSA_SHARD_WIDTH=$E timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider -m gpu --timeout 120 --timeout-method thread -k "not shift and not Shift" tests/test_gpu_executor.py tests/test_gpu_topn_exec.py > gpurun_out/r03_sw/pytest_w$E.log 2>&1
  rc=$?
  echo "width $E rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r03_sw/pytest_w$E.log | tail -15
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mesh.py > gpurun_out/r03_sw/pytest_mesh.log 2>&1 || { tail -c 3000 gpurun_out/r03_sw/pytest_mesh.log; exit 1; }
tail -2 gpurun_out/r03_sw/pytest_mesh.log
